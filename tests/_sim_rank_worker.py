"""Rank body for tests/test_gpu_scale.py::test_gloo_ranks_gather_real_sim_outputs (started by
urgym_amd.parallel.spawn_ranks through torch.distributed.run, every rank on GPU 0): each rank steps its shard
[r*n, (r+1)*n) of the batch -- a Sim handle with env_offset r*n -- with its slice of the global action stream,
all-gathers every return over gloo each step (urgym_amd.parallel.ReturnGather, the bench's collective), and
rank 0 saves the gathered batches (obs, final_obs, reward, terminated, truncated, success, substeps per step) to the
.npz path in argv[1]."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from urgym_amd._native import Sim  # noqa: E402
from urgym_amd.parallel import FIELDS, ReturnGather, shard  # noqa: E402


def main():
    out, task, total, steps, max_steps, seed = sys.argv[1], *map(int, sys.argv[2:7])
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    off, n = shard(total, world, rank)
    sim = Sim(task, n, device=0, seed=seed, env_offset=off)
    sim.set_autoreset(True, max_steps)
    sim.reset()
    rng = np.random.default_rng(seed)
    got = {k: [] for k in FIELDS}
    g = ReturnGather(n, sim.obs_dim, "cpu")
    for _ in range(steps):
        act = rng.uniform(-0.1, 0.1, size=(total, sim.act_dim)).astype(np.float32)
        r = sim.step(act[off:off + n])
        g.gather(*(torch.from_numpy(np.asarray(r[k])) for k in FIELDS))
        for k, v in g.decoded().items():
            got[k].append(v.numpy().copy())
    sim.close()
    if rank == 0:
        np.savez(out, world=world, **{k: np.stack(v) for k, v in got.items()})
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
