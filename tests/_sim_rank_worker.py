"""Rank body for tests/test_gpu_scale.py::test_ranks_gather_real_sim_outputs (started by
urgym_amd.parallel.spawn_ranks through torch.distributed.run, every rank on GPU 0): each rank steps its shard
[r*n, (r+1)*n) of the batch -- a Sim handle with env_offset r*n -- with its slice of the global action stream,
all-gathers every return each step (urgym_amd.parallel.ReturnGather, the bench's collective), and
rank 0 saves the gathered batches (obs, final_obs, reward, terminated, truncated, success, substeps per step) to the
.npz path in argv[1].  argv[7] (optional) is the backend: gloo (default: returns gathered through host memory) or
nccl (RCCL: the returns in device tensors on the rank's GPU, gathered from HBM -- the production branch)."""
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
    backend = sys.argv[7] if len(sys.argv) > 7 else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group(backend)
    rank, world = dist.get_rank(), dist.get_world_size()
    off, n = shard(total, world, rank)
    sim = Sim(task, n, device=0, seed=seed, env_offset=off)
    sim.set_autoreset(True, max_steps)
    sim.reset()
    rng = np.random.default_rng(seed)
    got = {k: [] for k in FIELDS}
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    g = ReturnGather(n, sim.obs_dim, dev)
    assert g.send.device.type == dev.type
    for _ in range(steps):
        act = rng.uniform(-0.1, 0.1, size=(total, sim.act_dim)).astype(np.float32)
        r = sim.step(act[off:off + n])
        g.gather(*(torch.from_numpy(np.asarray(r[k])).to(dev) for k in FIELDS))
        for k, v in g.decoded().items():
            got[k].append(v.cpu().numpy().copy())
    sim.close()
    if rank == 0:
        np.savez(out, world=world, backend=backend, **{k: np.stack(v) for k, v in got.items()})
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
