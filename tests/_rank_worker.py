"""Rank body for tests/test_distributed.py::test_spawn_ranks_world2 (started by urgym_amd.parallel.spawn_ranks
through torch.distributed.run): each rank builds its shard's returns (values derived from global env ids),
all-gathers them over gloo, and rank 0 writes the gathered batch to the JSON path in argv[1]."""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from urgym_amd.parallel import gather_returns, shard  # noqa: E402


def main():
    out, total, od = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    off, n = shard(total, world, rank)
    ids = torch.arange(off, off + n, dtype=torch.float64)
    obs = ids[:, None] * 10 + torch.arange(od, dtype=torch.float64)[None, :]
    g = gather_returns(obs, ids * 0.5, (ids.long() % 3) == 0, (ids.long() % 5) == 0, final_obs=-obs,
                       success=(ids.long() % 7) == 0, substeps=ids.to(torch.int32) + 10)
    t = gather_returns(obs, ids * 0.5, (ids.long() % 3) == 0, (ids.long() % 5) == 0, as_tuple=True)  # round-3 form
    assert len(t) == 4 and all(torch.equal(a, g[k]) for a, k in zip(t, ("obs", "reward", "terminated", "truncated")))
    if rank == 0:
        json.dump({"world": world, "obs": g["obs"].tolist(), "rew": g["reward"].tolist(), "term": g["terminated"].tolist(),
                   "trunc": g["truncated"].tolist(), "final": g["final_obs"].tolist(), "succ": g["success"].tolist(),
                   "sub": g["substeps"].tolist()}, open(out, "w"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
