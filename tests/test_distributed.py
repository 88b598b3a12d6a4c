"""Multi-process (world_size 2, gloo, CPU) coverage of the sharded path: shard bookkeeping and the
per-step all-gather of returns, which must reassemble the global batch in env-id order."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, obs_dim, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from urgym_amd.parallel import gather_returns, shard
    off, n = shard(total, world, rank)
    ids = torch.arange(off, off + n, dtype=torch.float64)
    obs = ids[:, None] * 10 + torch.arange(obs_dim, dtype=torch.float64)[None, :]
    rew = ids * 0.5
    term = (ids.long() % 3) == 0
    trunc = (ids.long() % 5) == 0
    o, r, t, tr = gather_returns(obs, rew, term, trunc)
    if rank == 0:
        q.put((o.numpy(), r.numpy(), t.numpy(), tr.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_bounds():
    from urgym_amd.parallel import shard
    assert shard(65536, 8, 3) == (3 * 8192, 8192)
    with pytest.raises(ValueError):
        shard(10, 3, 0)


def test_gather_returns_world2_gloo():
    import numpy as np
    world, total, od = 2, 16, 6
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, od, q)) for r in range(world)]
    for p in procs:
        p.start()
    o, r, t, tr = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ids = np.arange(total)
    assert np.array_equal(o, ids[:, None] * 10.0 + np.arange(od)[None, :])
    assert np.array_equal(r, ids * 0.5)
    assert np.array_equal(t, ids % 3 == 0) and np.array_equal(tr, ids % 5 == 0)
