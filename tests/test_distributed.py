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
    from urgym_amd.parallel import ReturnGather, shard
    off, n = shard(total, world, rank)
    ids = torch.arange(off, off + n, dtype=torch.float64)
    obs = ids[:, None] * 10 + torch.arange(obs_dim, dtype=torch.float64)[None, :]
    rew = ids * 0.5
    term = (ids.long() % 3) == 0
    trunc = (ids.long() % 5) == 0
    # the bench's form: one ReturnGather, several steps through the same preallocated buffers
    g = ReturnGather(n, obs_dim, "cpu")
    for step in range(3):
        v = g.gather(obs + step, -obs, rew, term, trunc, (ids.long() % 7) == 0, ids.to(torch.int32) + step)
    d = g.decoded()
    assert v["obs"].data_ptr() == g.recv.data_ptr()  # views of the preallocated buffer
    if rank == 0:
        q.put({k: x.numpy().copy() for k, x in d.items()})
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
    d = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ids = np.arange(total)
    obs = ids[:, None] * 10.0 + np.arange(od)[None, :]
    assert np.array_equal(d["obs"], obs + 2) and np.array_equal(d["final_obs"], -obs)
    assert np.array_equal(d["reward"], ids * 0.5)
    assert np.array_equal(d["terminated"], ids % 3 == 0) and np.array_equal(d["truncated"], ids % 5 == 0)
    assert np.array_equal(d["success"], ids % 7 == 0) and np.array_equal(d["substeps"], ids + 2)


def test_spawn_ranks_world2(tmp_path):
    """parallel.spawn_ranks (what `bench.py --gpus 2` uses) starts 2 ranks through torch.distributed.run;
    their gathered returns come back in global env-id order."""
    import json

    import numpy as np
    from urgym_amd.parallel import spawn_ranks
    out = tmp_path / "gathered.json"
    total, od = 12, 4
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_rank_worker.py")
    rc = spawn_ranks(2, worker, [str(out), str(total), str(od)])
    assert rc == 0
    g = json.load(open(out))
    ids = np.arange(total)
    assert g["world"] == 2
    assert np.array_equal(np.array(g["obs"]), ids[:, None] * 10.0 + np.arange(od)[None, :])
    assert np.array_equal(np.array(g["rew"]), ids * 0.5)
    assert np.array_equal(np.array(g["term"]), ids % 3 == 0) and np.array_equal(np.array(g["trunc"]), ids % 5 == 0)
    assert np.array_equal(np.array(g["final"]), -(ids[:, None] * 10.0 + np.arange(od)[None, :]))
    assert np.array_equal(np.array(g["succ"]), ids % 7 == 0) and np.array_equal(np.array(g["sub"]), ids + 10)


def test_bench_gpus_flag_spawns_or_refuses(monkeypatch):
    """bench.py --gpus N: outside a launcher it starts N ranks itself (before any GPU call); under a launcher a
    WORLD_SIZE that disagrees with --gpus is refused; --gpus 1 runs in-process."""
    import importlib
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    bench = importlib.import_module("bench")
    import urgym_amd.parallel as par
    calls = []
    monkeypatch.setattr(par, "spawn_ranks", lambda n, script, argv: calls.append((n, script, list(argv))) or 0)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    argv = ["--gpus", "2", "--steps", "3"]
    assert bench.main(argv) == 0
    assert calls == [(2, os.path.abspath(bench.__file__), argv)]
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert bench.main(["--gpus", "2"]) == 2
    monkeypatch.delenv("WORLD_SIZE")
    args = type("A", (), {"gpus": 1})()
    assert bench.maybe_spawn(args, []) is None
