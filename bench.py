#!/usr/bin/env python3
"""Headline benchmark: env-steps/sec of URGym/BallBalance-v0 x 4096 envs per MI355X.

Contract (see DESIGN.md "Measurement"):
  python bench.py --gpus N --steps K --warmup W
One process per GPU (torch.distributed.run for N>1, RCCL all-gather of the
per-step returns).  A step = one batched env.step() on every env of the shard:
IK + joint motors + wait_until_stable (<=480 physics substeps) + reward, and the
same-step autoreset of finished episodes (reset cost counted).  Actions are
synthetic (PCG64 seed 20241220 + rank, uniform in the action space) and are
resident in HBM before the timed region; outputs stay in HBM.  Rank 0 prints
one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

TASK_NAMES = {0: "URGym/BallBalance-v0", 1: "URGym/CubesPush-v0", 2: "URGym/CubesGrasp-v0", 3: "URGym/Golf-v0",
              4: "URGym/CubesPushDiff-v0", 5: "URGym/GolfJoints-v0"}
MAX_STEPS = {0: 500, 1: 50, 2: 20, 3: 100, 4: 50, 5: 100}
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_VALU_PEAK_TFLOPS = 78.6   # MI355X FP64 vector spec


def state_bytes():
    from urgym_amd._native import lib
    return lib().urgym_state_dim() * 8


def cpu_baseline(task, seconds=10.0):
    """CPU restatement (oracle/, test infrastructure) timed on this host's cores: a bounded sample
    of the same workload (same task, random actions, autoreset), OpenMP one env per thread."""
    import ctypes
    from oracle.pyoracle import OracleEnv, lib as olib
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    os.environ["OMP_NUM_THREADS"] = str(threads)
    n = 4 * threads
    envs = [OracleEnv(task, 20241220 + i) for i in range(n)]
    for e in envs:
        e.reset()
    arr = (ctypes.c_void_p * n)(*[e.h for e in envs])
    A, O = envs[0].act_dim, envs[0].obs_dim
    rng = np.random.default_rng(20241220)
    from urgym_amd.envs import spaces_for
    _, act_space = spaces_for(task)
    alo, ahi = np.asarray(act_space.low, np.float64), np.asarray(act_space.high, np.float64)
    obs = np.zeros((n, O)); rew = np.zeros(n); term = np.zeros(n, np.uint8); succ = np.zeros(n, np.uint8)
    sub = np.zeros(n, np.int32); el = np.zeros(n, np.int32)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    steps = 0
    substeps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        act = rng.uniform(alo, ahi, size=(n, A)).astype(np.float32)
        substeps += olib().ugo_batch_step(arr, n, p(act), p(obs), p(rew), p(term), p(succ), p(sub), 1,
                                          MAX_STEPS[task], p(el))
        steps += n
    dt = time.perf_counter() - t0
    return {"value": steps / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"{TASK_NAMES[task]} x {n} envs, {steps} env-steps incl. autoresets "
                      f"({substeps} substeps) in {dt:.1f}s; C restatement (oracle/), OpenMP {threads} threads"}


def pmc_traffic(task, n, K, W):
    """HBM bytes per k_step launch from the committed PMC summary of this same workload
    (profiles/traffic_k_step.json, made by tools/pmc_traffic.py from separate rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes of `bench.py --steps K --warmup W`); None if it does not match."""
    path = os.path.join(ROOT, "profiles", "traffic_k_step.json")
    try:
        t = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    if (t.get("task"), t.get("envs"), t.get("steps"), t.get("warmup")) != (task, n, K, W):
        return None, None
    return float(t["hbm_bytes_per_launch"]), "profiles/traffic_k_step.json (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE)"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--task", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world)
    dev = torch.device("cuda", local)

    from urgym_amd._native import Sim
    n = args.envs
    sim = Sim(args.task, n, device=local, seed=20241220, env_offset=rank * n)
    sim.set_autoreset(True, MAX_STEPS[args.task])
    sim.reset()
    A, O = sim.act_dim, sim.obs_dim
    rng = np.random.default_rng(20241220 + rank)
    K, W = args.steps, args.warmup
    from urgym_amd.envs import spaces_for
    _, act_space = spaces_for(args.task)
    lo, hi = np.asarray(act_space.low, np.float64), np.asarray(act_space.high, np.float64)
    acts = torch.from_numpy(rng.uniform(lo, hi, size=(W + K, n, A)).astype(np.float32)).to(dev)
    obs = torch.zeros(n, O, dtype=torch.float64, device=dev)
    fin = torch.zeros_like(obs)
    rew = torch.zeros(n, dtype=torch.float64, device=dev)
    term = torch.zeros(n, dtype=torch.uint8, device=dev)
    trunc = torch.zeros_like(term)
    succ = torch.zeros_like(term)
    sub = torch.zeros(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.ExternalStream(sim.L.urgym_stream(sim.h), device=dev)

    def one_step(t, e=None):
        sim.step_device(acts[t].data_ptr(), obs.data_ptr(), fin.data_ptr(), rew.data_ptr(), term.data_ptr(),
                        trunc.data_ptr(), succ.data_ptr(), sub.data_ptr())
        if e is not None:
            e.record(stream)
        if world > 1:
            # returns gathered over RCCL (xGMI): obs | reward | terminated | truncated
            from urgym_amd.parallel import gather_returns
            with torch.cuda.stream(stream):
                gather_returns(obs, rew, term, trunc)

    sub_tot = torch.zeros((), dtype=torch.int64, device=dev)
    res_tot = torch.zeros((), dtype=torch.int64, device=dev)
    for t in range(W):
        one_step(t)
        with torch.cuda.stream(stream):  # warm the bookkeeping ops too (first use loads their code objects)
            sub_tot += sub.sum()
            res_tot += (term | trunc).sum()
    sim.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # per-launch HIP events on the handle's stream (the stream k_step runs on); substep / reset counts
    # accumulate on the device, so the timed loop has no host round trip per step
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    sub_tot.zero_()
    res_tot.zero_()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k, t in enumerate(range(W, W + K)):
        ev[k][0].record(stream)
        one_step(t, ev[k][1])
        with torch.cuda.stream(stream):
            sub_tot += sub.sum()
            res_tot += (term | trunc).sum()
    sim.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kern_ms = [a.elapsed_time(b) for a, b in ev]
    substeps = int(sub_tot.item())
    resets = int(res_tot.item())
    dt_t = torch.tensor([dt], dtype=torch.float64, device=dev)
    tot = torch.tensor([float(substeps), float(resets)], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    dt = float(dt_t.item())
    env_steps = n * K * world
    value = env_steps / dt
    avg_kernel_ms = float(np.mean(kern_ms))
    # algorithmic HBM bytes per env-step: state in + out, actions, obs (+final obs), reward, flags, substeps
    S = state_bytes()
    bytes_per_env = 2 * S + 4 * A + 8 * O * 2 + 8 + 3 + 4
    achieved_gbs = bytes_per_env * n / (avg_kernel_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(args.task, n, K, W)
    line = {
        "metric": ("env-steps/sec at N parallel envs (BallBalance-v0, 4096 envs per MI355X)" if args.task == 0 and n == 4096
                   else f"env-steps/sec at N parallel envs ({TASK_NAMES[args.task].split('/')[1]}, {n} envs per MI355X)"),
        "value": value,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": dt / K * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: uniform random actions (PCG64 seed 20241220+rank), per-env MT19937 reset draws",
        "config": {"workload": f"{TASK_NAMES[args.task]} x {n} envs per GPU, autoreset, max_episode_steps "
                               f"{MAX_STEPS[args.task]}", "envs_per_gpu": n, "total_envs": n * world,
                   "parallelism": f"env-dp{world}"},
        "substeps_per_env_step": float(tot[0].item()) / env_steps,
        "resets": int(tot[1].item()),
        "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_unit": "bytes per launch", "traffic_source": traffic_src,
                     "kernel": "k_step", "avg_kernel_ms": avg_kernel_ms,
                     "algorithmic_bytes_per_env_step": bytes_per_env,
                     "note": "path is FP64-VALU/latency bound, not HBM bound (DESIGN.md); PMC traffic in profiles/"},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.task, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(line), flush=True)
    sim.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
