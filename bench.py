#!/usr/bin/env python3
"""Headline benchmark: env-steps/sec of URGym/BallBalance-v0 x 4096 envs per MI355X.

Contract:
  python bench.py --gpus N --steps K --warmup W [--reps R] [--task T --envs E]
One process per GPU.  With --gpus N > 1 and no torch.distributed environment, bench.py starts its N
ranks itself (torch.distributed.run, 127.0.0.1) as child processes before any GPU call; under a launcher
WORLD_SIZE must equal N.  A step = one batched env.step() on every env of the rank's shard: IK + joint
motors + wait_until_stable (<= 480 physics substeps) + reward, and the same-step autoreset of finished
episodes (reset cost counted); with N > 1 the per-step returns are all-gathered over RCCL (xGMI).
Actions are synthetic (PCG64 seed 20241220 + rank, uniform in the action space) and resident in HBM
before the timed region; outputs stay in HBM.  Protocol: W untimed warm-up steps, then R
repetitions of K timed steps, each bracketed by barrier + synchronize, time = max over ranks; `value` is
the median repetition.  Rank 0 prints one JSON line.
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
              4: "URGym/CubesPushDiff-v0", 5: "URGym/GolfJoints-v0", 6: "URGym/TwoBallsBalance-v0", 7: "URGym/Box-v0"}
MAX_STEPS = {0: 500, 1: 50, 2: 20, 3: 100, 4: 50, 5: 100, 6: 500, 7: 200}
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E (MI355X_MICROARCH.md)
FP64_VALU_PEAK_TFLOPS = 78.6   # MI355X FP64 vector peak (AMD spec; the path's bounding roofline)


def state_bytes():
    from urgym_amd._native import lib
    return lib().urgym_state_dim() * 8


def cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _oracle_sample(task, n, threads, seconds, flags=0, robot="ur5_robotiq_85"):
    import ctypes
    from oracle.pyoracle import LIB_PATH, LIB_PATH_R140, OracleEnv, lib
    from urgym_amd.envs import spaces_for
    lib_path = LIB_PATH_R140 if robot == "ur5_robotiq_140" else LIB_PATH
    olib = lambda: lib(lib_path)  # noqa: E731
    olib().ugo_set_threads.argtypes = [ctypes.c_int]
    olib().ugo_set_threads(threads)
    envs = [OracleEnv(task, 20241220 + i, lib_path=lib_path, flags=flags) for i in range(n)]
    for e in envs:
        e.reset()
    arr = (ctypes.c_void_p * n)(*[e.h for e in envs])
    A, O = envs[0].act_dim, envs[0].obs_dim
    rng = np.random.default_rng(20241220)
    _, act_space = spaces_for(task)
    alo, ahi = np.asarray(act_space.low, np.float64), np.asarray(act_space.high, np.float64)
    obs = np.zeros((n, O)); rew = np.zeros(n); term = np.zeros(n, np.uint8); succ = np.zeros(n, np.uint8)
    sub = np.zeros(n, np.int32); el = np.zeros(n, np.int32)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    steps = substeps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        act = rng.uniform(alo, ahi, size=(n, A)).astype(np.float32)
        substeps += olib().ugo_batch_step(arr, n, p(act), p(obs), p(rew), p(term), p(succ), p(sub), 1,
                                          MAX_STEPS[task], p(el))
        steps += n
    return steps, substeps, time.perf_counter() - t0


def usable_cores():
    """(cores this process can keep busy, how that was found): the affinity mask, capped by the cgroup v2 CPU quota
    (cpu.max "quota period") -- the GPU box's mask lists the whole machine while its quota is the box's share, and
    threads past the quota only queue"""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, -(-int(q) // int(per)))
            if quota < aff:
                return quota, f"cgroup cpu.max quota {quota} of {aff} affinity cores"
    except (OSError, ValueError):
        pass
    return aff, f"every core of the affinity mask ({aff})"


def cpu_baseline(task, seconds=10.0, seconds_1core=5.0, flags=0, robot="ur5_robotiq_85"):
    """CPU restatement (oracle/, test infrastructure) timed on this host's cores: bounded samples of the same
    workload (same task, random actions, autoreset) -- every core this process may use (usable_cores: the affinity
    mask within the cgroup quota; OpenMP, 4 envs per thread), the 16-thread figure of rounds 2-3 beside it for
    continuity, and the 1-env / 1-core analogue of config A."""
    cores, how = usable_cores()
    n = 4 * cores
    steps, substeps, dt = _oracle_sample(task, n, cores, seconds, flags, robot)
    t16 = min(16, cores)
    s16, sub16, dt16 = _oracle_sample(task, 4 * t16, t16, 0.6 * seconds, flags, robot)
    s1, sub1, dt1 = _oracle_sample(task, 1, 1, seconds_1core, flags, robot)
    return {"value": steps / dt, "unit": "env-steps/s", "cores": cores, "kind": "port",
            "cpu_model": cpu_model(),
            "sample": f"{TASK_NAMES[task]} x {n} envs, {steps} env-steps incl. autoresets ({substeps} substeps) in "
                      f"{dt:.1f}s; C restatement (oracle/), OpenMP {cores} threads ({how})",
            "threads_16": {"value": s16 / dt16, "unit": "env-steps/s", "cores": t16,
                           "sample": f"{4 * t16} envs, {s16} env-steps ({sub16} substeps) in {dt16:.1f}s"},
            "one_core": {"value": s1 / dt1, "unit": "env-steps/s", "cores": 1,
                         "sample": f"1 env, {s1} env-steps ({sub1} substeps) in {dt1:.1f}s, 1 thread"}}


def pmc_traffic(task, n, geometry, contact):
    """HBM bytes per k_step launch from the committed PMC summary of this workload (profiles/traffic_k_step.json,
    tools/pmc_traffic.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes), keyed on (task, envs,
    geometry, contact); a record without a geometry key is a round-2 LOD measurement, one without a contact key a
    vertex-in-hull (rounds 1-3) one."""
    path = os.path.join(ROOT, "profiles", "traffic_k_step.json")
    try:
        t = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    for rec in (t if isinstance(t, list) else [t]):
        if (rec.get("task"), rec.get("envs"), rec.get("geometry", "lod"), rec.get("contact", "vih")) == (task, n, geometry, contact):
            return float(rec["hbm_bytes_per_launch"]), \
                f"profiles/traffic_k_step.json ({rec.get('source', 'rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE')})"
    return None, None


def work_model(task, geometry, contact):
    """FP64 FLOPs per substep / per env-step outside substeps (profiles/work_model.json, tools/opcount.py), counted
    on the restatement in the same geometry and contact mode"""
    try:
        key = ("tasks_full" if geometry == "full" else "tasks") + ("_gjk" if contact == "gjk" else "")
        m = json.load(open(os.path.join(ROOT, "profiles", "work_model.json")))[key][str(task)]
        return float(m["F_sub"]), float(m["F_nonsub_per_env_step"])
    except (OSError, ValueError, KeyError):
        return None, None


def action_stream(kind, rng, lo, hi, T, n):
    """(T, n, A) float64 actions in [lo, hi].  uniform: the benchmark protocol.  ou: per env an
    Ornstein-Uhlenbeck process x += theta (c - x) + sigma sqrt(2 theta) h N(0,1) in units of the half-range h about the
    centre c (theta 0.15, sigma 0.5: lag-1 correlation 0.85, stationary spread half the half-range), clipped.  scaled:
    c + 0.3 (u - c) for u uniform -- a policy-like stream that stays near the centre."""
    A = lo.shape[0]
    c, h = (lo + hi) / 2.0, (hi - lo) / 2.0
    if kind == "uniform":
        return rng.uniform(lo, hi, size=(T, n, A))
    if kind == "scaled":
        return c + 0.3 * (rng.uniform(lo, hi, size=(T, n, A)) - c)
    theta, sigma = 0.15, 0.5
    out = np.empty((T, n, A))
    x = rng.uniform(-0.5, 0.5, size=(n, A))
    for t in range(T):
        x = x + theta * (0.0 - x) + sigma * np.sqrt(2.0 * theta) * rng.standard_normal((n, A))
        out[t] = np.clip(c + h * x, lo, hi)
    return out


def maybe_spawn(args, argv):
    """--gpus N > 1 outside a launcher: start the N ranks as children (before any GPU call) and return their
    exit code; under a launcher, refuse a WORLD_SIZE that disagrees with --gpus.  None: run in-process."""
    world = os.environ.get("WORLD_SIZE")
    if world is None:
        if args.gpus > 1:
            from urgym_amd.parallel import spawn_ranks
            return spawn_ranks(args.gpus, os.path.abspath(__file__), argv)
        return None
    if int(world) != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        return 2
    return None


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--task", type=int, default=0)
    ap.add_argument("--geometry", choices=("full", "lod"), default="full",
                    help="collision geometry: full (default: every vertex of PyBullet's mesh hulls, a true cylinder disc) "
                         "or lod (<= 48-vertex hulls, a 16-gon disc prism: URGYM_FLAG_LOD_GEOMETRY)")
    ap.add_argument("--contact", choices=("gjk", "vih"), default="gjk",
                    help="contact generation: gjk (default: Bullet's convex-convex GJK / EPA pair detector, one new point per "
                         "pair and substep) or vih (rounds 1-3's vertex-in-hull generator: URGYM_FLAG_CONTACT_VIH)")
    ap.add_argument("--robot", choices=("ur5_robotiq_85", "ur5_robotiq_140"), default="ur5_robotiq_85",
                    help="arm + gripper (robot.py): UR5Robotiq85 (every registered env; default) or UR5Robotiq140")
    ap.add_argument("--gather", action="store_true", help="all-gather the returns every step also at N=1 (a process "
                    "group of one rank: RCCL's all-gather timed on one GPU; with N>1 the gather always runs)")
    ap.add_argument("--actions", choices=("uniform", "ou", "scaled"), default="uniform",
                    help="synthetic action stream: uniform in the action space (SURVEY 8(d), the default), ou "
                         "(time-correlated Ornstein-Uhlenbeck around the space's centre, clipped) or scaled (uniform "
                         "shrunk x0.3 about the centre) -- the last two check the launch-order models off-distribution")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--backend", default="nccl", help="nccl (RCCL over xGMI); gloo only to rehearse several ranks "
                                                      "on one GPU (returns gathered through host memory)")
    args = ap.parse_args(argv)
    rc = maybe_spawn(args, argv)
    if rc is not None:
        return rc

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = local % max(torch.cuda.device_count(), 1)  # == local on a node with a GPU per rank
    use_pg = world > 1 or args.gather
    if use_pg:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            from urgym_amd.parallel import free_port
            os.environ["MASTER_PORT"] = str(free_port())
        torch.cuda.set_device(gpu)
        dist.init_process_group(args.backend, rank=rank, world_size=world)
        world = dist.get_world_size()
    dev = torch.device("cuda", gpu)

    from urgym_amd._native import CONTACT_VIH, GEOM_LOD, Sim
    n = args.envs
    geom_flags = (GEOM_LOD if args.geometry == "lod" else 0) | (CONTACT_VIH if args.contact == "vih" else 0)
    sim = Sim(args.task, n, device=gpu, seed=20241220, env_offset=rank * n, flags=geom_flags, robot=args.robot)
    sim.set_autoreset(True, MAX_STEPS[args.task])
    sim.reset()
    A, O = sim.act_dim, sim.obs_dim
    rng = np.random.default_rng(20241220 + rank)
    K, W, R = args.steps, args.warmup, args.reps
    from urgym_amd.envs import spaces_for
    _, act_space = spaces_for(args.task)
    lo, hi = np.asarray(act_space.low, np.float64), np.asarray(act_space.high, np.float64)
    acts = torch.from_numpy(action_stream(args.actions, rng, lo, hi, W + K * R, n).astype(np.float32)).to(dev)
    obs = torch.zeros(n, O, dtype=torch.float64, device=dev)
    fin = torch.zeros_like(obs)
    rew = torch.zeros(n, dtype=torch.float64, device=dev)
    term = torch.zeros(n, dtype=torch.uint8, device=dev)
    trunc = torch.zeros_like(term)
    succ = torch.zeros_like(term)
    sub = torch.zeros(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.ExternalStream(sim.L.urgym_stream(sim.h), device=dev)
    if use_pg:
        from urgym_amd.parallel import ReturnGather
        gat = ReturnGather(n, O, dev)

    def one_step(t, e=None):
        sim.step_device(acts[t].data_ptr(), obs.data_ptr(), fin.data_ptr(), rew.data_ptr(), term.data_ptr(),
                        trunc.data_ptr(), succ.data_ptr(), sub.data_ptr())
        if e is not None:
            e.record(stream)
        if use_pg:
            # every return gathered over RCCL (xGMI) into one preallocated global buffer, global env-id order
            with torch.cuda.stream(stream):
                gat.gather(obs, fin, rew, term, trunc, succ, sub)

    sub_tot = torch.zeros((), dtype=torch.int64, device=dev)
    res_tot = torch.zeros((), dtype=torch.int64, device=dev)
    for t in range(W):
        one_step(t)
        with torch.cuda.stream(stream):  # warm the bookkeeping ops too (first use loads their code objects)
            sub_tot += sub.sum()
            res_tot += (term | trunc).sum()
    sim.sync()
    torch.cuda.synchronize()

    reps = []
    for r in range(R):
        # per-launch HIP events on the handle's stream (the stream k_step runs on); substep / reset counts
        # accumulate on the device, so the timed loop has no host round trip per step
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
        sub_tot.zero_()
        res_tot.zero_()
        torch.cuda.synchronize()
        if use_pg:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(K):
            t = W + r * K + k
            ev[k][0].record(stream)
            one_step(t, ev[k][1])
            with torch.cuda.stream(stream):
                sub_tot += sub.sum()
                res_tot += (term | trunc).sum()
        sim.sync()
        torch.cuda.synchronize()
        if use_pg:
            dist.barrier()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        kern_ms = [a.elapsed_time(b) for a, b in ev]
        vals = torch.tensor([dt, float(sub_tot.item()), float(res_tot.item()), float(np.mean(kern_ms))],
                            dtype=torch.float64, device=dev if args.backend == "nccl" else "cpu")
        if use_pg:
            mx = vals.clone()
            dist.all_reduce(mx, op=dist.ReduceOp.MAX)
            dist.all_reduce(vals, op=dist.ReduceOp.SUM)
            vals[0] = mx[0]
            vals[3] = mx[3]
        reps.append([float(x) for x in vals.tolist()])
        if rank == 0:  # progress on stderr (a long repetition is otherwise silent)
            print(f"[bench] rep {r + 1}/{R}: {reps[-1][0]:.3f} s for {K} steps", file=sys.stderr, flush=True)
    order = sorted(range(R), key=lambda i: reps[i][0])
    med = reps[order[R // 2]]
    dt, substeps, resets, avg_kernel_ms = med
    env_steps = n * K * world
    value = env_steps / dt
    # roofline of the dominant kernel (k_step): FP64 VALU, algorithmic FLOPs per launch from the op-counted
    # restatement (profiles/work_model.json) with this run's substep count, over the HIP-event launch time
    F_sub, F_non = work_model(args.task, args.geometry, args.contact)
    flops_per_launch = None
    if F_sub is not None:
        flops_per_launch = (F_sub * substeps + F_non * env_steps) / (K * world)
    # algorithmic HBM bytes per env-step: state in + out, actions, obs (+final obs), reward, flags, substeps
    S = state_bytes()
    bytes_per_env = 2 * S + 4 * A + 8 * O * 2 + 8 + 3 + 4
    achieved_gbs = bytes_per_env * n / (avg_kernel_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(args.task, n, args.geometry, args.contact)
    if args.robot != "ur5_robotiq_85":  # the PMC record and the work model were measured on the Robotiq-85 build
        traffic, traffic_src = None, None
    if flops_per_launch is not None:
        tf = flops_per_launch / (avg_kernel_ms * 1e-3) / 1e12
        roof = {"bound": "fp64-valu", "achieved": tf, "peak": FP64_VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": tf / FP64_VALU_PEAK_TFLOPS, "traffic": traffic, "traffic_unit": "HBM bytes per launch",
                "traffic_source": traffic_src, "kernel": "k_step", "avg_kernel_ms": avg_kernel_ms,
                "flops_per_launch": flops_per_launch, "flops_per_substep": F_sub,
                "flops_nonsub_per_env_step": F_non, "work_model": "profiles/work_model.json (tools/opcount.py)",
                "hbm": {"achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved_gbs / HBM_PEAK_GBS, "algorithmic_bytes_per_env_step": bytes_per_env}}
    else:
        roof = {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic, "kernel": "k_step",
                "avg_kernel_ms": avg_kernel_ms, "algorithmic_bytes_per_env_step": bytes_per_env,
                "note": "work model missing (profiles/work_model.json): HBM fraction only"}
    line = {
        "metric": ("env-steps/sec at N parallel envs (BallBalance-v0, 4096 envs per MI355X)" if args.task == 0 and n == 4096
                   else f"env-steps/sec at N parallel envs ({TASK_NAMES[args.task].split('/')[1]}, {n} envs per MI355X)"),
        "value": value,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "reps": R,
        "ms_per_step": dt / K * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": f"synthetic: {args.actions} random actions (PCG64 seed 20241220+rank), per-env MT19937 reset draws",
        "config": {"workload": f"{TASK_NAMES[args.task]} x {n} envs per GPU, autoreset, max_episode_steps "
                               f"{MAX_STEPS[args.task]}", "envs_per_gpu": n, "total_envs": n * world,
                   "parallelism": f"env-dp{world}", "world_size": world, "geometry": args.geometry,
                   "contact": args.contact,
                   "backend": args.backend if use_pg else None, "returns_gathered": use_pg, "robot": args.robot,
                   "library": os.path.relpath(sim.L._name, ROOT), "actions": args.actions,
                   "launch_order": "fallback (URGYM_NO_PRIO_MODEL)" if os.environ.get("URGYM_NO_PRIO_MODEL", "0") not in
                                   ("", "0") else "k_prio models"},
        "rep_values": [env_steps / x[0] for x in reps],
        "substeps_per_env_step": substeps / env_steps,
        "resets": int(resets),
        "roofline": roof,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.task, args.cpu_seconds, flags=geom_flags, robot=args.robot)
    if rank == 0:
        print(json.dumps(line), flush=True)
    sim.close()
    if use_pg:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
