"""Block timeline of k_step launches (development aid for the critical path): per block (= env) its
start / end (s_memrealtime, 100 MHz), whether its env reset, its substeps.  Per launch it reports the launch time, the
balanced time (the blocks' summed durations over the slots that ran at once), the substep distribution, and what
list scheduling predicts for three block orders on those slots: the launch order (block index), the blocks sorted
by their measured durations (longest first: the bound any reordering can reach), and sorted by a predictor known
before the launch -- the env's substep count in the previous env-step.
Needs the -DUG_PROF library (tools/build_prof.sh).
usage: python tools/timeline.py [--task 0] [--envs 4096] [--steps 20] [--skip 5] [--json out.json]"""
import argparse
import ctypes
import heapq
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("URGYM_LIB", os.path.join(ROOT, "urgym_amd", "_lib", "liburgym_prof.so"))


def list_schedule(durations, order, slots):
    """makespan of dispatching blocks in `order` onto `slots` identical slots, each to the first free slot"""
    free = [0.0] * slots
    heapq.heapify(free)
    end = 0.0
    for k in order:
        t = heapq.heappop(free) + durations[k]
        end = max(end, t)
        heapq.heappush(free, t)
    return end


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--task", type=int, default=0)
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--skip", type=int, default=5)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from urgym_amd._native import Sim
    from urgym_amd.envs import spaces_for
    n = a.envs
    assert n <= 8192, "the timeline buffer holds 8192 blocks"
    sim = Sim(a.task, n, seed=20241220)
    from bench import MAX_STEPS
    sim.set_autoreset(True, MAX_STEPS[a.task])
    sim.reset()
    act = spaces_for(a.task)[1]
    lo, hi = np.asarray(act.low, np.float64), np.asarray(act.high, np.float64)
    rng = np.random.default_rng(0)
    buf = np.zeros(4 * 8192, np.uint64)
    rows, prev_ns = [], None
    for t in range(a.steps):
        sim.step(rng.uniform(lo, hi, size=(n, len(lo))).astype(np.float32))
        sim.sync()
        assert sim.L.urgym_debug_prof(sim.h, buf.ctypes.data_as(ctypes.c_void_p), 2) == 0
        b = buf[:4 * n].reshape(n, 4).astype(np.int64)
        t0 = b[:, 0].min()
        st, en = (b[:, 0] - t0) / 100.0, (b[:, 1] - t0) / 100.0  # microseconds
        rs = (b[:, 3] >> 16) & 1
        ns = (b[:, 3] & 0xFFFF).astype(np.float64)
        dur = en - st
        if t >= a.skip:
            # slots: the most blocks running at one instant
            ev = np.concatenate([np.stack([st, np.ones(n)], 1), np.stack([en, -np.ones(n)], 1)])
            ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
            slots = int(np.cumsum(ev[:, 1]).max())
            launch = en.max()
            r = {"step": t, "launch_ms": launch / 1e3, "slots": slots,
                 "balanced_ms": dur.sum() / slots / 1e3, "longest_block_ms": dur.max() / 1e3,
                 "resets": int(rs.sum()),
                 "substeps_p50_p90_p99_max": [float(np.percentile(ns, q)) for q in (50, 90, 99)] + [float(ns.max())],
                 "us_per_substep_median": float(np.median(dur / np.maximum(ns, 1))),
                 "sched_launch_order_ms": list_schedule(dur, range(n), slots) / 1e3,
                 "sched_longest_first_ms": list_schedule(dur, np.argsort(-dur, kind="stable"), slots) / 1e3}
            if prev_ns is not None:
                r["sched_prev_substeps_first_ms"] = list_schedule(dur, np.argsort(-prev_ns, kind="stable"), slots) / 1e3
                r["corr_substeps_vs_prev"] = float(np.corrcoef(ns, prev_ns)[0, 1])
            rows.append(r)
            print(json.dumps(r), flush=True)
        prev_ns = ns
    keys = [k for k in rows[0] if isinstance(rows[0][k], float) and k != "step"]
    summary = {"task": a.task, "envs": n, "steps": len(rows),
               "mean": {k: float(np.mean([r[k] for r in rows if k in r])) for k in keys},
               "launches": rows}
    print(json.dumps(summary["mean"]))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(summary, fh, indent=1)


if __name__ == "__main__":
    main()
