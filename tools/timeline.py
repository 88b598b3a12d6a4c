"""Block timeline of k_step launches (development aid for the critical path): per env, by its position
in the launch order, its start / end (s_memrealtime, 100 MHz), whether it reset, its substeps, and where it ran (XCD,
SIMD: the placement view below -- dispatch gaps on each SIMD, per-XCD work).  Per launch it reports the launch time, the
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


def placement(b, st, en, dur):
    """where the blocks ran (word 3: XCC_ID in bits 20-23, HW_ID in 32-63: SIMD 4-5, CU 8-11, SH 12, SE 13-15): per XCD
    its blocks, work and slots; list scheduling of each XCD's own blocks in block order on its own slots (the launch if
    the dispatcher deals blocks round-robin to the XCDs and each fills its slots greedily); and the dispatch delay --
    a block's start minus the end of the block that ran before it on the same SIMD"""
    xcc = (b[:, 3] >> 20) & 15
    hw = (b[:, 3] >> 32) & 0xFFFFFFFF
    slot = (xcc << 16) | ((hw >> 4) & 0xFFF)
    n = len(st)
    out = {"xcds": int(len(np.unique(xcc)))}
    mod = np.arange(n) % 8
    agree = sum(int(np.max(np.bincount(xcc[mod == m], minlength=16))) for m in range(8))
    out["blockidx_mod8_same_xcd_frac"] = agree / n
    per, ends = [], []
    for x in np.unique(xcc):
        sel = np.nonzero(xcc == x)[0]
        s, e = st[sel], en[sel]
        ev = np.concatenate([np.stack([s, np.ones(len(sel))], 1), np.stack([e, -np.ones(len(sel))], 1)])
        ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
        sl = int(np.cumsum(ev[:, 1]).max())
        per.append(list_schedule(dur[sel], np.arange(len(sel)), sl))
        ends.append(e.max())
        out.setdefault("xcd_blocks", []).append(int(len(sel)))
        out.setdefault("xcd_slots", []).append(sl)
        out.setdefault("xcd_work_per_slot_ms", []).append(float(dur[sel].sum() / sl / 1e3))
        out.setdefault("xcd_end_ms", []).append(float(e.max() / 1e3))
    out["sched_per_xcd_ms"] = float(max(per) / 1e3)
    gaps = []
    for k in np.unique(slot):
        sel = np.nonzero(slot == k)[0]
        sel = sel[np.argsort(st[sel])]
        if len(sel) > 1:
            gaps.extend((st[sel[1:]] - en[sel[:-1]]).tolist())
    g = np.asarray(gaps) if gaps else np.zeros(1)
    out["simd_slots"] = int(len(np.unique(slot)))
    out["dispatch_gap_us_mean_p99_max"] = [float(g.mean()), float(np.percentile(g, 99)), float(g.max())]
    out["dispatch_gap_total_ms_per_slot"] = float(g.sum() / max(1, len(np.unique(slot))) / 1e3)
    return out


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
    rows, prev_ns, prev_cls = [], None, None
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
                 "work_ms": float(dur.sum() / 1e3),  # the blocks' summed durations (co-runner contention A/B)
                 "reset_us_per_substep_median": float(np.median((dur / np.maximum(ns, 1))[rs == 1])) if rs.any() else 0.0,
                 "cus_used": int(len(np.unique(((b[:, 3] >> 20) & 15) << 16 | ((b[:, 3] >> 40) & 0xFF)))),
                 "sched_launch_order_ms": list_schedule(dur, range(n), slots) / 1e3,
                 "sched_longest_first_ms": list_schedule(dur, np.argsort(-dur, kind="stable"), slots) / 1e3}
            if prev_ns is not None:
                r["sched_prev_substeps_first_ms"] = list_schedule(dur, np.argsort(-prev_ns, kind="stable"), slots) / 1e3
                r["corr_substeps_vs_prev"] = float(np.corrcoef(ns, prev_ns)[0, 1])
            r.update(placement(b, st, en, dur))
            # the launch order against the resets: their positions (a reset placed past the first `slots` envs
            # starts its chain only when a slot frees), and the priority classes this launch was ordered by
            # (word 3 bits 24-31: the level the env had when this launch was ordered; 16 bands)
            kr = np.nonzero(rs)[0]
            r["reset_pos_past_slots"] = int((kr >= slots).sum())
            r["reset_pos_max"] = int(kr.max()) if len(kr) else -1
            if prev_cls is not None:
                cls = ((b[:, 3] >> 24) & 255) >> 4  # the level this launch was ordered by, in 16 bands
                r["class_hist"] = np.bincount(cls, minlength=16).tolist()
                r["reset_class_hist"] = np.bincount(cls[rs == 1], minlength=16).tolist()
                fresh = prev_rs[b[:, 2]] == 1  # the env reset in the last launch: its episode's first step now
                r["fresh_envs_resets"] = [int(fresh.sum()), int((fresh & (rs == 1)).sum())]
                r["fresh_class_hist"] = np.bincount(cls[fresh], minlength=16).tolist()
            rows.append(r)
            print(json.dumps(r), flush=True)
        cur = np.zeros(n, np.int64)
        cur[b[:, 2]] = (b[:, 3] >> 24) & 255
        prev_cls = cur
        prev_rs = np.zeros(n, np.int64)
        prev_rs[b[:, 2]] = rs
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
