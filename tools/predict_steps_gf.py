"""Collects Golf step-length rows under uniform random actions (development aid for its launch order; no result
depends on the order).  Per env and step, before the step: state[0:80] (q, qd, motor targets / enables, object
active flags, the objects' pos / quat / v / w), the task words state[945:949], the elapsed steps, the step's action;
after it: substeps and the reset flag.  Writes gpurun_out/r6_steps_task<task>.npy (float32, the first 4096 envs,
steps after a 10-step warm-up).
usage: python tools/predict_steps_gf.py [task=3] [envs=8192] [steps=40]"""
import os
import sys

import numpy as np

ROOT = __file__.rsplit("/tools/", 1)[0]
sys.path.insert(0, ROOT)
from urgym_amd import layout as LY  # noqa: E402
from urgym_amd._native import Sim  # noqa: E402
from urgym_amd.envs import spaces_for  # noqa: E402
from bench import MAX_STEPS  # noqa: E402


def main():
    task = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    sim = Sim(task, n, seed=20241220)
    sim.set_autoreset(True, MAX_STEPS[task])
    sim.reset()
    act = spaces_for(task)[1]
    lo, hi = np.asarray(act.low, np.float64), np.asarray(act.high, np.float64)
    rng = np.random.default_rng(0)
    keep = min(n, 4096)
    rows = []
    for t in range(steps):
        s = sim.get_state()
        el = sim.get_rng()[1]
        a = rng.uniform(lo, hi, size=(n, len(lo))).astype(np.float32)
        out = sim.step(a)
        d = (out["terminated"] | out["truncated"]).astype(np.float64)
        if t >= 10:
            rows.append(np.concatenate([s[:keep, 0:LY.F_NMAN], s[:keep, LY.F_TASK:LY.F_TASK + 4],
                                        el[:keep, None].astype(np.float64), a[:keep].astype(np.float64),
                                        out["substeps"][:keep, None].astype(np.float64), d[:keep, None]], 1)
                        .astype(np.float32))
        print("step", t, "substeps p50 / max", int(np.median(out["substeps"])), int(out["substeps"].max()), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.save(os.path.join(ROOT, "gpurun_out", f"r6_steps_task{task}.npy"), np.concatenate(rows))
    print("saved", sum(len(r) for r in rows))


if __name__ == "__main__":
    main()
