"""Collects (joint state, observation, action, substeps of the step) rows for a task under uniform random actions
(development aid for an action-aware launch order: the step's wait_until_stable length is what orders the launch).
Writes gpurun_out/r5_steps_task<task>.npy: per env and step q[12], qd[12], obs[O], action[A], substeps, reset.
usage: python tools/predict_steps.py task envs steps"""
import os
import sys

import numpy as np

ROOT = __file__.rsplit("/tools/", 1)[0]
sys.path.insert(0, ROOT)
from urgym_amd import layout as LY
from urgym_amd._native import Sim
from urgym_amd.envs import spaces_for
from bench import MAX_STEPS

task, n, steps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
sim = Sim(task, n, seed=20241220)
sim.set_autoreset(True, MAX_STEPS[task])
obs = sim.reset()
act = spaces_for(task)[1]
lo, hi = np.asarray(act.low, np.float64), np.asarray(act.high, np.float64)
rng = np.random.default_rng(0)
rows = []
for t in range(steps):
    s = sim.get_state()
    q, qd = s[:, LY.F_Q:LY.F_Q + 12], s[:, LY.F_QD:LY.F_QD + 12]
    a = rng.uniform(lo, hi, size=(n, len(lo))).astype(np.float32)
    out = sim.step(a)
    d = (out["terminated"] | out["truncated"]).astype(float)
    if t >= 2:
        rows.append(np.concatenate([q, qd, np.asarray(obs, np.float64).reshape(n, -1), a.astype(np.float64),
                                    out["substeps"][:, None].astype(np.float64), d[:, None]], 1))
    obs = out["obs"]
    print("step", t, "substeps p50 / max", int(np.median(out["substeps"])), int(out["substeps"].max()), flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.save(os.path.join(ROOT, "gpurun_out", f"r5_steps_task{task}.npy"), np.concatenate(rows))
print("saved", sum(len(r) for r in rows))
