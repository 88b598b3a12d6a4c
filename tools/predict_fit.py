"""Collects (predictor features, reset-in-next-step) pairs (development aid for the launch-order priority):
per ball, its paddle-frame offset, velocities, height over the paddle and in-plane gravity, before each step of
random actions drawn from the task's action space; then the step's termination.  BallBalance (task 0) writes
gpurun_out/r6_predict_feats.npy (10 features, label, substeps per row); TwoBallsBalance (task 6)
gpurun_out/r5_predict_feats_task6.npy (10 features of ball 1, 10 of ball 2, elapsed steps, paddle vz, label,
substeps).
usage: python tools/predict_fit.py [task] [steps]"""
import os
import sys

import numpy as np

ROOT = __file__.rsplit("/tools/", 1)[0]
sys.path.insert(0, ROOT)
from urgym_amd import layout as LY
from urgym_amd._native import Sim
from urgym_amd.envs import spaces_for
HX, HY = 0.05, 0.1  # the paddle's half extents


def qmat(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


task = int(sys.argv[1]) if len(sys.argv) > 1 else 0
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
nb = 2 if task == 6 else 1
n = 4096
sim = Sim(task, n, seed=20241220)
sim.set_autoreset(True, 500)
sim.reset()
act = spaces_for(task)[1]
lo, hi = np.asarray(act.low, np.float64), np.asarray(act.high, np.float64)
rng = np.random.default_rng(0)
rows = []
for t in range(steps):
    s = sim.get_state()
    p0 = LY.obj(0)
    pp, pq, pv = s[:, p0:p0 + 3], s[:, p0 + 3:p0 + 7], s[:, p0 + 7:p0 + 10]
    feats = np.zeros((n, 10 * nb))
    gw = np.array([0.0, 0.0, -9.81])
    for i in range(n):
        R = qmat(pq[i])
        gl = R.T @ gw  # gravity in the paddle frame (its in-plane part rolls the ball)
        for k in range(nb):
            b0 = LY.obj(1 + k)
            bp, bv = s[i, b0:b0 + 3], s[i, b0 + 7:b0 + 10]
            l = R.T @ (bp - pp[i])
            lv = R.T @ (bv - pv[i])
            feats[i, 10 * k:10 * k + 10] = [abs(l[0]) / HX, abs(l[1]) / HY, l[2], lv[0] * np.sign(l[0]),
                                            lv[1] * np.sign(l[1]), lv[2], bp[2] - pp[i, 2], bv[2],
                                            gl[0] * np.sign(l[0]), gl[1] * np.sign(l[1])]
    extra = np.zeros((n, 0))
    if task == 6:  # the episode's elapsed steps and the paddle's world vertical velocity
        extra = np.stack([sim.get_rng()[1].astype(np.float64), pv[:, 2]], 1)
    out = sim.step(rng.uniform(lo, hi, size=(n, len(lo))).astype(np.float32))
    d = (out["terminated"] | out["truncated"]).astype(float)
    if t >= 5:
        rows.append(np.concatenate([feats, extra, d[:, None], out["substeps"][:, None]], 1))
    print("step", t, "resets", int(d.sum()), flush=True)
name = "r6_predict_feats.npy" if task == 0 else f"r5_predict_feats_task{task}.npy"
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.save(os.path.join(ROOT, "gpurun_out", name), np.concatenate(rows))
print("saved", sum(len(r) for r in rows))
