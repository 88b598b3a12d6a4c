"""Collects (predictor features, reset-in-next-step) pairs on BallBalance x 4096 (development aid for the
launch-order priority): paddle-frame ball offset now and extrapolated, height over the paddle, velocities."""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from urgym_amd import layout as LY
from urgym_amd._native import Sim
sys.path.insert(0, __file__.rsplit("/", 1)[0])
from predict_quality import qmat, HX, HY

n = 4096
sim = Sim(0, n, seed=20241220)
sim.set_autoreset(True, 500)
sim.reset()
rng = np.random.default_rng(0)
rows = []
for t in range(40):
    s = sim.get_state()
    p0, b0 = LY.obj(0), LY.obj(1)
    feats = np.zeros((n, 10))
    for i, st in enumerate(s):
        pp, pq, pv, pw = st[p0:p0 + 3], st[p0 + 3:p0 + 7], st[p0 + 7:p0 + 10], st[p0 + 10:p0 + 13]
        bp, bv = st[b0:b0 + 3], st[b0 + 7:b0 + 10]
        R = qmat(pq)
        l = R.T @ (bp - pp)
        lv = R.T @ (bv - pv)
        gl = R.T @ np.array([0.0, 0.0, -9.81])  # gravity in the paddle frame (its in-plane part rolls the ball)
        feats[i] = [abs(l[0]) / HX, abs(l[1]) / HY, l[2], lv[0] * np.sign(l[0]), lv[1] * np.sign(l[1]), lv[2],
                    bp[2] - pp[2], bv[2], gl[0] * np.sign(l[0]), gl[1] * np.sign(l[1])]
    out = sim.step(rng.uniform(-0.1, 0.1, size=(n, 3)).astype(np.float32))
    d = (out["terminated"] | out["truncated"]).astype(float)
    if t >= 5:
        rows.append(np.concatenate([feats, d[:, None], out["substeps"][:, None]], 1))
np.save("gpurun_out/r6_predict_feats.npy", np.concatenate(rows))
print("saved", sum(len(r) for r in rows))
