"""How well the launch-order priority (ug_team.h team_priority) predicts BallBalance's same-step resets
(development aid): before each step the predictor is recomputed from the state, envs are ranked
as k_order ranks them, and the ranks of the envs that then reset are reported (a reset dispatched in the first
1024 blocks starts its chain at once; later ones start a block-round later)."""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from urgym_amd import layout as LY
from urgym_amd._native import Sim

HX, HY, HZ, DT = 0.05, 0.1, 0.005, 1.0 / 240.0


def qmat(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def prio(s, f_scale=10.0, T=24.0 * DT):
    out = np.zeros(len(s), int)
    for i, st in enumerate(s):
        p0, b0 = LY.obj(0), LY.obj(1)
        pp, pq, pv = st[p0:p0 + 3], st[p0 + 3:p0 + 7], st[p0 + 7:p0 + 10]
        bp, bv = st[b0:b0 + 3], st[b0 + 7:b0 + 10]
        R = qmat(pq)
        f = 0.0
        for k in range(2):
            l = R.T @ ((bp - pp) + (bv - pv) * T * k)
            g = max(abs(l[0]) / HX, abs(l[1]) / HY)
            if l[2] < HZ:
                g = max(g, 1.0)
            f = max(f, g)
        out[i] = min(14, max(0, int(f * f_scale)))
    return out


n = 4096
sim = Sim(0, n, seed=20241220)
sim.set_autoreset(True, 500)
sim.reset()
rng = np.random.default_rng(0)
for t in range(25):
    s = sim.get_state()
    p = prio(s)
    order = np.argsort(-p, kind="stable")
    rank = np.empty(n, int)
    rank[order] = np.arange(n)
    out = sim.step(rng.uniform(-0.1, 0.1, size=(n, 3)).astype(np.float32))
    d = (out["terminated"] | out["truncated"]).astype(bool)
    r = np.sort(rank[d])
    if t >= 5:
        print(t, "resets", int(d.sum()), "rank<256", int((r < 256).sum()), "<512", int((r < 512).sum()), "<1024",
              int((r < 1024).sum()), "max rank", int(r.max()) if len(r) else -1,
              "prio hist of resets", np.bincount(p[d], minlength=15).tolist(), flush=True)
