"""Per-step substep distribution of BallBalance x 4096 (development aid): the launch time is the longest env
chain, so the max with / without a same-step autoreset matters more than the mean."""
import sys
import time

import numpy as np

sys.path.insert(0, '/root/repo')
from urgym_amd._native import Sim

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
task = int(sys.argv[2]) if len(sys.argv) > 2 else 0
sim = Sim(task, n, seed=20241220)
sim.set_autoreset(True, 500)
sim.reset()
rng = np.random.default_rng(0)
A = sim.act_dim
for t in range(30):
    a = rng.uniform(-0.1, 0.1, size=(n, A)).astype(np.float32)
    sim.sync()
    t0 = time.perf_counter()
    out = sim.step(a)
    sim.sync()
    ms = (time.perf_counter() - t0) * 1e3
    s = out["substeps"]
    d = (out["terminated"] | out["truncated"]).astype(bool)
    print(t, f"{ms:6.1f} ms", "sum", int(s.sum()), "max", s.max(), "p99", np.percentile(s, 99), "p50", np.median(s),
          "resets", int(d.sum()), "max(no reset)", s[~d].max() if (~d).any() else -1,
          "max(reset)", s[d].max() if d.any() else -1, "mean(reset)", round(float(s[d].mean()), 1) if d.any() else -1,
          flush=True)
