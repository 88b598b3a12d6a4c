import sys, numpy as np
sys.path.insert(0, '/root/repo')
from urgym_amd._native import Sim
n = 4096
sim = Sim(0, n, seed=20241220)
sim.set_autoreset(True, 500)
sim.reset()
rng = np.random.default_rng(0)
for t in range(12):
    out = sim.step(rng.uniform(-0.1, 0.1, size=(n, 3)).astype(np.float32))
    s = out["substeps"]; d = out["terminated"] | out["truncated"]
    print(t, "max", s.max(), "p99", np.percentile(s, 99), "p50", np.median(s), "resets", int(d.sum()),
          "max(no reset)", s[~d.astype(bool)].max() if (~d.astype(bool)).any() else -1, "max(reset)", s[d.astype(bool)].max() if d.any() else -1)
