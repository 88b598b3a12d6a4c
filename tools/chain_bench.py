"""Reset-chain and step-chain timings of one task (development aid for the critical path).

  reset   urgym_reset of every env (the autoreset's chain: robot reset + settling, ~171 substeps on
          BallBalance): ms per call and per reset substep
  step    env-steps with the autoreset off (no reset chains in the launch): ms per launch and per substep
usage: python tools/chain_bench.py [task] [envs]
"""
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from urgym_amd._native import Sim

task = int(sys.argv[1]) if len(sys.argv) > 1 else 0
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
sim = Sim(task, n, seed=20241220)
sim.reset()
sim.sync()
res = []
for r in range(3):
    t0 = time.perf_counter()
    sim.reset()
    sim.sync()
    res.append((time.perf_counter() - t0) * 1e3)
print(f"reset: {np.median(res):.2f} ms per call (reps {[round(x, 2) for x in res]})", flush=True)
sim.set_autoreset(False, 0)
rng = np.random.default_rng(0)
ms, subs = [], []
for t in range(12):
    a = rng.uniform(-0.1, 0.1, size=(n, sim.act_dim)).astype(np.float32)
    sim.sync()
    t0 = time.perf_counter()
    out = sim.step(a)
    sim.sync()
    if t >= 2:
        ms.append((time.perf_counter() - t0) * 1e3)
        subs.append(int(out["substeps"].max()))
print(f"step (no autoreset): {np.median(ms):.2f} ms per launch, max substeps per env {subs}", flush=True)
