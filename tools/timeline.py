"""Block timeline of one k_step launch (development aid for the critical path): per block its
start / end (s_memrealtime, 100 MHz), whether its env reset, its substeps.  Prints when the launch's last
blocks end and what they were, the reset blocks' start times, and the step-only blocks' spread.
Needs the -DUG_PROF library (tools/build_prof.sh).  usage: python tools/timeline.py [envs] [steps]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("URGYM_LIB", os.path.join(ROOT, "urgym_amd", "_lib", "liburgym_prof.so"))
from urgym_amd._native import Sim

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
sim = Sim(0, n, seed=20241220)
sim.set_autoreset(True, 500)
sim.reset()
rng = np.random.default_rng(0)
buf = np.zeros(4 * 8192, np.uint64)
agg = []
for t in range(steps):
    sim.step(rng.uniform(-0.1, 0.1, size=(n, 3)).astype(np.float32))
    sim.sync()
    assert sim.L.urgym_debug_prof(sim.h, buf.ctypes.data_as(ctypes.c_void_p), 2) == 0
    b = buf[:4 * n].reshape(n, 4).astype(np.int64)
    t0 = b[:, 0].min()
    st, en = (b[:, 0] - t0) / 100.0, (b[:, 1] - t0) / 100.0  # microseconds
    rs = (b[:, 3] >> 16) & 1
    ns = b[:, 3] & 0xFFFF
    if t < 5:
        continue
    last = np.argsort(-en)[:8]
    rb = np.nonzero(rs)[0]
    agg.append((en.max(), len(rb), en[rs == 0].max() if (rs == 0).any() else 0.0,
                en[rb].max() if len(rb) else 0.0, st[rb].max() if len(rb) else 0.0))
    print(f"step {t}: launch {en.max() / 1e3:.2f} ms, resets {len(rb)}, step-only blocks end by "
          f"{agg[-1][2] / 1e3:.2f} ms, reset blocks end by {agg[-1][3] / 1e3:.2f} ms; latest reset start "
          f"{agg[-1][4] / 1e3:.2f} ms (block {int(rb[np.argmax(st[rb])]) if len(rb) else -1}); reset chain "
          f"durations ms median {np.median(en[rb] - st[rb]) / 1e3 if len(rb) else 0:.2f} max "
          f"{(en[rb] - st[rb]).max() / 1e3 if len(rb) else 0:.2f}; last 8 blocks (block, reset, substeps, start ms): "
          f"{[(int(k), int(rs[k]), int(ns[k]), round(st[k] / 1e3, 2)) for k in last[:4]]}", flush=True)
a = np.array(agg)
print("mean launch ms", a[:, 0].mean() / 1e3, "mean step-only end", a[:, 2].mean() / 1e3, "mean reset end",
      a[:, 3].mean() / 1e3)
