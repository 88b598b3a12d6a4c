"""Histogram of the PGS row layouts (n, nnc, nn, nf, nr) and sweep counts of BallBalance's solves, split into
reset settling and env-steps (development aid for the solver's specialised paths).  Uses an
oracle build with -DUG_ROWHIST (oracle/_dev/libugoracle_rowhist.so), whose solves log their layout to fd 2.
usage: python tools/row_hist.py [episodes] [steps]"""
import collections
import os
import sys
import tempfile

import numpy as np

ROOT = __file__.rsplit("/tools/", 1)[0]
sys.path.insert(0, ROOT)
from oracle.pyoracle import OracleEnv

eps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
fd, path = tempfile.mkstemp()
saved = os.dup(2)
os.dup2(fd, 2)
marks = []
task = int(os.environ.get("UG_TASK", "0"))
env = OracleEnv(task, 20241220, lib_path=os.path.join(ROOT, "oracle/_dev/libugoracle_rowhist.so"))
rng = np.random.default_rng(0)
for e in range(eps):
    marks.append(("reset", os.lseek(fd, 0, os.SEEK_CUR)))
    env.reset()
    marks.append(("step", os.lseek(fd, 0, os.SEEK_CUR)))
    for t in range(steps):
        env.step(rng.uniform(-0.1, 0.1, size=env.act_dim))
        if env.terminated():
            break
marks.append(("end", os.lseek(fd, 0, os.SEEK_CUR)))
os.dup2(saved, 2)
data = open(path, "rb").read()
os.unlink(path)
for kind in ("reset", "step"):
    h = collections.Counter()
    sweeps = collections.Counter()
    for (k, a), (_, b) in zip(marks, marks[1:]):
        if k != kind:
            continue
        for line in data[a:b].decode().splitlines():
            if line.startswith("ROWS"):
                v = tuple(map(int, line.split()[1:]))
                h[v[:5]] += 1
                sweeps[v[:5]] += v[5]
    tot = sum(h.values())
    print(f"{kind}: {tot} solves")
    for v, c in h.most_common(15):
        print(f"  n={v[0]:3d} nnc={v[1]:2d} nn={v[2]:2d} nf={v[3]:2d} nr={v[4]:2d}: {c / tot:6.1%}  sweeps {sweeps[v] / c:5.1f}")
