"""Debug aid (GPU): find the first substep where the HIP path and the CPU restatement diverge.

Runs a few batched env-steps on the GPU, then single substeps (k_substep) from the GPU state, each
checked against the oracle's substep from the same input state.  Prints the first mismatching
(env, substep) with the oracle's PGS shape (rows per kind, sweeps, split sweeps) and the differing
state fields.  Usage: python tools/debug_substeps.py [task] [n_envs] [steps] [substeps]
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from urgym_amd._native import Sim  # noqa: E402
from oracle.pyoracle import OracleEnv, lib as olib  # noqa: E402
from urgym_amd.envs import spaces_for  # noqa: E402


def main():
    task = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    T = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    K = int(sys.argv[4]) if len(sys.argv) > 4 else 60
    seed = 20241220
    sim = Sim(task, n, seed=seed)
    sim.set_autoreset(True, 500)
    sim.reset()
    _, asp = spaces_for(task)
    rng = np.random.default_rng(seed)
    for t in range(T):
        sim.step(rng.uniform(asp.low, asp.high, size=(n, len(asp.low))).astype(np.float32))
    ref = OracleEnv(task, seed)
    dbg = (ctypes.c_int * 8)()
    bad = 0
    shapes = {}
    for k in range(K):
        st = sim.get_state()
        sim.substep()
        st2 = sim.get_state()
        for i in range(n):
            ref.set_state(st[i])
            ref.substep()
            olib().ugo_debug_rows(dbg)
            shp = tuple(dbg[:7])
            key = (shp[0] > 64, shp[0] > 96, shp[6] > 0)
            shapes[key] = shapes.get(key, 0) + 1
            o = ref.get_state()
            if not np.array_equal(o, st2[i]):
                d = np.nonzero(o != st2[i])[0]
                print(f"substep {k} env {i}: shape n,nnc,nn,nf,nr,sweeps,split = {shp}; "
                      f"{len(d)} fields differ, first {d[:8].tolist()}, max |d| {np.abs(o - st2[i]).max():.3e}")
                bad += 1
                if bad > 12:
                    print("shapes seen:", shapes)
                    return 1
    print("shapes seen (n>64, n>96, split):", shapes)
    print("all substeps bit-identical" if bad == 0 else f"{bad} mismatches")
    return 0 if bad == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
