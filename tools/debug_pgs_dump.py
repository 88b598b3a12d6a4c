"""Debug aid (GPU, needs a -DUG_DEBUG_DUMP build in URGYM_LIB): compare one substep's PGS internals
(Delassus rows A, w after the warm start, w and impulses after the sweeps) between the HIP kernel and
the CPU restatement, for every env of a small batch.  Usage: URGYM_LIB=... python tools/debug_pgs_dump.py"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from urgym_amd._native import Sim, lib  # noqa: E402
from oracle.pyoracle import OracleEnv, lib as olib  # noqa: E402
from urgym_amd.envs import spaces_for  # noqa: E402

M = 128


def main():
    task, n, T = 0, 64, 3
    seed = 20241220
    sim = Sim(task, n, seed=seed)
    sim.set_autoreset(True, 500)
    sim.reset()
    _, asp = spaces_for(task)
    rng = np.random.default_rng(seed)
    for t in range(T):
        sim.step(rng.uniform(asp.low, asp.high, size=(n, len(asp.low))).astype(np.float32))
    st = sim.get_state()
    sim.substep()
    wsd = lib().urgym_debug_ws_doubles()
    dbg_off = wsd - (M * M + 8 * M)
    ref = OracleEnv(task, seed)
    dbg = (ctypes.c_int * 8)()
    A = np.zeros((M, M))
    w4 = np.zeros(4 * M)
    ws = np.zeros(wsd)
    for i in range(n):
        ref.set_state(st[i])
        ref.substep()
        olib().ugo_debug_rows(dbg)
        olib().ugo_debug_pgs(A.ctypes.data_as(ctypes.c_void_p), w4.ctypes.data_as(ctypes.c_void_p))
        lib().urgym_debug_workspace(sim.h, i, ws.ctypes.data_as(ctypes.c_void_p), wsd)
        d = ws[dbg_off:]
        nr = dbg[0]
        GA = d[:M * M].reshape(M, M).T  # dbg[J*128 + row] = A[row][J]
        p = min(nr, 96)
        badA = np.argwhere(GA[:nr, :p] != A[:nr, :p])
        w0 = d[M * M:M * M + M]
        wf = d[M * M + M:M * M + 2 * M]
        imp = d[M * M + 2 * M:M * M + 3 * M]
        msg = []
        if len(badA):
            msg.append(f"A differs at {len(badA)} entries, first {badA[:4].tolist()}")
        if not np.array_equal(w0[:nr], w4[:nr]):
            msg.append(f"w(warm) differs at {np.nonzero(w0[:nr] != w4[:nr])[0][:8].tolist()}")
        if not np.array_equal(wf[:nr], w4[M:M + nr]):
            msg.append(f"w(final) differs at {np.nonzero(wf[:nr] != w4[M:M + nr])[0][:8].tolist()}")
        if not np.array_equal(imp[:nr], w4[2 * M:2 * M + nr]):
            msg.append(f"imp differs at {np.nonzero(imp[:nr] != w4[2 * M:2 * M + nr])[0][:8].tolist()}")
        print(f"env {i} shape {tuple(dbg[:7])}: " + ("OK" if not msg else "; ".join(msg)))


if __name__ == "__main__":
    main()
