"""Debug aid (GPU): replay a crafted env-step substep by substep on the device.

tests/test_gpu_failures.py's folded arm: the crafted state is set on both sides, the oracle runs the whole env-step
with its substep trace on (ugo_trace: the state before every wait_until_stable substep), then the GPU runs one
substep (urgym_substep) from every traced state and is compared with the next traced state; at the first mismatch
the oracle's convex-convex queries of that substep are replayed one wave each (urgym_debug_gjk).
Usage: python tools/debug_gjk.py [task] [q1] [q2] [seed offset]"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from urgym_amd._native import Sim, lib, ptr  # noqa: E402
from urgym_amd import layout as LY  # noqa: E402
from oracle.pyoracle import OracleEnv  # noqa: E402


def main():
    task = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    q1 = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
    q2 = float(sys.argv[3]) if len(sys.argv) > 3 else 2.5
    seed = 20241220 + (int(sys.argv[4]) if len(sys.argv) > 4 else 0)
    sim = Sim(task, 1, seed=seed)
    sim.reset()
    ref = OracleEnv(task, seed)
    ref.reset()
    st = sim.get_state()[0]
    st[LY.F_Q + 1] = q1
    st[LY.F_Q + 2] = q2
    st[LY.F_QD:LY.F_QD + 12] = 0.0
    ref.set_state(st)
    L = ref.L
    for f, a, r in (("ugo_gjk_record", [ctypes.c_int], None), ("ugo_gjk_records", [ctypes.c_void_p, ctypes.c_int], ctypes.c_int),
                    ("ugo_trace", [ctypes.c_int], None), ("ugo_traced", [ctypes.c_void_p, ctypes.c_int], ctypes.c_int)):
        getattr(L, f).argtypes = a
        getattr(L, f).restype = r
    L.ugo_trace(1)
    o, rew, term, succ, ns = ref.step(np.zeros(ref.act_dim, np.float32))
    L.ugo_trace(0)
    tr = np.zeros((600, len(st)))
    nt = L.ugo_traced(tr.ctypes.data_as(ctypes.c_void_p), 600)
    final = ref.get_state()
    print(f"oracle step: {ns} substeps, {nt} traced, obs {o}, flags {ref.flags()}", flush=True)
    for k in range(nt):
        nxt = tr[k + 1] if k + 1 < nt else final
        sim.set_state(tr[k][None, :])
        sim.substep()
        g = sim.get_state()[0]
        same = np.array_equal(g, nxt, equal_nan=True)
        if not same or k % 20 == 0:
            print(f"substep {k}: state equal {same}; oracle finite {np.all(np.isfinite(nxt))}, gpu finite {np.all(np.isfinite(g))}", flush=True)
        if not same:
            d = np.nonzero(~((g == nxt) | (np.isnan(g) & np.isnan(nxt))))[0]
            print("  differing fields:", d[:60])
            ref.set_state(tr[k])
            L.ugo_gjk_record(1)
            ref.substep()
            rec = np.zeros((512, 47))
            nq = L.ugo_gjk_records(rec.ctypes.data_as(ctypes.c_void_p), 512)
            L.ugo_gjk_record(0)
            q = np.ascontiguousarray(rec[:nq, :39])
            out = np.zeros((nq, 7))
            ok = np.zeros(nq, np.int32)
            assert lib().urgym_debug_gjk(nq, ptr(q), ptr(out), ptr(ok)) == 0
            for i in range(nq):
                if ok[i] != rec[i, 39] or (ok[i] and not np.array_equal(out[i], rec[i, 40:47])):
                    print("  query", i, "kinds", rec[i, 0], rec[i, 19], "oracle", rec[i, 39:47], "gpu", ok[i], out[i])
            print("  nman gpu/oracle", g[LY.F_NMAN], nxt[LY.F_NMAN])
            for m in range(int(max(g[LY.F_NMAN], nxt[LY.F_NMAN]))):
                b = LY.F_MAN + m * LY.MAN_DOUBLES
                print("   man", m, "gpu", g[b:b + 2], g[b + 2:b + 2 + 13], "oracle", nxt[b:b + 2], nxt[b + 2:b + 2 + 13])
            break


if __name__ == "__main__":
    main()
