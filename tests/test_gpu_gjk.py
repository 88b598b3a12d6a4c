"""The kernels' convex-convex narrowphase on MI355X (ug_gjk.h through urgym_debug_gjk: one wave per query, the hull
support as a lane-strided max-dot + DPP arg-max) against the oracle's independent restatement (oracle/ug_gjk_ref.h),
bit for bit, on the same randomised shape pairs tests/test_gjk.py runs on the CPU: robot hulls (full and LOD), boxes,
spheres and cylinders at poses within a centimetre of contact, separated and penetrating (EPA)."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import test_gjk as T  # noqa: E402


def pack(A, TA, B, TB, thr):
    q = []
    for S, (R, p) in ((A, TA), (B, TB)):
        q += [S[0], S[1], S[2], *np.asarray(S[3], float), S[4], *np.asarray(R, float).ravel(), *np.asarray(p, float)]
    q.append(thr)
    assert len(q) == 39
    return q


@pytest.mark.parametrize("task", [None, 3], ids=["gjk16", "gjk8"])
def test_gpu_gjk_matches_oracle(built, task):
    """task None: the default library (16-lane groups); task 3 (Golf): liburgym_g8.so, the 8-lane build the Golf tasks
    load (two cell candidates per lane, half-row reductions, the GJK / EPA stores in the hull-candidate LDS union)"""
    from urgym_amd._native import lib, ptr
    oracle = T._lib("libugoracle.so", "ugo_gjk_pair")
    import re
    txt = open(os.path.join(T.ROOT, "urgym_amd", "csrc", "model_data.h")).read()
    model = {}
    for m in re.finditer(r"UG_CONST (int|double) (UG_\w+)\[(\d+)\] = \{([^}]*)\};", txt):
        vals = [float(x) for x in m.group(4).split(",")]
        model[m.group(2)] = np.array(vals, dtype=np.int64 if m.group(1) == "int" else np.float64)
    rng = np.random.default_rng(2024)
    cases = list(T._cases(model, rng, 4000))
    thrs = [(0.002, 0.004, 0.01)[k % 3] for k in range(len(cases))]
    q = np.array([pack(A, TA, B, TB, thr) for (A, TA, B, TB), thr in zip(cases, thrs)], np.float64)
    out = np.zeros((len(cases), 7))
    ok = np.zeros(len(cases), np.int32)
    assert lib(task=task).urgym_debug_gjk(len(cases), ptr(q), ptr(out), ptr(ok)) == 0
    n_pt = n_pen = 0
    for k, ((A, TA, B, TB), thr) in enumerate(zip(cases, thrs)):
        r, o = T.query(oracle, A, TA, B, TB, thr)
        assert r == ok[k], (k, A[:3], B[:3])
        if r:
            n_pt += 1
            n_pen += o[6] < -(A[4] + B[4])
            assert np.array_equal(o, out[k]), (k, A[:3], B[:3], o, out[k])
    assert n_pt > 800 and n_pen > 150, (n_pt, n_pen)
