"""The restatement alone (CPU) on tests/test_gpu_failures.py's crafted states: the arm folded into the table in both
contact modes (manifold and row capacity overflow, the 480-substep cap, the split pass), the deep folds the coordinate-velocity
clamp keeps finite, an absurd joint velocity that ends at the non-finite guard, a cube sunk into the table.  Each case checks the counter it targets, as the GPU test does.  These
are the states tools/oracle_asan.sh runs under AddressSanitizer / UBSan (make -C oracle asan), where every capacity
branch, clamp and NaN path of oracle/ug_oracle.c executes with bounds and undefined-behaviour checks."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import test_gpu_failures as F  # noqa: E402  (its POSES / _fold; its tests stay GPU-marked there)


def _run(task, edits, action, flags=0):
    from oracle.pyoracle import OracleEnv
    out = []
    for i, edit in enumerate(edits):
        r = OracleEnv(task, F.SEED + i, flags=flags)
        r.reset()
        st = r.get_state()
        edit(st)
        r.set_state(st)
        s0 = np.asarray(r.stats(), np.int64).copy()
        o, rew, term, succ, ns = r.step(np.asarray(action, np.float32))
        out.append((np.asarray(o), int(r.flags()), np.asarray(r.stats(), np.int64) - s0, ns))
    return out


@pytest.mark.parametrize("task", [0, 1])
def test_oracle_manifold_capacity_overflow(task):
    res = _run(task, [F._fold(*p) for p in F.POSES[task]], np.zeros(3))
    d = np.array([r[2] for r in res])
    assert (d[:, F.MANCAP] > 0).sum() >= 3 and all(r[1] & F.FLAG_DROPPED for r in res), d.tolist()
    assert (d[:, F.SPLIT] > 0).all()
    assert all(np.all(np.isfinite(r[0])) for r in res)


@pytest.mark.parametrize("task", [0, 1])
def test_oracle_row_capacity_overflow_vih(task):
    res = _run(task, [F._fold(*p) for p in F.POSES_VIH[task]], np.zeros(3), flags=F.CONTACT_VIH)
    d = np.array([r[2] for r in res])
    assert (d[:, F.MANCAP] > 0).sum() >= 3 and (d[:, F.ROWCAP] > 0).sum() >= 4, d.tolist()
    assert (d[:, F.UNSTABLE] > 0).any()


def test_oracle_nonfinite_guard():
    res = _run(0, [F._spin(5, 1e200), F._spin(0, 1e200)], np.zeros(3))
    for o, fl, d, ns in res:
        assert fl & F.FLAG_NONFINITE and d[F.NONFINITE] == 1 and ns == 1, (fl, d.tolist(), ns)
        assert not np.all(np.isfinite(o))


def test_oracle_deep_folds_stay_finite():
    """the folds that ran away in round 4: btMultiBody's coordinate-velocity clamp (+-100, every dof, after
    the force step and after the solve) bounds them; they end at the 480 cap with finite states"""
    res = _run(0, [F._fold(0.5, 2.5), F._fold(1.0, 2.0)], np.zeros(3))
    for o, fl, d, ns in res:
        assert np.all(np.isfinite(o)) and not fl & F.FLAG_NONFINITE, (fl, d.tolist())
        assert ns == 480 and fl & F.FLAG_UNSTABLE


def test_oracle_split_impulse():
    from urgym_amd import layout as LY

    def sink(dz):
        def e(s):
            s[LY.obj(0) + 2] = dz
        return e
    (o0, f0, d0, _), (o1, f1, d1, _) = _run(1, [sink(-0.03), sink(0.019)], np.zeros(3))
    assert d0[F.SPLIT] >= 1 and d1[F.SPLIT] == 0
