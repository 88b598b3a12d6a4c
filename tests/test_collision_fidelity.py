"""The collision-fidelity builds of the restatement (tools/collision_fidelity.py, oracle/ug_fidelity.h): the
Bullet SAT-polyhedral narrowphase (the sat variant) pinned by box-box known answers (face contact: 4 clipped corners at the penetration
depth; edge-edge: one contact at the crossing), and every variant steps each task family with finite state.
These builds measure the product's collision substitutes (profiles/collision_fidelity.json);
they need the reference meshes, so the module skips where /root/reference is absent (the GPU box)."""
import ctypes
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.skipif(not os.path.isdir("/root/reference/urgym"), reason="needs the reference meshes")


@pytest.fixture(scope="module")
def fid():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import collision_fidelity as cf
    src = os.path.join(ROOT, "oracle", "ug_oracle.c")
    if not all(os.path.exists(p) and os.path.getmtime(p) >= os.path.getmtime(src) for p in cf.LIBS.values()):
        cf.build()
    return cf


def _rot(axis, ang):
    a = np.asarray(axis, float) / np.linalg.norm(axis)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * K @ K


def _box_box(fid, ha, Ra, pa, hb, Rb, pb, thr=0.02):
    L = ctypes.CDLL(fid.LIBS["sat"])
    P = ctypes.c_void_p
    L.ugo_fid_box_box.argtypes = [P] * 6 + [ctypes.c_double, P, ctypes.c_int]
    arrs = [np.ascontiguousarray(x, np.float64) for x in (ha, Ra, pa, hb, Rb, pb)]
    out = np.zeros((64, 7))
    n = L.ugo_fid_box_box(*[a.ctypes.data_as(P) for a in arrs], thr, out.ctypes.data_as(P), 64)
    return out[:n]


def test_face_contact_clips_the_incident_face(fid):
    # A (0.1 cube half 0.05) resting 1 mm into B (a slab) -- A's bottom face is the incident face
    c = _box_box(fid, [0.05] * 3, np.eye(3), [0, 0, 0.05 - 0.001], [0.5, 0.5, 0.05], np.eye(3), [0, 0, -0.05])
    assert len(c) == 4
    np.testing.assert_allclose(c[:, :3], [[0, 0, 1]] * 4, atol=1e-12)    # normal on B towards A
    np.testing.assert_allclose(c[:, 6], [-0.001] * 4, atol=1e-12)         # penetration depth
    np.testing.assert_allclose(np.sort(np.abs(c[:, 3:5]).ravel()), [0.05] * 8, atol=1e-12)  # A's corners
    np.testing.assert_allclose(c[:, 5], [0.0] * 4, atol=1e-12)            # on B's top face


def test_edge_edge_contact(fid):
    # A rotated 45 deg about x, B rotated 45 deg about y: A's bottom edge (along x) crosses B's top edge (along y)
    h = [0.05] * 3
    e = 0.05 * np.sqrt(2.0)
    c = _box_box(fid, h, _rot([1, 0, 0], np.pi / 4), [0, 0, e + e - 0.0005], h, _rot([0, 1, 0], np.pi / 4), [0, 0, 0])
    assert len(c) >= 1
    # the edge-edge point: at the crossing, on B's edge, along the axis, at the penetration depth (the clipped
    # face points that accompany it are no deeper)
    k = int(np.argmin(np.linalg.norm(c[:, 3:6] - [0, 0, e], axis=1)))
    np.testing.assert_allclose(c[k, 3:6], [0, 0, e], atol=1e-9)
    np.testing.assert_allclose(c[k, :3], [0, 0, 1], atol=1e-9)
    np.testing.assert_allclose(c[k, 6], -0.0005, atol=1e-9)
    assert c[:, 6].min() >= -0.0005 - 1e-12


def test_separated_boxes_give_nothing(fid):
    c = _box_box(fid, [0.05] * 3, np.eye(3), [0, 0, 0.2], [0.05] * 3, np.eye(3), [0, 0, 0], thr=0.02)
    assert len(c) == 0


@pytest.mark.parametrize("task", [0, 2, 3])
def test_variants_step_finite(fid, task):
    from oracle.pyoracle import OracleEnv
    e0 = OracleEnv(task, 1000)
    e0.reset()
    s0 = e0.get_state()
    acts = fid.actions(task, 2, 3)
    for v in ("lod", "vih", "sat"):
        e = OracleEnv(task, 1000, lib_path=fid.LIBS.get(v), flags=fid.FLAGS.get(v, 0))
        e.set_state(s0)
        for a in acts:
            e.step(a)
        assert np.all(np.isfinite(e.get_state()))
