"""The convex-convex narrowphase (Bullet's btGjkPairDetector: GJK + EPA), CPU side.

Two implementations of the same restatement exist: the oracle's (oracle/ug_gjk_ref.h, plain C, pointers and
recursion as in Bullet3's btGjkPairDetector / btVoronoiSimplexSolver / btGjkEpa2) and the kernels'
(urgym_amd/csrc/ug_gjk.h: register-resident simplex with explicit selects, EPA in a flat store, the horizon walk on an
explicit stack).  tools/gjk_host.cpp builds the kernels' header for the host with a serial hull support, so this file
can check them against each other bit for bit on the CPU; tests/test_gpu_gjk.py repeats the comparison on MI355X
with the wave-parallel support.

Known answers (the oracle alone): separated spheres, boxes and spheres across a face, a hull against a box along an
axis (the hull's own extreme vertex), the penetration depth of a sphere centre inside a box core (EPA) -- what the
margin-expanded shapes must give whatever the iteration path.  Parity with PyBullet itself is unpinned (pybullet is
absent); these pin the restatement to the geometry it claims.
"""
import ctypes
import math
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BOX, HULL, SPHERE, CYL = 0, 1, 2, 3
DP = ctypes.POINTER(ctypes.c_double)
ARGS = [ctypes.c_int, ctypes.c_int, ctypes.c_int, DP, ctypes.c_double, DP, DP,
        ctypes.c_int, ctypes.c_int, ctypes.c_int, DP, ctypes.c_double, DP, DP, ctypes.c_double, DP]


def _lib(name, fn):
    path = os.path.join(ROOT, "oracle", "_build", name)
    if name == "libugoracle.so" and os.environ.get("URGYM_ORACLE_LIB"):  # tools/oracle_asan.sh's instrumented build
        path = os.environ["URGYM_ORACLE_LIB"]
    L = ctypes.CDLL(path)
    f = getattr(L, fn)
    f.argtypes = ARGS
    f.restype = ctypes.c_int
    return f


@pytest.fixture(scope="module")
def libs():
    return _lib("libugoracle.so", "ugo_gjk_pair"), _lib("libgjk_host.so", "ugk_host_pair")


@pytest.fixture(scope="module")
def model():
    txt = open(os.path.join(ROOT, "urgym_amd", "csrc", "model_data.h")).read()
    M = {}
    for m in re.finditer(r"UG_CONST (int|double) (UG_\w+)\[(\d+)\] = \{([^}]*)\};", txt):
        vals = [float(x) for x in m.group(4).split(",")]
        M[m.group(2)] = np.array(vals, dtype=np.int64 if m.group(1) == "int" else np.float64)
    return M


def _p(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a, a.ctypes.data_as(DP)


def query(f, A, TA, B, TB, thr):
    """A, B: (kind, v0, nv, imp3, margin); TA, TB: (R 3x3, p 3)"""
    keep = []

    def P(x):
        a, p = _p(x)
        keep.append(a)
        return p

    out = np.zeros(7)
    ok = f(A[0], A[1], A[2], P(A[3]), A[4], P(TA[0].ravel()), P(TA[1]),
           B[0], B[1], B[2], P(B[3]), B[4], P(TB[0].ravel()), P(TB[1]), thr, out.ctypes.data_as(DP))
    return ok, out


def rot(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


I3 = np.eye(3)
Z3 = np.zeros(3)


def sphere(r):
    return (SPHERE, 0, 0, Z3, r)


def box(h, m):
    return (BOX, 0, 0, np.asarray(h, float) - m, m)


def cyl(r, hh, m):
    return (CYL, 0, 0, np.array([r - m, r - m, hh - m]), m)


def hulls(model, full):
    k = model["UG_SHAPE_KIND"]
    v0 = model["UG_SHAPE_FV0" if full else "UG_SHAPE_V0"]
    nv = model["UG_SHAPE_FNV" if full else "UG_SHAPE_NV"]
    return [(HULL, int(v0[i]), int(nv[i]), Z3, 0.001) for i in range(len(k)) if k[i] == 1 and nv[i] > 0]


def test_separated_spheres(libs):
    oracle, _ = libs
    rng = np.random.default_rng(3)
    for _ in range(50):
        r1, r2 = rng.uniform(0.005, 0.05, 2)
        u = rng.normal(size=3)
        u /= np.linalg.norm(u)
        gap = rng.uniform(0.0, 0.01)
        cB = rng.uniform(-1, 1, 3)
        cA = cB + u * (r1 + r2 + gap)
        ok, out = query(oracle, sphere(r1), (rot(rng), cA), sphere(r2), (rot(rng), cB), 0.02)
        assert ok
        assert abs(out[6] - gap) < 1e-12
        assert np.allclose(out[:3], u, atol=1e-9)
        assert np.allclose(out[3:6], cB + u * r2, atol=1e-9)


def test_box_sphere_and_box_box_across_a_face(libs):
    oracle, _ = libs
    h = np.array([0.05, 0.1, 0.02])
    for gap in (0.0, 0.0005, 0.003, 0.015):
        # sphere above the +z face, off the face centre
        r = 0.02
        ok, out = query(oracle, sphere(r), (I3, np.array([0.01, -0.03, h[2] + r + gap])), box(h, 0.001), (I3, Z3), 0.02)
        assert ok and abs(out[6] - gap) < 1e-12 and np.allclose(out[:3], [0, 0, 1], atol=1e-12)
        # a smaller box resting face to face (rounded edges do not matter face on)
        g = np.array([0.02, 0.02, 0.02])
        ok, out = query(oracle, box(g, 0.001), (I3, np.array([0.0, 0.0, h[2] + g[2] + gap])), box(h, 0.001), (I3, Z3), 0.02)
        assert ok and abs(out[6] - gap) < 1e-12 and abs(out[2] - 1.0) < 1e-12
    # beyond margins + threshold: no point
    ok, _ = query(oracle, sphere(0.02), (I3, np.array([0, 0, h[2] + 0.02 + 0.05])), box(h, 0.001), (I3, Z3), 0.02)
    assert not ok


def test_sphere_centre_inside_box_core_takes_epa(libs):
    oracle, _ = libs
    h, m, r = np.array([0.05, 0.1, 0.02]), 0.001, 0.01
    for z in (0.002, 0.005, 0.012):
        c = np.array([0.003, -0.002, z])
        ok, out = query(oracle, sphere(r), (I3, c), box(h, m), (I3, Z3), 0.02)
        assert ok
        # nearest core face is +z (core half z = 0.019): depth = (0.019 - z) + m + r of the expanded shapes
        want = -((h[2] - m - z) + m + r)
        assert abs(out[6] - want) < 1e-9, (z, out[6], want)
        assert np.allclose(out[:3], [0, 0, 1], atol=1e-9)


def test_hull_against_box_along_an_axis(libs, model):
    """A robot hull hovering above a box face: the distance is the face's height above the hull's lowest vertex,
    less both margins (the hull's extreme vertex along -z is found by its own support)."""
    oracle, _ = libs
    V = model["UG_HULL_V"].reshape(-1, 3)
    h = np.array([0.5, 0.5, 0.25])
    for H in hulls(model, True)[:6]:
        verts = V[H[1]:H[1] + H[2]]
        zmin = verts[:, 2].min()
        for gap in (0.001, 0.004):
            p = np.array([0.01, 0.02, h[2] - zmin + 0.001 + gap])  # the box margin lies inside its extents
            ok, out = query(oracle, H, (I3, p), box(h, 0.001), (I3, Z3), 0.02)
            assert ok and abs(out[6] - gap) < 1e-9 and abs(out[2] - 1) < 1e-9


def _cases(model, rng, n):
    shapesA = hulls(model, True) + hulls(model, False) + [box([0.03, 0.02, 0.01], 0.001), cyl(0.04, 0.005, 0.0005)]
    shapesB = [box([0.05, 0.1, 0.005], 0.0005), box([0.02, 0.02, 0.02], 0.001), box([0.5, 1.0, 0.25], 0.025),
               sphere(0.02), sphere(0.003), cyl(0.04, 0.005, 0.0005), cyl(0.02, 0.025, 0.002)] + hulls(model, True)[:3]
    V = model["UG_HULL_V"].reshape(-1, 3)
    for k in range(n):
        A = shapesA[rng.integers(len(shapesA))]
        B = shapesB[rng.integers(len(shapesB))]
        RA = I3 if k % 7 == 0 else rot(rng)
        RB = I3 if k % 5 == 0 else rot(rng)
        pB = rng.uniform(-0.5, 0.5, 3)
        # place A near B: along a random direction at about the sum of the two shapes' reaches, +- a few mm
        u = rng.normal(size=3)
        if k % 11 == 0:
            u = np.array([0.0, 0.0, 1.0])
        u /= np.linalg.norm(u)

        def reach(S, R, d):
            dl = R.T @ d
            if S[0] == HULL:
                return float(np.max(V[S[1]:S[1] + S[2]] @ dl)) + S[4]
            if S[0] == SPHERE:
                return S[4]
            if S[0] == BOX:
                return float(np.abs(dl) @ S[3]) + S[4]
            q = math.hypot(dl[0], dl[1])
            return S[3][0] * q + S[3][2] * abs(dl[2]) + S[4]

        d = reach(A, RA, -u) + reach(B, RB, u) + rng.uniform(-0.01, 0.01)
        pA = pB + u * d
        yield A, (RA, pA), B, (RB, pB)


def test_kernel_header_matches_oracle_bit_for_bit(libs, model):
    oracle, host = libs
    rng = np.random.default_rng(2024)
    n_pt = n_pen = 0
    for k, (A, TA, B, TB) in enumerate(_cases(model, rng, 20000)):
        thr = (0.002, 0.004, 0.01)[k % 3]  # 0.02 x the angular-motion discs of the task shapes
        ok1, o1 = query(oracle, A, TA, B, TB, thr)
        ok2, o2 = query(host, A, TA, B, TB, thr)
        assert ok1 == ok2, (A, B, TA, TB)
        if ok1:
            n_pt += 1
            n_pen += o1[6] < -(A[4] + B[4])
            assert np.array_equal(o1, o2), (A[:3], B[:3], o1, o2)
    assert n_pt > 4000 and n_pen > 1000, (n_pt, n_pen)
