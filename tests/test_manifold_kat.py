"""Known answers for the persistent manifold update (btPersistentManifold [ext]: getCacheEntry, replaceContactPoint,
addManifoldPoint, sortCachedPoints with KEEP_DEEPEST_POINT and gContactCalcArea3Points), on crafted manifolds.

The restatement's manifold_add (oracle/ug_oracle.c) is called through the ugo_manifold_add hook; the expected outcome
is computed here from the rules themselves:
  * a new point whose local point on A lies within the breaking threshold of a cached one replaces the nearest, keeping
    its accumulated impulses (warm start);
  * otherwise it is appended while the manifold has room;
  * into a full manifold (4 points) it replaces point i = argmax |res_i|, where res_i is the squared area spanned with
    the other three (the 3-point cross-product rule), the deepest cached point -- deeper than the new one -- excluded.
The kernels run the same update (ug_team.h manifold_add) and are bit-exact against the restatement in every GPU test.
"""
import ctypes
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def add():
    L = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libugoracle.so"))
    f = L.ugo_manifold_add
    f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_double]
    f.restype = ctypes.c_int

    def run(pts, TA, TB, c, thr):
        buf = np.zeros((4, 13))
        if len(pts):
            buf[:len(pts)] = pts
        ta = np.concatenate([TA[0].ravel(), TA[1]])
        tb = np.concatenate([TB[0].ravel(), TB[1]])
        cc = np.asarray(c, np.float64)
        n = f(buf.ctypes.data, len(pts), ta.ctypes.data, tb.ctypes.data, cc.ctypes.data, thr)
        return buf[:n]
    return run


I3 = np.eye(3)


def point(lpA, dist, imp=(0.0, 0.0, 0.0), n=(0.0, 0.0, 1.0)):
    lpA = np.asarray(lpA, float)
    return np.concatenate([lpA, lpA - np.asarray(n) * dist, n, [dist], imp])


def cross(a, b):
    return np.array([a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]])


def area_rule(pts, new_lpA, new_dist):
    """sortCachedPoints: the slot the new point takes in a full manifold"""
    deepest, pen = -1, new_dist
    for i in range(4):
        if pts[i][9] < pen:
            deepest, pen = i, pts[i][9]
    P = [p[:3] for p in pts]
    combos = {0: (new_lpA - P[1], P[3] - P[2]), 1: (new_lpA - P[0], P[3] - P[2]),
              2: (new_lpA - P[0], P[3] - P[1]), 3: (new_lpA - P[0], P[2] - P[1])}
    res = []
    for i in range(4):
        if i == deepest:
            res.append(0.0)
            continue
        c = cross(*combos[i])
        res.append(c[0] * c[0] + c[1] * c[1] + c[2] * c[2])
    best, bv = -1, -1e30
    for i in range(4):
        if abs(res[i]) > bv:
            best, bv = i, abs(res[i])
    return best, deepest


def new_cand(lpA_world, d, n=(0.0, 0.0, 1.0)):
    """a candidate whose point on A (pB + n d) is lpA_world, with identity transforms"""
    n = np.asarray(n, float)
    pB = np.asarray(lpA_world, float) - n * d
    return np.concatenate([n, pB, [d]])


def test_fifth_point_replaces_by_the_area_rule(add):
    rng = np.random.default_rng(11)
    thr = 0.004
    seen = set()
    for trial in range(400):
        # four cached points spread over a 6 cm patch (pairwise > thr apart), a fifth away from all of them
        while True:
            P = rng.uniform(-0.03, 0.03, (5, 3)) * [1, 1, 0.1]
            if min(np.linalg.norm(P[i] - P[j]) for i in range(5) for j in range(i)) > 2 * thr:
                break
        dist = rng.uniform(-0.004, 0.003, 5)
        pts = [point(P[i], dist[i], imp=(i + 1.0, 10.0 * i, -i)) for i in range(4)]
        c = new_cand(P[4], dist[4])
        out = add(pts, (I3, np.zeros(3)), (I3, np.zeros(3)), c, thr)
        assert len(out) == 4
        lpA = c[3:6] + c[:3] * c[6]  # the point on A as addContactPoint forms it (pB + n d)
        want, deepest = area_rule(pts, lpA, dist[4])
        for i in range(4):
            if i == want:
                assert np.array_equal(out[i][:3], lpA) and out[i][9] == dist[4] and not out[i][10:].any()
            else:
                assert np.array_equal(out[i], pts[i]), (trial, i, want)
        assert want != deepest
        seen.add((want, deepest >= 0))
    assert len(seen) >= 6  # every slot replaced, with and without a deeper cached point


def test_deepest_cached_point_is_kept(add):
    """the deepest cached point survives even when dropping it would give the largest area"""
    thr = 0.004
    P = np.array([[0.0, 0.0, 0], [0.05, 0.0, 0], [0.05, 0.05, 0], [0.0, 0.05, 0]])
    pts = [point(P[i], -0.001) for i in range(4)]
    pts[0][9] = -0.02  # slot 0 deepest
    shallow0 = [np.concatenate([pts[0][:9], [0.0], pts[0][10:]])] + pts[1:]
    rng = np.random.default_rng(5)
    while True:  # a new point for which, without the depth rule, slot 0 would go
        new = np.concatenate([rng.uniform(-0.2, 0.2, 2), [0.0]])
        if np.linalg.norm(P - new, axis=1).min() > thr and area_rule(shallow0, new, -0.001)[0] == 0:
            break
    out = add(pts, (I3, np.zeros(3)), (I3, np.zeros(3)), new_cand(new, -0.001), thr)
    want, deepest = area_rule(pts, new, -0.001)
    assert deepest == 0 and want != 0
    assert np.array_equal(out[0], pts[0]) and np.allclose(out[want][:3], new, atol=1e-16)
    # with the new point the deepest, no cached point is protected: all four areas compete
    out2 = add(pts, (I3, np.zeros(3)), (I3, np.zeros(3)), new_cand(new, -0.05), thr)
    want2, deepest2 = area_rule(pts, new, -0.05)
    assert deepest2 == -1 and np.allclose(out2[want2][:3], new, atol=1e-16)


def test_near_point_replaces_the_nearest_and_keeps_its_impulses(add):
    thr = 0.004
    P = np.array([[0.0, 0.0, 0], [0.01, 0.0, 0], [0.02, 0.0, 0]])
    pts = [point(P[i], -0.001, imp=(1.0 + i, 2.0 + i, 3.0 + i)) for i in range(3)]
    new = np.array([0.011, 0.0005, 0.0])  # within thr of point 1 (nearest) and of no other... and 0.009 from point 0
    out = add(pts, (I3, np.zeros(3)), (I3, np.zeros(3)), new_cand(new, -0.002), thr)
    assert len(out) == 3
    assert np.allclose(out[1][:3], new, atol=1e-16) and out[1][9] == -0.002
    assert np.array_equal(out[1][10:], pts[1][10:])  # warm-start impulses carried over
    assert np.array_equal(out[0], pts[0]) and np.array_equal(out[2], pts[2])
    # two cached points within thr: the nearer wins
    new2 = np.array([0.0052, 0.0, 0.0])
    out = add([point(P[0], -0.001), point([0.008, 0, 0], -0.001, imp=(7, 8, 9))], (I3, np.zeros(3)), (I3, np.zeros(3)),
              new_cand(new2, -0.002), thr)
    assert len(out) == 2 and np.allclose(out[1][:3], new2, atol=1e-16) and np.array_equal(out[1][10:], [7, 8, 9])


def test_append_and_breaking_threshold(add):
    thr = 0.004
    out = add([point([0, 0, 0], -0.001)], (I3, np.zeros(3)), (I3, np.zeros(3)), new_cand([0.02, 0, 0], -0.001), thr)
    assert len(out) == 2 and np.allclose(out[1][:3], [0.02, 0, 0], atol=1e-16)
    # a candidate beyond the breaking threshold is not added (btManifoldResult::addContactPoint)
    out = add([point([0, 0, 0], -0.001)], (I3, np.zeros(3)), (I3, np.zeros(3)), new_cand([0.02, 0, 0], thr * 1.01), thr)
    assert len(out) == 1


def test_local_points_follow_the_transforms(add):
    """the stored local points are the candidate's world points mapped into each body's frame"""
    rng = np.random.default_rng(3)
    for _ in range(50):
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        x, y, z, w = q
        R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                      [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                      [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
        pa, pb = rng.normal(size=3), rng.normal(size=3)
        n = rng.normal(size=3)
        n /= np.linalg.norm(n)
        c = np.concatenate([n, rng.normal(size=3), [-0.001]])
        out = add([], (R, pa), (I3, pb), c, 0.004)
        wA = c[3:6] + n * c[6]
        assert np.allclose(R @ out[0][:3] + pa, wA, atol=1e-14) and np.allclose(out[0][3:6] + pb, c[3:6], atol=1e-14)
