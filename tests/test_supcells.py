"""The accelerated hull support (support-cell tables, tools/build_supcells.py) returns the full scan's vertex.

btConvexHullShape's support is btVector3::maxDot: the first maximal dot product over every hull vertex.  The kernels dot
only the candidates of the direction's cube-map cell.  These tests run the host build of the same lookup
(tools/gjk_host.cpp: ug_supcell.h's classification, the generated tables) against the full scan on >= 1e6 directions per
full hull -- random, axis-aligned, on cell and cube-face boundaries, at extreme scales, zero and non-finite -- and pin
the C full scan itself to numpy on a sample.  The tables are data generated from model_data.h: a stale table (a hull
changed without re-running the tool) fails here.
"""
import ctypes
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import build_supcells as B  # noqa: E402

N_DIRS = 1_000_000


ROBOTS = {"r85": ("libgjk_host.so", "model_data.h", "supcell_data.h"),
          "r140": ("libgjk_host_r140.so", "model_data_r140.h", "supcell_data_r140.h")}


def _host(lib):
    L = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", lib))
    L.ugk_host_support.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    L.ugk_host_cell.argtypes = [ctypes.c_double] * 3 + [ctypes.c_int]
    L.ugk_host_cell.restype = ctypes.c_int
    return L


@pytest.fixture(scope="module")
def host():
    return _host(ROBOTS["r85"][0])


@pytest.fixture(scope="module")
def model():
    return B.read_model(os.path.join(ROOT, "urgym_amd", "csrc", "model_data.h"))


def tabled(model, table="supcell_data.h"):
    txt = open(os.path.join(ROOT, "urgym_amd", "csrc", table)).read()
    scb = [int(x) for x in txt.split("UG_SHAPE_SCB[")[1].split("{")[1].split("}")[0].split(",")]
    return [si for si, b in enumerate(scb) if b >= 0]


def support(host, si, dirs, table):
    dirs = np.ascontiguousarray(dirs, np.float64)
    out = np.empty(len(dirs), np.int32)
    host.ugk_host_support(si, 1 if table else 0, len(dirs), dirs.ctypes.data, out.ctypes.data)
    return out


def directions(rng, n):
    """a mix that stresses the classification: random, near-axis, on cell / face boundaries, extreme scales, special"""
    parts = [rng.normal(size=(n * 6 // 10, 3))]
    # near-axis: one dominant component, the others 0 or tiny (the flat faces' ties sit here)
    m = n // 10
    ax = np.zeros((m, 3))
    ax[np.arange(m), rng.integers(0, 3, m)] = rng.choice([-1.0, 1.0], m) * rng.uniform(0.1, 10, m)
    ax += rng.normal(size=(m, 3)) * (10.0 ** rng.integers(-18, -3, (m, 1))) * rng.integers(0, 2, (m, 3))
    parts.append(ax)
    # exactly on (or one rounding off) cell edges of K = 8 and 12, on a random cube face
    m = n // 10
    f = rng.integers(0, 6, m)
    K = rng.choice([8, 12], m)
    ei = rng.integers(0, K + 1)
    u = -1.0 + 2.0 * ei / K + rng.choice([0.0, 1e-16, -1e-16, 1e-9], m)
    v = rng.uniform(-1, 1, m)
    sw = rng.integers(0, 2, m).astype(bool)
    u, v = np.where(sw, v, u), np.where(sw, u, v)
    fd = np.empty((m, 3))
    for face in range(6):
        k = f == face
        fd[k] = B.face_dirs(face, u[k], v[k])
    parts.append(fd * rng.uniform(0.01, 100, (m, 1)))
    # equal magnitudes in two or three components (cube-face boundaries)
    m = n // 10
    t = rng.uniform(0.1, 10, m)
    e = np.stack([t, t * rng.choice([-1.0, 1.0], m), rng.uniform(-1, 1, m) * t], 1)
    e[: m // 4, 2] = -t[: m // 4]  # a quarter with all three magnitudes equal (a cube corner)
    parts.append(np.take_along_axis(e, np.argsort(rng.uniform(size=(m, 3)), 1), 1))
    # extreme scales, inside and outside the tables' [1e-30, 1e30] range
    m = n - sum(len(p) for p in parts) - 8
    parts.append(rng.normal(size=(m, 3)) * 10.0 ** rng.uniform(-40, 40, (m, 1)))
    parts.append(np.array([[0, 0, 0], [-0.0, 0, 0], [np.nan, 1, 0], [1, np.inf, 0], [-np.inf, 0, 0], [1e-300, 0, 0],
                           [5e-324, -5e-324, 0], [1e308, -1e308, 1e308]]))
    return np.concatenate(parts)


def test_tables_are_current(tmp_path):
    """the committed tables are what tools/build_supcells.py generates from the committed model headers"""
    for m in ("model_data.h", "model_data_r140.h"):
        out = tmp_path / m.replace("model_data", "supcell_data")
        B.build(os.path.join(ROOT, "urgym_amd", "csrc", m), str(out))
        assert out.read_text() == open(os.path.join(ROOT, "urgym_amd", "csrc", out.name)).read(), m


def test_classification_lands_in_the_enlarged_cell(host):
    """the FP32 cell of a direction contains it once the cell is enlarged by UG_SC_GUARD (what the tables assume)"""
    rng = np.random.default_rng(7)
    D = directions(rng, 100_000)
    D = D[np.all(np.isfinite(D), 1)]
    for K in (8, 12):
        for d in D[:: 7]:
            c = host.ugk_host_cell(d[0], d[1], d[2], K)
            a = np.abs(d)
            if not (a.max() >= 1e-30 and a.max() <= 1e30):
                assert c == -1
                continue
            f, i, j = c // (K * K), (c // K) % K, c % K
            ax, b, cc = B.FACE_AX[f >> 1]
            m = abs(d[ax])
            assert m == a.max() and (d[ax] < 0) == bool(f & 1)
            u, v = d[b] / m, d[cc] / m
            lo = -1.0 + 2.0 * np.array([i, j]) / K - B.GUARD
            hi = -1.0 + 2.0 * (np.array([i, j]) + 1) / K + B.GUARD
            assert lo[0] <= u <= hi[0] and lo[1] <= v <= hi[1], (d, K, c, u, v)


@pytest.mark.parametrize("robot", ["r85", "r140"])
def test_cell_support_equals_full_scan(robot):
    """>= 1e6 directions per full hull (both robots' builds): the cell's candidates give the full scan's first maximum
    (bit-identical index)"""
    lib, mh, th = ROBOTS[robot]
    host = _host(lib)
    model = B.read_model(os.path.join(ROOT, "urgym_amd", "csrc", mh))
    X = model["UG_HULL_V"].reshape(-1, 3)
    rng = np.random.default_rng(2025)
    shapes = tabled(model, th)
    assert len(shapes) >= 6
    for si in shapes:
        D = directions(rng, N_DIRS)
        a = support(host, si, D, True)
        b = support(host, si, D, False)
        bad = np.nonzero(a != b)[0]
        assert len(bad) == 0, (si, len(bad), D[bad[:5]], a[bad[:5]], b[bad[:5]])
        # the C full scan against numpy's first maximum, same operation order, on a sample of finite directions
        S = D[np.all(np.isfinite(D), 1)][:20_000]
        H = X[model["UG_SHAPE_FV0"][si]:model["UG_SHAPE_FV0"][si] + model["UG_SHAPE_FNV"][si]]
        assert np.array_equal(B.first_max(H, S), support(host, si, S, False)), si


def test_ties_resolve_to_the_lowest_index(host, model):
    """directions normal to a flat face of a hull (many exactly tied vertices): the table keeps every tied vertex and the
    lowest index wins, as in maxDot"""
    X = model["UG_HULL_V"].reshape(-1, 3)
    n_tied = 0
    for si in tabled(model):
        H = X[model["UG_SHAPE_FV0"][si]:model["UG_SHAPE_FV0"][si] + model["UG_SHAPE_FNV"][si]]
        D = np.concatenate([np.eye(3), -np.eye(3)])
        dots = (H[None, :, 0] * D[:, None, 0] + H[None, :, 1] * D[:, None, 1]) + H[None, :, 2] * D[:, None, 2]
        n_tied += int(((dots == dots.max(1, keepdims=True)).sum(1) > 1).sum())
        assert np.array_equal(support(host, si, D, True), np.argmax(dots, 1)), si
    assert n_tied > 0  # some axis directions hit exact ties on these meshes


@pytest.mark.parametrize("robot", ["r85", "r140"])
def test_inline_coordinates_are_the_listed_vertices(robot):
    """the kernels read a cell's candidates' coordinates from UG_SC_XYZ (the host build reads UG_SC_IDX): slot by slot
    they are the listed vertices' coordinates, bit for bit"""
    import re
    _, mh, th = ROBOTS[robot]
    model = B.read_model(os.path.join(ROOT, "urgym_amd", "csrc", mh))
    X = model["UG_HULL_V"].reshape(-1, 3)
    txt = open(os.path.join(ROOT, "urgym_amd", "csrc", th)).read()

    def arr(name, dt):
        m = re.search(r"%s\[\d+\] = \{([^}]*)\}" % name, txt)
        return np.array([float(x) for x in m.group(1).split(",")], dt)
    scb, sck = arr("UG_SHAPE_SCB", np.int64), arr("UG_SHAPE_SCK", np.int64)
    idx, xyz = arr("UG_SC_IDX", np.int64), arr("UG_SC_XYZ", np.float64).reshape(-1, B.SLOTS, 3)
    for si in np.nonzero(scb >= 0)[0]:
        H = X[model["UG_SHAPE_FV0"][si]:model["UG_SHAPE_FV0"][si] + model["UG_SHAPE_FNV"][si]]
        for c in range(scb[si], scb[si] + 6 * sck[si] ** 2):
            sl = idx[c * B.SLOTS:(c + 1) * B.SLOTS]
            if sl[0] != B.OVF:
                assert np.array_equal(xyz[c], H[sl]), (si, c)
