"""Support-cell tables for the full hulls: an exact, accelerated btConvexHullShape support query.

Bullet's hull support (btConvexHullShape::localGetSupportingVertexWithoutMargin -> btVector3::maxDot) scans every
vertex and keeps the first maximal dot product.  On a full robot hull that is up to 865 dot products per query.  This
tool precomputes, for every hull and every cell of a cube map over the direction sphere, the short list of vertices that
can win that scan for some direction in the cell.  The kernels then dot only the cell's list (<= UG_SC_SLOTS vertices,
one per lane of the query's 16-lane group) and get the same vertex as the full scan, ties included.

Why the list is exact.  A direction d with major axis a (|d_a| the largest component, sign s) and face coordinates
u = d_b / |d_a|, v = d_c / |d_a| falls into cell (i, j) = floor((u + 1) / 2 * K), floor((v + 1) / 2 * K).  The set of
directions the kernels may classify into a cell is contained in the cone spanned by the cell's four corner rays
c_k = s e_a + u_k e_b + v_k e_c, each corner pushed out by GUARD in (u, v) (the kernels classify in FP32: their error is
< 1e-6 in u, v).  A vertex x is left out of the list only if some vertex y dominates it on all four corners:
c_k . (y - x) >= TAU |c_k| for k = 1..4.  Every d in the cone is sum_k lam_k c_k with lam_k >= 0, so
d . (y - x) >= TAU sum_k lam_k |c_k| >= TAU |d|, while the kernels' computed dot products ((x d_x + y d_y) + z d_z, no fma)
are within 3 eps |d| |x|_1 < 1e-15 |d| of the exact ones for these hulls (|x| < 0.5 m).  With TAU = 1e-12 the left-out
vertex's computed dot is strictly below y's: it can neither win nor tie, and the full scan's first maximum is always on
the list.  The list is sorted by vertex index, so the lane group's arg-max (larger dot, then lower index) returns the
full scan's vertex.  Directions the kernels cannot classify (zero, non-finite, |d|_inf outside [1e-30, 1e30]) fall
back to the full scan.  tests/test_supcells.py checks the claim on 1e6 random directions per hull (incl. axis-aligned
and face-boundary directions) against the full scan.

Input: urgym_amd/csrc/model_data.h (or model_data_r140.h); output: supcell_data.h (supcell_data_r140.h) next to it.
Data, not code: read by the kernels (ug_team.h) and by the host build of the GJK header (tools/gjk_host.cpp).
"""
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SLOTS = 16      # one candidate per lane of a GJK lane group
GUARD = 1e-4    # cell enlargement in face coordinates (FP32 classification error < 1e-6)
TAU = 1e-12     # dominance margin per unit |d| (dot-product rounding < 1e-15 |d| for |x| < 0.5 m)
SCAN_TRIP = 128  # vertices one trip of the kernels' full scan covers (8 per lane of a 16-lane group)
OVF = 0xFFFF     # slot 0 of a cell whose list is longer than SLOTS: slot 1 count, slots 2-3 offset (lo, hi) of the list
SAMPLES = 9     # sample directions per cell side whose full-scan supports serve as dominators


def read_model(path):
    txt = open(path).read()
    M = {}
    for m in re.finditer(r"UG_CONST (int|double) (UG_\w+)\[(\d+)\] = \{([^}]*)\};", txt):
        vals = [float(x) for x in m.group(4).split(",")]
        M[m.group(2)] = np.array(vals, dtype=np.int64 if m.group(1) == "int" else np.float64)
    return M


FACE_AX = [(0, 1, 2), (1, 0, 2), (2, 0, 1)]  # major axis a, then the face coordinates' axes (b, c)


def face_dirs(f, u, v):
    """directions of face f (axis f >> 1, sign + for even f) at face coordinates u, v (broadcast arrays)"""
    a, b, c = FACE_AX[f >> 1]
    s = -1.0 if f & 1 else 1.0
    u, v = np.broadcast_arrays(np.asarray(u, float), np.asarray(v, float))
    d = np.zeros(u.shape + (3,))
    d[..., a] = s
    d[..., b] = u
    d[..., c] = v
    return d


def first_max(X, D):
    """btVector3::maxDot's first maximum for each direction (rows of D), the kernels' operation order"""
    dots = (X[None, :, 0] * D[:, None, 0] + X[None, :, 1] * D[:, None, 1]) + X[None, :, 2] * D[:, None, 2]
    return np.argmax(dots, axis=1)  # numpy's argmax returns the first maximum


def cell_lists(X, K):
    """candidate lists (ascending vertex indices) of the 6 K K cells of hull X (n x 3)"""
    n = len(X)
    lists = []
    edges = -1.0 + 2.0 * np.arange(K + 1) / K
    t = np.linspace(0.0, 1.0, SAMPLES)
    for f in range(6):
        for i in range(K):
            for j in range(K):
                u0, u1 = edges[i] - GUARD, edges[i + 1] + GUARD
                v0, v1 = edges[j] - GUARD, edges[j + 1] + GUARD
                C = face_dirs(f, np.array([u0, u1, u0, u1]), np.array([v0, v0, v1, v1]))
                Cn = C / np.linalg.norm(C, axis=1, keepdims=True)
                U, V = np.meshgrid(u0 + (u1 - u0) * t, v0 + (v1 - v0) * t)
                doms = np.unique(first_max(X, face_dirs(f, U.ravel(), V.ravel())))
                alive = np.ones(n, bool)
                P = X @ Cn.T  # n x 4: each vertex's extent along each (unit) corner ray
                for y in doms:
                    # x is dominated by y on every corner: c_k.(y - x) >= TAU |c_k|
                    dom = np.all(P[y][None, :] - P >= TAU, axis=1)
                    alive &= ~dom
                lists.append(np.nonzero(alive)[0])
    return lists


def build(model_path, out_path):
    M = read_model(model_path)
    X = M["UG_HULL_V"].reshape(-1, 3)
    kind, fv0, fnv = M["UG_SHAPE_KIND"], M["UG_SHAPE_FV0"], M["UG_SHAPE_FNV"]
    scb, sck, idx = [], [], []
    report = []
    ovf = []
    for si in range(len(kind)):
        if kind[si] != 1 or fnv[si] <= SCAN_TRIP:  # a box, or a hull the full scan covers in one trip
            scb.append(-1)
            sck.append(0)
            continue
        H = X[fv0[si]:fv0[si] + fnv[si]]
        assert np.abs(H).max() < 0.5, "the rounding bound in the docstring assumes |x| < 0.5 m"
        K = 12 if len(H) > 400 else 8
        L = cell_lists(H, K)
        scb.append(len(idx) // SLOTS)
        sck.append(K)
        counts = np.array([len(c) for c in L])
        for c in L:
            if len(c) <= SLOTS:  # pad with the list's last vertex: a repeated candidate never changes the first maximum
                idx.extend(list(c) + [int(c[-1])] * (SLOTS - len(c)))
            else:
                idx.extend([OVF, len(c), 0, 0] + [0] * (SLOTS - 4))
                ovf.append((len(idx) - SLOTS, c))
        report.append("shape %2d: %3d vertices, K %2d (%4d cells), candidates per cell mean %.2f p99 %d max %d, "
                      "%d cells over %d" % (si, len(H), K, 6 * K * K, counts.mean(), np.percentile(counts, 99),
                                            counts.max(), (counts > SLOTS).sum(), SLOTS))
    for at, c in ovf:  # the long lists after every cell, each padded to whole SLOTS trips
        off = len(idx)
        idx[at + 2], idx[at + 3] = off & 0xFFFF, off >> 16
        n = -(-len(c) // SLOTS) * SLOTS
        idx.extend(list(c) + [int(c[-1])] * (n - len(c)))
    assert max(idx) < 65536
    # each cell's candidates' coordinates, slot by slot (the kernels read a cell's vertices in one memory round; an
    # overflow cell's slots are unused zeros, its long list goes through UG_SC_IDX)
    xyz = []
    for si in range(len(kind)):
        if scb[si] < 0:
            continue
        H = X[fv0[si]:fv0[si] + fnv[si]]
        for c in range(6 * sck[si] * sck[si]):
            sl = idx[(scb[si] + c) * SLOTS:(scb[si] + c + 1) * SLOTS]
            if sl[0] == OVF:
                xyz.extend([0.0] * (3 * SLOTS))
            else:
                for v in sl:
                    xyz.extend(H[v].tolist())
    name = os.path.basename(model_path)
    out = ["/* GENERATED by tools/build_supcells.py from %s. Do not edit. */" % name,
           "/* Support-cell tables of the full hulls (exactness argument: tools/build_supcells.py).  Per shape: the first",
           " * cell (-1: no table) and K (a cube map of 6 K K direction cells); per cell UG_SC_SLOTS vertex indices into the",
           " * hull, ascending, padded by repeating the last; a longer list: slot 0 UG_SC_OVF, slot 1 its length, slots 2-3",
           " * its offset in UG_SC_IDX (low, high 16 bits), the list padded to whole UG_SC_SLOTS trips. */",
           "#ifndef URGYM_SUPCELL_DATA_H", "#define URGYM_SUPCELL_DATA_H",
           "#define UG_SC_SLOTS %d" % SLOTS,
           "#define UG_SC_GUARD %.17g" % GUARD,
           "#define UG_SC_OVF %d" % OVF,
           "UG_CONST int UG_SHAPE_SCB[%d] = {%s};" % (len(scb), ", ".join(map(str, scb))),
           "UG_CONST int UG_SHAPE_SCK[%d] = {%s};" % (len(sck), ", ".join(map(str, sck))),
           "UG_CONST unsigned short UG_SC_IDX[%d] = {%s};" % (len(idx), ", ".join(map(str, idx))),
           "/* per cell (in UG_SC_IDX's cell order): its UG_SC_SLOTS candidates' x y z (zeros for a long list) */",
           "UG_CONST double UG_SC_XYZ[%d] = {%s};" % (len(xyz), ", ".join("%.17g" % x for x in xyz)),
           "#endif"]
    open(out_path, "w").write("\n".join(out) + "\n")
    print("\n".join(report))
    print("%d cells, %d bytes -> %s" % (len(idx) // SLOTS, 2 * len(idx), out_path))


def main():
    csrc = os.path.join(ROOT, "urgym_amd", "csrc")
    which = sys.argv[1:] or ["model_data.h", "model_data_r140.h"]
    for m in which:
        build(os.path.join(csrc, m), os.path.join(csrc, m.replace("model_data", "supcell_data")))


if __name__ == "__main__":
    main()
