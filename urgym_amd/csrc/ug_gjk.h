/* ug_gjk.h -- Bullet3's default convex-convex narrowphase as the kernels run it (one wavefront per pair).
 *
 * What it restates [ext, Bullet3; the CPU statement of the same algorithm is
 * oracle/ug_gjk_ref.h, a separate implementation that the kernels match bit for bit]:
 *   btGjkPairDetector::getClosestPointsNonVirtual (BT_USE_DOUBLE_PRECISION): a libccd-style intersection test of the
 *   core shapes, the classic margin GJK over btVoronoiSimplexSolver, btGjkEpaPenetrationDepthSolver (btGjkEpa2's GJK +
 *   EPA, 9 guess directions, ::Distance as fallback) when the cores intersect or the GJK degenerates, the
 *   normal-direction fix, and the one point btConvexConvexAlgorithm hands to btManifoldResult::addContactPoint.
 *
 * How it runs on CDNA4: every lane of the env's wavefront executes the same (uniform) scalar chain, so the wave is
 * one pair's solver; the only wave-parallel step is the hull support query (max-dot over up to 865 vertices), which
 * the includer supplies as ugk_hull_support(shape, d) (ug_team.h: the direction cell's candidate list from the full
 * hulls' support-cell tables, ug_supcell.h / tools/build_supcells.py, or every vertex; lane-strided dot products + a
 * DPP arg-max with the lowest index winning ties, as btVector3::maxDot's first maximum).  The common path (intersection test, Voronoi
 * GJK, normal fix) keeps its small state in registers: every run-time index into the simplex arrays is an explicit
 * select, so no private array is dynamically indexed.  The penetration path (btGjkEpa2 GJK + EPA:
 * 132 support vertices, 256 faces, their lists) lives in the env's global workspace (EpaMem, L2-resident); EPA's
 * recursive horizon walk (expand) runs on an explicit stack.
 *
 * Provenance: the algorithms and constants are Bullet3's (zlib licence, (c) Erwin Coumans and contributors; its GJK
 * intersection test follows libccd, BSD licence, (c) Daniel Fiser), restated -- no Bullet source is copied here.
 *
 * The includer defines UGK_FN (the function qualifier: `__device__ static inline` in the kernels, `static inline` in
 * tools/gjk_host.cpp, the host build that checks this file against the oracle on the CPU) and, after including it,
 * ugk_hull_support (declared below).
 */
#ifndef UG_GJK_H
#define UG_GJK_H

#include "scene_data.h"
#include "ug_detmath.h"

#ifndef UGK_FN_PAIR /* the includer's linkage for gjk_pair (the kernels: forced inline into its one caller, team_gjk) */
#define UGK_FN_PAIR UGK_FN
#endif
#ifndef UGK_GMEM /* the address space of the EPA store (the kernels: global, so its accesses are global_*, not flat_*) */
#define UGK_GMEM
#endif
#ifndef UGK_OPAQUE /* the includer's register pin: the value stays in registers, never re-read from where it came */
#define UGK_OPAQUE(x)
#endif
#ifndef UGK_LMEM /* the address space of the hull-slot table (the kernels: LDS) */
#define UGK_LMEM
#endif
#ifndef UGK_COUNT /* the includer's event counter and timer hooks (the kernels' -DUG_PROF build) */
#define UGK_COUNT(k, v) do { } while (0)
#define UGK_T0(v)
#define UGK_ADD(k, v) do { } while (0)
#endif

namespace ugk {

struct gv { double x, y, z; };
struct gm { double m[9]; }; /* row-major */
struct gx { gm R; gv p; };  /* rigid transform: x -> R x + p */

UGK_FN gv V3(double x, double y, double z) { gv r; r.x = x; r.y = y; r.z = z; return r; }
UGK_FN gv add(gv a, gv b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
UGK_FN gv sub(gv a, gv b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
UGK_FN gv scl(gv a, double s) { return V3(a.x * s, a.y * s, a.z * s); }
UGK_FN gv neg(gv a) { return V3(-a.x, -a.y, -a.z); }
UGK_FN double dot(gv a, gv b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
UGK_FN gv cross(gv a, gv b) { return V3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
UGK_FN double len(gv a) { return ug_sqrt(dot(a, a)); }
UGK_FN gv mulinv(gv a, double l) { const double inv = 1.0 / l; return V3(a.x * inv, a.y * inv, a.z * inv); }
UGK_FN gv mv(const gm& M, gv v) {
    const double* m = M.m;
    return V3(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[3] * v.x + m[4] * v.y + m[5] * v.z, m[6] * v.x + m[7] * v.y + m[8] * v.z);
}
UGK_FN gv mtv(const gm& M, gv v) {
    const double* m = M.m;
    return V3(m[0] * v.x + m[3] * v.y + m[6] * v.z, m[1] * v.x + m[4] * v.y + m[7] * v.z, m[2] * v.x + m[5] * v.y + m[8] * v.z);
}
UGK_FN gm mtm(const gm& A, const gm& B) {
    gm C;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) C.m[3 * i + j] = A.m[i] * B.m[j] + A.m[3 + i] * B.m[3 + j] + A.m[6 + i] * B.m[6 + j];
    return C;
}
UGK_FN gv xfa(const gx& T, gv x) { return add(mv(T.R, x), T.p); }
UGK_FN bool veq(gv a, gv b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
UGK_FN gv vsel(bool c, gv a, gv b) { return V3(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z); }

/* a convex shape as GJK sees it (kind: UG_SHAPE_*; imp: box / cylinder implicit dimensions; margin: getMargin;
 * scb, sck: a hull's support-cell table -- first cell in UG_SC_IDX and K -- or scb = -1 for none, supcell_data.h) */
struct GShape { int kind, v0, nv; gv imp; double margin; int scb, sck; };

} /* namespace ugk */

/* the includer's hull support: the vertex of hull [s.v0, s.v0 + s.nv) with the first maximal dot product with d
 * (btVector3::maxDot), over the whole hull or over the direction cell's candidates (s.scb >= 0, ug_supcell.h) */
UGK_FN ugk::gv ugk_hull_support(const ugk::GShape& s, ugk::gv d);
#ifdef UGK_GROUP_PARALLEL
/* the includer's lane-group hooks (kernels): this lane's index in its group, and v as lane j of the group holds it.
 * With them the solver evaluates a few independent sub-results on separate lanes at once (the tetrahedron's faces,
 * libccd's five triangle distances) and reads them back in the serial order; the host build runs them in turn. */
UGK_FN int ugk_glane();
UGK_FN double ugk_gread(double v, int j);
UGK_FN int ugk_greadi(int v, int j);
UGK_FN bool ugk_gany(bool p); /* p on any lane of the group */
UGK_FN int ugk_gsize();       /* lanes per group */
#endif

namespace ugk {

constexpr double kEps = 2.220446049250313e-16; /* SIMD_EPSILON */
constexpr double kLarge = 1e30;                /* BT_LARGE_FLOAT */
constexpr double kRelError2 = 1.0e-12;
constexpr double kPenTol = 1.0e-12;
constexpr double kEqVertex = (double)1e-12f;
constexpr int kMaxIter = 1000;
constexpr double kGjkMinDist = 1e-12, kGjkDupEps = 1e-12, kGjkAccuracy = 1e-12;
constexpr int kGjkMaxIterations = 128;
constexpr double kEpaAccuracy = 1e-12, kEpaPlaneEps = 1e-14; /* btGjkEpa2.cpp double block (single: 1e-4, 1e-5) */
constexpr int kEpaMaxVertices = 128, kEpaMaxFaces = 256, kEpaMaxIterations = 255;
constexpr int kTetra = 4 + kEpaMaxVertices; /* E->sv slots of the EPA's first tetrahedron */

/* localGetSupportVertexWithoutMarginNonVirtual */
UGK_FN gv support0(const GShape& s, gv d) {
    if (s.kind == UG_SHAPE_SPHERE) return V3(0.0, 0.0, 0.0);
    if (s.kind == UG_SHAPE_BOX)
        return V3(d.x >= 0.0 ? s.imp.x : -s.imp.x, d.y >= 0.0 ? s.imp.y : -s.imp.y, d.z >= 0.0 ? s.imp.z : -s.imp.z);
    if (s.kind == UG_SHAPE_CYL) {
        const double q = ug_sqrt(d.x * d.x + d.y * d.y);
        const double z = d.z < 0.0 ? -s.imp.z : s.imp.z;
        if (q != 0.0) {
            const double k = s.imp.x / q;
            return V3(d.x * k, d.y * k, z);
        }
        return V3(s.imp.x, 0.0, z);
    }
    return ugk_hull_support(s, d);
}
/* localGetSupportVertexNonVirtual */
UGK_FN gv support(const GShape& s, gv d) {
    gv n = d;
    if (dot(n, n) < kEps * kEps) n = V3(-1.0, -1.0, -1.0);
    n = mulinv(n, ug_sqrt(dot(n, n)));
    const gv p = support0(s, n);
    const double m = s.margin;
    return V3(p.x + m * n.x, p.y + m * n.y, p.z + m * n.z);
}

/* ---------------- btVoronoiSimplexSolver (registers; run-time indices are explicit selects) ---------------- */
enum { UA = 1, UB = 2, UC = 4, UD = 8 };
struct Sub { gv closest; int used; double bc[4]; int degenerate; };
UGK_FN void sub_reset(Sub& r) { r.degenerate = 0; r.bc[0] = r.bc[1] = r.bc[2] = r.bc[3] = 0.0; r.used = 0; }
UGK_FN void sub_set(Sub& r, double a, double b, double c, double d) { r.bc[0] = a; r.bc[1] = b; r.bc[2] = c; r.bc[3] = d; }
UGK_FN bool sub_valid(const Sub& r) { return r.bc[0] >= 0.0 && r.bc[1] >= 0.0 && r.bc[2] >= 0.0 && r.bc[3] >= 0.0; }

struct Voronoi {
    int n;
    gv W[4], P[4], Q[4];
    gv cP1, cP2, cV, lastW;
    bool needsUpdate, validClosest;
    Sub bc;
};
UGK_FN void vs_reset(Voronoi& s) {
    s.validClosest = false;
    s.n = 0;
    s.needsUpdate = true;
    s.lastW = V3(kLarge, kLarge, kLarge);
    sub_reset(s.bc);
}
UGK_FN void vs_add(Voronoi& s, gv w, gv p, gv q) {
    s.lastW = w;
    s.needsUpdate = true;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const bool h = i == s.n;
        s.W[i] = vsel(h, w, s.W[i]);
        s.P[i] = vsel(h, p, s.P[i]);
        s.Q[i] = vsel(h, q, s.Q[i]);
    }
    s.n++;
}
/* removeVertex(I): n--, slot I <- slot n (I a compile-time index, n a run-time one; vs_reduce removes slot I only
 * while n > I, so the source is a slot j >= I: slot I itself when it was the last) */
template <int I>
UGK_FN void vs_remove(Voronoi& s) {
    s.n--;
    gv w = s.W[I], p = s.P[I], q = s.Q[I];
#pragma unroll
    for (int j = I + 1; j < 4; j++) {
        const bool h = j == s.n;
        w = vsel(h, s.W[j], w);
        p = vsel(h, s.P[j], p);
        q = vsel(h, s.Q[j], q);
    }
    s.W[I] = w; s.P[I] = p; s.Q[I] = q;
}
UGK_FN void vs_reduce(Voronoi& s, int used) {
    if (s.n >= 4 && !(used & UD)) vs_remove<3>(s);
    if (s.n >= 3 && !(used & UC)) vs_remove<2>(s);
    if (s.n >= 2 && !(used & UB)) vs_remove<1>(s);
    if (s.n >= 1 && !(used & UA)) vs_remove<0>(s);
}
/* closestPtPointTriangle, p = the origin */
UGK_FN void vs_tri(gv p, gv a, gv b, gv c, Sub& r) {
    r.used = 0;
    const gv ab = sub(b, a), ac = sub(c, a), ap = sub(p, a);
    const double d1 = dot(ab, ap), d2 = dot(ac, ap);
    if (d1 <= 0.0 && d2 <= 0.0) { r.closest = a; r.used = UA; sub_set(r, 1, 0, 0, 0); return; }
    const gv bp = sub(p, b);
    const double d3 = dot(ab, bp), d4 = dot(ac, bp);
    if (d3 >= 0.0 && d4 <= d3) { r.closest = b; r.used = UB; sub_set(r, 0, 1, 0, 0); return; }
    const double vc = d1 * d4 - d3 * d2;
    if (vc <= 0.0 && d1 >= 0.0 && d3 <= 0.0) {
        const double v = d1 / (d1 - d3);
        r.closest = add(a, scl(ab, v));
        r.used = UA | UB;
        sub_set(r, 1 - v, v, 0, 0);
        return;
    }
    const gv cp = sub(p, c);
    const double d5 = dot(ab, cp), d6 = dot(ac, cp);
    if (d6 >= 0.0 && d5 <= d6) { r.closest = c; r.used = UC; sub_set(r, 0, 0, 1, 0); return; }
    const double vb = d5 * d2 - d1 * d6;
    if (vb <= 0.0 && d2 >= 0.0 && d6 <= 0.0) {
        const double w = d2 / (d2 - d6);
        r.closest = add(a, scl(ac, w));
        r.used = UA | UC;
        sub_set(r, 1 - w, 0, w, 0);
        return;
    }
    const double va = d3 * d6 - d5 * d4;
    if (va <= 0.0 && (d4 - d3) >= 0.0 && (d5 - d6) >= 0.0) {
        const double w = (d4 - d3) / ((d4 - d3) + (d5 - d6));
        r.closest = add(b, scl(sub(c, b), w));
        r.used = UB | UC;
        sub_set(r, 0, 1 - w, w, 0);
        return;
    }
    const double denom = 1.0 / (va + vb + vc);
    const double v = vb * denom, w = vc * denom;
    r.closest = add(add(a, scl(ab, v)), scl(ac, w));
    r.used = UA | UB | UC;
    sub_set(r, 1 - v - w, v, w, 0);
}
UGK_FN int vs_outside(gv p, gv a, gv b, gv c, gv d) {
    const gv normal = cross(sub(b, a), sub(c, a));
    const double signp = dot(sub(p, a), normal);
    const double signd = dot(sub(d, a), normal);
    if (signd * signd < (1e-8 * 1e-8)) return -1;
    return signp * signd < 0.0;
}
/* closestPtPointTetrahedron: the candidate faces in Bullet's order, each relabelled into the tetrahedron's slots */
UGK_FN bool vs_tet(gv p, gv a, gv b, gv c, gv d, Sub& fr) {
    fr.closest = p;
    fr.used = UA | UB | UC | UD;
#ifdef UGK_GROUP_PARALLEL
    {
        /* lane j of the group takes face j (ABC, ACD, ADB, BDC with its opposite vertex): its outside test and its
         * closest point, all four at once; the serial selection then runs on the gathered values */
        const int j = ugk_glane() & 3;
        const gv x = j == 3 ? b : a;
        const gv y = j == 0 ? b : (j == 1 ? c : d);
        const gv z = j == 0 ? c : (j == 1 ? d : (j == 2 ? b : c));
        const gv w = j == 0 ? d : (j == 1 ? b : (j == 2 ? c : a));
        const int oj = vs_outside(p, x, y, z, w);
        Sub t;
        vs_tri(p, x, y, z, t);
        const double sqj = dot(sub(t.closest, p), sub(t.closest, p));
        const int o0 = ugk_greadi(oj, 0), o1 = ugk_greadi(oj, 1), o2 = ugk_greadi(oj, 2), o3 = ugk_greadi(oj, 3);
        if (o0 < 0 || o1 < 0 || o2 < 0 || o3 < 0) { fr.degenerate = 1; return false; }
        if (!o0 && !o1 && !o2 && !o3) return false;
        const double s0 = ugk_gread(sqj, 0), s1 = ugk_gread(sqj, 1), s2 = ugk_gread(sqj, 2), s3 = ugk_gread(sqj, 3);
        double best = 3.4028234663852886e+38; /* FLT_MAX */
        int k = -1;
        if (o0 && s0 < best) { best = s0; k = 0; }
        if (o1 && s1 < best) { best = s1; k = 1; }
        if (o2 && s2 < best) { best = s2; k = 2; }
        if (o3 && s3 < best) { best = s3; k = 3; }
        if (k >= 0) {
            fr.closest = V3(ugk_gread(t.closest.x, k), ugk_gread(t.closest.y, k), ugk_gread(t.closest.z, k));
            const int u = ugk_greadi(t.used, k);
            const double b0 = ugk_gread(t.bc[0], k), b1 = ugk_gread(t.bc[1], k), b2 = ugk_gread(t.bc[2], k);
            if (k == 0) {
                fr.used = u & (UA | UB | UC);
                sub_set(fr, b0, b1, b2, 0);
            } else if (k == 1) {
                fr.used = ((u & UA) ? UA : 0) | ((u & UB) ? UC : 0) | ((u & UC) ? UD : 0);
                sub_set(fr, b0, 0, b1, b2);
            } else if (k == 2) {
                fr.used = ((u & UA) ? UA : 0) | ((u & UC) ? UB : 0) | ((u & UB) ? UD : 0);
                sub_set(fr, b0, b2, 0, b1);
            } else {
                fr.used = ((u & UA) ? UB : 0) | ((u & UC) ? UC : 0) | ((u & UB) ? UD : 0);
                sub_set(fr, 0, b0, b2, b1);
            }
        }
        return true;
    }
#endif
    const int oABC = vs_outside(p, a, b, c, d);
    const int oACD = vs_outside(p, a, c, d, b);
    const int oADB = vs_outside(p, a, d, b, c);
    const int oBDC = vs_outside(p, b, d, c, a);
    if (oABC < 0 || oACD < 0 || oADB < 0 || oBDC < 0) { fr.degenerate = 1; return false; }
    if (!oABC && !oACD && !oADB && !oBDC) return false;
    double best = 3.4028234663852886e+38; /* FLT_MAX */
    Sub t;
    if (oABC) {
        vs_tri(p, a, b, c, t);
        const double sq = dot(sub(t.closest, p), sub(t.closest, p));
        if (sq < best) {
            best = sq;
            fr.closest = t.closest;
            fr.used = t.used & (UA | UB | UC);
            sub_set(fr, t.bc[0], t.bc[1], t.bc[2], 0);
        }
    }
    if (oACD) {
        vs_tri(p, a, c, d, t);
        const double sq = dot(sub(t.closest, p), sub(t.closest, p));
        if (sq < best) {
            best = sq;
            fr.closest = t.closest;
            fr.used = ((t.used & UA) ? UA : 0) | ((t.used & UB) ? UC : 0) | ((t.used & UC) ? UD : 0);
            sub_set(fr, t.bc[0], 0, t.bc[1], t.bc[2]);
        }
    }
    if (oADB) {
        vs_tri(p, a, d, b, t);
        const double sq = dot(sub(t.closest, p), sub(t.closest, p));
        if (sq < best) {
            best = sq;
            fr.closest = t.closest;
            fr.used = ((t.used & UA) ? UA : 0) | ((t.used & UC) ? UB : 0) | ((t.used & UB) ? UD : 0);
            sub_set(fr, t.bc[0], t.bc[2], 0, t.bc[1]);
        }
    }
    if (oBDC) {
        vs_tri(p, b, d, c, t);
        const double sq = dot(sub(t.closest, p), sub(t.closest, p));
        if (sq < best) {
            best = sq;
            fr.closest = t.closest;
            fr.used = ((t.used & UA) ? UB : 0) | ((t.used & UC) ? UC : 0) | ((t.used & UB) ? UD : 0);
            sub_set(fr, 0, t.bc[0], t.bc[2], t.bc[1]);
        }
    }
    return true;
}
/* updateClosestVectorAndPoints */
UGK_FN bool vs_update(Voronoi& s) {
    if (!s.needsUpdate) return s.validClosest;
    sub_reset(s.bc);
    s.needsUpdate = false;
    const gv O = V3(0.0, 0.0, 0.0);
    if (s.n == 0) {
        s.validClosest = false;
    } else if (s.n == 1) {
        s.cP1 = s.P[0];
        s.cP2 = s.Q[0];
        s.cV = sub(s.cP1, s.cP2);
        sub_reset(s.bc);
        sub_set(s.bc, 1.0, 0.0, 0.0, 0.0);
        s.validClosest = sub_valid(s.bc);
    } else if (s.n == 2) {
        const gv from = s.W[0], to = s.W[1];
        const gv diff = sub(O, from);
        const gv v = sub(to, from);
        double t = dot(v, diff);
        if (t > 0) {
            const double dotVV = dot(v, v);
            if (t < dotVV) {
                t /= dotVV;
                s.bc.used |= UA | UB;
            } else {
                t = 1;
                s.bc.used |= UB;
            }
        } else {
            t = 0;
            s.bc.used |= UA;
        }
        sub_set(s.bc, 1 - t, t, 0, 0);
        s.cP1 = add(s.P[0], scl(sub(s.P[1], s.P[0]), t));
        s.cP2 = add(s.Q[0], scl(sub(s.Q[1], s.Q[0]), t));
        s.cV = sub(s.cP1, s.cP2);
        vs_reduce(s, s.bc.used);
        s.validClosest = sub_valid(s.bc);
    } else if (s.n == 3) {
        vs_tri(O, s.W[0], s.W[1], s.W[2], s.bc);
        const double* b = s.bc.bc;
        s.cP1 = add(add(scl(s.P[0], b[0]), scl(s.P[1], b[1])), scl(s.P[2], b[2]));
        s.cP2 = add(add(scl(s.Q[0], b[0]), scl(s.Q[1], b[1])), scl(s.Q[2], b[2]));
        s.cV = sub(s.cP1, s.cP2);
        vs_reduce(s, s.bc.used);
        s.validClosest = sub_valid(s.bc);
    } else if (s.n == 4) {
        if (vs_tet(O, s.W[0], s.W[1], s.W[2], s.W[3], s.bc)) {
            const double* b = s.bc.bc;
            s.cP1 = add(add(add(scl(s.P[0], b[0]), scl(s.P[1], b[1])), scl(s.P[2], b[2])), scl(s.P[3], b[3]));
            s.cP2 = add(add(add(scl(s.Q[0], b[0]), scl(s.Q[1], b[1])), scl(s.Q[2], b[2])), scl(s.Q[3], b[3]));
            s.cV = sub(s.cP1, s.cP2);
            vs_reduce(s, s.bc.used);
            s.validClosest = sub_valid(s.bc);
        } else if (s.bc.degenerate) {
            s.validClosest = false;
        } else {
            s.validClosest = true;
            s.cV = V3(0.0, 0.0, 0.0);
        }
    } else {
        s.validClosest = false;
    }
    return s.validClosest;
}
UGK_FN bool vs_in(const Voronoi& s, gv w) {
    bool found = false;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const gv d = sub(w, s.W[i]);
        found = found || (i < s.n && dot(d, d) <= kEqVertex);
    }
    return veq(w, s.lastW) || found;
}

/* ---------------- btGjkEpa2: GJK + EPA in the global workspace ---------------- */
struct ESv { gv d, w; };
/* a face; Bullet's two intrusive lists become: the free faces a stack (m_stock is only ever popped at its root and
 * pushed there; it starts as faces 0, 1, 2, ... from the root, kept implicit as a 'fresh' counter below the pushed
 * ones), the hull an unordered array of (d, append stamp, face) with swap-removal (m_hull's list order is most
 * recently appended first, so its first minimum is the largest stamp among the minima -- what ugk_epa_findbest
 * returns from the array) */
struct EFace {
    gv n;
    double d;
    unsigned char c[3], f[3]; /* vertex ids (< 136), neighbour faces (< 256) */
    unsigned char e[3];       /* the neighbours' edge indices, one byte each: a link is two plain byte stores (a packed
                                 field made every e_bind a read-modify-write, a dependent load on the EPA's chain) */
    unsigned char pass;       /* expand()'s visit mark (<= 255 iterations) */
};
static_assert(sizeof(EFace) == 48, "the face record");
UGK_FN int fe(const EFace& F, int j) { return F.e[j]; }
UGK_FN void set_fe(EFace& F, int j, int v) { F.e[j] = (unsigned char)v; }
struct EHull { double d; int stamp, f; };
/* copies in and out of the store's address space (a struct does not convert between address spaces implicitly) */
UGK_FN gv ldw(const UGK_GMEM ESv& s) { return V3(s.w.x, s.w.y, s.w.z); }
UGK_FN gv ldd(const UGK_GMEM ESv& s) { return V3(s.d.x, s.d.y, s.d.z); }
UGK_FN ESv ldsv(const UGK_GMEM ESv& s) { ESv v; v.d = ldd(s); v.w = ldw(s); return v; }
UGK_FN void stsv(UGK_GMEM ESv& s, const ESv& v) {
    s.d.x = v.d.x; s.d.y = v.d.y; s.d.z = v.d.z;
    s.w.x = v.w.x; s.w.y = v.w.y; s.w.z = v.w.z;
}
struct EpaMem {
    ESv sv[4 + kEpaMaxVertices + 4]; /* [0, 4) the GJK's store, then the EPA's, [132, 136) its first tetrahedron */
    EFace fc[kEpaMaxFaces];
    int sc[2][4];                /* the GJK's two simplices: vertex indices, weights, ranks */
    double sp[2][4];
    int srank[2];
    int freev[4];
    EHull hl[kEpaMaxFaces];      /* the hull faces [0, hcount), unordered */
    unsigned char hpos[kEpaMaxFaces]; /* a hull face's slot in hl (< 256) */
    int stk[kEpaMaxFaces];       /* expand()'s parent frames, packed (e_frame) */
    int stock[kEpaMaxFaces];     /* the faces pushed back to the stock, top = the list root */
    int evm[2 * kEpaMaxFaces];   /* e_expand_group's event log and marked faces beyond their register slots */
    int mkm[kEpaMaxFaces];
};
} /* namespace ugk */
/* the includer's EPA record hooks: face f's record and hull slot i (the kernels keep the first few of each in LDS,
 * the rest in E) */
UGK_FN ugk::EFace ugk_face_get(UGK_GMEM ugk::EpaMem* E, int f);
UGK_FN void ugk_face_put(UGK_GMEM ugk::EpaMem* E, int f, const ugk::EFace& F);
UGK_FN void ugk_face_pass(UGK_GMEM ugk::EpaMem* E, int f, int pass);
UGK_FN void ugk_face_link(UGK_GMEM ugk::EpaMem* E, int f, int j, int nf, int ne); /* neighbour j of face f := (nf, edge ne) */
UGK_FN ugk::EHull ugk_hull_get(UGK_GMEM ugk::EpaMem* E, int i);
UGK_FN void ugk_hull_put(UGK_GMEM ugk::EpaMem* E, int i, const ugk::EHull& h);
UGK_FN UGK_LMEM unsigned char* ugk_hpos(UGK_GMEM ugk::EpaMem* E); /* the hull-slot table, kEpaMaxFaces entries */
/* support vertices: the btGjkEpa2 GJK's store 0..3 (svl: the kernels keep it in LDS) and the EPA's (svg, in E: the
 * EPA copies the GJK's final simplex to 132..135 first, so it never reads the store) */
UGK_FN ugk::ESv ugk_svl_get(UGK_GMEM ugk::EpaMem* E, int i);
UGK_FN void ugk_svl_put(UGK_GMEM ugk::EpaMem* E, int i, const ugk::ESv& v);
namespace ugk {
struct Mink { GShape s0, s1; gm toshape1; gx toshape0; bool margins; };
UGK_FN gv mk_ls(const Mink& M, int i, gv d) {
    const GShape& s = i ? M.s1 : M.s0;
    return M.margins ? support(s, d) : support0(s, d);
}
UGK_FN gv mk_support0(const Mink& M, gv d) { return mk_ls(M, 0, d); }
UGK_FN gv mk_support1(const Mink& M, gv d) { return xfa(M.toshape0, mk_ls(M, 1, mv(M.toshape1, d))); }
UGK_FN gv mk_support(const Mink& M, gv d) { return sub(mk_support0(M, d), mk_support1(M, neg(d))); }
UGK_FN void mk_init(Mink& M, const GShape& s0, const gx& w0, const GShape& s1, const gx& w1, bool margins) {
    M.s0 = s0;
    M.s1 = s1;
    M.toshape1 = mtm(w1.R, w0.R);
    M.toshape0.R = mtm(w0.R, w1.R);
    M.toshape0.p = mtv(w0.R, sub(w1.p, w0.p));
    M.margins = margins;
}

struct Gjk2 { /* btGjkEpa2's GJK: the scalar fields (the stores are in EpaMem) */
    gv ray;
    double distance;
    int nfree, current, simplex, status;
};
enum { GJK_VALID = 0, GJK_INSIDE, GJK_FAILED };
enum { EPA_VALID = 0, EPA_TOUCHING, EPA_DEGENERATED, EPA_NONCONVEX, EPA_INVALIDHULL, EPA_OUTOFFACES, EPA_OUTOFVERTICES,
       EPA_ACCURACYREACHED, EPA_FALLBACK, EPA_FAILED };

UGK_FN ESv g2_support(const Mink& M, gv d) {
    const gv dd = mulinv(d, len(d));
    ESv v;
    v.d = dd;
    v.w = mk_support(M, dd);
    return v;
}
UGK_FN void g2_getsupport(UGK_GMEM EpaMem* E, const Mink& M, gv d, int sv) { ugk_svl_put(E, sv, g2_support(M, d)); }
UGK_FN void g2_remove(UGK_GMEM EpaMem* E, Gjk2& g, int s) { E->freev[g.nfree++] = E->sc[s][--E->srank[s]]; }
UGK_FN void g2_append(UGK_GMEM EpaMem* E, Gjk2& g, const Mink& M, int s, gv v) {
    const int r = E->srank[s];
    E->sp[s][r] = 0;
    E->sc[s][r] = E->freev[--g.nfree];
    E->srank[s] = r + 1;
    g2_getsupport(E, M, v, E->sc[s][r]);
}
UGK_FN double g2_det(gv a, gv b, gv c) {
    return a.y * b.z * c.x + a.z * b.x * c.y - a.x * b.z * c.y - a.y * b.x * c.z + a.x * b.y * c.z - a.z * b.y * c.x;
}
UGK_FN double g2_proj2(gv a, gv b, double* w, int& m) {
    const gv d = sub(b, a);
    const double l = dot(d, d);
    if (l > 0.0) {
        const double t = l > 0 ? -dot(a, d) / l : 0;
        if (t >= 1) { w[0] = 0; w[1] = 1; m = 2; return dot(b, b); }
        if (t <= 0) { w[0] = 1; w[1] = 0; m = 1; return dot(a, a); }
        w[1] = t;
        w[0] = 1 - t;
        m = 3;
        const gv q = add(a, scl(d, t));
        return dot(q, q);
    }
    return -1;
}
UGK_FN double g2_proj3(gv a, gv b, gv c, double* w, int& m) {
    const gv vt[3] = {a, b, c};
    const gv dl[3] = {sub(a, b), sub(b, c), sub(c, a)};
    const gv n = cross(dl[0], dl[1]);
    const double l = dot(n, n);
    if (l > 0.0) {
        double mindist = -1;
        double subw[2] = {0.0, 0.0};
        int subm = 0;
#pragma unroll
        for (int i = 0; i < 3; i++) {
            if (dot(vt[i], cross(dl[i], n)) > 0) {
                const int j = i == 2 ? 0 : i + 1;
                const double subd = g2_proj2(vt[i], vt[j], subw, subm);
                if (mindist < 0 || subd < mindist) {
                    mindist = subd;
                    m = ((subm & 1) ? 1 << i : 0) + ((subm & 2) ? 1 << j : 0);
                    w[i] = subw[0];
                    w[j] = subw[1];
                    w[j == 2 ? 0 : j + 1] = 0;
                }
            }
        }
        if (mindist < 0) {
            const double d = dot(a, n);
            const double s = ug_sqrt(l);
            const gv p = scl(n, d / l);
            mindist = dot(p, p);
            m = 7;
            w[0] = len(cross(dl[1], sub(b, p))) / s;
            w[1] = len(cross(dl[2], sub(c, p))) / s;
            w[2] = 1 - (w[0] + w[1]);
        }
        return mindist;
    }
    return -1;
}
UGK_FN double g2_proj4(gv a, gv b, gv c, gv d, double* w, int& m) {
    const gv vt[4] = {a, b, c, d};
    const gv dl[3] = {sub(a, d), sub(b, d), sub(c, d)};
    const double vl = g2_det(dl[0], dl[1], dl[2]);
    const bool ng = (vl * dot(a, cross(sub(b, c), sub(a, b)))) <= 0;
    if (ng && ug_fabs(vl) > 0.0) {
        double mindist = -1;
        double subw[3] = {0.0, 0.0, 0.0};
        int subm = 0;
#pragma unroll
        for (int i = 0; i < 3; i++) {
            const int j = i == 2 ? 0 : i + 1;
            const double s = vl * dot(d, cross(dl[i], dl[j]));
            if (s > 0) {
                const double subd = g2_proj3(vt[i], vt[j], d, subw, subm);
                if (mindist < 0 || subd < mindist) {
                    mindist = subd;
                    m = ((subm & 1) ? 1 << i : 0) + ((subm & 2) ? 1 << j : 0) + ((subm & 4) ? 8 : 0);
                    w[i] = subw[0];
                    w[j] = subw[1];
                    w[j == 2 ? 0 : j + 1] = 0;
                    w[3] = subw[2];
                }
            }
        }
        if (mindist < 0) {
            mindist = 0;
            m = 15;
            w[0] = g2_det(c, b, d) / vl;
            w[1] = g2_det(a, c, d) / vl;
            w[2] = g2_det(b, a, d) / vl;
            w[3] = 1 - (w[0] + w[1] + w[2]);
        }
        return mindist;
    }
    return -1;
}
/* GJK::Evaluate */
UGK_FN int g2_evaluate(UGK_GMEM EpaMem* E, Gjk2& g, const Mink& M, gv guess) {
    int iterations = 0;
    double sqdist = 0, alpha = 0;
    gv lastw[4];
    int clastw = 0;
    for (int i = 0; i < 4; i++) E->freev[i] = i;
    g.nfree = 4;
    g.current = 0;
    g.status = GJK_VALID;
    g.distance = 0;
    E->srank[0] = 0;
    g.ray = guess;
    const double sqrl = dot(g.ray, g.ray);
    g2_append(E, g, M, 0, sqrl > 0 ? neg(g.ray) : V3(1, 0, 0));
    E->sp[0][0] = 1;
    g.ray = ugk_svl_get(E, E->sc[0][0]).w;
    sqdist = sqrl;
    lastw[0] = lastw[1] = lastw[2] = lastw[3] = g.ray;
    do {
        const int cs = g.current, ns = 1 - g.current;
        const double rl = len(g.ray);
        if (rl < kGjkMinDist) { g.status = GJK_INSIDE; break; }
        g2_append(E, g, M, cs, neg(g.ray));
        const gv w = ugk_svl_get(E, E->sc[cs][E->srank[cs] - 1]).w;
        bool found = false;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const gv dd = sub(w, lastw[i]);
            found = found || dot(dd, dd) < kGjkDupEps;
        }
        if (found) { g2_remove(E, g, cs); break; }
        clastw = (clastw + 1) & 3;
#pragma unroll
        for (int i = 0; i < 4; i++) lastw[i] = vsel(i == clastw, w, lastw[i]);
        const double omega = dot(g.ray, w) / rl;
        alpha = omega > alpha ? omega : alpha;
        if (((rl - alpha) - (kGjkAccuracy * rl)) <= 0) { g2_remove(E, g, cs); break; }
        double weights[4];
        int mask = 0;
        const int rank = E->srank[cs];
        const gv w0 = ugk_svl_get(E, E->sc[cs][0]).w, w1 = ugk_svl_get(E, E->sc[cs][1]).w;
        if (rank == 2) sqdist = g2_proj2(w0, w1, weights, mask);
        else if (rank == 3) sqdist = g2_proj3(w0, w1, ugk_svl_get(E, E->sc[cs][2]).w, weights, mask);
        else if (rank == 4) sqdist = g2_proj4(w0, w1, ugk_svl_get(E, E->sc[cs][2]).w, ugk_svl_get(E, E->sc[cs][3]).w, weights, mask);
        if (sqdist >= 0) {
            E->srank[ns] = 0;
            g.ray = V3(0, 0, 0);
            g.current = ns;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                if (i >= rank) continue;
                if (mask & (1 << i)) {
                    const int r = E->srank[ns]++;
                    E->sc[ns][r] = E->sc[cs][i];
                    E->sp[ns][r] = weights[i];
                    g.ray = add(g.ray, scl(ugk_svl_get(E, E->sc[cs][i]).w, weights[i]));
                } else {
                    E->freev[g.nfree++] = E->sc[cs][i];
                }
            }
            if (mask == 15) g.status = GJK_INSIDE;
        } else {
            g2_remove(E, g, cs);
            break;
        }
        g.status = (++iterations) < kGjkMaxIterations ? g.status : GJK_FAILED;
    } while (g.status == GJK_VALID);
    g.simplex = g.current;
    if (g.status == GJK_VALID) g.distance = len(g.ray);
    else if (g.status == GJK_INSIDE) g.distance = 0;
    return g.status;
}
/* GJK::EncloseOrigin, its recursion unrolled by rank (rank r tries the simplices of rank r + 1) */
UGK_FN gv g2_axis(int i) { return V3(i == 0 ? 1.0 : 0.0, i == 1 ? 1.0 : 0.0, i == 2 ? 1.0 : 0.0); }
UGK_FN bool g2_enc4(UGK_GMEM EpaMem* E, const Gjk2& g) {
    const int s = g.simplex;
    const gv w3 = ugk_svl_get(E, E->sc[s][3]).w;
    return ug_fabs(g2_det(sub(ugk_svl_get(E, E->sc[s][0]).w, w3), sub(ugk_svl_get(E, E->sc[s][1]).w, w3), sub(ugk_svl_get(E, E->sc[s][2]).w, w3))) > 0;
}
UGK_FN bool g2_enc3(UGK_GMEM EpaMem* E, Gjk2& g, const Mink& M) {
    const int s = g.simplex;
    const gv w0 = ugk_svl_get(E, E->sc[s][0]).w;
    const gv n = cross(sub(ugk_svl_get(E, E->sc[s][1]).w, w0), sub(ugk_svl_get(E, E->sc[s][2]).w, w0));
    if (dot(n, n) > 0) {
        g2_append(E, g, M, s, n);
        if (g2_enc4(E, g)) return true;
        g2_remove(E, g, s);
        g2_append(E, g, M, s, neg(n));
        if (g2_enc4(E, g)) return true;
        g2_remove(E, g, s);
    }
    return false;
}
UGK_FN bool g2_enc2(UGK_GMEM EpaMem* E, Gjk2& g, const Mink& M) {
    const int s = g.simplex;
    const gv d = sub(ugk_svl_get(E, E->sc[s][1]).w, ugk_svl_get(E, E->sc[s][0]).w);
    for (int i = 0; i < 3; i++) {
        const gv p = cross(d, g2_axis(i));
        if (dot(p, p) > 0) {
            g2_append(E, g, M, s, p);
            if (g2_enc3(E, g, M)) return true;
            g2_remove(E, g, s);
            g2_append(E, g, M, s, neg(p));
            if (g2_enc3(E, g, M)) return true;
            g2_remove(E, g, s);
        }
    }
    return false;
}
UGK_FN bool g2_enc1(UGK_GMEM EpaMem* E, Gjk2& g, const Mink& M) {
    const int s = g.simplex;
    for (int i = 0; i < 3; i++) {
        const gv axis = g2_axis(i);
        g2_append(E, g, M, s, axis);
        if (g2_enc2(E, g, M)) return true;
        g2_remove(E, g, s);
        g2_append(E, g, M, s, neg(axis));
        if (g2_enc2(E, g, M)) return true;
        g2_remove(E, g, s);
    }
    return false;
}
UGK_FN bool g2_enclose(UGK_GMEM EpaMem* E, Gjk2& g, const Mink& M) {
    const int r = E->srank[g.simplex];
    if (r == 1) return g2_enc1(E, g, M);
    if (r == 2) return g2_enc2(E, g, M);
    if (r == 3) return g2_enc3(E, g, M);
    if (r == 4) return g2_enc4(E, g);
    return false;
}

/* a small stack of ints (the free-face stack, expand()'s parent frames) whose lowest slots may live in registers */
struct LStack { int reg; };
struct Epa { int status, nextsv, hcount, nstock, nfresh, stampctr; LStack stock; gv normal; double depth; int rc[3]; double rp[3]; int rrank; };

} /* namespace ugk */
/* the includer's EPA hook: of the hull faces hl[0, hcount), the one with the smallest d * d, ties to the largest stamp
 * (m_hull's first minimum), except that a NaN at the list root (the largest stamp) keeps the root (Bullet's loop never
 * replaces a NaN) */
UGK_FN int ugk_epa_findbest(const UGK_GMEM ugk::EpaMem* E, int hcount);
/* the includer's LStack hooks: slot i of the stack whose memory is mem (the kernels hold slots [0, 16) in the lane
 * group's registers, lane i slot i) */
UGK_FN void ugk_ls_put(UGK_GMEM int* mem, ugk::LStack& s, int i, int v);
UGK_FN int ugk_ls_get(const UGK_GMEM int* mem, const ugk::LStack& s, int i);
namespace ugk {

UGK_FN void e_bind(UGK_GMEM EpaMem* E, int fa, int ea, int fb, int eb) {
    ugk_face_link(E, fa, ea, fb, eb);
    ugk_face_link(E, fb, eb, fa, ea);
}
UGK_FN void h_append(UGK_GMEM EpaMem* E, Epa& P, int f, double d, int stamp) {
    EHull h;
    h.d = d; h.stamp = stamp; h.f = f;
    ugk_hull_put(E, P.hcount, h);
    ugk_hpos(E)[f] = (unsigned char)P.hcount++;
}
UGK_FN void h_remove(UGK_GMEM EpaMem* E, Epa& P, int f) {
    UGK_LMEM unsigned char* hp = ugk_hpos(E);
    const int i = hp[f], last = --P.hcount;
    if (i != last) {
        const EHull t = ugk_hull_get(E, last);
        ugk_hull_put(E, i, t);
        hp[t.f] = (unsigned char)i;
    }
}
UGK_FN void s_push(UGK_GMEM EpaMem* E, Epa& P, int f) { ugk_ls_put(E->stock, P.stock, P.nstock++, f); }
UGK_FN bool e_edgedist(gv aw, gv bw, gv fn, double& dist) {
    const gv ba = sub(bw, aw);
    const gv n_ab = cross(ba, fn);
    if (dot(aw, n_ab) < 0) {
        const double ba_l2 = dot(ba, ba);
        const double a_dot_ba = dot(aw, ba);
        const double b_dot_ba = dot(bw, ba);
        if (a_dot_ba > 0) dist = len(aw);
        else if (b_dot_ba < 0) dist = len(bw);
        else {
            const double a_dot_b = dot(aw, bw);
            const double x = (dot(aw, aw) * dot(bw, bw) - a_dot_b * a_dot_b) / ba_l2;
            dist = ug_sqrt(x > 0 ? x : 0);
        }
        return true;
    }
    return false;
}
/* a new face's plane from its vertices: false when degenerate (|n| <= EPA_ACCURACY: nOut = the raw normal) */
UGK_FN bool e_plane(gv aw, gv bw, gv cw, gv& nOut, double& dOut) {
    const gv n = cross(sub(bw, aw), sub(cw, aw));
    const double l = len(n);
    if (l > kEpaAccuracy) {
        double d;
        if (!(e_edgedist(aw, bw, n, d) || e_edgedist(bw, cw, n, d) || e_edgedist(cw, aw, n, d)))
            d = dot(aw, n) / l;
        dOut = d;
        nOut = mulinv(n, l);
        return true;
    }
    nOut = n;
    return false;
}
UGK_FN int e_newface(UGK_GMEM EpaMem* E, Epa& P, int a, int b, int c, bool forced) {
    if (P.nstock > 0 || P.nfresh < kEpaMaxFaces) {
        const int f = P.nstock > 0 ? ugk_ls_get(E->stock, P.stock, P.nstock - 1) : P.nfresh;
        if (P.nstock > 0) P.nstock--;
        else P.nfresh++;
        const int stamp = ++P.stampctr; /* m_hull.append: the face joins the hull before its plane is known */
        const gv aw = ldw(E->sv[a]), bw = ldw(E->sv[b]), cw = ldw(E->sv[c]);
        EFace F; /* its three links are all set by e_bind before the hull is read again */
        F.f[0] = F.f[1] = F.f[2] = 0;
        F.e[0] = F.e[1] = F.e[2] = 0;
        F.d = 0.0;
        F.pass = 0;
        F.c[0] = (unsigned char)a; F.c[1] = (unsigned char)b; F.c[2] = (unsigned char)c;
        gv n;
        double d = 0.0;
        const bool nondeg = e_plane(aw, bw, cw, n, d);
        F.n = n;
        if (nondeg) F.d = d;
        ugk_face_put(E, f, F);
        if (nondeg) {
            if (forced || d >= -kEpaPlaneEps) {
                h_append(E, P, f, d, stamp);
                return f;
            }
            P.status = EPA_NONCONVEX;
        } else {
            P.status = EPA_DEGENERATED;
        }
        s_push(E, P, f); /* m_hull.remove + m_stock.append: back on top of the stock */
        return -1;
    }
    P.status = EPA_OUTOFFACES;
    return -1;
}
/* EPA::expand as an explicit depth-first walk.  The current frame (face, edge, stage; stage 0 = entry, 1 = the first
 * neighbour's answer is in r, 2 = the second's) lives in registers, its parents on E->stk packed as face | edge << 8 |
 * stage << 10 | second neighbour << 12 | its edge << 20 (read at entry: a visited face's other edges are not rebound
 * while its subtree runs, the pass mark stops every re-entry).  The same visits, face allocations and list operations
 * as the recursion. */
UGK_FN bool e_expand(UGK_GMEM EpaMem* E, Epa& P, int pass, int w, gv ww, int f0, int e0, int& hcf, int& hff, int& hnf) {
    int sp = 0, f = f0, e = e0, stage = 0, f2 = 0, e2 = 0;
    bool r = false;
    LStack fs;
    fs.reg = 0;
    for (;;) {
        bool pop = true;
        if (stage == 0) {
            const EFace F = ugk_face_get(E, f); /* the face's record in one batch of loads */
            const int e1 = e == 2 ? 0 : e + 1, em = e == 0 ? 2 : e - 1;
            if (F.pass == pass) {
                r = false;
            } else if ((dot(F.n, ww) - F.d) < -kEpaPlaneEps) {
                const int nf = e_newface(E, P, F.c[e1], F.c[e], w, false);
                r = false;
                if (nf >= 0) {
                    e_bind(E, nf, 0, f, e);
                    if (hcf >= 0) e_bind(E, hcf, 1, nf, 2);
                    else hff = nf;
                    hcf = nf;
                    hnf++;
                    r = true;
                }
            } else {
                ugk_face_pass(E, f, pass);
                ugk_ls_put(E->stk, fs, sp++, f | (e << 8) | (1 << 10) | (F.f[em] << 12) | (fe(F, em) << 20));
                f = F.f[e1];
                e = fe(F, e1);
                pop = false;
            }
        } else if (stage == 1) {
            if (r) {
                ugk_ls_put(E->stk, fs, sp++, f | (e << 8) | (2 << 10));
                f = f2;
                e = e2;
                stage = 0;
                pop = false;
            }
        } else if (r) {
            h_remove(E, P, f);
            s_push(E, P, f);
        }
        if (pop) {
            if (sp == 0) break;
            const int fr = ugk_ls_get(E->stk, fs, --sp);
            f = fr & 255;
            e = (fr >> 8) & 3;
            stage = (fr >> 10) & 3;
            f2 = (fr >> 12) & 255;
            e2 = (fr >> 20) & 3;
        }
    }
    return r;
}
#ifdef UGK_GROUP_PARALLEL
/* One EPA iteration's three expand() calls with the new faces' planes computed on separate lanes of the group.
 * The walk runs first and logs, in its order, the faces it would create (horizon edge: its vertices and the
 * neighbour it binds to) and the visible faces it would return to the stock, assuming every new face succeeds: the
 * walk's decisions never read what those calls change (a new face only rebinds the horizon face's edge, which the
 * walk never descends through; a removed face is never reached again).  Then lane k computes event k's plane; when
 * none is degenerate or non-convex (and the faces suffice) the log is replayed in order -- stock pops and pushes,
 * stamps, records, hull appends / removals, bindings -- which is exactly what the serial walk does.  Otherwise the
 * walk's marks are cleared and the serial expand() runs. */
UGK_FN bool e_walk(UGK_GMEM EpaMem* E, int pass, gv ww, int f0, int e0, LStack& ev, int& nev, int& nnew, LStack& mk, int& nmk) {
    int sp = 0, f = f0, e = e0, stage = 0, f2 = 0, e2 = 0;
    bool r = false;
    LStack fs;
    fs.reg = 0;
    for (;;) {
        bool pop = true;
        if (stage == 0) {
            const EFace F = ugk_face_get(E, f);
            const int e1 = e == 2 ? 0 : e + 1, em = e == 0 ? 2 : e - 1;
            if (F.pass == pass) {
                r = false;
            } else if ((dot(F.n, ww) - F.d) < -kEpaPlaneEps) {
                ugk_ls_put(E->evm, ev, nev++, f | (e << 8) | (F.c[e1] << 10) | (F.c[e] << 18));
                nnew++;
                r = true;
            } else {
                ugk_face_pass(E, f, pass);
                ugk_ls_put(E->mkm, mk, nmk++, f);
                ugk_ls_put(E->stk, fs, sp++, f | (e << 8) | (1 << 10) | (F.f[em] << 12) | (fe(F, em) << 20));
                f = F.f[e1];
                e = fe(F, e1);
                pop = false;
            }
        } else if (stage == 1) {
            if (r) {
                ugk_ls_put(E->stk, fs, sp++, f | (e << 8) | (2 << 10));
                f = f2;
                e = e2;
                stage = 0;
                pop = false;
            }
        } else if (r) {
            ugk_ls_put(E->evm, ev, nev++, f | (1 << 28)); /* back to the stock */
        }
        if (pop) {
            if (sp == 0) break;
            const int fr = ugk_ls_get(E->stk, fs, --sp);
            f = fr & 255;
            e = (fr >> 8) & 3;
            stage = (fr >> 10) & 3;
            f2 = (fr >> 12) & 255;
            e2 = (fr >> 20) & 3;
        }
    }
    return r;
}
UGK_FN bool e_expand_group(UGK_GMEM EpaMem* E, Epa& P, int pass, int w, gv ww, const EFace& B, int& hcf, int& hff, int& hnf) {
    LStack ev, mk;
    ev.reg = 0;
    mk.reg = 0;
    int nev = 0, nnew = 0, nmk = 0;
    bool valid = true;
    for (int j = 0; j < 3 && valid; j++) valid = e_walk(E, pass, ww, B.f[j], fe(B, j), ev, nev, nnew, mk, nmk) && valid;
    /* lane k: event k's plane (its own register slot holds the event) */
    const int k = ugk_glane();
    const int my = ev.reg;
    gv pn = V3(0.0, 0.0, 0.0);
    double pd = 0.0;
    bool fail = false;
    if (k < nev && !((my >> 28) & 1)) {
        const int a = (my >> 10) & 255, b = (my >> 18) & 255;
        const bool nondeg = e_plane(ldw(E->sv[a]), ldw(E->sv[b]), ww, pn, pd);
        fail = !nondeg || !(pd >= -kEpaPlaneEps);
    }
    const bool serial = ugk_gany(fail) || nev > ugk_gsize() || nnew > P.nstock + (kEpaMaxFaces - P.nfresh);
    if (serial) {
        for (int i = 0; i < nmk; i++) ugk_face_pass(E, ugk_ls_get(E->mkm, mk, i), 0);
        hcf = -1;
        hff = -1;
        hnf = 0;
        valid = true;
        for (int j = 0; j < 3 && valid; j++) valid = e_expand(E, P, pass, w, ww, B.f[j], fe(B, j), hcf, hff, hnf) && valid;
        return valid;
    }
    for (int i = 0; i < nev; i++) {
        const int x = ugk_greadi(my, i);
        const int f = x & 255;
        if ((x >> 28) & 1) {
            h_remove(E, P, f);
            s_push(E, P, f);
            continue;
        }
        const int e = (x >> 8) & 3;
        const int nf = P.nstock > 0 ? ugk_ls_get(E->stock, P.stock, P.nstock - 1) : P.nfresh;
        if (P.nstock > 0) P.nstock--;
        else P.nfresh++;
        const int stamp = ++P.stampctr;
        EFace F;
        F.f[0] = F.f[1] = F.f[2] = 0;
        F.e[0] = F.e[1] = F.e[2] = 0;
        F.pass = 0;
        F.c[0] = (unsigned char)((x >> 10) & 255); F.c[1] = (unsigned char)((x >> 18) & 255); F.c[2] = (unsigned char)w;
        const double d = ugk_gread(pd, i);
        F.n = V3(ugk_gread(pn.x, i), ugk_gread(pn.y, i), ugk_gread(pn.z, i));
        F.d = d;
        ugk_face_put(E, nf, F);
        h_append(E, P, nf, d, stamp);
        e_bind(E, nf, 0, f, e);
        if (hcf >= 0) e_bind(E, hcf, 1, nf, 2);
        else hff = nf;
        hcf = nf;
        hnf++;
    }
    return valid;
}
#endif
/* EPA::Evaluate */
UGK_FN int e_evaluate(UGK_GMEM EpaMem* E, Epa& P, Gjk2& g, const Mink& M, gv guess) {
    const int s = g.simplex;
    UGK_T0(t_setup);
    if (E->srank[s] > 1 && g2_enclose(E, g, M)) {
        /* Bullet first moves every hull face back to the stock: a fresh EPA (e_init) has none */
        P.status = EPA_VALID;
        P.nextsv = 0;
        UGK_GMEM int* c = E->sc[s];
        {
            const gv w3 = ugk_svl_get(E, c[3]).w;
            if (g2_det(sub(ugk_svl_get(E, c[0]).w, w3), sub(ugk_svl_get(E, c[1]).w, w3), sub(ugk_svl_get(E, c[2]).w, w3)) < 0) {
                const int t = c[0]; c[0] = c[1]; c[1] = t;
                const double tp = E->sp[s][0]; E->sp[s][0] = E->sp[s][1]; E->sp[s][1] = tp;
            }
        }
        /* the simplex's vertices as EPA vertices 132..135 (the same values; the EPA only ever reads E->sv) */
        for (int k = 0; k < 4; k++) stsv(E->sv[kTetra + k], ugk_svl_get(E, c[k]));
        int tetra[4];
        tetra[0] = e_newface(E, P, kTetra + 0, kTetra + 1, kTetra + 2, true);
        tetra[1] = e_newface(E, P, kTetra + 1, kTetra + 0, kTetra + 3, true);
        tetra[2] = e_newface(E, P, kTetra + 2, kTetra + 1, kTetra + 3, true);
        tetra[3] = e_newface(E, P, kTetra + 0, kTetra + 2, kTetra + 3, true);
        if (P.hcount == 4) {
            int best = ugk_epa_findbest(E, P.hcount);
            UGK_ADD(PF_EPA_SETUP, t_setup);
            int pass = 0;
            e_bind(E, tetra[0], 0, tetra[1], 0);
            e_bind(E, tetra[0], 1, tetra[2], 0);
            e_bind(E, tetra[0], 2, tetra[3], 0);
            e_bind(E, tetra[1], 1, tetra[3], 2);
            e_bind(E, tetra[1], 2, tetra[2], 1);
            e_bind(E, tetra[2], 2, tetra[3], 1);
            EFace outer = ugk_face_get(E, best); /* after the bindings: the loop walks from its links */
            P.status = EPA_VALID;
            for (int it = 0; it < kEpaMaxIterations; it++) {
                UGK_COUNT(PC_EPA_IT, 1);
                if (P.nextsv >= kEpaMaxVertices) { P.status = EPA_OUTOFVERTICES; break; }
                int hcf = -1, hff = -1, hnf = 0;
                const int w = 4 + P.nextsv++;
                bool valid = true;
                ugk_face_pass(E, best, ++pass);
                UGK_T0(t_sup);
                /* the best face is `outer` (read after findbest; only its mark changed since), the new vertex the
                 * value just stored: neither is read back from the store (each reread was a dependent load) */
                const ESv sw = g2_support(M, outer.n);
                stsv(E->sv[w], sw);
                UGK_ADD(PF_EPA_SUP, t_sup);
                const gv ww = sw.w;
                EFace B = outer;
                B.pass = (unsigned char)pass;
                const double wdist = dot(B.n, ww) - B.d;
                if (!(wdist > kEpaAccuracy)) { P.status = EPA_ACCURACYREACHED; break; }
                UGK_T0(t_exp);
#ifdef UGK_GROUP_PARALLEL
                valid = e_expand_group(E, P, pass, w, ww, B, hcf, hff, hnf);
#else
                for (int j = 0; j < 3 && valid; j++)
                    valid = e_expand(E, P, pass, w, ww, B.f[j], fe(B, j), hcf, hff, hnf) && valid;
#endif
                UGK_ADD(PF_EPA_EXPAND, t_exp);
                if (!(valid && hnf >= 3)) { P.status = EPA_INVALIDHULL; break; }
                e_bind(E, hcf, 1, hff, 2);
                h_remove(E, P, best);
                s_push(E, P, best);
                UGK_T0(t_best);
                best = ugk_epa_findbest(E, P.hcount);
                UGK_ADD(PF_EPA_BEST, t_best);
                outer = ugk_face_get(E, best);
            }
            const gv projection = scl(outer.n, outer.d);
            P.normal = outer.n;
            P.depth = outer.d;
            P.rrank = 3;
            P.rc[0] = outer.c[0]; P.rc[1] = outer.c[1]; P.rc[2] = outer.c[2];
            const gv a = sub(ldw(E->sv[outer.c[0]]), projection), b = sub(ldw(E->sv[outer.c[1]]), projection),
                     cc = sub(ldw(E->sv[outer.c[2]]), projection);
            P.rp[0] = len(cross(b, cc));
            P.rp[1] = len(cross(cc, a));
            P.rp[2] = len(cross(a, b));
            const double sum = P.rp[0] + P.rp[1] + P.rp[2];
            P.rp[0] /= sum;
            P.rp[1] /= sum;
            P.rp[2] /= sum;
            return P.status;
        }
    }
    P.status = EPA_FALLBACK;
    P.normal = neg(guess);
    const double nl = len(P.normal);
    P.normal = nl > 0 ? mulinv(P.normal, nl) : V3(1, 0, 0);
    P.depth = 0;
    P.rrank = 1;
    P.rc[0] = E->sc[s][0];
    P.rp[0] = 1;
    return P.status;
}
UGK_FN void e_init(UGK_GMEM EpaMem* E, Epa& P) {
    P.status = EPA_FAILED;
    P.normal = V3(0, 0, 0);
    P.depth = 0;
    P.nextsv = 0;
    P.hcount = 0;
    P.nstock = 0; /* the stock: faces 0, 1, 2, ... from the root (fresh), nothing pushed back yet */
    P.stock.reg = 0;
    P.nfresh = 0;
    P.stampctr = 0;
}
struct Res { gv w0, w1, normal; double distance; };
UGK_FN bool g2_penetration(UGK_GMEM EpaMem* E, const GShape& s0, const gx& w0, const GShape& s1, const gx& w1, gv guess, Res& r) {
    Mink M;
    mk_init(M, s0, w0, s1, w1, true);
    Gjk2 g;
    UGK_T0(t_g2);
    const int gs = g2_evaluate(E, g, M, neg(guess));
    UGK_ADD(PF_EPA_GJK, t_g2);
    if (gs == GJK_INSIDE) {
        Epa P;
        e_init(E, P);
        if (e_evaluate(E, P, g, M, neg(guess)) != EPA_FAILED) {
            gv a = V3(0, 0, 0);
            /* the witness: EPA vertices, or the GJK store's for the fallback */
            for (int i = 0; i < P.rrank; i++)
                a = add(a, scl(mk_support0(M, P.rc[i] < 4 ? ugk_svl_get(E, P.rc[i]).d : ldd(E->sv[P.rc[i]])), P.rp[i]));
            r.w0 = xfa(w0, a);
            r.w1 = xfa(w0, sub(a, scl(P.normal, P.depth)));
            r.normal = neg(P.normal);
            r.distance = -P.depth;
            return true;
        }
    }
    return false;
}
UGK_FN bool g2_distance(UGK_GMEM EpaMem* E, const GShape& s0, const gx& w0, const GShape& s1, const gx& w1, gv guess, Res& r) {
    Mink M;
    mk_init(M, s0, w0, s1, w1, false);
    Gjk2 g;
    if (g2_evaluate(E, g, M, guess) == GJK_VALID) {
        gv a = V3(0, 0, 0), b = V3(0, 0, 0);
        const int s = g.simplex;
        for (int i = 0; i < E->srank[s]; i++) {
            const double p = E->sp[s][i];
            const gv d = ugk_svl_get(E, E->sc[s][i]).d;
            a = add(a, scl(mk_support0(M, d), p));
            b = add(b, scl(mk_support1(M, neg(d)), p));
        }
        r.w0 = xfa(w0, a);
        r.w1 = xfa(w0, b);
        r.normal = sub(a, b);
        r.distance = len(r.normal);
        r.normal = mulinv(r.normal, r.distance > kGjkMinDist ? r.distance : 1);
        return true;
    }
    return false;
}
UGK_FN gv safe_normalize(gv d) {
    const double l2 = dot(d, d);
    return l2 >= kEps * kEps ? mulinv(d, ug_sqrt(l2)) : V3(1, 0, 0);
}
/* btGjkEpaPenetrationDepthSolver::calcPenDepth */
UGK_FN bool calc_pen_depth(UGK_GMEM EpaMem* E, const GShape& A, const GShape& B, const gx& TA, const gx& TB, gv& v, gv& wA, gv& wB) {
    for (int i = 0; i < 9; i++) {
        gv guess;
        if (i == 0) guess = safe_normalize(sub(TB.p, TA.p));
        else if (i == 1) guess = safe_normalize(sub(TA.p, TB.p));
        else if (i == 2) guess = V3(0, 0, 1);
        else if (i == 3) guess = V3(0, 1, 0);
        else if (i == 4) guess = V3(1, 0, 0);
        else if (i == 5) guess = V3(1, 1, 0);
        else if (i == 6) guess = V3(1, 1, 1);
        else if (i == 7) guess = V3(0, 1, 1);
        else guess = V3(1, 0, 1);
        Res r;
        if (g2_penetration(E, A, TA, B, TB, guess, r)) { wA = r.w0; wB = r.w1; v = r.normal; return true; }
        if (g2_distance(E, A, TA, B, TB, guess, r)) { wA = r.w0; wB = r.w1; v = r.normal; return false; }
    }
    wA = wB = v = V3(0, 0, 0);
    return false;
}

/* ---------------- btGjkPairDetector: the libccd intersection test ---------------- */
UGK_FN bool fuzzy0(double x) { return ug_fabs(x) < kEps; }
UGK_FN bool ccd_eq(double a_, double b_) {
    const double ab = a_ - b_;
    if (ug_fabs(ab) < kEps) return true;
    const double a = ug_fabs(a_), b = ug_fabs(b_);
    return b > a ? ug_fabs(ab) < kEps * b : ug_fabs(ab) < kEps * a;
}
UGK_FN int ccd_sign(double v) { return fuzzy0(v) ? 0 : (v < 0.0 ? -1 : 1); }
UGK_FN bool ccd_veq(gv a, gv b) { return ccd_eq(a.x, b.x) && ccd_eq(a.y, b.y) && ccd_eq(a.z, b.z); }
UGK_FN gv neg1(gv a) { return V3(a.x * -1.0, a.y * -1.0, a.z * -1.0); }
UGK_FN gv triple(gv a, gv b, gv c) { return cross(cross(a, b), c); }
UGK_FN double seg_dist2(gv P, gv x0, gv b, bool witness) {
    const gv d = sub(b, x0);
    const gv a = sub(x0, P);
    double t = -1.0 * dot(a, d);
    t /= dot(d, d);
    if (t < 0.0 || fuzzy0(t)) { const gv q = sub(x0, P); return dot(q, q); }
    if (t > 1.0 || ccd_eq(t, 1.0)) { const gv q = sub(b, P); return dot(q, q); }
    if (witness) {
        gv wv = V3(d.x * t, d.y * t, d.z * t);
        wv = V3(wv.x + x0.x, wv.y + x0.y, wv.z + x0.z);
        const gv q = sub(wv, P);
        return dot(q, q);
    }
    gv dd = V3(d.x * t, d.y * t, d.z * t);
    dd = V3(dd.x + a.x, dd.y + a.y, dd.z + a.z);
    return dot(dd, dd);
}
UGK_FN double tri_dist2(gv P, gv x0, gv B, gv C) {
    const gv d1 = sub(B, x0), d2 = sub(C, x0), a = sub(x0, P);
    const double u = dot(a, a), v = dot(d1, d1), w = dot(d2, d2);
    const double p = dot(a, d1), q = dot(a, d2), r = dot(d1, d2);
    const double s = (q * r - w * p) / (w * v - r * r);
    const double t = (-s * r - q) / w;
    if ((fuzzy0(s) || s > 0.0) && (ccd_eq(s, 1.0) || s < 1.0) && (fuzzy0(t) || t > 0.0) && (ccd_eq(t, 1.0) || t < 1.0) &&
        (ccd_eq(t + s, 1.0) || t + s < 1.0)) {
        double dist = s * s * v;
        dist += t * t * w;
        dist += 2.0 * s * t * r;
        dist += 2.0 * s * p;
        dist += 2.0 * t * q;
        dist += u;
        return dist;
    }
    double dist = seg_dist2(P, x0, B, false);
    double dist2 = seg_dist2(P, x0, C, true);
    if (dist2 < dist) dist = dist2;
    dist2 = seg_dist2(P, B, C, true);
    if (dist2 < dist) dist = dist2;
    return dist;
}
/* libccd's simplex: the points ps0..ps3 (registers), n = size; every update below names its slots explicitly */
struct Ccd { gv p0, p1, p2, p3; int n; };
UGK_FN int ccd_do3(Ccd& s, gv A, gv& dir) { /* size 3: A = p2, B = p1, C = p0 */
    const gv B = s.p1, C = s.p0;
    if (fuzzy0(tri_dist2(V3(0.0, 0.0, 0.0), A, B, C))) return 1;
    if (ccd_veq(A, B) || ccd_veq(A, C)) return -1;
    const gv AO = neg1(A);
    const gv AB = sub(B, A), AC = sub(C, A);
    const gv ABC = cross(AB, AC);
    double d = dot(cross(ABC, AC), AO);
    if (fuzzy0(d) || d > 0.0) {
        d = dot(AC, AO);
        if (fuzzy0(d) || d > 0.0) {
            s.p1 = A; s.n = 2;
            dir = triple(AC, AO, AC);
        } else {
            d = dot(AB, AO);
            if (fuzzy0(d) || d > 0.0) {
                s.p0 = B; s.p1 = A; s.n = 2;
                dir = triple(AB, AO, AB);
            } else {
                s.p0 = A; s.n = 1;
                dir = AO;
            }
        }
    } else {
        d = dot(cross(AB, ABC), AO);
        if (fuzzy0(d) || d > 0.0) {
            d = dot(AB, AO);
            if (fuzzy0(d) || d > 0.0) {
                s.p0 = B; s.p1 = A; s.n = 2;
                dir = triple(AB, AO, AB);
            } else {
                s.p0 = A; s.n = 1;
                dir = AO;
            }
        } else {
            d = dot(ABC, AO);
            if (fuzzy0(d) || d > 0.0) {
                dir = ABC;
            } else {
                s.p0 = B; s.p1 = C;
                dir = neg1(ABC);
            }
        }
    }
    return 0;
}
UGK_FN int ccd_do(Ccd& s, gv& dir) {
    if (s.n == 2) { /* A = p1, B = p0 */
        const gv A = s.p1, B = s.p0;
        const gv AB = sub(B, A);
        const gv AO = neg1(A);
        const double d = dot(AB, AO);
        const gv tmp = cross(AB, AO);
        if (fuzzy0(dot(tmp, tmp)) && d > 0.0) return 1;
        if (fuzzy0(d) || d < 0.0) {
            s.p0 = A; s.n = 1;
            dir = AO;
        } else {
            dir = triple(AB, AO, AB);
        }
        return 0;
    }
    if (s.n == 3) return ccd_do3(s, s.p2, dir);
    /* size 4: A = p3, B = p2, C = p1, D = p0 */
    const gv A = s.p3, B = s.p2, C = s.p1, D = s.p0;
    const gv O = V3(0.0, 0.0, 0.0);
#ifdef UGK_GROUP_PARALLEL
    {
        /* the five distances on lanes 0..4 of the group at once (the others repeat lane 2's), tested in order */
        const int j = ugk_glane();
        const double rj = tri_dist2(j == 0 ? A : O, (j == 0 || j == 4) ? B : A, (j == 1 || j == 3) ? B : C, j == 1 ? C : D);
        if (fuzzy0(ugk_gread(rj, 0))) return -1;
        if (fuzzy0(ugk_gread(rj, 1)) || fuzzy0(ugk_gread(rj, 2)) || fuzzy0(ugk_gread(rj, 3)) || fuzzy0(ugk_gread(rj, 4)))
            return 1;
    }
#else
    if (fuzzy0(tri_dist2(A, B, C, D))) return -1;
    if (fuzzy0(tri_dist2(O, A, B, C))) return 1;
    if (fuzzy0(tri_dist2(O, A, C, D))) return 1;
    if (fuzzy0(tri_dist2(O, A, B, D))) return 1;
    if (fuzzy0(tri_dist2(O, B, C, D))) return 1;
#endif
    const gv AO = neg1(A);
    const gv AB = sub(B, A), AC = sub(C, A), AD = sub(D, A);
    const gv ABC = cross(AB, AC), ACD = cross(AC, AD), ADB = cross(AD, AB);
    const int B_on_ACD = ccd_sign(dot(ACD, AB));
    const int C_on_ADB = ccd_sign(dot(ADB, AC));
    const int D_on_ABC = ccd_sign(dot(ABC, AD));
    const bool AB_O = ccd_sign(dot(ACD, AO)) == B_on_ACD;
    const bool AC_O = ccd_sign(dot(ADB, AO)) == C_on_ADB;
    const bool AD_O = ccd_sign(dot(ABC, AO)) == D_on_ABC;
    if (AB_O && AC_O && AD_O) return 1;
    if (!AB_O) { s.p2 = A; }
    else if (!AC_O) { s.p1 = D; s.p0 = B; s.p2 = A; }
    else { s.p0 = C; s.p1 = B; s.p2 = A; }
    s.n = 3;
    return ccd_do3(s, s.p2, dir);
}

/* support of A - B in world: A along dir, B along -dir (cores) */
UGK_FN gv support_ab(const GShape& A, const gx& TA, const GShape& B, const gx& TB, gv dir) {
    const gv pA = support0(A, mtv(TA.R, dir));
    const gv qB = support0(B, mtv(TB.R, neg(dir)));
    return sub(xfa(TA, pA), xfa(TB, qB));
}

/* btGjkPairDetector::getClosestPointsNonVirtual: one point (normal on B, point on B, distance) or none */
UGK_FN_PAIR bool gjk_pair(UGK_GMEM EpaMem* E, const GShape& A0, const gx& TA0, const GShape& B0, const gx& TB0, double thr,
                     gv& nOut, gv& pOut, double& dOut, gv* sepAxis = nullptr) {
    UGK_COUNT(PC_GJK, 1);
    UGK_T0(t_all);
    const GShape A = A0, B = B0; /* by value: the caller's records are not re-read through its stack in the loops */
    const double marginA = A.margin, marginB = B.margin;
    double maxd2 = marginA + marginB + thr;
    maxd2 *= maxd2;
    gx TA = TA0, TB = TB0;
    /* pinned: the caller's records sit on its stack, and a re-read through that generic address is a flat load that
     * waits for every outstanding memory access of the wave */
    for (int i = 0; i < 9; i++) { UGK_OPAQUE(TA.R.m[i]); UGK_OPAQUE(TB.R.m[i]); }
    UGK_OPAQUE(TA.p.x); UGK_OPAQUE(TA.p.y); UGK_OPAQUE(TA.p.z);
    UGK_OPAQUE(TB.p.x); UGK_OPAQUE(TB.p.y); UGK_OPAQUE(TB.p.z);
    const gv off = scl(add(TA.p, TB.p), 0.5);
    TA.p = sub(TA.p, off);
    TB.p = sub(TB.p, off);
    double distance = 0.0;
    gv normalInB = V3(0.0, 0.0, 0.0), pointOnB = V3(0, 0, 0);
    gv axis = V3(0.0, 1.0, 0.0);
    bool isValid = false, checkSimplex = false;
    int degenerate = 0, status = -2;
    gv orgNormalInB = V3(0, 0, 0);
    const double margin = marginA + marginB;
    UGK_T0(t_ccd);
    {
        Ccd s;
        gv dir = V3(1, 0, 0);
        gv sup = support_ab(A, TA, B, TB, dir);
        s.p0 = sup;
        s.p1 = s.p2 = s.p3 = sup;
        s.n = 1;
        dir = neg(sup);
        for (int it = 0; it < kMaxIter; it++) {
            UGK_COUNT(PC_GJK_CCD, 1);
            UGK_T0(t_cs);
            sup = support_ab(A, TA, B, TB, dir);
            UGK_ADD(PF_CCD_SUP, t_cs);
            if (dot(sup, dir) < 0) { status = -1; break; }
            if (s.n == 1) s.p1 = sup;
            else if (s.n == 2) s.p2 = sup;
            else s.p3 = sup;
            s.n++;
            UGK_T0(t_cd);
            const int res = ccd_do(s, dir);
            UGK_ADD(PF_CCD_DO, t_cd);
            if (res == 1) { status = 0; break; }
            if (res == -1) { status = -1; break; }
            if (fuzzy0(dot(dir, dir))) status = -1;
            if (dot(dir, dir) < kEps) { status = -1; break; }
            if (dot(dir, dir) < kEps * kEps) { status = -1; break; }
        }
    }
    UGK_ADD(PF_GJK_CCD, t_ccd);
    UGK_T0(t_cls);
    Voronoi vs;
    vs_reset(vs);
    {
        double squaredDistance = kLarge, delta = 0.0;
        int curIter = 0;
        for (;;) {
            UGK_COUNT(PC_GJK_IT, 1);
            UGK_T0(t_ks);
            const gv pW = xfa(TA, support0(A, mtv(TA.R, neg(axis))));
            const gv qW = xfa(TB, support0(B, mtv(TB.R, axis)));
            const gv w = sub(pW, qW);
            UGK_ADD(PF_CLS_SUP, t_ks);
            UGK_T0(t_kv);
            delta = dot(axis, w);
            if (delta > 0.0 && delta * delta > squaredDistance * maxd2) { degenerate = 10; checkSimplex = true; break; }
            if (vs_in(vs, w)) { degenerate = 1; checkSimplex = true; break; }
            const double f0 = squaredDistance - delta, f1 = squaredDistance * kRelError2;
            if (f0 <= f1) { degenerate = f0 <= 0.0 ? 2 : 11; checkSimplex = true; break; }
            vs_add(vs, w, pW, qW);
            const bool ok = vs_update(vs);
            UGK_ADD(PF_CLS_VS, t_kv);
            const gv nax = vs.cV;
            if (!ok) { degenerate = 3; checkSimplex = true; break; }
            if (dot(nax, nax) < kRelError2) { axis = nax; degenerate = 6; checkSimplex = true; break; }
            const double prev = squaredDistance;
            squaredDistance = dot(nax, nax);
            if (prev - squaredDistance <= kEps * prev) { checkSimplex = true; degenerate = 12; break; }
            axis = nax;
            if (curIter++ > kMaxIter) break;
            if (vs.n == 4) { degenerate = 13; break; }
        }
        if (checkSimplex) {
            vs_update(vs);
            gv pointOnA = vs.cP1;
            pointOnB = vs.cP2;
            normalInB = axis;
            const double lenSqr = dot(axis, axis);
            if (lenSqr < kRelError2) degenerate = 5;
            if (lenSqr > kEps * kEps) {
                const double rlen = 1.0 / ug_sqrt(lenSqr);
                normalInB = scl(normalInB, rlen);
                const double s = ug_sqrt(squaredDistance);
                pointOnA = sub(pointOnA, scl(axis, marginA / s));
                pointOnB = add(pointOnB, scl(axis, marginB / s));
                distance = (1.0 / rlen) - margin;
                isValid = true;
                orgNormalInB = normalInB;
            }
        }
    }
    UGK_ADD(PF_GJK_CLASSIC, t_cls);
    /* the classic GJK's last separating axis (from B towards A): the caller's separation certificate, when the query
     * ends without a point it keeps (an observer only: nothing below reads it) */
    if (sepAxis) *sepAxis = status == 0 ? V3(0, 0, 0) : axis;
    const bool catchDegenerate = degenerate && ((distance + margin) < kPenTol);
    if ((!isValid || catchDegenerate) || status == 0) {
        UGK_COUNT(PC_GJK_EPA, 1);
        UGK_T0(t_pen);
        gv tA, tB;
        axis = V3(0, 0, 0);
        const bool isValid2 = calc_pen_depth(E, A, B, TA, TB, axis, tA, tB);
        UGK_ADD(PF_GJK_PEN, t_pen);
        if (dot(axis, axis) != 0.0) {
            if (isValid2) {
                gv tn = sub(tB, tA);
                double lenSqr = dot(tn, tn);
                if (lenSqr <= kEps * kEps) { tn = axis; lenSqr = dot(axis, axis); }
                if (lenSqr > kEps * kEps) {
                    tn = mulinv(tn, ug_sqrt(lenSqr));
                    const double distance2 = -len(sub(tA, tB));
                    if (!isValid || distance2 < distance) {
                        distance = distance2;
                        pointOnB = tB;
                        normalInB = tn;
                        isValid = true;
                    }
                }
            } else if (dot(axis, axis) > 0.0) {
                const double distance2 = len(sub(tA, tB)) - margin;
                if (!isValid || distance2 < distance) {
                    distance = distance2;
                    pointOnB = add(tB, scl(axis, marginB));
                    normalInB = mulinv(axis, len(axis));
                    isValid = true;
                }
            }
        }
    }
    if (!(isValid && (distance < 0 || distance * distance < maxd2))) return false;
    {
        double d2 = 0.0;
        const bool org = dot(orgNormalInB, orgNormalInB) != 0.0;
        if (org) {
            const gv w = sub(xfa(TA, support0(A, mtv(TA.R, neg(orgNormalInB)))), xfa(TB, support0(B, mtv(TB.R, orgNormalInB))));
            d2 = dot(orgNormalInB, w) - margin;
        }
        const gv w1 = sub(xfa(TA, support0(A, mtv(TA.R, normalInB))), xfa(TB, support0(B, mtv(TB.R, neg(normalInB)))));
        const double d1 = dot(neg(normalInB), w1) - margin;
        const gv w0 = sub(xfa(TA, support0(A, mtv(TA.R, neg(normalInB)))), xfa(TB, support0(B, mtv(TB.R, normalInB))));
        const double d0 = dot(normalInB, w0) - margin;
        if (d1 > d0) normalInB = V3(normalInB.x * -1.0, normalInB.y * -1.0, normalInB.z * -1.0);
        if (org && d2 > d0 && d2 > d1 && d2 > distance) {
            normalInB = orgNormalInB;
            distance = d2;
        }
    }
    nOut = normalInB;
    pOut = add(pointOnB, off);
    dOut = distance;
    UGK_ADD(PF_GJK_ALL, t_all);
    return true;
}

} /* namespace ugk */

#endif
