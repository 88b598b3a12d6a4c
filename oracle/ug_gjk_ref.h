/* ug_gjk_ref.h -- CPU restatement of Bullet3's default convex-convex narrowphase (TEST INFRASTRUCTURE ONLY).
 *
 * Included by ug_oracle.c (it uses that file's v3 / m3 / xf helpers).  What PyBullet runs for a pair of convex
 * shapes that has no dedicated algorithm [ext, Bullet3 src/BulletCollision, restated from its published source,
 * unverifiable here -- pybullet is absent]:
 *
 *   btConvexConvexAlgorithm::processCollision   the robot's URDF meshes are btConvexHullShapes without polyhedral
 *                                               features (robot.py:186-187 passes no URDF_INITIALIZE_SAT_FEATURES), so
 *                                               the SAT / clipping branch is not taken: one btGjkPairDetector query per
 *                                               pair and call, m_numPerturbationIterations = 0 (btDefaultCollision-
 *                                               Configuration) -> at most ONE new point per pair per substep, merged
 *                                               into the persistent manifold by btManifoldResult::addContactPoint
 *   btGjkPairDetector::getClosestPointsNonVirtual   (BT_USE_DOUBLE_PRECISION, as pybullet is built)
 *       1. a libccd-style GJK intersection test of the core shapes (no margins): btComputeSupport, btDoSimplex2/3/4
 *       2. the classic margin GJK over btVoronoiSimplexSolver (REL_ERROR2 1e-12, equal-vertex threshold 1e-12f)
 *       3. penetration: btGjkEpaPenetrationDepthSolver::calcPenDepth -> btGjkEpaSolver2::Penetration (btGjkEpa2's
 *          GJK + EPA on the margin-expanded shapes; 9 guess directions), ::Distance as its fallback
 *       4. the normal-direction fix (d0 / d1 / d2 support probes) and addContactPoint(normalInB, pointOnB, distance)
 *
 * Shapes (localGetSupportVertexWithoutMarginNonVirtual + getMarginNonVirtual):
 *   hull      max-dot over the vertices, the first maximum (btVector3::maxDot)        margin 0.001 (URDF)
 *   box       btFsels per axis over the implicit half extents (outer - margin)        its collision margin
 *   sphere    the centre                                                               margin = radius
 *   cylinder  CylinderLocalSupportZ over the implicit dimensions (outer - margin)      its collision margin
 * The kernels restate the same algorithm in urgym_amd/csrc/ug_gjk.h (a separate implementation: wave-parallel
 * support queries, indices instead of pointers, the recursions unrolled); GPU == this file bit for bit.
 *
 * Provenance: the algorithms and constants are Bullet3's (btGjkPairDetector, btVoronoiSimplexSolver, btGjkEpa2, the
 * libccd-derived intersection test; Bullet3 is zlib-licensed, (c) Erwin Coumans and contributors; libccd is
 * BSD-licensed, (c) Daniel Fiser), restated from their published description -- no Bullet source is in this
 * repository or in /root/reference.  tests/test_gjk_independent.py pins the answers to exact geometry.
 */
#ifndef UG_GJK_REF_H
#define UG_GJK_REF_H

#define G_EPS 2.220446049250313e-16       /* SIMD_EPSILON (double) */
#define G_LARGE 1e30                      /* BT_LARGE_FLOAT (double) */
#define G_REL_ERROR2 1.0e-12              /* btGjkPairDetector.cpp REL_ERROR2 (double) */
#define G_PEN_TOL 1.0e-12                 /* gGjkEpaPenetrationTolerance (double) */
#define G_EQ_VERTEX ((double)1e-12f)      /* VORONOI_DEFAULT_EQUAL_VERTEX_THRESHOLD (double build: a float literal) */
#define G_MAX_ITER 1000                   /* gGjkMaxIter */
#define G_GJK_MIN_DISTANCE 1e-12          /* btGjkEpa2.cpp (double) */
#define G_GJK_DUPLICATED_EPS 1e-12
#define G_GJK_ACCURACY 1e-12
#define G_GJK_MAX_ITERATIONS 128
#define G_EPA_ACCURACY 1e-12
#define G_EPA_PLANE_EPS 1e-14         /* btGjkEpa2.cpp, BT_USE_DOUBLE_PRECISION block (single: 0.00001) */
#define G_EPA_MAX_VERTICES 128
#define G_EPA_MAX_FACES (G_EPA_MAX_VERTICES * 2)
#define G_EPA_MAX_ITERATIONS 255

typedef struct {
    int kind;          /* UG_SHAPE_HULL / BOX / SPHERE / CYL */
    const double* v;   /* hull: local vertices (x, y, z) */
    int nv;
    v3 imp;            /* box / cylinder: implicit dimensions (outer minus margin) */
    double margin;     /* getMarginNonVirtual: collision margin; the sphere's radius */
} gshape;

/* localGetSupportVertexWithoutMarginNonVirtual */
static v3 gs_support0(const gshape* s, v3 d) {
    if (s->kind == UG_SHAPE_SPHERE) return V(0.0, 0.0, 0.0);
    if (s->kind == UG_SHAPE_BOX) /* btFsels(a, b, c) = a >= 0 ? b : c */
        return V(d.x >= 0.0 ? s->imp.x : -s->imp.x, d.y >= 0.0 ? s->imp.y : -s->imp.y, d.z >= 0.0 ? s->imp.z : -s->imp.z);
    if (s->kind == UG_SHAPE_CYL) { /* CylinderLocalSupportZ (up axis z: XX 0, YY 2, ZZ 1) */
        const double radius = s->imp.x, hh = s->imp.z;
        const double q = ug_sqrt(d.x * d.x + d.y * d.y);
        const double z = d.z < 0.0 ? -hh : hh;
        if (q != 0.0) {
            const double k = radius / q;
            return V(d.x * k, d.y * k, z);
        }
        return V(radius, 0.0, z);
    }
    /* btConvexHullShape::localGetSupportingVertexWithoutMargin -> btVector3::maxDot (scalar build) */
    double best = -INFINITY;
    int bi = 0;
    for (int i = 0; i < s->nv; i++) {
        const double* p = s->v + 3 * i;
        const double dot = p[0] * d.x + p[1] * d.y + p[2] * d.z;
        if (dot > best) { best = dot; bi = i; }
    }
    return V(s->v[3 * bi], s->v[3 * bi + 1], s->v[3 * bi + 2]);
}
/* localGetSupportVertexNonVirtual: normalised direction, support + margin * direction */
static v3 gs_support(const gshape* s, v3 d) {
    v3 n = d;
    if (vdot(n, n) < G_EPS * G_EPS) n = V(-1.0, -1.0, -1.0);
    const double inv = 1.0 / ug_sqrt(vdot(n, n));
    n = V(n.x * inv, n.y * inv, n.z * inv);
    const v3 p = gs_support0(s, n);
    const double m = s->margin;
    return V(p.x + m * n.x, p.y + m * n.y, p.z + m * n.z);
}

/* ======================================================================== */
/* btVoronoiSimplexSolver                                                    */
/* ======================================================================== */
#define UA 1
#define UB 2
#define UC 4
#define UD 8
typedef struct { v3 closest; int used; double bc[4]; int degenerate; } gsub; /* btSubSimplexClosestResult */
typedef struct {
    int n;
    v3 W[5], P[5], Q[5];
    v3 cP1, cP2, cV, lastW;
    int needsUpdate, validClosest;
    gsub bc;
} vsolver;

static void gsub_reset(gsub* r) {
    r->degenerate = 0;
    r->bc[0] = r->bc[1] = r->bc[2] = r->bc[3] = 0.0;
    r->used = 0;
}
static void gsub_set(gsub* r, double a, double b, double c, double d) { r->bc[0] = a; r->bc[1] = b; r->bc[2] = c; r->bc[3] = d; }
static int gsub_valid(const gsub* r) { return r->bc[0] >= 0.0 && r->bc[1] >= 0.0 && r->bc[2] >= 0.0 && r->bc[3] >= 0.0; }

static void vs_reset(vsolver* s) {
    s->validClosest = 0;
    s->n = 0;
    s->needsUpdate = 1;
    s->lastW = V(G_LARGE, G_LARGE, G_LARGE);
    gsub_reset(&s->bc);
}
static void vs_add(vsolver* s, v3 w, v3 p, v3 q) {
    s->lastW = w;
    s->needsUpdate = 1;
    s->W[s->n] = w; s->P[s->n] = p; s->Q[s->n] = q;
    s->n++;
}
static void vs_remove(vsolver* s, int i) {
    s->n--;
    s->W[i] = s->W[s->n]; s->P[i] = s->P[s->n]; s->Q[i] = s->Q[s->n];
}
static void vs_reduce(vsolver* s, int used) {
    if (s->n >= 4 && !(used & UD)) vs_remove(s, 3);
    if (s->n >= 3 && !(used & UC)) vs_remove(s, 2);
    if (s->n >= 2 && !(used & UB)) vs_remove(s, 1);
    if (s->n >= 1 && !(used & UA)) vs_remove(s, 0);
}
/* closestPtPointTriangle (p = the origin in every call here, kept general as in Bullet) */
static void vs_tri(v3 p, v3 a, v3 b, v3 c, gsub* r) {
    r->used = 0;
    const v3 ab = vsub(b, a), ac = vsub(c, a), ap = vsub(p, a);
    const double d1 = vdot(ab, ap), d2 = vdot(ac, ap);
    if (d1 <= 0.0 && d2 <= 0.0) { r->closest = a; r->used = UA; gsub_set(r, 1, 0, 0, 0); return; }
    const v3 bp = vsub(p, b);
    const double d3 = vdot(ab, bp), d4 = vdot(ac, bp);
    if (d3 >= 0.0 && d4 <= d3) { r->closest = b; r->used = UB; gsub_set(r, 0, 1, 0, 0); return; }
    const double vc = d1 * d4 - d3 * d2;
    if (vc <= 0.0 && d1 >= 0.0 && d3 <= 0.0) {
        const double v = d1 / (d1 - d3);
        r->closest = vadd(a, vscale(ab, v));
        r->used = UA | UB;
        gsub_set(r, 1 - v, v, 0, 0);
        return;
    }
    const v3 cp = vsub(p, c);
    const double d5 = vdot(ab, cp), d6 = vdot(ac, cp);
    if (d6 >= 0.0 && d5 <= d6) { r->closest = c; r->used = UC; gsub_set(r, 0, 0, 1, 0); return; }
    const double vb = d5 * d2 - d1 * d6;
    if (vb <= 0.0 && d2 >= 0.0 && d6 <= 0.0) {
        const double w = d2 / (d2 - d6);
        r->closest = vadd(a, vscale(ac, w));
        r->used = UA | UC;
        gsub_set(r, 1 - w, 0, w, 0);
        return;
    }
    const double va = d3 * d6 - d5 * d4;
    if (va <= 0.0 && (d4 - d3) >= 0.0 && (d5 - d6) >= 0.0) {
        const double w = (d4 - d3) / ((d4 - d3) + (d5 - d6));
        r->closest = vadd(b, vscale(vsub(c, b), w));
        r->used = UB | UC;
        gsub_set(r, 0, 1 - w, w, 0);
        return;
    }
    const double denom = 1.0 / (va + vb + vc);
    const double v = vb * denom, w = vc * denom;
    r->closest = vadd(vadd(a, vscale(ab, v)), vscale(ac, w));
    r->used = UA | UB | UC;
    gsub_set(r, 1 - v - w, v, w, 0);
}
/* pointOutsideOfPlane (CATCH_DEGENERATE_TETRAHEDRON, double: 1e-8) */
static int vs_outside(v3 p, v3 a, v3 b, v3 c, v3 d) {
    const v3 normal = vcross(vsub(b, a), vsub(c, a));
    const double signp = vdot(vsub(p, a), normal);
    const double signd = vdot(vsub(d, a), normal);
    if (signd * signd < (1e-8 * 1e-8)) return -1;
    return signp * signd < 0.0;
}
/* closestPtPointTetrahedron; returns hasSeparation */
static int vs_tet(v3 p, v3 a, v3 b, v3 c, v3 d, gsub* fr) {
    gsub t;
    fr->closest = p;
    fr->used = UA | UB | UC | UD;
    const int oABC = vs_outside(p, a, b, c, d);
    const int oACD = vs_outside(p, a, c, d, b);
    const int oADB = vs_outside(p, a, d, b, c);
    const int oBDC = vs_outside(p, b, d, c, a);
    if (oABC < 0 || oACD < 0 || oADB < 0 || oBDC < 0) { fr->degenerate = 1; return 0; }
    if (!oABC && !oACD && !oADB && !oBDC) return 0;
    double best = 3.4028234663852886e+38; /* FLT_MAX */
    if (oABC) {
        vs_tri(p, a, b, c, &t);
        const v3 q = t.closest;
        const double sq = vdot(vsub(q, p), vsub(q, p));
        if (sq < best) {
            best = sq;
            fr->closest = q;
            fr->used = t.used & (UA | UB | UC);
            gsub_set(fr, t.bc[0], t.bc[1], t.bc[2], 0);
        }
    }
    if (oACD) {
        vs_tri(p, a, c, d, &t);
        const v3 q = t.closest;
        const double sq = vdot(vsub(q, p), vsub(q, p));
        if (sq < best) {
            best = sq;
            fr->closest = q;
            fr->used = ((t.used & UA) ? UA : 0) | ((t.used & UB) ? UC : 0) | ((t.used & UC) ? UD : 0);
            gsub_set(fr, t.bc[0], 0, t.bc[1], t.bc[2]);
        }
    }
    if (oADB) {
        vs_tri(p, a, d, b, &t);
        const v3 q = t.closest;
        const double sq = vdot(vsub(q, p), vsub(q, p));
        if (sq < best) {
            best = sq;
            fr->closest = q;
            fr->used = ((t.used & UA) ? UA : 0) | ((t.used & UC) ? UB : 0) | ((t.used & UB) ? UD : 0);
            gsub_set(fr, t.bc[0], t.bc[2], 0, t.bc[1]);
        }
    }
    if (oBDC) {
        vs_tri(p, b, d, c, &t);
        const v3 q = t.closest;
        const double sq = vdot(vsub(q, p), vsub(q, p));
        if (sq < best) {
            best = sq;
            fr->closest = q;
            fr->used = ((t.used & UA) ? UB : 0) | ((t.used & UC) ? UC : 0) | ((t.used & UB) ? UD : 0);
            gsub_set(fr, 0, t.bc[0], t.bc[2], t.bc[1]);
        }
    }
    return 1;
}
/* updateClosestVectorAndPoints */
static int vs_update(vsolver* s) {
    if (!s->needsUpdate) return s->validClosest;
    gsub_reset(&s->bc);
    s->needsUpdate = 0;
    const v3 O = V(0.0, 0.0, 0.0);
    switch (s->n) {
    case 0: s->validClosest = 0; break;
    case 1:
        s->cP1 = s->P[0];
        s->cP2 = s->Q[0];
        s->cV = vsub(s->cP1, s->cP2);
        gsub_reset(&s->bc);
        gsub_set(&s->bc, 1.0, 0.0, 0.0, 0.0);
        s->validClosest = gsub_valid(&s->bc);
        break;
    case 2: {
        const v3 from = s->W[0], to = s->W[1];
        const v3 diff = vsub(O, from);
        const v3 v = vsub(to, from);
        double t = vdot(v, diff);
        if (t > 0) {
            const double dotVV = vdot(v, v);
            if (t < dotVV) {
                t /= dotVV;
                s->bc.used |= UA | UB;
            } else {
                t = 1;
                s->bc.used |= UB;
            }
        } else {
            t = 0;
            s->bc.used |= UA;
        }
        gsub_set(&s->bc, 1 - t, t, 0, 0);
        s->cP1 = vadd(s->P[0], vscale(vsub(s->P[1], s->P[0]), t));
        s->cP2 = vadd(s->Q[0], vscale(vsub(s->Q[1], s->Q[0]), t));
        s->cV = vsub(s->cP1, s->cP2);
        vs_reduce(s, s->bc.used);
        s->validClosest = gsub_valid(&s->bc);
        break;
    }
    case 3: {
        vs_tri(O, s->W[0], s->W[1], s->W[2], &s->bc);
        const double* b = s->bc.bc;
        s->cP1 = vadd(vadd(vscale(s->P[0], b[0]), vscale(s->P[1], b[1])), vscale(s->P[2], b[2]));
        s->cP2 = vadd(vadd(vscale(s->Q[0], b[0]), vscale(s->Q[1], b[1])), vscale(s->Q[2], b[2]));
        s->cV = vsub(s->cP1, s->cP2);
        vs_reduce(s, s->bc.used);
        s->validClosest = gsub_valid(&s->bc);
        break;
    }
    case 4: {
        const int sep = vs_tet(O, s->W[0], s->W[1], s->W[2], s->W[3], &s->bc);
        if (sep) {
            const double* b = s->bc.bc;
            s->cP1 = vadd(vadd(vadd(vscale(s->P[0], b[0]), vscale(s->P[1], b[1])), vscale(s->P[2], b[2])), vscale(s->P[3], b[3]));
            s->cP2 = vadd(vadd(vadd(vscale(s->Q[0], b[0]), vscale(s->Q[1], b[1])), vscale(s->Q[2], b[2])), vscale(s->Q[3], b[3]));
            s->cV = vsub(s->cP1, s->cP2);
            vs_reduce(s, s->bc.used);
        } else {
            if (s->bc.degenerate) s->validClosest = 0;
            else { s->validClosest = 1; s->cV = V(0.0, 0.0, 0.0); }
            break;
        }
        s->validClosest = gsub_valid(&s->bc);
        break;
    }
    default: s->validClosest = 0;
    }
    return s->validClosest;
}
static int vs_closest(vsolver* s, v3* v) {
    const int ok = vs_update(s);
    *v = s->cV;
    return ok;
}
static int vs_in(const vsolver* s, v3 w) {
    int found = 0;
    for (int i = 0; i < s->n; i++) {
        const v3 d = vsub(w, s->W[i]);
        if (vdot(d, d) <= G_EQ_VERTEX) { found = 1; break; }
    }
    if (w.x == s->lastW.x && w.y == s->lastW.y && w.z == s->lastW.z) return 1;
    return found;
}

/* ======================================================================== */
/* btGjkEpa2 (GJK + EPA on the Minkowski difference in shape 0's frame)      */
/* ======================================================================== */
typedef struct { v3 d, w; } gsv;
typedef struct { int c[4]; double p[4]; int rank; } gsimplex;
typedef struct { v3 n; double d; int c[3], f[3], l[2]; int e[3]; int pass; } gface;
typedef struct { int root, count; } glist;
typedef struct {
    const gshape* s[2];
    m3 toshape1;
    xf toshape0;
    int margins;
    /* GJK */
    v3 ray;
    double distance;
    gsimplex simplices[2];
    int freev[4], nfree, current, simplex, status;
    /* vertex store: [0, 4) the GJK's, [4, 4 + EPA_MAX_VERTICES) the EPA's */
    gsv sv[4 + G_EPA_MAX_VERTICES];
    /* EPA */
    int estatus;
    gsimplex result;
    v3 normal;
    double depth;
    gface fc[G_EPA_MAX_FACES];
    int nextsv;
    glist hull, stock;
} gepa;
enum { GJK_VALID = 0, GJK_INSIDE, GJK_FAILED };
enum { EPA_VALID = 0, EPA_TOUCHING, EPA_DEGENERATED, EPA_NONCONVEX, EPA_INVALIDHULL, EPA_OUTOFFACES, EPA_OUTOFVERTICES,
       EPA_ACCURACYREACHED, EPA_FALLBACK, EPA_FAILED };

static v3 gm_ls(const gepa* g, int i, v3 d) { return g->margins ? gs_support(g->s[i], d) : gs_support0(g->s[i], d); }
static v3 gm_support0(const gepa* g, v3 d) { return gm_ls(g, 0, d); }
static v3 gm_support1(const gepa* g, v3 d) { return xf_apply(&g->toshape0, gm_ls(g, 1, mv(&g->toshape1, d))); }
static v3 gm_support(const gepa* g, v3 d) { return vsub(gm_support0(g, d), gm_support1(g, vneg(d))); }
static v3 gm_support_i(const gepa* g, v3 d, int i) { return i ? gm_support1(g, d) : gm_support0(g, d); }

/* Initialize(shape0, wtrs0, shape1, wtrs1, results, shape, withmargins) */
static void gm_init(gepa* g, const gshape* s0, const xf* w0, const gshape* s1, const xf* w1, int margins) {
    g->s[0] = s0;
    g->s[1] = s1;
    g->toshape1 = mtm(&w1->R, &w0->R);
    g->toshape0.R = mtm(&w0->R, &w1->R);
    g->toshape0.p = mtv(&w0->R, vsub(w1->p, w0->p));
    g->margins = margins;
}
static void gjk_getsupport(gepa* g, v3 d, int sv) {
    const double inv = 1.0 / vlen(d);
    g->sv[sv].d = V(d.x * inv, d.y * inv, d.z * inv);
    g->sv[sv].w = gm_support(g, g->sv[sv].d);
}
static void gjk_remove(gepa* g, gsimplex* s) { g->freev[g->nfree++] = s->c[--s->rank]; }
static void gjk_append(gepa* g, gsimplex* s, v3 v) {
    s->p[s->rank] = 0;
    s->c[s->rank] = g->freev[--g->nfree];
    gjk_getsupport(g, v, s->c[s->rank++]);
}
static double gdet(v3 a, v3 b, v3 c) {
    return a.y * b.z * c.x + a.z * b.x * c.y - a.x * b.z * c.y - a.y * b.x * c.z + a.x * b.y * c.z - a.z * b.y * c.x;
}
static double gproj2(v3 a, v3 b, double* w, int* m) {
    const v3 d = vsub(b, a);
    const double l = vdot(d, d);
    if (l > 0.0) { /* GJK_SIMPLEX2_EPS 0 */
        const double t = l > 0 ? -vdot(a, d) / l : 0;
        if (t >= 1) { w[0] = 0; w[1] = 1; *m = 2; return vdot(b, b); }
        else if (t <= 0) { w[0] = 1; w[1] = 0; *m = 1; return vdot(a, a); }
        else {
            w[0] = 1 - (w[1] = t);
            *m = 3;
            const v3 q = vadd(a, vscale(d, t));
            return vdot(q, q);
        }
    }
    return -1;
}
static double gproj3(v3 a, v3 b, v3 c, double* w, int* m) {
    static const int imd3[] = {1, 2, 0};
    const v3 vt[] = {a, b, c};
    const v3 dl[] = {vsub(a, b), vsub(b, c), vsub(c, a)};
    const v3 n = vcross(dl[0], dl[1]);
    const double l = vdot(n, n);
    if (l > 0.0) { /* GJK_SIMPLEX3_EPS 0 */
        double mindist = -1;
        double subw[2] = {0.0, 0.0};
        int subm = 0;
        for (int i = 0; i < 3; i++) {
            if (vdot(vt[i], vcross(dl[i], n)) > 0) {
                const int j = imd3[i];
                const double subd = gproj2(vt[i], vt[j], subw, &subm);
                if (mindist < 0 || subd < mindist) {
                    mindist = subd;
                    *m = ((subm & 1) ? 1 << i : 0) + ((subm & 2) ? 1 << j : 0);
                    w[i] = subw[0];
                    w[j] = subw[1];
                    w[imd3[j]] = 0;
                }
            }
        }
        if (mindist < 0) {
            const double d = vdot(a, n);
            const double s = ug_sqrt(l);
            const v3 p = vscale(n, d / l);
            mindist = vdot(p, p);
            *m = 7;
            w[0] = vlen(vcross(dl[1], vsub(b, p))) / s;
            w[1] = vlen(vcross(dl[2], vsub(c, p))) / s;
            w[2] = 1 - (w[0] + w[1]);
        }
        return mindist;
    }
    return -1;
}
static double gproj4(v3 a, v3 b, v3 c, v3 d, double* w, int* m) {
    static const int imd3[] = {1, 2, 0};
    const v3 vt[] = {a, b, c, d};
    const v3 dl[] = {vsub(a, d), vsub(b, d), vsub(c, d)};
    const double vl = gdet(dl[0], dl[1], dl[2]);
    const int ng = (vl * vdot(a, vcross(vsub(b, c), vsub(a, b)))) <= 0;
    if (ng && ug_fabs(vl) > 0.0) { /* GJK_SIMPLEX4_EPS 0 */
        double mindist = -1;
        double subw[3] = {0.0, 0.0, 0.0};
        int subm = 0;
        for (int i = 0; i < 3; i++) {
            const int j = imd3[i];
            const double s = vl * vdot(d, vcross(dl[i], dl[j]));
            if (s > 0) {
                const double subd = gproj3(vt[i], vt[j], d, subw, &subm);
                if (mindist < 0 || subd < mindist) {
                    mindist = subd;
                    *m = ((subm & 1) ? 1 << i : 0) + ((subm & 2) ? 1 << j : 0) + ((subm & 4) ? 8 : 0);
                    w[i] = subw[0];
                    w[j] = subw[1];
                    w[imd3[j]] = 0;
                    w[3] = subw[2];
                }
            }
        }
        if (mindist < 0) {
            mindist = 0;
            *m = 15;
            w[0] = gdet(c, b, d) / vl;
            w[1] = gdet(a, c, d) / vl;
            w[2] = gdet(b, a, d) / vl;
            w[3] = 1 - (w[0] + w[1] + w[2]);
        }
        return mindist;
    }
    return -1;
}
/* GJK::Evaluate */
static int gjk_evaluate(gepa* g, v3 guess) {
    int iterations = 0;
    double sqdist = 0, alpha = 0;
    v3 lastw[4];
    int clastw = 0;
    for (int i = 0; i < 4; i++) g->freev[i] = i;
    g->nfree = 4;
    g->current = 0;
    g->status = GJK_VALID;
    g->distance = 0;
    g->simplices[0].rank = 0;
    g->ray = guess;
    const double sqrl = vdot(g->ray, g->ray);
    gjk_append(g, &g->simplices[0], sqrl > 0 ? vneg(g->ray) : V(1, 0, 0));
    g->simplices[0].p[0] = 1;
    g->ray = g->sv[g->simplices[0].c[0]].w;
    sqdist = sqrl;
    lastw[0] = lastw[1] = lastw[2] = lastw[3] = g->ray;
    do {
        const int next = 1 - g->current;
        gsimplex* cs = &g->simplices[g->current];
        gsimplex* ns = &g->simplices[next];
        const double rl = vlen(g->ray);
        if (rl < G_GJK_MIN_DISTANCE) { g->status = GJK_INSIDE; break; }
        gjk_append(g, cs, vneg(g->ray));
        const v3 w = g->sv[cs->c[cs->rank - 1]].w;
        int found = 0;
        for (int i = 0; i < 4; i++) {
            const v3 dd = vsub(w, lastw[i]);
            if (vdot(dd, dd) < G_GJK_DUPLICATED_EPS) { found = 1; break; }
        }
        if (found) { gjk_remove(g, &g->simplices[g->current]); break; }
        else lastw[clastw = (clastw + 1) & 3] = w;
        const double omega = vdot(g->ray, w) / rl;
        alpha = omega > alpha ? omega : alpha;
        if (((rl - alpha) - (G_GJK_ACCURACY * rl)) <= 0) { gjk_remove(g, &g->simplices[g->current]); break; }
        double weights[4];
        int mask = 0;
        switch (cs->rank) {
        case 2: sqdist = gproj2(g->sv[cs->c[0]].w, g->sv[cs->c[1]].w, weights, &mask); break;
        case 3: sqdist = gproj3(g->sv[cs->c[0]].w, g->sv[cs->c[1]].w, g->sv[cs->c[2]].w, weights, &mask); break;
        case 4:
            sqdist = gproj4(g->sv[cs->c[0]].w, g->sv[cs->c[1]].w, g->sv[cs->c[2]].w, g->sv[cs->c[3]].w, weights, &mask);
            break;
        }
        if (sqdist >= 0) {
            ns->rank = 0;
            g->ray = V(0, 0, 0);
            g->current = next;
            for (int i = 0, ni = cs->rank; i < ni; i++) {
                if (mask & (1 << i)) {
                    ns->c[ns->rank] = cs->c[i];
                    ns->p[ns->rank++] = weights[i];
                    g->ray = vadd(g->ray, vscale(g->sv[cs->c[i]].w, weights[i]));
                } else {
                    g->freev[g->nfree++] = cs->c[i];
                }
            }
            if (mask == 15) g->status = GJK_INSIDE;
        } else {
            gjk_remove(g, &g->simplices[g->current]);
            break;
        }
        g->status = (++iterations) < G_GJK_MAX_ITERATIONS ? g->status : GJK_FAILED;
    } while (g->status == GJK_VALID);
    g->simplex = g->current;
    if (g->status == GJK_VALID) g->distance = vlen(g->ray);
    else if (g->status == GJK_INSIDE) g->distance = 0;
    return g->status;
}
/* GJK::EncloseOrigin */
static int gjk_enclose(gepa* g) {
    gsimplex* s = &g->simplices[g->simplex];
    switch (s->rank) {
    case 1:
        for (int i = 0; i < 3; i++) {
            v3 axis = V(0, 0, 0);
            if (i == 0) axis.x = 1; else if (i == 1) axis.y = 1; else axis.z = 1;
            gjk_append(g, s, axis);
            if (gjk_enclose(g)) return 1;
            gjk_remove(g, s);
            gjk_append(g, s, vneg(axis));
            if (gjk_enclose(g)) return 1;
            gjk_remove(g, s);
        }
        break;
    case 2: {
        const v3 d = vsub(g->sv[s->c[1]].w, g->sv[s->c[0]].w);
        for (int i = 0; i < 3; i++) {
            v3 axis = V(0, 0, 0);
            if (i == 0) axis.x = 1; else if (i == 1) axis.y = 1; else axis.z = 1;
            const v3 p = vcross(d, axis);
            if (vdot(p, p) > 0) {
                gjk_append(g, s, p);
                if (gjk_enclose(g)) return 1;
                gjk_remove(g, s);
                gjk_append(g, s, vneg(p));
                if (gjk_enclose(g)) return 1;
                gjk_remove(g, s);
            }
        }
        break;
    }
    case 3: {
        const v3 n = vcross(vsub(g->sv[s->c[1]].w, g->sv[s->c[0]].w), vsub(g->sv[s->c[2]].w, g->sv[s->c[0]].w));
        if (vdot(n, n) > 0) {
            gjk_append(g, s, n);
            if (gjk_enclose(g)) return 1;
            gjk_remove(g, s);
            gjk_append(g, s, vneg(n));
            if (gjk_enclose(g)) return 1;
            gjk_remove(g, s);
        }
        break;
    }
    case 4:
        if (ug_fabs(gdet(vsub(g->sv[s->c[0]].w, g->sv[s->c[3]].w), vsub(g->sv[s->c[1]].w, g->sv[s->c[3]].w),
                         vsub(g->sv[s->c[2]].w, g->sv[s->c[3]].w))) > 0)
            return 1;
        break;
    }
    return 0;
}

/* EPA (faces in an array, -1 = null; the linked lists and their order as Bullet's) */
static void epa_bind(gepa* g, int fa, int ea, int fb, int eb) {
    g->fc[fa].e[ea] = eb; g->fc[fa].f[ea] = fb;
    g->fc[fb].e[eb] = ea; g->fc[fb].f[eb] = fa;
}
static void epa_append(gepa* g, glist* L, int f) {
    g->fc[f].l[0] = -1;
    g->fc[f].l[1] = L->root;
    if (L->root >= 0) g->fc[L->root].l[0] = f;
    L->root = f;
    L->count++;
}
static void epa_remove(gepa* g, glist* L, int f) {
    if (g->fc[f].l[1] >= 0) g->fc[g->fc[f].l[1]].l[0] = g->fc[f].l[0];
    if (g->fc[f].l[0] >= 0) g->fc[g->fc[f].l[0]].l[1] = g->fc[f].l[1];
    if (f == L->root) L->root = g->fc[f].l[1];
    L->count--;
}
static void epa_init(gepa* g) {
    g->estatus = EPA_FAILED;
    g->normal = V(0, 0, 0);
    g->depth = 0;
    g->nextsv = 0;
    g->hull.root = g->stock.root = -1;
    g->hull.count = g->stock.count = 0;
    for (int i = 0; i < G_EPA_MAX_FACES; i++) epa_append(g, &g->stock, G_EPA_MAX_FACES - i - 1);
}
static int epa_edgedist(gepa* g, int f, int a, int b, double* dist) {
    const v3 aw = g->sv[a].w, bw = g->sv[b].w;
    const v3 ba = vsub(bw, aw);
    const v3 n_ab = vcross(ba, g->fc[f].n);
    const double a_dot_nab = vdot(aw, n_ab);
    if (a_dot_nab < 0) {
        const double ba_l2 = vdot(ba, ba);
        const double a_dot_ba = vdot(aw, ba);
        const double b_dot_ba = vdot(bw, ba);
        if (a_dot_ba > 0) *dist = vlen(aw);
        else if (b_dot_ba < 0) *dist = vlen(bw);
        else {
            const double a_dot_b = vdot(aw, bw);
            const double x = (vdot(aw, aw) * vdot(bw, bw) - a_dot_b * a_dot_b) / ba_l2;
            *dist = ug_sqrt(x > 0 ? x : 0);
        }
        return 1;
    }
    return 0;
}
static int epa_newface(gepa* g, int a, int b, int c, int forced) {
    if (g->stock.root >= 0) {
        const int f = g->stock.root;
        epa_remove(g, &g->stock, f);
        epa_append(g, &g->hull, f);
        gface* F = &g->fc[f];
        F->pass = 0;
        F->c[0] = a; F->c[1] = b; F->c[2] = c;
        F->n = vcross(vsub(g->sv[b].w, g->sv[a].w), vsub(g->sv[c].w, g->sv[a].w));
        const double l = vlen(F->n);
        const int v = l > G_EPA_ACCURACY;
        if (v) {
            if (!(epa_edgedist(g, f, a, b, &F->d) || epa_edgedist(g, f, b, c, &F->d) || epa_edgedist(g, f, c, a, &F->d)))
                F->d = vdot(g->sv[a].w, F->n) / l;
            const double inv = 1.0 / l;
            F->n = V(F->n.x * inv, F->n.y * inv, F->n.z * inv);
            if (forced || F->d >= -G_EPA_PLANE_EPS) return f;
            g->estatus = EPA_NONCONVEX;
        } else {
            g->estatus = EPA_DEGENERATED;
        }
        epa_remove(g, &g->hull, f);
        epa_append(g, &g->stock, f);
        return -1;
    }
    g->estatus = g->stock.root >= 0 ? EPA_OUTOFVERTICES : EPA_OUTOFFACES;
    return -1;
}
static int epa_findbest(gepa* g) {
    int minf = g->hull.root;
    double mind = g->fc[minf].d * g->fc[minf].d;
    for (int f = g->fc[minf].l[1]; f >= 0; f = g->fc[f].l[1]) {
        const double sqd = g->fc[f].d * g->fc[f].d;
        if (sqd < mind) { minf = f; mind = sqd; }
    }
    return minf;
}
typedef struct { int cf, ff, nf; } ghorizon;
static int epa_expand(gepa* g, int pass, int w, int f, int e, ghorizon* h) {
    static const int i1m3[] = {1, 2, 0};
    static const int i2m3[] = {2, 0, 1};
    if (g->fc[f].pass != pass) {
        const int e1 = i1m3[e];
        if ((vdot(g->fc[f].n, g->sv[w].w) - g->fc[f].d) < -G_EPA_PLANE_EPS) {
            const int nf = epa_newface(g, g->fc[f].c[e1], g->fc[f].c[e], w, 0);
            if (nf >= 0) {
                epa_bind(g, nf, 0, f, e);
                if (h->cf >= 0) epa_bind(g, h->cf, 1, nf, 2);
                else h->ff = nf;
                h->cf = nf;
                h->nf++;
                return 1;
            }
        } else {
            const int e2 = i2m3[e];
            g->fc[f].pass = pass;
            if (epa_expand(g, pass, w, g->fc[f].f[e1], g->fc[f].e[e1], h) &&
                epa_expand(g, pass, w, g->fc[f].f[e2], g->fc[f].e[e2], h)) {
                epa_remove(g, &g->hull, f);
                epa_append(g, &g->stock, f);
                return 1;
            }
        }
    }
    return 0;
}
/* EPA::Evaluate */
static int epa_evaluate(gepa* g, v3 guess) {
    gsimplex* simplex = &g->simplices[g->simplex];
    if (simplex->rank > 1 && gjk_enclose(g)) {
        while (g->hull.root >= 0) {
            const int f = g->hull.root;
            epa_remove(g, &g->hull, f);
            epa_append(g, &g->stock, f);
        }
        g->estatus = EPA_VALID;
        g->nextsv = 0;
        if (gdet(vsub(g->sv[simplex->c[0]].w, g->sv[simplex->c[3]].w), vsub(g->sv[simplex->c[1]].w, g->sv[simplex->c[3]].w),
                 vsub(g->sv[simplex->c[2]].w, g->sv[simplex->c[3]].w)) < 0) {
            int t = simplex->c[0]; simplex->c[0] = simplex->c[1]; simplex->c[1] = t;
            double tp = simplex->p[0]; simplex->p[0] = simplex->p[1]; simplex->p[1] = tp;
        }
        int tetra[4];
        tetra[0] = epa_newface(g, simplex->c[0], simplex->c[1], simplex->c[2], 1);
        tetra[1] = epa_newface(g, simplex->c[1], simplex->c[0], simplex->c[3], 1);
        tetra[2] = epa_newface(g, simplex->c[2], simplex->c[1], simplex->c[3], 1);
        tetra[3] = epa_newface(g, simplex->c[0], simplex->c[2], simplex->c[3], 1);
        if (g->hull.count == 4) {
            int best = epa_findbest(g);
            gface outer = g->fc[best];
            int pass = 0;
            epa_bind(g, tetra[0], 0, tetra[1], 0);
            epa_bind(g, tetra[0], 1, tetra[2], 0);
            epa_bind(g, tetra[0], 2, tetra[3], 0);
            epa_bind(g, tetra[1], 1, tetra[3], 2);
            epa_bind(g, tetra[1], 2, tetra[2], 1);
            epa_bind(g, tetra[2], 2, tetra[3], 1);
            g->estatus = EPA_VALID;
            for (int iterations = 0; iterations < G_EPA_MAX_ITERATIONS; iterations++) {
                if (g->nextsv < G_EPA_MAX_VERTICES) {
                    ghorizon h = {-1, -1, 0};
                    const int w = 4 + g->nextsv++;
                    int valid = 1;
                    g->fc[best].pass = ++pass;
                    gjk_getsupport(g, g->fc[best].n, w);
                    const double wdist = vdot(g->fc[best].n, g->sv[w].w) - g->fc[best].d;
                    if (wdist > G_EPA_ACCURACY) {
                        for (int j = 0; j < 3 && valid; j++) valid &= epa_expand(g, pass, w, g->fc[best].f[j], g->fc[best].e[j], &h);
                        if (valid && h.nf >= 3) {
                            epa_bind(g, h.cf, 1, h.ff, 2);
                            epa_remove(g, &g->hull, best);
                            epa_append(g, &g->stock, best);
                            best = epa_findbest(g);
                            outer = g->fc[best];
                        } else {
                            g->estatus = EPA_INVALIDHULL;
                            break;
                        }
                    } else {
                        g->estatus = EPA_ACCURACYREACHED;
                        break;
                    }
                } else {
                    g->estatus = EPA_OUTOFVERTICES;
                    break;
                }
            }
            const v3 projection = vscale(outer.n, outer.d);
            g->normal = outer.n;
            g->depth = outer.d;
            g->result.rank = 3;
            g->result.c[0] = outer.c[0]; g->result.c[1] = outer.c[1]; g->result.c[2] = outer.c[2];
            g->result.p[0] = vlen(vcross(vsub(g->sv[outer.c[1]].w, projection), vsub(g->sv[outer.c[2]].w, projection)));
            g->result.p[1] = vlen(vcross(vsub(g->sv[outer.c[2]].w, projection), vsub(g->sv[outer.c[0]].w, projection)));
            g->result.p[2] = vlen(vcross(vsub(g->sv[outer.c[0]].w, projection), vsub(g->sv[outer.c[1]].w, projection)));
            const double sum = g->result.p[0] + g->result.p[1] + g->result.p[2];
            g->result.p[0] /= sum;
            g->result.p[1] /= sum;
            g->result.p[2] /= sum;
            return g->estatus;
        }
    }
    g->estatus = EPA_FALLBACK;
    g->normal = vneg(guess);
    const double nl = vlen(g->normal);
    if (nl > 0) { const double inv = 1.0 / nl; g->normal = V(g->normal.x * inv, g->normal.y * inv, g->normal.z * inv); }
    else g->normal = V(1, 0, 0);
    g->depth = 0;
    g->result.rank = 1;
    g->result.c[0] = simplex->c[0];
    g->result.p[0] = 1;
    return g->estatus;
}

/* btGjkEpaSolver2::Penetration / ::Distance: witnesses in world, normal, distance */
typedef struct { v3 w0, w1, normal; double distance; } gres;
static int gepa_penetration(gepa* g, const gshape* s0, const xf* w0, const gshape* s1, const xf* w1, v3 guess, gres* r) {
    gm_init(g, s0, w0, s1, w1, 1);
    const int st = gjk_evaluate(g, vneg(guess));
    if (st == GJK_INSIDE) {
        epa_init(g);
        const int es = epa_evaluate(g, vneg(guess));
        if (es != EPA_FAILED) {
            v3 a = V(0, 0, 0);
            for (int i = 0; i < g->result.rank; i++) a = vadd(a, vscale(gm_support_i(g, g->sv[g->result.c[i]].d, 0), g->result.p[i]));
            r->w0 = xf_apply(w0, a);
            r->w1 = xf_apply(w0, vsub(a, vscale(g->normal, g->depth)));
            r->normal = vneg(g->normal);
            r->distance = -g->depth;
            return 1;
        }
    }
    return 0;
}
static int gepa_distance(gepa* g, const gshape* s0, const xf* w0, const gshape* s1, const xf* w1, v3 guess, gres* r) {
    gm_init(g, s0, w0, s1, w1, 0);
    const int st = gjk_evaluate(g, guess);
    if (st == GJK_VALID) {
        v3 a = V(0, 0, 0), b = V(0, 0, 0);
        const gsimplex* s = &g->simplices[g->simplex];
        for (int i = 0; i < s->rank; i++) {
            const double p = s->p[i];
            a = vadd(a, vscale(gm_support_i(g, g->sv[s->c[i]].d, 0), p));
            b = vadd(b, vscale(gm_support_i(g, vneg(g->sv[s->c[i]].d), 1), p));
        }
        r->w0 = xf_apply(w0, a);
        r->w1 = xf_apply(w0, b);
        r->normal = vsub(a, b);
        r->distance = vlen(r->normal);
        const double dv = r->distance > G_GJK_MIN_DISTANCE ? r->distance : 1;
        const double inv = 1.0 / dv;
        r->normal = V(r->normal.x * inv, r->normal.y * inv, r->normal.z * inv);
        return 1;
    }
    return 0;
}
/* btGjkEpaPenetrationDepthSolver::calcPenDepth: returns 1 penetrating (witnesses + normal), 0 otherwise (witnesses +
 * normal from the distance query, or all zero) */
static int gepa_calc_pen_depth(gepa* g, const gshape* A, const gshape* B, const xf* TA, const xf* TB, v3* v, v3* wA, v3* wB) {
    v3 guess[9];
    {
        v3 d = vsub(TB->p, TA->p);
        double l2 = vdot(d, d);
        if (l2 >= G_EPS * G_EPS) { const double inv = 1.0 / ug_sqrt(l2); guess[0] = V(d.x * inv, d.y * inv, d.z * inv); }
        else guess[0] = V(1, 0, 0);
        d = vsub(TA->p, TB->p);
        l2 = vdot(d, d);
        if (l2 >= G_EPS * G_EPS) { const double inv = 1.0 / ug_sqrt(l2); guess[1] = V(d.x * inv, d.y * inv, d.z * inv); }
        else guess[1] = V(1, 0, 0);
    }
    guess[2] = V(0, 0, 1); guess[3] = V(0, 1, 0); guess[4] = V(1, 0, 0); guess[5] = V(1, 1, 0);
    guess[6] = V(1, 1, 1); guess[7] = V(0, 1, 1); guess[8] = V(1, 0, 1);
    for (int i = 0; i < 9; i++) {
        gres r;
        if (gepa_penetration(g, A, TA, B, TB, guess[i], &r)) { *wA = r.w0; *wB = r.w1; *v = r.normal; return 1; }
        if (gepa_distance(g, A, TA, B, TB, guess[i], &r)) { *wA = r.w0; *wB = r.w1; *v = r.normal; return 0; }
    }
    *wA = *wB = *v = V(0, 0, 0);
    return 0;
}

/* ======================================================================== */
/* btGjkPairDetector: libccd intersection test (btDoSimplex*)                */
/* ======================================================================== */
static int g_fuzzy0(double x) { return ug_fabs(x) < G_EPS; }
static int g_eq(double a_, double b_) {
    const double ab = a_ - b_;
    if (ug_fabs(ab) < G_EPS) return 1;
    const double a = ug_fabs(a_), b = ug_fabs(b_);
    if (b > a) return ug_fabs(ab) < G_EPS * b;
    return ug_fabs(ab) < G_EPS * a;
}
static int g_sign(double v) { return g_fuzzy0(v) ? 0 : (v < 0.0 ? -1 : 1); }
static int g_veq(v3 a, v3 b) { return g_eq(a.x, b.x) && g_eq(a.y, b.y) && g_eq(a.z, b.z); }
static v3 g_neg1(v3 a) { return V(a.x * -1.0, a.y * -1.0, a.z * -1.0); } /* btVec3Scale(v, -1) */
static v3 g_triple(v3 a, v3 b, v3 c) { return vcross(vcross(a, b), c); }
/* btVec3PointSegmentDist2 (witness != NULL selects the witness arithmetic) */
static double g_seg_dist2(v3 P, v3 x0, v3 b, int want_witness) {
    const v3 d = vsub(b, x0);
    const v3 a = vsub(x0, P);
    double t = -1.0 * vdot(a, d);
    t /= vdot(d, d);
    if (t < 0.0 || g_fuzzy0(t)) { const v3 q = vsub(x0, P); return vdot(q, q); }
    if (t > 1.0 || g_eq(t, 1.0)) { const v3 q = vsub(b, P); return vdot(q, q); }
    if (want_witness) {
        v3 wv = V(d.x * t, d.y * t, d.z * t);
        wv = V(wv.x + x0.x, wv.y + x0.y, wv.z + x0.z);
        const v3 q = vsub(wv, P);
        return vdot(q, q);
    }
    v3 dd = V(d.x * t, d.y * t, d.z * t);
    dd = V(dd.x + a.x, dd.y + a.y, dd.z + a.z);
    return vdot(dd, dd);
}
/* btVec3PointTriDist2 without a witness */
static double g_tri_dist2(v3 P, v3 x0, v3 B, v3 C) {
    const v3 d1 = vsub(B, x0), d2 = vsub(C, x0), a = vsub(x0, P);
    const double u = vdot(a, a), v = vdot(d1, d1), w = vdot(d2, d2);
    const double p = vdot(a, d1), q = vdot(a, d2), r = vdot(d1, d2);
    const double s = (q * r - w * p) / (w * v - r * r);
    const double t = (-s * r - q) / w;
    if ((g_fuzzy0(s) || s > 0.0) && (g_eq(s, 1.0) || s < 1.0) && (g_fuzzy0(t) || t > 0.0) && (g_eq(t, 1.0) || t < 1.0) &&
        (g_eq(t + s, 1.0) || t + s < 1.0)) {
        double dist = s * s * v;
        dist += t * t * w;
        dist += 2.0 * s * t * r;
        dist += 2.0 * s * p;
        dist += 2.0 * t * q;
        dist += u;
        return dist;
    }
    double dist = g_seg_dist2(P, x0, B, 0);
    double dist2 = g_seg_dist2(P, x0, C, 1);
    if (dist2 < dist) dist = dist2;
    dist2 = g_seg_dist2(P, B, C, 1);
    if (dist2 < dist) dist = dist2;
    return dist;
}
typedef struct { v3 ps[4]; int last; } gccd; /* btSimplex (only the Minkowski points are read) */
static int g_do2(gccd* s, v3* dir) {
    const v3 A = s->ps[s->last], B = s->ps[0];
    const v3 AB = vsub(B, A);
    const v3 AO = g_neg1(A);
    const double dot = vdot(AB, AO);
    const v3 tmp = vcross(AB, AO);
    if (g_fuzzy0(vdot(tmp, tmp)) && dot > 0.0) return 1;
    if (g_fuzzy0(dot) || dot < 0.0) {
        s->ps[0] = A;
        s->last = 0;
        *dir = AO;
    } else {
        *dir = g_triple(AB, AO, AB);
    }
    return 0;
}
static int g_do3(gccd* s, v3* dir) {
    const v3 A = s->ps[s->last], B = s->ps[1], C = s->ps[0];
    const double dist = g_tri_dist2(V(0.0, 0.0, 0.0), A, B, C);
    if (g_fuzzy0(dist)) return 1;
    if (g_veq(A, B) || g_veq(A, C)) return -1;
    const v3 AO = g_neg1(A);
    const v3 AB = vsub(B, A), AC = vsub(C, A);
    const v3 ABC = vcross(AB, AC);
    v3 tmp = vcross(ABC, AC);
    double dot = vdot(tmp, AO);
    if (g_fuzzy0(dot) || dot > 0.0) {
        dot = vdot(AC, AO);
        if (g_fuzzy0(dot) || dot > 0.0) {
            s->ps[1] = A;
            s->last = 1;
            *dir = g_triple(AC, AO, AC);
        } else {
            dot = vdot(AB, AO);
            if (g_fuzzy0(dot) || dot > 0.0) {
                s->ps[0] = B;
                s->ps[1] = A;
                s->last = 1;
                *dir = g_triple(AB, AO, AB);
            } else {
                s->ps[0] = A;
                s->last = 0;
                *dir = AO;
            }
        }
    } else {
        tmp = vcross(AB, ABC);
        dot = vdot(tmp, AO);
        if (g_fuzzy0(dot) || dot > 0.0) {
            dot = vdot(AB, AO);
            if (g_fuzzy0(dot) || dot > 0.0) {
                s->ps[0] = B;
                s->ps[1] = A;
                s->last = 1;
                *dir = g_triple(AB, AO, AB);
            } else {
                s->ps[0] = A;
                s->last = 0;
                *dir = AO;
            }
        } else {
            dot = vdot(ABC, AO);
            if (g_fuzzy0(dot) || dot > 0.0) {
                *dir = ABC;
            } else {
                const v3 t = C;
                s->ps[0] = B;
                s->ps[1] = t;
                *dir = g_neg1(ABC);
            }
        }
    }
    return 0;
}
static int g_do4(gccd* s, v3* dir) {
    const v3 A = s->ps[s->last], B = s->ps[2], C = s->ps[1], D = s->ps[0];
    double dist = g_tri_dist2(A, B, C, D);
    if (g_fuzzy0(dist)) return -1;
    const v3 O = V(0.0, 0.0, 0.0);
    dist = g_tri_dist2(O, A, B, C);
    if (g_fuzzy0(dist)) return 1;
    dist = g_tri_dist2(O, A, C, D);
    if (g_fuzzy0(dist)) return 1;
    dist = g_tri_dist2(O, A, B, D);
    if (g_fuzzy0(dist)) return 1;
    dist = g_tri_dist2(O, B, C, D);
    if (g_fuzzy0(dist)) return 1;
    const v3 AO = g_neg1(A);
    const v3 AB = vsub(B, A), AC = vsub(C, A), AD = vsub(D, A);
    const v3 ABC = vcross(AB, AC), ACD = vcross(AC, AD), ADB = vcross(AD, AB);
    const int B_on_ACD = g_sign(vdot(ACD, AB));
    const int C_on_ADB = g_sign(vdot(ADB, AC));
    const int D_on_ABC = g_sign(vdot(ABC, AD));
    const int AB_O = g_sign(vdot(ACD, AO)) == B_on_ACD;
    const int AC_O = g_sign(vdot(ADB, AO)) == C_on_ADB;
    const int AD_O = g_sign(vdot(ABC, AO)) == D_on_ABC;
    if (AB_O && AC_O && AD_O) return 1;
    if (!AB_O) {
        s->ps[2] = A;
        s->last = 2;
    } else if (!AC_O) {
        s->ps[1] = D;
        s->ps[0] = B;
        s->ps[2] = A;
        s->last = 2;
    } else {
        s->ps[0] = C;
        s->ps[1] = B;
        s->ps[2] = A;
        s->last = 2;
    }
    return g_do3(s, dir);
}
static int g_do_simplex(gccd* s, v3* dir) {
    if (s->last + 1 == 2) return g_do2(s, dir);
    if (s->last + 1 == 3) return g_do3(s, dir);
    return g_do4(s, dir);
}

/* support of A - B in world (the pair detector's frames): A along dir, B along -dir */
static v3 g_support_ab(const gshape* A, const xf* TA, const gshape* B, const xf* TB, v3 dir) {
    const v3 pA = gs_support0(A, mtv(&TA->R, dir));
    const v3 qB = gs_support0(B, mtv(&TB->R, vneg(dir)));
    return vsub(xf_apply(TA, pA), xf_apply(TB, qB));
}

/* btGjkPairDetector::getClosestPointsNonVirtual + the btManifoldResult input it forms.  TA / TB: world transforms of
 * the two shapes; thr: the manifold's contact breaking threshold.  Returns 1 with (normal on B, point on B, distance)
 * when the detector reports a point (the caller's addContactPoint still drops distance > thr), else 0. */
/* test hook (tests/test_gjk_independent.py): the last query's exits -- the classic GJK's degenerate code and iteration
 * count, the libccd status, whether the penetration path ran */
static _Thread_local int g_gjk_dbg[4];
static int gjk_pair(const gshape* A, const xf* TA0, const gshape* B, const xf* TB0, double thr, v3* nOut, v3* pOut,
                    double* dOut) {
    static _Thread_local gepa g; /* the EPA's stores (btGjkEpaSolver2 keeps them on its stack) */
    const double marginA = A->margin, marginB = B->margin;
    double maxd2 = marginA + marginB + thr;
    maxd2 *= maxd2;
    xf TA = *TA0, TB = *TB0;
    const v3 off = vscale(vadd(TA.p, TB.p), 0.5);
    TA.p = vsub(TA.p, off);
    TB.p = vsub(TB.p, off);
    double distance = 0.0;
    v3 normalInB = V(0.0, 0.0, 0.0), pointOnA = V(0, 0, 0), pointOnB = V(0, 0, 0);
    v3 axis = V(0.0, 1.0, 0.0); /* m_cachedSeparatingAxis of a fresh detector */
    int isValid = 0, checkSimplex = 0, degenerate = 0, status = -2;
    v3 orgNormalInB = V(0, 0, 0);
    const double margin = marginA + marginB;
    /* 1. libccd intersection test of the core shapes */
    {
        gccd s;
        s.last = -1;
        v3 dir = V(1, 0, 0);
        v3 sup = g_support_ab(A, &TA, B, &TB, dir);
        s.ps[++s.last] = sup;
        dir = vneg(sup);
        for (int it = 0; it < G_MAX_ITER; it++) {
            sup = g_support_ab(A, &TA, B, &TB, dir);
            const double delta = vdot(sup, dir);
            if (delta < 0) { status = -1; break; }
            s.ps[++s.last] = sup;
            const int res = g_do_simplex(&s, &dir);
            if (res == 1) { status = 0; break; }
            else if (res == -1) { status = -1; break; }
            if (g_fuzzy0(vdot(dir, dir))) status = -1;
            if (vdot(dir, dir) < G_EPS) { status = -1; break; }
            if (vdot(dir, dir) < G_EPS * G_EPS) { status = -1; break; }
        }
    }
    /* 2. the classic GJK with margins */
    vsolver vs;
    vs_reset(&vs);
    {
        double squaredDistance = G_LARGE, delta = 0.0;
        int curIter = 0;
        for (;;) {
            const v3 sepA = mtv(&TA.R, vneg(axis));
            const v3 sepB = mtv(&TB.R, axis);
            const v3 pW = xf_apply(&TA, gs_support0(A, sepA));
            const v3 qW = xf_apply(&TB, gs_support0(B, sepB));
            const v3 w = vsub(pW, qW);
            delta = vdot(axis, w);
            if (delta > 0.0 && delta * delta > squaredDistance * maxd2) { degenerate = 10; checkSimplex = 1; break; }
            if (vs_in(&vs, w)) { degenerate = 1; checkSimplex = 1; break; }
            const double f0 = squaredDistance - delta, f1 = squaredDistance * G_REL_ERROR2;
            if (f0 <= f1) { degenerate = f0 <= 0.0 ? 2 : 11; checkSimplex = 1; break; }
            vs_add(&vs, w, pW, qW);
            v3 nax;
            if (!vs_closest(&vs, &nax)) { degenerate = 3; checkSimplex = 1; break; }
            if (vdot(nax, nax) < G_REL_ERROR2) { axis = nax; degenerate = 6; checkSimplex = 1; break; }
            const double prev = squaredDistance;
            squaredDistance = vdot(nax, nax);
            if (prev - squaredDistance <= G_EPS * prev) { checkSimplex = 1; degenerate = 12; break; }
            axis = nax;
            if (curIter++ > G_MAX_ITER) break;
            if (vs.n == 4) { degenerate = 13; break; }
        }
        g_gjk_dbg[0] = degenerate;
        g_gjk_dbg[1] = curIter;
        if (checkSimplex) {
            vs_update(&vs); /* compute_points */
            pointOnA = vs.cP1;
            pointOnB = vs.cP2;
            normalInB = axis;
            const double lenSqr = vdot(axis, axis);
            if (lenSqr < G_REL_ERROR2) degenerate = 5;
            if (lenSqr > G_EPS * G_EPS) {
                const double rlen = 1.0 / ug_sqrt(lenSqr);
                normalInB = vscale(normalInB, rlen);
                const double s = ug_sqrt(squaredDistance);
                pointOnA = vsub(pointOnA, vscale(axis, marginA / s));
                pointOnB = vadd(pointOnB, vscale(axis, marginB / s));
                distance = (1.0 / rlen) - margin;
                isValid = 1;
                orgNormalInB = normalInB;
            }
        }
    }
    /* 3. penetration (EPA) */
    const int catchDegenerate = degenerate && ((distance + margin) < G_PEN_TOL);
    g_gjk_dbg[2] = status;
    g_gjk_dbg[3] = (!isValid || catchDegenerate) || status == 0;
    if ((!isValid || catchDegenerate) || status == 0) {
        v3 tA, tB;
        axis = V(0, 0, 0);
        const int isValid2 = gepa_calc_pen_depth(&g, A, B, &TA, &TB, &axis, &tA, &tB);
        if (vdot(axis, axis) != 0.0) {
            if (isValid2) {
                v3 tn = vsub(tB, tA);
                double lenSqr = vdot(tn, tn);
                if (lenSqr <= G_EPS * G_EPS) { tn = axis; lenSqr = vdot(axis, axis); }
                if (lenSqr > G_EPS * G_EPS) {
                    const double inv = 1.0 / ug_sqrt(lenSqr);
                    tn = V(tn.x * inv, tn.y * inv, tn.z * inv);
                    const double distance2 = -vlen(vsub(tA, tB));
                    if (!isValid || distance2 < distance) {
                        distance = distance2;
                        pointOnA = tA;
                        pointOnB = tB;
                        normalInB = tn;
                        isValid = 1;
                    }
                }
            } else {
                if (vdot(axis, axis) > 0.0) {
                    const double distance2 = vlen(vsub(tA, tB)) - margin;
                    if (!isValid || distance2 < distance) {
                        distance = distance2;
                        pointOnA = vsub(tA, vscale(axis, marginA));
                        pointOnB = vadd(tB, vscale(axis, marginB));
                        const double inv = 1.0 / vlen(axis);
                        normalInB = V(axis.x * inv, axis.y * inv, axis.z * inv);
                        isValid = 1;
                    }
                }
            }
        }
    }
    (void)pointOnA;
    if (!(isValid && (distance < 0 || distance * distance < maxd2))) return 0;
    /* 4. the normal-direction fix */
    {
        double d2 = 0.0;
        if (vdot(orgNormalInB, orgNormalInB) != 0.0) {
            const v3 w = vsub(xf_apply(&TA, gs_support0(A, mtv(&TA.R, vneg(orgNormalInB)))),
                              xf_apply(&TB, gs_support0(B, mtv(&TB.R, orgNormalInB))));
            d2 = vdot(orgNormalInB, w) - margin;
        }
        double d1;
        {
            const v3 w = vsub(xf_apply(&TA, gs_support0(A, mtv(&TA.R, normalInB))),
                              xf_apply(&TB, gs_support0(B, mtv(&TB.R, vneg(normalInB)))));
            d1 = vdot(vneg(normalInB), w) - margin;
        }
        double d0;
        {
            const v3 w = vsub(xf_apply(&TA, gs_support0(A, mtv(&TA.R, vneg(normalInB)))),
                              xf_apply(&TB, gs_support0(B, mtv(&TB.R, normalInB))));
            d0 = vdot(normalInB, w) - margin;
        }
        if (d1 > d0) normalInB = V(normalInB.x * -1.0, normalInB.y * -1.0, normalInB.z * -1.0);
        if (vdot(orgNormalInB, orgNormalInB) != 0.0) {
            if (d2 > d0 && d2 > d1 && d2 > distance) {
                normalInB = orgNormalInB;
                distance = d2;
            }
        }
    }
    *nOut = normalInB;
    *pOut = vadd(pointOnB, off);
    *dOut = distance;
    return 1;
}

#endif
