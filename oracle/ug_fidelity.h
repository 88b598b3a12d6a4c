/* ug_fidelity.h -- collision-fidelity narrowphase of the CPU restatement (TEST / MEASUREMENT ONLY).
 *
 * Included by ug_oracle.c when built with -DUG_FIDELITY (tools/collision_fidelity.py), together with the
 * fidelity model header (full, undecimated hulls; face vertex loops; a 128-sided club-disc prism).  It
 * replaces the product's hull narrowphases -- vertex-in-box / corner-in-hull / vertex-in-hull with the
 * face planes, deepest + farthest-spread 4 points (nc_hull_box, nc_hull_hull) and the deepest face plane
 * for spheres (nc_hull_sphere) -- by a restatement of Bullet's polyhedral path [ext]:
 *
 *   btPolyhedralContactClipping::findSeparatingAxis   separating axis over the face normals of both hulls
 *       and the cross products of their edges (edge pairs restricted to Minkowski-difference faces, which
 *       never changes the least-overlap axis), oriented from B to A by the centroids;
 *   btPolyhedralContactClipping::clipHullAgainstHull  incident face of B (most aligned with the axis)
 *       clipped (Sutherland-Hodgman) against the side planes of A's witness face (most anti-aligned),
 *       points behind the witness plane kept with their signed depth (clamped below at the axis overlap);
 *   the edge-edge closest-point contact when the axis is an edge pair;
 *   btGjkPairDetector for hull-sphere: the exact closest point of the hull surface to the sphere centre.
 *
 * Every produced point goes to the persistent manifold (which keeps 4 by sortCachedPoints), as Bullet's
 * btManifoldResult does.  Margins are applied as in the product path (hull + 0.001 outside, box inside),
 * so the comparison isolates geometry (LOD, edge contacts, exact distances) from margin policy.
 * Not used by any kernel, by bench.py's measured path or by the parity tests.
 */
#ifndef UG_FIDELITY_H
#define UG_FIDELITY_H
#ifndef UG_HULL_POLYS
#error "the fidelity build needs the model header made with URGYM_HULL_POLYS=1 (tools/collision_fidelity.py)"
/* known-answer hook for tests/test_collision_fidelity.py: box A (half extents ha, pose qa/pa) vs box B through the
 * polyhedral path; writes up to max_pts candidates as (n3, pB3, d) and returns their count */
int ugo_fid_box_box(const double* ha, const double* Ra, const double* pa, const double* hb, const double* Rb,
                    const double* pb, double thr, double* out, int max_pts) {
    collider A, B;
    memset(&A, 0, sizeof(A));
    memset(&B, 0, sizeof(B));
    for (int i = 0; i < 3; i++) { A.half[i] = ha[i]; B.half[i] = hb[i]; }
    xf TA, TB;
    memcpy(TA.R.m, Ra, sizeof(TA.R.m));
    memcpy(TB.R.m, Rb, sizeof(TB.R.m));
    TA.p = V(pa[0], pa[1], pa[2]);
    TB.p = V(pb[0], pb[1], pb[2]);
    fp_box(&g_fpA, &TA, &A);
    fp_box(&g_fpB, &TB, &B);
    static candlist L;
    cand_init(&L, MAXCAND);
    fp_hull_hull(&g_fpA, &g_fpB, 0.0, 0.0, thr, &L);
    int n = L.n < max_pts ? L.n : max_pts;
    for (int i = 0; i < n; i++) {
        double* o = out + 7 * i;
        o[0] = L.c[i].n.x; o[1] = L.c[i].n.y; o[2] = L.c[i].n.z;
        o[3] = L.c[i].pB.x; o[4] = L.c[i].pB.y; o[5] = L.c[i].pB.z;
        o[6] = L.c[i].d;
    }
    return L.n;
}
#endif

#define FP_MAXV 1024
#define FP_MAXF 2048
#define FP_MAXE 4096
#define FP_MAXLOOP 2048

typedef struct {
    int nv, nf, ne;
    v3 v[FP_MAXV];        /* world vertices */
    v3 fn[FP_MAXF];       /* world outward face normals */
    double fd[FP_MAXF];   /* plane: fn . x <= fd */
    int fv0[FP_MAXF], fvn[FP_MAXF];
    int loop[FP_MAXLOOP * 4]; /* local vertex indices of the face loops */
    int e[FP_MAXE][4];    /* edge: v0, v1, face0, face1 */
    v3 c;                 /* centroid of the vertices */
} fpoly;

/* edges with their two faces from the face loops (each edge appears in exactly two loops); computed once per
 * shape (key: the hull's first face, -1 for boxes) and cached */
static struct { int key, ne; int (*e)[4]; } g_ecache[64];
static int g_necache;
static void fp_edges(fpoly* P, int key) {
    for (int c = 0; c < g_necache; c++)
        if (g_ecache[c].key == key) {
            P->ne = g_ecache[c].ne;
            memcpy(P->e, g_ecache[c].e, sizeof(int[4]) * P->ne);
            return;
        }
    P->ne = 0;
    for (int f = 0; f < P->nf; f++) {
        const int n = P->fvn[f];
        for (int k = 0; k < n; k++) {
            int a = P->loop[P->fv0[f] + k], b = P->loop[P->fv0[f] + (k + 1) % n];
            int found = -1;
            for (int i = 0; i < P->ne; i++)
                if ((P->e[i][0] == a && P->e[i][1] == b) || (P->e[i][0] == b && P->e[i][1] == a)) { found = i; break; }
            if (found >= 0) { if (P->e[found][3] < 0) P->e[found][3] = f; }
            else if (P->ne < FP_MAXE) { P->e[P->ne][0] = a; P->e[P->ne][1] = b; P->e[P->ne][2] = f; P->e[P->ne][3] = -1; P->ne++; }
        }
    }
    if (g_necache < 64) {
        g_ecache[g_necache].key = key;
        g_ecache[g_necache].ne = P->ne;
        g_ecache[g_necache].e = malloc(sizeof(int[4]) * (P->ne > 0 ? P->ne : 1));
        memcpy(g_ecache[g_necache].e, P->e, sizeof(int[4]) * P->ne);
        g_necache++;
    }
}
static void fp_finish(fpoly* P) {
    v3 c = V(0, 0, 0);
    for (int i = 0; i < P->nv; i++) c = vadd(c, P->v[i]);
    P->c = vscale(c, 1.0 / P->nv);
}
/* hull collider in world space (full hull + face loops from the fidelity model header) */
static void fp_hull(fpoly* P, const xf* T, const collider* A) {
    P->nv = A->nv;
    P->nf = A->nf;
    for (int i = 0; i < A->nv; i++) {
        const double* vv = &UG_HULL_V[3 * (A->v0 + i)];
        P->v[i] = xf_apply(T, V(vv[0], vv[1], vv[2]));
    }
    int k = 0;
    for (int f = 0; f < A->nf; f++) {
        const double* F = &UG_HULL_F[4 * (A->f0 + f)];
        P->fn[f] = mv(&T->R, V(F[0], F[1], F[2]));
        P->fd[f] = F[3] + vdot(P->fn[f], T->p);
        P->fv0[f] = k;
        P->fvn[f] = UG_HULL_FVN[A->f0 + f];
        for (int j = 0; j < P->fvn[f]; j++) P->loop[k++] = UG_HULL_FV[UG_HULL_FV0[A->f0 + f] + j] - A->v0;
    }
    fp_edges(P, A->f0);
    fp_finish(P);
}
/* box collider (half extents, margin inside) as a polyhedron: corner c = (x:bit0, y:bit1, z:bit2) */
static void fp_box(fpoly* P, const xf* T, const collider* B) {
    static const int loops[6][4] = {{1, 3, 7, 5}, {0, 4, 6, 2}, {2, 6, 7, 3}, {0, 1, 5, 4}, {4, 5, 7, 6}, {0, 2, 3, 1}};
    static const double nrm[6][3] = {{1, 0, 0}, {-1, 0, 0}, {0, 1, 0}, {0, -1, 0}, {0, 0, 1}, {0, 0, -1}};
    const double* h = B->half;
    P->nv = 8;
    P->nf = 6;
    for (int c = 0; c < 8; c++)
        P->v[c] = xf_apply(T, V((c & 1) ? h[0] : -h[0], (c & 2) ? h[1] : -h[1], (c & 4) ? h[2] : -h[2]));
    for (int f = 0; f < 6; f++) {
        P->fn[f] = mv(&T->R, V(nrm[f][0], nrm[f][1], nrm[f][2]));
        P->fd[f] = h[f >> 1] + vdot(P->fn[f], T->p);
        P->fv0[f] = 4 * f;
        P->fvn[f] = 4;
        for (int j = 0; j < 4; j++) P->loop[4 * f + j] = loops[f][j];
    }
    fp_edges(P, -1);
    fp_finish(P);
}
static void fp_project(const fpoly* P, v3 n, double* lo, double* hi) {
    double a = 1e300, b = -1e300;
    for (int i = 0; i < P->nv; i++) {
        double x = vdot(P->v[i], n);
        if (x < a) a = x;
        if (x > b) b = x;
    }
    *lo = a;
    *hi = b;
}
/* Minkowski-face test of edge (faces a, b of A) against edge (faces c, d of B): their Gauss-map arcs cross */
static int fp_minkowski(v3 a, v3 b, v3 c, v3 d) {
    c = vneg(c);
    d = vneg(d);
    v3 bxa = vcross(b, a), dxc = vcross(d, c);
    double cba = vdot(c, bxa), dba = vdot(d, bxa), adc = vdot(a, dxc), bdc = vdot(b, dxc);
    return cba * dba < 0.0 && adc * bdc < 0.0 && cba * bdc > 0.0;
}

typedef struct { v3 n; double depth; int ea, eb; } fp_axis; /* n from B towards A; depth = overlap */

/* findSeparatingAxis: least projection overlap over the candidate axes; returns 0 when separated by more
 * than `slack` (margins + breaking threshold) along some axis */
static int fp_sep_axis(const fpoly* A, const fpoly* B, double slack, fp_axis* out) {
    v3 dc = vsub(A->c, B->c);
    double dmin = 1e300;
    int found = 0;
#define FP_TEST(axis, EA, EB)                                                   \
    do {                                                                        \
        v3 n_ = (axis);                                                         \
        if (vdot(dc, n_) < 0.0) n_ = vneg(n_);                                  \
        double a0, a1, b0, b1;                                                  \
        fp_project(A, n_, &a0, &a1);                                            \
        fp_project(B, n_, &b0, &b1);                                            \
        double d0 = a1 - b0, d1 = b1 - a0;                                      \
        double d = d0 < d1 ? d0 : d1;                                           \
        if (d < -slack) return 0;                                               \
        if (d < dmin) { dmin = d; out->n = n_; out->ea = (EA); out->eb = (EB); found = 1; } \
    } while (0)
    for (int f = 0; f < A->nf; f++) FP_TEST(A->fn[f], -1, -1);
    for (int f = 0; f < B->nf; f++) FP_TEST(B->fn[f], -1, -1);
    /* edge pairs (Gregorius' edge query): the axis is oriented outward from A at A's edge and the pair's own
     * separation dot(N, pB - pA) is used, so among parallel axes the supporting pair wins (a full-projection
     * overlap is the same for every pair sharing the axis and cannot tell them apart) */
    for (int i = 0; i < A->ne; i++) {
        if (A->e[i][3] < 0) continue;
        v3 pa = A->v[A->e[i][0]];
        v3 ea = vsub(A->v[A->e[i][1]], pa);
        for (int j = 0; j < B->ne; j++) {
            if (B->e[j][3] < 0) continue;
            if (!fp_minkowski(A->fn[A->e[i][2]], A->fn[A->e[i][3]], B->fn[B->e[j][2]], B->fn[B->e[j][3]])) continue;
            v3 pb = B->v[B->e[j][0]];
            v3 eb = vsub(B->v[B->e[j][1]], pb);
            v3 x = vcross(ea, eb);
            double l = vlen(x);
            if (l < 1e-9 * vlen(ea) * vlen(eb)) continue;
            x = vscale(x, 1.0 / l);
            if (vdot(x, vsub(pa, A->c)) < 0.0) x = vneg(x); /* outward from A */
            double d = -vdot(x, vsub(pb, pa));               /* overlap of the pair along x */
            if (d < -slack) return 0;
            if (d < dmin) { dmin = d; out->n = vneg(x); out->ea = i; out->eb = j; found = 1; }
        }
    }
#undef FP_TEST
    out->depth = dmin;
    return found;
}
/* Sutherland-Hodgman: keep the part of the polygon with m . x <= off */
static int fp_clip(const v3* in, int n, v3 m, double off, v3* out) {
    int k = 0;
    if (n == 0) return 0;
    v3 a = in[n - 1];
    double da = vdot(m, a) - off;
    for (int i = 0; i < n; i++) {
        v3 b = in[i];
        double db = vdot(m, b) - off;
        if (da <= 0.0) {
            if (db <= 0.0) out[k++] = b;
            else out[k++] = vadd(a, vscale(vsub(b, a), da / (da - db)));
        } else if (db <= 0.0) {
            out[k++] = vadd(a, vscale(vsub(b, a), da / (da - db)));
            out[k++] = b;
        }
        a = b;
        da = db;
    }
    return k;
}
/* closest points of segments p0 + s (p1 - p0) and q0 + t (q1 - q0) */
static void fp_seg_closest(v3 p0, v3 p1, v3 q0, v3 q1, v3* cp, v3* cq) {
    v3 d1 = vsub(p1, p0), d2 = vsub(q1, q0), r = vsub(p0, q0);
    double a = vdot(d1, d1), e = vdot(d2, d2), f = vdot(d2, r), c = vdot(d1, r), b = vdot(d1, d2);
    double den = a * e - b * b, s = den > 1e-300 ? (b * f - c * e) / den : 0.0;
    s = s < 0.0 ? 0.0 : (s > 1.0 ? 1.0 : s);
    double t = (b * s + f) / e;
    if (t < 0.0) { t = 0.0; s = -c / a; s = s < 0.0 ? 0.0 : (s > 1.0 ? 1.0 : s); }
    else if (t > 1.0) { t = 1.0; s = (b - c) / a; s = s < 0.0 ? 0.0 : (s > 1.0 ? 1.0 : s); }
    *cp = vadd(p0, vscale(d1, s));
    *cq = vadd(q0, vscale(d2, t));
}
/* convex A (margin mA) vs convex B (margin mB): candidates (n on B towards A, point on B, depth incl. margins) */
static void fp_hull_hull(const fpoly* A, const fpoly* B, double mA, double mB, double thr, candlist* out) {
    fp_axis ax;
    const double m = mA + mB;
    if (!fp_sep_axis(A, B, m + thr, &ax)) return;
    v3 n = ax.n;
    /* edge-edge axis: the segments' closest points */
    if (ax.ea >= 0) {
        v3 ca, cb;
        fp_seg_closest(A->v[A->e[ax.ea][0]], A->v[A->e[ax.ea][1]], B->v[B->e[ax.eb][0]], B->v[B->e[ax.eb][1]], &ca, &cb);
        double d = vdot(vsub(ca, cb), n) - m;
        if (d < thr) cand_add(out, n, cb, d);
    }
    /* incident face of B (most aligned with n), witness face of A (most anti-aligned) */
    int fb = 0, fa = 0;
    double bmax = -1e300, amin = 1e300;
    for (int f = 0; f < B->nf; f++) { double d = vdot(B->fn[f], n); if (d > bmax) { bmax = d; fb = f; } }
    for (int f = 0; f < A->nf; f++) { double d = vdot(A->fn[f], n); if (d < amin) { amin = d; fa = f; } }
    static v3 buf0[FP_MAXLOOP + 64], buf1[FP_MAXLOOP + 64];
    int k = B->fvn[fb];
    for (int j = 0; j < k; j++) buf0[j] = B->v[B->loop[B->fv0[fb] + j]];
    v3* in = buf0;
    v3* o = buf1;
    const int na = A->fvn[fa];
    v3 ctr = V(0, 0, 0);
    for (int j = 0; j < na; j++) ctr = vadd(ctr, A->v[A->loop[A->fv0[fa] + j]]);
    ctr = vscale(ctr, 1.0 / na);
    for (int j = 0; j < na && k > 0; j++) {
        v3 a = A->v[A->loop[A->fv0[fa] + j]], b = A->v[A->loop[A->fv0[fa] + (j + 1) % na]];
        v3 sn = vcross(vsub(b, a), A->fn[fa]);
        double l = vlen(sn);
        if (l < 1e-15) continue;
        sn = vscale(sn, 1.0 / l);
        if (vdot(sn, vsub(ctr, a)) > 0.0) sn = vneg(sn); /* side plane faces out of the witness face */
        k = fp_clip(in, k, sn, vdot(sn, a), o);
        v3* t = in; in = o; o = t;
    }
    const double dclamp = -ax.depth - m; /* minDist: no point deeper than the axis overlap */
    for (int j = 0; j < k; j++) {
        double d = vdot(A->fn[fa], in[j]) - A->fd[fa] - m;
        if (d < dclamp) d = dclamp;
        if (d < thr) cand_add(out, n, in[j], d);
    }
}
static fpoly g_fpA, g_fpB; /* single-threaded fidelity runs (the tool drives one env per process) */
static void nc_hull_box(const xf* TA, const collider* A, const xf* TB, const collider* B, double thr, candlist* out) {
    fp_hull(&g_fpA, TA, A);
    fp_box(&g_fpB, TB, B);
    fp_hull_hull(&g_fpA, &g_fpB, A->margin, 0.0, thr, out);
}
static void nc_hull_hull(const xf* TA, const collider* A, const xf* TB, const collider* B, double thr, candlist* out) {
    fp_hull(&g_fpA, TA, A);
    fp_hull(&g_fpB, TB, B);
    fp_hull_hull(&g_fpA, &g_fpB, A->margin, B->margin, thr, out);
}
/* hull (A) vs sphere (B): exact closest point of the hull surface to the centre (GJK), deepest face inside */
static void nc_hull_sphere(const xf* TA, const collider* A, const xf* TB, const collider* B, double thr, candlist* out) {
    fp_hull(&g_fpA, TA, A);
    const fpoly* P = &g_fpA;
    v3 c = TB->p;
    const double r = B->half[0];
    double smax = -1e300;
    int fm = 0;
    for (int f = 0; f < P->nf; f++) {
        double sd = vdot(P->fn[f], c) - P->fd[f];
        if (sd > smax) { smax = sd; fm = f; }
    }
    v3 u;      /* unit normal from the hull towards the centre */
    double dist;
    if (smax <= 0.0) { u = P->fn[fm]; dist = smax; }
    else {
        double best = 1e300;
        v3 q = c;
        for (int f = 0; f < P->nf; f++) {
            double sd = vdot(P->fn[f], c) - P->fd[f];
            if (sd <= 0.0) continue;
            v3 p = vsub(c, vscale(P->fn[f], sd)); /* projection onto the face plane */
            int inside = 1;
            const int nf = P->fvn[f];
            v3 ctr = V(0, 0, 0);
            for (int t = 0; t < nf; t++) ctr = vadd(ctr, P->v[P->loop[P->fv0[f] + t]]);
            ctr = vscale(ctr, 1.0 / nf);
            for (int j = 0; j < nf && inside; j++) {
                v3 a = P->v[P->loop[P->fv0[f] + j]], b = P->v[P->loop[P->fv0[f] + (j + 1) % nf]];
                v3 sn = vcross(vsub(b, a), P->fn[f]);
                if (vdot(sn, vsub(ctr, a)) > 0.0) sn = vneg(sn);
                if (vdot(sn, vsub(p, a)) > 0.0) inside = 0;
            }
            if (inside) { if (sd < best) { best = sd; q = p; } continue; }
            for (int j = 0; j < nf; j++) {
                v3 a = P->v[P->loop[P->fv0[f] + j]], b = P->v[P->loop[P->fv0[f] + (j + 1) % nf]];
                v3 ab = vsub(b, a);
                double t = vdot(vsub(c, a), ab) / vdot(ab, ab);
                t = t < 0.0 ? 0.0 : (t > 1.0 ? 1.0 : t);
                v3 x = vadd(a, vscale(ab, t));
                double d = vlen(vsub(c, x));
                if (d < best) { best = d; q = x; }
            }
        }
        dist = best;
        u = vscale(vsub(c, q), 1.0 / best);
    }
    double depth = dist - r - A->margin;
    if (depth >= thr) return;
    v3 nw = vneg(u);
    cand_add(out, nw, vadd(c, vscale(nw, r)), depth);
}
/* known-answer hook for tests/test_collision_fidelity.py: box A (half extents ha, pose qa/pa) vs box B through the
 * polyhedral path; writes up to max_pts candidates as (n3, pB3, d) and returns their count */
int ugo_fid_box_box(const double* ha, const double* Ra, const double* pa, const double* hb, const double* Rb,
                    const double* pb, double thr, double* out, int max_pts) {
    collider A, B;
    memset(&A, 0, sizeof(A));
    memset(&B, 0, sizeof(B));
    for (int i = 0; i < 3; i++) { A.half[i] = ha[i]; B.half[i] = hb[i]; }
    xf TA, TB;
    memcpy(TA.R.m, Ra, sizeof(TA.R.m));
    memcpy(TB.R.m, Rb, sizeof(TB.R.m));
    TA.p = V(pa[0], pa[1], pa[2]);
    TB.p = V(pb[0], pb[1], pb[2]);
    fp_box(&g_fpA, &TA, &A);
    fp_box(&g_fpB, &TB, &B);
    static candlist L;
    cand_init(&L, MAXCAND);
    fp_hull_hull(&g_fpA, &g_fpB, 0.0, 0.0, thr, &L);
    int n = L.n < max_pts ? L.n : max_pts;
    for (int i = 0; i < n; i++) {
        double* o = out + 7 * i;
        o[0] = L.c[i].n.x; o[1] = L.c[i].n.y; o[2] = L.c[i].n.z;
        o[3] = L.c[i].pB.x; o[4] = L.c[i].pB.y; o[5] = L.c[i].pB.z;
        o[6] = L.c[i].d;
    }
    return L.n;
}
#endif
