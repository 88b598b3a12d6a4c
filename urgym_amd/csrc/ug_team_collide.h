/* ug_team_collide.h -- part of ug_team.h: collision: broadphase, the hull / box / cylinder / GJK narrowphases, the manifold update (team_collide).
 * Included by ug_team.h inside namespace ugd, in this order (the kernel is one translation unit); not self-contained. */
/* ---------------- collision ---------------- */
#define HB_FACE_UNROLL 12 /* covers hulls of up to 96 faces (the model's largest has 89) */
/* hull (A, robot link) vs box (B): the whole wave.  Produces cand k (<= 4 points) in sh.u.cand. */
__device__ __forceinline__ static void team_reduce4(int n, int k);
__device__ __forceinline__ static void team_hull_box(const HullArg& A, const HullArg& B, const XF& TA, const XF& TB,
                                     double thr, int k, unsigned char* hcert) {
    Shared& sh = g_sh;
    const int lane = threadIdx.x;
    PROF_T0(t_hv);
    m3 RAB = mtm(TB.R, TA.R);
    v3 pAB = mtv(TB.R, vsub(TA.p, TB.p));
    v3 h = V(B.half[0], B.half[1], B.half[2]);
    double mA = A.margin;
    /* vertices (lane i = vertex i) */
    int vvalid = 0;
    Cand vc;
    if (lane < A.nv) {
        const double* vv = &UG_HULL_V[3 * (A.v0 + lane)];
        v3 x = vadd(mv(RAB, V(vv[0], vv[1], vv[2])), pAB);
        v3 d = V(ug_fabs(x.x) - h.x, ug_fabs(x.y) - h.y, ug_fabs(x.z) - h.z);
        double dist = 0.0;
        v3 nl = V(0, 0, 0), pl = V(0, 0, 0);
        int ok = 1;
        if (d.x < 0 && d.y < 0 && d.z < 0) {
            int kk = 0;
            double dm = d.x;
            if (d.y > dm) { dm = d.y; kk = 1; }
            if (d.z > dm) { dm = d.z; kk = 2; }
            dist = dm;
            double sg = vget(x, kk) < 0 ? -1.0 : 1.0;
            vsetc(nl, kk, sg);
            pl = x; vsetc(pl, kk, sg * vget(h, kk));
        } else {
            v3 q = V(ug_max(-h.x, ug_min(h.x, x.x)), ug_max(-h.y, ug_min(h.y, x.y)), ug_max(-h.z, ug_min(h.z, x.z)));
            v3 df = vsub(x, q);
            double dl = vlen(df);
            if (dl - mA >= thr) ok = 0;
            else { dist = dl; nl = vscale(df, 1.0 / dl); pl = q; }
        }
        double depth = dist - mA;
        if (ok && depth < thr) {
            vvalid = 1;
            vc.n = mv(TB.R, nl);
            vc.pB = xf_apply(TB, pl);
            vc.d = depth;
        }
    }
    PROF_ADD(PF_HB_VERT, t_hv);
    PROF_T0(t_hc);
    /* box corners: 8 lanes per corner, faces strided over the group, then a group arg-max */
    int c = lane >> 3, j = lane & 7;
    m3 RBA = mtm(TA.R, TB.R);
    v3 pBA = mtv(TA.R, vsub(TB.p, TA.p));
    v3 cl = V((c & 1) ? h.x : -h.x, (c & 2) ? h.y : -h.y, (c & 4) ? h.z : -h.z);
    v3 y = vadd(mv(RBA, cl), pBA);
    double smax = -1e300;
    int fm = 0x7fffffff;
    const int nf = A.nf;
    /* certificate: a corner is rejected (smax - margin >= thr) as soon as one face's plane distance, formed
     * with the scan's own expression, clears it -- the scan's max is at least that value and the subtraction
     * is monotone.  The faces that maximised the corners last time usually still do: when all 8 corners are
     * rejected by them the face scan is skipped, with the same (empty) corner result. */
    bool certified = false;
    if (nf > 0) {
        int fc = hcert[c];
        fc = fc < nf ? fc : nf - 1;
        const double* F = &UG_HULL_F[4 * (A.f0 + fc)];
        const double sd = F[0] * y.x + F[1] * y.y + F[2] * y.z - F[3];
        certified = ballot(j == 0 && sd - mA >= thr) == 0x0101010101010101ull;
    }
    if (!certified) {
    /* the first HB_FACE_UNROLL x 8 faces with every plane load issued up front (clamped index, predicated
     * update: one load latency instead of one per face); faces beyond that (none in this model) in a loop */
    {
        double F[HB_FACE_UNROLL][4];
#pragma unroll
        for (int i = 0; i < HB_FACE_UNROLL; i++) {
            const int f = j + 8 * i;
#pragma unroll
            for (int c = 0; c < 4; c++) F[i][c] = UG_HULL_F[4 * (A.f0 + (f < nf ? f : 0)) + c];
        }
#pragma unroll
        for (int i = 0; i < HB_FACE_UNROLL; i++)
#pragma unroll
            for (int c = 0; c < 4; c++) asm volatile("" : "+v"(F[i][c])); /* one memory latency for all planes */
#pragma unroll
        for (int i = 0; i < HB_FACE_UNROLL; i++) {
            const int f = j + 8 * i;
            double sd = F[i][0] * y.x + F[i][1] * y.y + F[i][2] * y.z - F[i][3];
            if (f < nf && sd > smax) { smax = sd; fm = f; }
        }
    }
    for (int f = j + 8 * HB_FACE_UNROLL; f < nf; f += 8) {
        const double* F = &UG_HULL_F[4 * (A.f0 + f)];
        double sd = F[0] * y.x + F[1] * y.y + F[2] * y.z - F[3];
        if (sd > smax) { smax = sd; fm = f; }
    }
    {
        double w; int jj;
        w = dpp<0xB1>(smax); jj = dppi<0xB1>(fm);
        if (!better(smax, fm, w, jj, true)) { smax = w; fm = jj; }
        w = dpp<0x4E>(smax); jj = dppi<0x4E>(fm);
        if (!better(smax, fm, w, jj, true)) { smax = w; fm = jj; }
        w = dpp<0x141>(smax); jj = dppi<0x141>(fm);
        if (!better(smax, fm, w, jj, true)) { smax = w; fm = jj; }
    }
    if (j == 0 && fm != 0x7fffffff) hcert[c] = (unsigned char)fm;
    }
    int cvalid = 0;
    Cand cc;
    if (j == 0 && fm != 0x7fffffff) {
        double depth = smax - mA;
        if (depth < thr) {
            const double* F = &UG_HULL_F[4 * (A.f0 + fm)];
            v3 nw = mv(TA.R, V(F[0], F[1], F[2]));
            cvalid = 1;
            cc.n = vneg(nw);
            cc.pB = xf_apply(TB, cl);
            cc.d = depth;
        }
    }
    PROF_ADD(PF_HB_CORNER, t_hc);
    PROF_T0(t_hr);
    /* collect in canonical order: vertices by index, then corners by index */
    unsigned long long vb = ballot(vvalid), cb = ballot(cvalid);
    int nv = __popcll(vb), nc = __popcll(cb);
    if (vvalid) sh.hc[lane_prefix(vb)] = vc;
    if (cvalid) sh.hc[nv + lane_prefix(cb)] = cc;
    __syncthreads();
    team_reduce4(nv + nc, k);
    PROF_ADD(PF_HB_REDUCE, t_hr);
}

/* hull (A) vs hull (B) (oracle nc_hull_hull): lane per A vertex against B's planes, lane per B vertex against
 * A's planes; candidates in canonical order (A vertices, then B vertices; at most 64 kept), then reduce4 */
__device__ __forceinline__ static void team_hull_hull(const HullArg& A, const HullArg& B, const XF& TA, const XF& TB,
                                                   double thr, int k, unsigned char* hcert) {
    Shared& sh = g_sh;
    const int lane = threadIdx.x;
    double mA = A.margin, mB = B.margin;
    int avalid = 0, bvalid = 0;
    Cand ac, bc;
    if (lane < A.nv) {
        m3 RAB = mtm(TB.R, TA.R);
        v3 pAB = mtv(TB.R, vsub(TA.p, TB.p));
        const double* vv = &UG_HULL_V[3 * (A.v0 + lane)];
        v3 x = vadd(mv(RAB, V(vv[0], vv[1], vv[2])), pAB);
        double smax = -1e300;
        int fm = -1;
        hull_plane_max(B, x, smax, fm);
        double depth = smax - mA - mB;
        if (depth < thr) {
            const double* F = &UG_HULL_F[4 * (B.f0 + fm)];
            v3 nl = V(F[0], F[1], F[2]);
            v3 pl = vsub(x, vscale(nl, smax));
            avalid = 1;
            ac.n = mv(TB.R, nl);
            ac.pB = xf_apply(TB, pl);
            ac.d = depth;
        }
    }
    if (lane < B.nv) {
        m3 RBA = mtm(TA.R, TB.R);
        v3 pBA = mtv(TA.R, vsub(TB.p, TA.p));
        const double* vv = &UG_HULL_V[3 * (B.v0 + lane)];
        v3 yl = V(vv[0], vv[1], vv[2]);
        v3 y = vadd(mv(RBA, yl), pBA);
        double smax = -1e300;
        int fm = -1;
        /* certificate: the face that last maximised this vertex's plane distance; when its plane (the scan's own
         * expression) already clears thr + margins, the scan's maximum does too -- no candidate, scan skipped */
        int fc = lane < 64 ? hcert[lane] : 0;
        fc = fc < A.nf ? fc : A.nf - 1;
        const double* Fc = &UG_HULL_F[4 * (A.f0 + fc)];
        const double sdc = Fc[0] * y.x + Fc[1] * y.y + Fc[2] * y.z - Fc[3];
        if (sdc - mA - mB < thr) {
            hull_plane_max(A, y, smax, fm);
            hcert[lane] = (unsigned char)fm;
        } else {
            smax = sdc; /* rejected below */
        }
        double depth = smax - mA - mB;
        if (depth < thr) {
            const double* F = &UG_HULL_F[4 * (A.f0 + fm)];
            v3 nw = mv(TA.R, V(F[0], F[1], F[2]));
            bvalid = 1;
            bc.n = vneg(nw);
            bc.pB = xf_apply(TB, yl);
            bc.d = depth;
        }
    }
    unsigned long long amask = ballot(avalid), bmask = ballot(bvalid);
    int na = __popcll(amask), nb = __popcll(bmask);
    if (avalid) { int pos = lane_prefix(amask); if (pos < 64) sh.hc[pos] = ac; }
    if (bvalid) { int pos = na + lane_prefix(bmask); if (pos < 64) sh.hc[pos] = bc; }
    __syncthreads();
    int n = na + nb;
    team_reduce4(n < 64 ? n : 64, k);
}

/* candidates sh.hc[0..n) -> at most 4 in sh.u.cand.c[k] (oracle reduce4: deepest, then farthest-spread) */
__device__ __forceinline__ static void team_reduce4(int n, int k) {
    Shared& sh = g_sh;
    const int lane = threadIdx.x;
    if (n <= 4) {
        if (lane < n) sh.u.cand.c[k][lane] = sh.hc[lane];
        if (lane == 0) sh.u.cand.n[k] = n;
        __syncthreads();
        return;
    }
    /* reduce4: deepest first, then farthest-spread (oracle reduce4) */
    Cand mine;
    if (lane < n) mine = sh.hc[lane];
    double v = lane < n ? mine.d : 0.0;
    int idx = lane < n ? lane : 0x7fffffff;
    wave_best(v, idx, false);
    int sel[4];
    sel[0] = idx;
    double md = 1e300; /* squared distance to the nearest selected point, folded in one point per round (a min:
                        * the same value as the oracle's scan over all selected points) */
    for (int s = 1; s < 4; s++) {
        {
            const Cand& st = sh.hc[sel[s - 1]];
            v3 dd = vsub(mine.pB, st.pB);
            double x = vdot(dd, dd);
            if (x < md) md = x;
        }
        bool used = false;
        for (int t = 0; t < s; t++) used = used || (sel[t] == lane);
        double mv2 = md;
        int mi = (lane < n && !used) ? lane : 0x7fffffff;
        wave_best(mv2, mi, true);
        sel[s] = mi;
    }
    if (lane < 4) sh.u.cand.c[k][lane] = sh.hc[sel[lane]];
    if (lane == 0) sh.u.cand.n[k] = 4;
    __syncthreads();
}

/* ---- full-geometry mode (UG_GEOM_FULL): hulls with more vertices than lanes (up to UG_FULL_HULL_MAXV) and more
 * candidates than the LDS list holds.  Same arithmetic as the LOD functions above and as the oracle's nc_hull_box /
 * nc_hull_hull with every candidate kept (collider.full): vertices in chunks of 64 lanes, candidates in canonical
 * order (vertices by index, then corners / the other hull's vertices) in the env's global workspace, reduce4 over
 * that list (per-lane strided scans, then the wave-wide arg-min / arg-max with ties to the lower index). */
__device__ __forceinline__ void gc_put(gdouble* gc, int i, const Cand& c) {
    gdouble* o = gc + 7 * i;
    o[0] = c.n.x; o[1] = c.n.y; o[2] = c.n.z; o[3] = c.pB.x; o[4] = c.pB.y; o[5] = c.pB.z; o[6] = c.d;
}
__device__ __forceinline__ Cand gc_get(const gdouble* gc, int i) {
    const gdouble* o = gc + 7 * i;
    Cand c;
    c.n = V(o[0], o[1], o[2]);
    c.pB = V(o[3], o[4], o[5]);
    c.d = o[6];
    return c;
}
__device__ __forceinline__ void gc_publish() { /* the wave's workspace stores, visible to its later loads */
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
}
/* candidate i to the workspace list, and to the LDS list (g_sh.hc) while it fits: a pair that ends with at most 64
 * candidates is reduced from LDS (team_reduce4), a larger one from the workspace (team_reduce4_g) */
__device__ __forceinline__ void fc_put(gdouble* gc, int i, const Cand& c) {
    if (i < FC_MAX) gc_put(gc, i, c); /* beyond the list's capacity a candidate is dropped, as the oracle's cand_add */
    if (i < 64) g_sh.hc[i] = c;
}
/* the list length after a chunk's m candidates were appended at n (capped at the capacity, oracle cand_add) */
__device__ __forceinline__ int fc_count(int n, unsigned long long m) {
    const int t = n + __popcll(m);
    return t < FC_MAX ? t : FC_MAX;
}
__device__ __forceinline__ static void team_reduce4(int n, int k);
__device__ __forceinline__ void fc_reduce(int n, int k, gdouble* gc);
/* candidates gc[0..n) -> at most 4 in sh.u.cand.c[k] (oracle reduce4) */
__device__ __noinline__ static void team_reduce4_g(int n, int k, gdouble* gc) {
    PROF_CALL(CALL_REDUCE4);
    Shared& sh = g_sh;
    const int lane = threadIdx.x;
    if (n <= 4) {
        if (lane < n) sh.u.cand.c[k][lane] = gc_get(gc, lane);
        if (lane == 0) sh.u.cand.n[k] = n;
        __syncthreads();
        return;
    }
    /* deepest: the first minimum of d */
    double v = 0.0;
    int idx = 0x7fffffff;
    for (int i = lane; i < n; i += TEAM) {
        const double d = gc[7 * i + 6];
        if (idx == 0x7fffffff || d < v) { v = d; idx = i; }
    }
    wave_best(v, idx, false);
    int s0 = idx, s1 = -1, s2 = -1;
    v3 p0 = V(gc[7 * s0 + 3], gc[7 * s0 + 4], gc[7 * s0 + 5]), p1 = V(0, 0, 0), p2 = V(0, 0, 0);
    for (int s = 1; s < 4; s++) {
        /* farthest-spread: the first maximum of the squared distance to the nearest selected point */
        double mv2 = 0.0;
        int mi = 0x7fffffff;
        for (int i = lane; i < n; i += TEAM) {
            if (i == s0 || i == s1 || i == s2) continue;
            const v3 pb = V(gc[7 * i + 3], gc[7 * i + 4], gc[7 * i + 5]);
            double md = 1e300;
            {
                v3 dd = vsub(pb, p0);
                double x = vdot(dd, dd);
                if (x < md) md = x;
            }
            if (s > 1) {
                v3 dd = vsub(pb, p1);
                double x = vdot(dd, dd);
                if (x < md) md = x;
            }
            if (s > 2) {
                v3 dd = vsub(pb, p2);
                double x = vdot(dd, dd);
                if (x < md) md = x;
            }
            if (mi == 0x7fffffff || md > mv2) { mv2 = md; mi = i; }
        }
        wave_best(mv2, mi, true);
        const v3 pm = V(gc[7 * mi + 3], gc[7 * mi + 4], gc[7 * mi + 5]);
        if (s == 1) { s1 = mi; p1 = pm; }
        else if (s == 2) { s2 = mi; p2 = pm; }
        else {
            const int si = lane == 0 ? s0 : lane == 1 ? s1 : lane == 2 ? s2 : mi;
            if (lane < 4) sh.u.cand.c[k][lane] = gc_get(gc, si);
        }
    }
    if (lane == 0) sh.u.cand.n[k] = 4;
    __syncthreads();
}
__device__ __forceinline__ void fc_reduce(int n, int k, gdouble* gc) {
    if (n <= 64) { /* the LDS copy is complete: the LOD path's reduce4 (same selection, same arithmetic) */
        __syncthreads();
        team_reduce4(n, k);
    } else {
        gc_publish();
        team_reduce4_g(n, k, gc);
    }
}
/* hull (A, robot link) vs box (B), full geometry (oracle nc_hull_box).  A candidate-free evaluation whose every
 * chunk sphere and every box corner clears the threshold by a positive slack leaves a separation certificate
 * (pcert, WS_PC): team_collide skips the pair while the relative pose has moved less than that slack from the
 * certificate's pose (the skipped evaluation would produce no candidate; the manifold update still runs). */
__device__ __forceinline__ static void team_hull_box_full(const HullArg& A, const HullArg& B, const XF& TA, const XF& TB,
                                                       double thr, int k, unsigned short* hcert, gdouble* gc,
                                                       gdouble* pcert) {
    const int lane = threadIdx.x;
    const m3 RAB = mtm(TB.R, TA.R);
    const v3 pAB = mtv(TB.R, vsub(TA.p, TB.p));
    const v3 h = V(B.half[0], B.half[1], B.half[2]);
    const double mA = A.margin;
    int n = 0;
    PROF_T0(t_hv);
    /* exact chunk cull, every chunk at once (lane c tests chunk c): every vertex of a chunk lies in its bounding
     * sphere (UG_HULL_CS); when the sphere is farther than thr + margin from the box (with 1e-9 for rounding), no
     * vertex is inside the box or within the threshold, so the chunk adds no candidate -- the skipped work would
     * have produced none */
    unsigned long long live;
    /* certificate accumulators: this lane's lowest extent of the hull along each box face normal (culled chunks by
     * their spheres, surviving chunks vertex by vertex), and its chunk's vertex radius */
    double mf[6] = {1e300, 1e300, 1e300, 1e300, 1e300, 1e300};
    double crad = 0.0;
    {
        bool keep = false;
        if (lane < (A.nv + TEAM - 1) / TEAM) {
            const double* S = &UG_HULL_CS[4 * (A.c0 + lane)];
            const v3 cc = vadd(mv(RAB, V(S[0], S[1], S[2])), pAB);
            const v3 q = V(ug_max(-h.x, ug_min(h.x, cc.x)), ug_max(-h.y, ug_min(h.y, cc.y)), ug_max(-h.z, ug_min(h.z, cc.z)));
            keep = !(vlen(vsub(cc, q)) - S[3] >= thr + mA + 1e-9);
            crad = vlen(V(S[0], S[1], S[2])) + S[3];
            if (!keep) {
                mf[0] = -cc.x - S[3]; mf[1] = cc.x - S[3]; mf[2] = -cc.y - S[3];
                mf[3] = cc.y - S[3]; mf[4] = -cc.z - S[3]; mf[5] = cc.z - S[3];
            }
        }
        live = ballot(keep);
    }
    for (; live != 0ull; live &= live - 1ull) {
        const int v0 = TEAM * __builtin_ctzll(live);
        const int vi = v0 + lane;
        int vvalid = 0;
        Cand vc;
        if (vi < A.nv) {
            const double* vv = &UG_HULL_V[3 * (A.v0 + vi)];
            v3 x = vadd(mv(RAB, V(vv[0], vv[1], vv[2])), pAB);
            mf[0] = ug_min(mf[0], -x.x); mf[1] = ug_min(mf[1], x.x); mf[2] = ug_min(mf[2], -x.y);
            mf[3] = ug_min(mf[3], x.y); mf[4] = ug_min(mf[4], -x.z); mf[5] = ug_min(mf[5], x.z);
            v3 d = V(ug_fabs(x.x) - h.x, ug_fabs(x.y) - h.y, ug_fabs(x.z) - h.z);
            double dist = 0.0;
            v3 nl = V(0, 0, 0), pl = V(0, 0, 0);
            int ok = 1;
            if (d.x < 0 && d.y < 0 && d.z < 0) {
                int kk = 0;
                double dm = d.x;
                if (d.y > dm) { dm = d.y; kk = 1; }
                if (d.z > dm) { dm = d.z; kk = 2; }
                dist = dm;
                double sg = vget(x, kk) < 0 ? -1.0 : 1.0;
                vsetc(nl, kk, sg);
                pl = x; vsetc(pl, kk, sg * vget(h, kk));
            } else {
                v3 q = V(ug_max(-h.x, ug_min(h.x, x.x)), ug_max(-h.y, ug_min(h.y, x.y)), ug_max(-h.z, ug_min(h.z, x.z)));
                v3 df = vsub(x, q);
                double dl = vlen(df);
                if (dl - mA >= thr) ok = 0;
                else { dist = dl; nl = vscale(df, 1.0 / dl); pl = q; }
            }
            double depth = dist - mA;
            if (ok && depth < thr) {
                vvalid = 1;
                vc.n = mv(TB.R, nl);
                vc.pB = xf_apply(TB, pl);
                vc.d = depth;
            }
        }
        const unsigned long long vb = ballot(vvalid);
        if (vvalid) fc_put(gc, n + lane_prefix(vb), vc);
        n = fc_count(n, vb);
    }
    PROF_ADD(PF_HB_VERT, t_hv);
    PROF_T0(t_hc);
    /* box corners: 8 lanes per corner, faces strided over the group, group arg-max (first maximum) */
    const int c = lane >> 3, j = lane & 7;
    const m3 RBA = mtm(TA.R, TB.R);
    const v3 pBA = mtv(TA.R, vsub(TB.p, TA.p));
    const v3 cl = V((c & 1) ? h.x : -h.x, (c & 2) ? h.y : -h.y, (c & 4) ? h.z : -h.z);
    const v3 y = vadd(mv(RBA, cl), pBA);
    double smax = -1e300;
    int fm = 0x7fffffff;
    const int nf = A.nf;
    bool certified = false;
    double csd; /* the corner's distance beyond a separating face of A (the cached one, or the scanned maximum) */
    {
        int fc = hcert[c];
        fc = fc < nf ? fc : nf - 1;
        const double* F = &UG_HULL_F[4 * (A.f0 + fc)];
        const double sd = F[0] * y.x + F[1] * y.y + F[2] * y.z - F[3];
        certified = ballot(j == 0 && sd - mA >= thr) == 0x0101010101010101ull;
        csd = sd;
    }
    if (!certified) {
        /* faces strided over the 8-lane group, HB_FACE_UNROLL planes per lane per batch with their loads issued
         * together (clamped index, predicated update), as team_hull_box */
        for (int fb = 0; fb < nf; fb += 8 * HB_FACE_UNROLL) {
            double F[HB_FACE_UNROLL][4];
#pragma unroll
            for (int i = 0; i < HB_FACE_UNROLL; i++) {
                const int f = fb + j + 8 * i;
#pragma unroll
                for (int cc = 0; cc < 4; cc++) F[i][cc] = UG_HULL_F[4 * (A.f0 + (f < nf ? f : 0)) + cc];
            }
#pragma unroll
            for (int i = 0; i < HB_FACE_UNROLL; i++)
#pragma unroll
                for (int cc = 0; cc < 4; cc++) asm volatile("" : "+v"(F[i][cc]));
#pragma unroll
            for (int i = 0; i < HB_FACE_UNROLL; i++) {
                const int f = fb + j + 8 * i;
                const double sd = F[i][0] * y.x + F[i][1] * y.y + F[i][2] * y.z - F[i][3];
                if (f < nf && sd > smax) { smax = sd; fm = f; }
            }
        }
        double w;
        int jj;
        w = dpp<0xB1>(smax); jj = dppi<0xB1>(fm);
        if (!better(smax, fm, w, jj, true)) { smax = w; fm = jj; }
        w = dpp<0x4E>(smax); jj = dppi<0x4E>(fm);
        if (!better(smax, fm, w, jj, true)) { smax = w; fm = jj; }
        w = dpp<0x141>(smax); jj = dppi<0x141>(fm);
        if (!better(smax, fm, w, jj, true)) { smax = w; fm = jj; }
        if (j == 0 && fm != 0x7fffffff) hcert[c] = (unsigned short)fm;
        csd = smax;
    }
    int cvalid = 0;
    Cand cc;
    if (j == 0 && fm != 0x7fffffff) {
        const double depth = smax - mA;
        if (depth < thr) {
            const double* F = &UG_HULL_F[4 * (A.f0 + fm)];
            const v3 nw = mv(TA.R, V(F[0], F[1], F[2]));
            cvalid = 1;
            cc.n = vneg(nw);
            cc.pB = xf_apply(TB, cl);
            cc.d = depth;
        }
    }
    const unsigned long long cb = ballot(cvalid);
    if (cvalid) fc_put(gc, n + lane_prefix(cb), cc);
    n = fc_count(n, cb);
    if (n == 0) {
        /* candidate-free: certify when every box corner clears its face of A and the whole hull lies beyond one box
         * face plane, each by a positive margin (a vertex beyond a face plane by more than thr + margin is that far
         * from the box; the plane's margin changes only by the motion along its normal) */
        const double ks = j == 0 ? csd - mA - thr - 1e-9 : 1e300;
        if (ballot(!(ks > 0.0)) == 0ull) {
            double best = -1e300;
            int bf = 0;
#pragma unroll
            for (int f = 0; f < 6; f++) {
                const double hf = (f >> 1) == 0 ? h.x : ((f >> 1) == 1 ? h.y : h.z);
                const double sf = wave_min_d(mf[f]) - hf - thr - mA - 1e-9;
                if (sf > best) { best = sf; bf = f; }
            }
            if (best > 0.0) {
                const double sc = wave_min_d(ks);
                const double rA = wave_max_d(crad);
                if (lane == 0) {
                    pcert[0] = sc;
#pragma unroll
                    for (int i = 0; i < 9; i++) pcert[1 + i] = RAB.m[i];
                    pcert[10] = pAB.x; pcert[11] = pAB.y; pcert[12] = pAB.z;
                    pcert[13] = pBA.x; pcert[14] = pBA.y; pcert[15] = pBA.z;
                    pcert[16] = rA;
                    pcert[17] = vlen(h);
                    pcert[18] = best;
                    pcert[19] = (double)bf;
                }
            }
        }
    }
    PROF_ADD(PF_HB_CORNER, t_hc);
    PROF_T0(t_hr);
    fc_reduce(n, k, gc);
    PROF_ADD(PF_HB_REDUCE, t_hr);
}
/* hull (A, robot link) vs hull (B), full geometry (oracle nc_hull_hull, every candidate kept) */
__device__ __forceinline__ static void team_hull_hull_full(const HullArg& A, const HullArg& B, const XF& TA, const XF& TB,
                                                        double thr, int k, gdouble* gc) {
    const int lane = threadIdx.x;
    const double mA = A.margin, mB = B.margin;
    int n = 0;
    const m3 RAB = mtm(TB.R, TA.R);
    const v3 pAB = mtv(TB.R, vsub(TA.p, TB.p));
    for (int v0 = 0; v0 < A.nv; v0 += TEAM) {
        const int vi = v0 + lane;
        int valid = 0;
        Cand ac;
        if (vi < A.nv) {
            const double* vv = &UG_HULL_V[3 * (A.v0 + vi)];
            const v3 x = vadd(mv(RAB, V(vv[0], vv[1], vv[2])), pAB);
            double smax = -1e300;
            int fm = -1;
            hull_plane_max(B, x, smax, fm);
            const double depth = smax - mA - mB;
            if (depth < thr) {
                const double* F = &UG_HULL_F[4 * (B.f0 + fm)];
                const v3 nl = V(F[0], F[1], F[2]);
                const v3 pl = vsub(x, vscale(nl, smax));
                valid = 1;
                ac.n = mv(TB.R, nl);
                ac.pB = xf_apply(TB, pl);
                ac.d = depth;
            }
        }
        const unsigned long long m = ballot(valid);
        if (valid) fc_put(gc, n + lane_prefix(m), ac);
        n = fc_count(n, m);
    }
    const m3 RBA = mtm(TA.R, TB.R);
    const v3 pBA = mtv(TA.R, vsub(TB.p, TA.p));
    for (int v0 = 0; v0 < B.nv; v0 += TEAM) {
        const int vi = v0 + lane;
        int valid = 0;
        Cand bc;
        if (vi < B.nv) {
            const double* vv = &UG_HULL_V[3 * (B.v0 + vi)];
            const v3 yl = V(vv[0], vv[1], vv[2]);
            const v3 y = vadd(mv(RBA, yl), pBA);
            double smax = -1e300;
            int fm = -1;
            hull_plane_max(A, y, smax, fm);
            const double depth = smax - mA - mB;
            if (depth < thr) {
                const double* F = &UG_HULL_F[4 * (A.f0 + fm)];
                const v3 nw = mv(TA.R, V(F[0], F[1], F[2]));
                valid = 1;
                bc.n = vneg(nw);
                bc.pB = xf_apply(TB, yl);
                bc.d = depth;
            }
        }
        const unsigned long long m = ballot(valid);
        if (valid) fc_put(gc, n + lane_prefix(m), bc);
        n = fc_count(n, m);
    }
    fc_reduce(n, k, gc);
}

/* polytope (A: full robot hull or box) vs the disc cylinder (B), full geometry (oracle nc_poly_cyl): A's vertices
 * (chunks of 64 lanes, chunk spheres culled exactly) against the cylinder, then lane per face f of A: the cylinder's
 * support points along -n_f when its centre is in front of f, each scanned against all of A's planes (lane-serial,
 * the oracle's loop with its early exit), candidates face-major in the workspace list, reduce4.  swapped: the pair is
 * (cylinder, box) -- the 4 results get the oracle's role swap (normal flipped, point moved onto the box). */
__device__ __forceinline__ void poly_face(const HullArg& A, bool hull, int f, v3& n, double& off) {
    if (!hull) {
        const int ax = f >> 1;
        const double sg = (f & 1) ? 1.0 : -1.0;
        n = V(ax == 0 ? sg : 0.0, ax == 1 ? sg : 0.0, ax == 2 ? sg : 0.0);
        off = ax == 0 ? A.half[0] : ax == 1 ? A.half[1] : A.half[2];
        return;
    }
    const double* F = &UG_HULL_F[4 * (A.f0 + f)];
    n = V(F[0], F[1], F[2]);
    off = F[3];
}
__device__ __forceinline__ static void team_poly_cyl(int k, bool swapped, gdouble* gc) {
    Shared& sh = g_sh;
    const int lane = threadIdx.x;
    /* the pair's record straight from LDS, sides picked there: a run-time pick between two private copies is the
     * pattern this compiler miscompiles (tools/scc_audit.py, tests/test_isa_audit.py) */
    const PairInfo& P = sh.pinfo[k];
    const HullArg A = swapped ? P.B : P.A, B = swapped ? P.A : P.B;
    const XF TA = swapped ? P.TB : P.TA, TB = swapped ? P.TA : P.TB;
    const int akind = swapped ? P.kb : P.ka;
    const double thr = P.thr;
    const double r = B.half[0], hh = B.half[2];
    const bool hull = akind == UG_SHAPE_HULL;
    const double mA = hull ? A.margin : 0.0;
    const int nv = hull ? A.nv : 8, nf = hull ? A.nf : 6;
    const m3 RAB = mtm(TB.R, TA.R);
    const v3 pAB = mtv(TB.R, vsub(TA.p, TB.p));
    int n = 0;
    unsigned long long live = 1ull; /* a box: its 8 corners, one chunk */
    if (hull) { /* exact chunk cull, all chunks at once (the cylinder distance is 1-Lipschitz) */
        bool keep = false;
        if (lane < (nv + TEAM - 1) / TEAM) {
            const double* S = &UG_HULL_CS[4 * (A.c0 + lane)];
            const v3 cc = vadd(mv(RAB, V(S[0], S[1], S[2])), pAB);
            v3 t0, t1;
            keep = !(cyl_point(r, hh, cc, t0, t1) - S[3] >= thr + mA + 1e-9);
        }
        live = ballot(keep);
    }
    for (; live != 0ull; live &= live - 1ull) {
        const int v0 = TEAM * __builtin_ctzll(live);
        const int vi = v0 + lane;
        int valid = 0;
        Cand c;
        if (vi < nv) {
            v3 xa;
            if (hull) {
                const double* vv = &UG_HULL_V[3 * (A.v0 + vi)];
                xa = V(vv[0], vv[1], vv[2]);
            } else {
                xa = V((vi & 1) ? A.half[0] : -A.half[0], (vi & 2) ? A.half[1] : -A.half[1], (vi & 4) ? A.half[2] : -A.half[2]);
            }
            const v3 x = vadd(mv(RAB, xa), pAB);
            v3 nl, pl;
            const double depth = cyl_point(r, hh, x, nl, pl) - mA;
            if (depth < thr) {
                valid = 1;
                c.n = mv(TB.R, nl);
                c.pB = xf_apply(TB, pl);
                c.d = depth;
            }
        }
        const unsigned long long m = ballot(valid);
        if (valid) fc_put(gc, n + lane_prefix(m), c);
        n = fc_count(n, m);
    }
    const m3 RBA = mtm(TA.R, TB.R);
    const v3 pBA = mtv(TA.R, vsub(TB.p, TA.p));
    PROF_CNT(PC_CYPAIR, 1);
    PROF_T0(t_cy1);
    /* pass 1, lane per face f: the filter and the support points' own-plane test; the surviving (face, point) codes
     * 4 f + j go to a list in the workspace in (face, point) order.  Pass 2, lane per survivor: the plane scan
     * (lane-serial, the oracle's loop with its early exit), candidates appended in survivor order */
    typedef __attribute__((address_space(1))) int gint;
    gint* sv = (gint*)(gc + (WS_SV - WS_FC));
    int ns = 0;
    /* the largest margin by which a face of A separates the whole cylinder (its support points along -n_f are the
     * cylinder's lowest points under that plane); every vertex of A lies behind each of its face planes */
    double sepm = -1e300;
    for (int f0 = 0; f0 < nf; f0 += TEAM) {
        const int f = f0 + lane;
        bool ok[4] = {false, false, false, false};
        if (f < nf) {
            v3 nf_;
            double off;
            poly_face(A, hull, f, nf_, off);
            if (vdot(nf_, pBA) - off > 0) {
                const v3 u = mtv(RBA, vneg(nf_));
                const int ks = cyl_support_n(u);
                double fs = 1e300;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    if (j >= ks) break;
                    const v3 y = vadd(mv(RBA, cyl_support_pt(r, hh, u, j)), pBA);
                    const double sj = vdot(nf_, y) - off - mA;
                    ok[j] = !(sj >= thr);
                    fs = ug_min(fs, sj - thr - 1e-9);
                }
                sepm = ug_max(sepm, fs); /* fs > 0: face f's plane separates the whole cylinder with that margin */
            }
        }
        const int cnt = (int)ok[0] + (int)ok[1] + (int)ok[2] + (int)ok[3];
        const unsigned long long b0 = ballot(cnt & 1), b1 = ballot(cnt & 2), b2 = ballot(cnt & 4);
        int pos = ns + lane_prefix(b0) + 2 * lane_prefix(b1) + 4 * lane_prefix(b2);
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (ok[j]) sv[pos++] = 4 * f + j;
        ns += __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
    }
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
    PROF_ADD(PF_CY1, t_cy1);
    /* a separating face: every survivor is a point of the cylinder, so its plane scan would reach that face (or an
     * earlier separating one) and reject it -- pass 2 would add nothing (and, by the same plane, the vertex pass found
     * nothing).  The margin is the pair's separation certificate while the cylinder moves less than it in A's frame
     * (team_collide skips the pair then). */
    const double sep = wave_max_d(sepm);
    if (sep > 0.0 && n == 0) {
        ns = 0;
        if (hull && !swapped && lane == 0) {
            gdouble* pc = (gdouble*)(gc + (WS_PC - WS_FC)) + PC_DOUBLES * sh.ov[sh.is[3] + k];
            pc[0] = sep;
#pragma unroll
            for (int i = 0; i < 9; i++) pc[1 + i] = RAB.m[i];
            pc[10] = pAB.x; pc[11] = pAB.y; pc[12] = pAB.z;
            pc[13] = pBA.x; pc[14] = pBA.y; pc[15] = pBA.z;
            pc[16] = 0.0; /* the hull's vertices stay behind the face: only the cylinder's motion counts */
            pc[17] = ug_sqrt(r * r + hh * hh);
        }
    }
    PROF_T0(t_cy2);
    PROF_CNT(PC_CYSV, ns);
    for (int s0 = 0; s0 < ns; s0 += TEAM) {
        const int si = s0 + lane;
        int valid = 0;
        Cand c;
#ifdef UG_PROF
        int iters = 0;
#endif
        if (si < ns) {
            const int code = sv[si], f = code >> 2, j = code & 3;
            v3 nf_;
            double off;
            poly_face(A, hull, f, nf_, off);
            const v3 sp = cyl_support_pt(r, hh, mtv(RBA, vneg(nf_)), j);
            const v3 y = vadd(mv(RBA, sp), pBA);
            double smax = -1e300;
            int fm = -1;
            for (int g = 0; g < nf; g++) {
                v3 ng;
                double og;
                poly_face(A, hull, g, ng, og);
                const double sd = ng.x * y.x + ng.y * y.y + ng.z * y.z - og;
                if (sd > smax) { smax = sd; fm = g; }
#ifdef UG_PROF
                iters = g + 1;
#endif
                if (sd - mA >= thr) break;
            }
            const double depth = smax - mA;
            if (depth < thr) {
                v3 nm;
                double om;
                poly_face(A, hull, fm, nm, om);
                valid = 1;
                c.n = vneg(mv(TA.R, nm));
                c.pB = xf_apply(TB, sp);
                c.d = depth;
            }
        }
        const unsigned long long m = ballot(valid);
        if (valid) fc_put(gc, n + lane_prefix(m), c);
        n = fc_count(n, m);
#ifdef UG_PROF
        PROF_CNT(PC_CYIT, (int)wave_max_d((double)iters));
#endif
    }
    PROF_ADD(PF_CY2, t_cy2);
    fc_reduce(n, k, gc);
    if (swapped) { /* cylinder-box: the oracle's role swap on the kept points */
        if (lane < sh.u.cand.n[k]) {
            Cand c = sh.u.cand.c[k][lane];
            const v3 n0 = c.n;
            c.n = vneg(n0);
            c.pB = vadd(c.pB, vscale(n0, c.d));
            sh.u.cand.c[k][lane] = c;
        }
        __syncthreads();
    }
}

/* box (A) vs box (B) (oracle nc_box_box: ODE dBoxBox2 as btBoxBoxDetector), the whole wave per pair.  The same
 * operations on the same values as the serial routine, spread over lanes:
 *   - the 15 separating-axis tests in lanes 0..14 (any positive separation ends the pair, as the serial early
 *     return does whichever test it is), then the serial selection order -- faces by strict max, edges by the
 *     fudge-weighted test -- replayed on the broadcast values;
 *   - the face case's rectangle-quad clipping (intersectRectQuad2) one polygon vertex per lane per pass: each
 *     vertex emits [itself if inside][the crossing if its edge crosses], prefix sums give the serial emission
 *     order, and the serial cap at 8 points keeps the first 8 items and ends the clipping;
 *   - the contact points one per lane (kept ones compacted in order); cullPoints: the centroid as the serial
 *     chain, the angles one point per lane, each pick an arg-min whose ties go to the lower index (the serial
 *     scan's first minimum).
 * Writes cand k (0..4 points). */
/* column / element picks by selects: run-time indices into register-resident matrices made team_box_box read wrong
 * values (measured: the face normal and clip frame came out of the wrong column), so every pick is explicit */
#ifndef UG_BB_DYNIDX
__device__ __forceinline__ v3 colsel(const m3& A, int i) {
    return i == 0 ? V(A.m[0], A.m[3], A.m[6]) : i == 1 ? V(A.m[1], A.m[4], A.m[7]) : V(A.m[2], A.m[5], A.m[8]);
}
__device__ __forceinline__ double sel3(const double (&a)[3], int i) { return i == 0 ? a[0] : i == 1 ? a[1] : a[2]; }
__device__ __forceinline__ m3 msel(bool c, const m3& a, const m3& b) {
    m3 r;
#pragma unroll
    for (int i = 0; i < 9; i++) r.m[i] = c ? a.m[i] : b.m[i];
    return r;
}
#else /* investigation build (tools/bb_dynidx.sh): the run-time-indexed picks the selects replaced */
__device__ __forceinline__ v3 colsel(const m3& A, int i) { return V(A.m[i], A.m[3 + i], A.m[6 + i]); }
__device__ __forceinline__ double sel3(const double (&a)[3], int i) { return a[i]; }
__device__ __forceinline__ m3 msel(bool c, const m3& a, const m3& b) { return c ? a : b; }
#endif
#ifdef UG_BB_CHECK
static __shared__ int g_bbdbg[8];
#endif
__device__ __forceinline__ static void team_box_box(const XF& TA, const double (&Ah)[3], const XF& TB,
                                                    const double (&Bh)[3], int k) {
    Shared& sh = g_sh;
    const int lane = threadIdx.x;
    const double fudge = 1.05;
    const m3& R1 = TA.R;
    const m3& R2 = TB.R;
    const v3 p1 = TA.p, p2 = TB.p;
    const v3 p = vsub(p2, p1);
    const v3 pp = mtv(R1, p);
    const double R11 = col_dot(R1, 0, R2, 0), R12 = col_dot(R1, 0, R2, 1), R13 = col_dot(R1, 0, R2, 2);
    const double R21 = col_dot(R1, 1, R2, 0), R22 = col_dot(R1, 1, R2, 1), R23 = col_dot(R1, 1, R2, 2);
    const double R31 = col_dot(R1, 2, R2, 0), R32 = col_dot(R1, 2, R2, 1), R33 = col_dot(R1, 2, R2, 2);
    const double Q11 = ug_fabs(R11), Q12 = ug_fabs(R12), Q13 = ug_fabs(R13);
    const double Q21 = ug_fabs(R21), Q22 = ug_fabs(R22), Q23 = ug_fabs(R23);
    const double Q31 = ug_fabs(R31), Q32 = ug_fabs(R32), Q33 = ug_fabs(R33);
    /* lane t: test t (code t + 1) */
    double e1 = 0.0, x2 = 0.0, n1 = 0.0, n2 = 0.0, n3 = 0.0;
    switch (lane) {
    case 0: e1 = pp.x; x2 = (Ah[0] + Bh[0] * Q11 + Bh[1] * Q12 + Bh[2] * Q13); break;
    case 1: e1 = pp.y; x2 = (Ah[1] + Bh[0] * Q21 + Bh[1] * Q22 + Bh[2] * Q23); break;
    case 2: e1 = pp.z; x2 = (Ah[2] + Bh[0] * Q31 + Bh[1] * Q32 + Bh[2] * Q33); break;
    case 3: e1 = col_dotv(R2, 0, p); x2 = (Ah[0] * Q11 + Ah[1] * Q21 + Ah[2] * Q31 + Bh[0]); break;
    case 4: e1 = col_dotv(R2, 1, p); x2 = (Ah[0] * Q12 + Ah[1] * Q22 + Ah[2] * Q32 + Bh[1]); break;
    case 5: e1 = col_dotv(R2, 2, p); x2 = (Ah[0] * Q13 + Ah[1] * Q23 + Ah[2] * Q33 + Bh[2]); break;
    case 6: e1 = pp.z * R21 - pp.y * R31; x2 = (Ah[1] * Q31 + Ah[2] * Q21 + Bh[1] * Q13 + Bh[2] * Q12); n1 = 0; n2 = -R31; n3 = R21; break;
    case 7: e1 = pp.z * R22 - pp.y * R32; x2 = (Ah[1] * Q32 + Ah[2] * Q22 + Bh[0] * Q13 + Bh[2] * Q11); n1 = 0; n2 = -R32; n3 = R22; break;
    case 8: e1 = pp.z * R23 - pp.y * R33; x2 = (Ah[1] * Q33 + Ah[2] * Q23 + Bh[0] * Q12 + Bh[1] * Q11); n1 = 0; n2 = -R33; n3 = R23; break;
    case 9: e1 = pp.x * R31 - pp.z * R11; x2 = (Ah[0] * Q31 + Ah[2] * Q11 + Bh[1] * Q23 + Bh[2] * Q22); n1 = R31; n2 = 0; n3 = -R11; break;
    case 10: e1 = pp.x * R32 - pp.z * R12; x2 = (Ah[0] * Q32 + Ah[2] * Q12 + Bh[0] * Q23 + Bh[2] * Q21); n1 = R32; n2 = 0; n3 = -R12; break;
    case 11: e1 = pp.x * R33 - pp.z * R13; x2 = (Ah[0] * Q33 + Ah[2] * Q13 + Bh[0] * Q22 + Bh[1] * Q21); n1 = R33; n2 = 0; n3 = -R13; break;
    case 12: e1 = pp.y * R11 - pp.x * R21; x2 = (Ah[0] * Q21 + Ah[1] * Q11 + Bh[1] * Q33 + Bh[2] * Q32); n1 = -R21; n2 = R11; n3 = 0; break;
    case 13: e1 = pp.y * R12 - pp.x * R22; x2 = (Ah[0] * Q22 + Ah[1] * Q12 + Bh[0] * Q33 + Bh[2] * Q31); n1 = -R22; n2 = R12; n3 = 0; break;
    case 14: e1 = pp.y * R13 - pp.x * R23; x2 = (Ah[0] * Q23 + Ah[1] * Q13 + Bh[0] * Q32 + Bh[1] * Q31); n1 = -R23; n2 = R13; n3 = 0; break;
    default: break;
    }
    const bool test = lane < 15;
    const double s2 = ug_fabs(e1) - x2;
    if (ballot(test && s2 > 0) != 0ull) { /* a separating axis: no contact */
        if (lane == 0) sh.u.cand.n[k] = 0;
        __syncthreads();
        return;
    }
    double l = 0.0, s2n = 0.0;
    v3 nc = V(0, 0, 0);
    if (lane >= 6 && lane < 15) {
        l = ug_sqrt((n1) * (n1) + (n2) * (n2) + (n3) * (n3));
        if (l > 0) {
            s2n = s2 / l;
            nc = V((n1) / l, (n2) / l, (n3) / l);
        }
    }
    const unsigned long long neg = ballot(test && e1 < 0), lpos = ballot(lane >= 6 && lane < 15 && l > 0);
    double s = -1e300;
    int nR = -1, tsel = -1, invert_normal = 0, code = 0;
    for (int t = 0; t < 6; t++) {
        const double v = readlane_d(s2, t);
        if (v > s) { s = v; nR = t; invert_normal = (int)((neg >> t) & 1ull); code = t + 1; }
    }
    for (int t = 6; t < 15; t++) {
        if ((lpos >> t) & 1ull) {
            const double v = readlane_d(s2n, t);
            if (v * fudge > s) { s = v; nR = -1; tsel = t; invert_normal = (int)((neg >> t) & 1ull); code = t + 1; }
        }
    }
    int nout = 0;
    if (code) {
        v3 normal;
        if (nR >= 0) { /* column nR % 3 of R1 (nR < 3) or R2, by selects (no dynamic register indexing) */
            const m3& Rn = nR < 3 ? R1 : R2;
            const int c = nR % 3;
#ifndef UG_BB_DYNIDX
            normal = c == 0 ? V(Rn.m[0], Rn.m[3], Rn.m[6]) : c == 1 ? V(Rn.m[1], Rn.m[4], Rn.m[7]) : V(Rn.m[2], Rn.m[5], Rn.m[8]);
#else
            normal = V(Rn.m[c], Rn.m[3 + c], Rn.m[6 + c]);
#endif
        } else {
            normal = mv(R1, V(readlane_d(nc.x, tsel), readlane_d(nc.y, tsel), readlane_d(nc.z, tsel)));
        }
        if (invert_normal) normal = vneg(normal);
        const double depth = -s;
        if (code > 6) { /* edge-edge: one point (uniform arithmetic; lane 0 stores it) */
            v3 pa = p1;
            for (int j = 0; j < 3; j++) {
                double sign = (col_dotv(R1, j, normal) > 0) ? 1.0 : -1.0;
                pa = vadd(pa, V(sign * Ah[j] * R1.m[j], sign * Ah[j] * R1.m[3 + j], sign * Ah[j] * R1.m[6 + j]));
            }
            v3 pb = p2;
            for (int j = 0; j < 3; j++) {
                double sign = (col_dotv(R2, j, normal) > 0) ? -1.0 : 1.0;
                pb = vadd(pb, V(sign * Bh[j] * R2.m[j], sign * Bh[j] * R2.m[3 + j], sign * Bh[j] * R2.m[6 + j]));
            }
            const int ia = (code - 7) / 3, ib = (code - 7) % 3;
            const v3 ua = colsel(R1, ia);
            const v3 ub = colsel(R2, ib);
            const v3 pd = vsub(pb, pa);
            double uaub = vdot(ua, ub), q1 = vdot(ua, pd), q2 = -vdot(ub, pd);
            double d = 1.0 - uaub * uaub, beta;
            if (d <= 0.0001) { beta = 0; }
            else { d = 1.0 / d; beta = (uaub * q1 + q2) * d; }
            pb = vadd(pb, vscale(ub, beta));
            if (lane == 0) {
                Cand c;
                c.n = vneg(normal);
                c.pB = pb;
                c.d = -depth;
                sh.u.cand.c[k][0] = c;
            }
            nout = 1;
        } else { /* face: clip the incident face against the reference face's rectangle */
            const m3 Ra = msel(code <= 3, R1, R2);
            const m3 Rb = msel(code <= 3, R2, R1);
            const v3 pa = code <= 3 ? p1 : p2, pb = code <= 3 ? p2 : p1;
            const double Sa[3] = {code <= 3 ? Ah[0] : Bh[0], code <= 3 ? Ah[1] : Bh[1], code <= 3 ? Ah[2] : Bh[2]};
            const double Sb[3] = {code <= 3 ? Bh[0] : Ah[0], code <= 3 ? Bh[1] : Ah[1], code <= 3 ? Bh[2] : Ah[2]};
            const v3 normal2 = code <= 3 ? normal : vneg(normal);
            const v3 nr = mtv(Rb, normal2);
            const v3 anr = V(ug_fabs(nr.x), ug_fabs(nr.y), ug_fabs(nr.z));
            int lanr, a1, a2;
            if (anr.y > anr.x) {
                if (anr.y > anr.z) { a1 = 0; lanr = 1; a2 = 2; }
                else { a1 = 0; a2 = 1; lanr = 2; }
            } else {
                if (anr.x > anr.z) { lanr = 0; a1 = 1; a2 = 2; }
                else { a1 = 0; a2 = 1; lanr = 2; }
            }
            v3 center;
            const v3 rbl = colsel(Rb, lanr);
            if (vget(nr, lanr) < 0) center = vadd(vsub(pb, pa), vscale(rbl, sel3(Sb, lanr)));
            else center = vsub(vsub(pb, pa), vscale(rbl, sel3(Sb, lanr)));
            const int codeN = code <= 3 ? code - 1 : code - 4;
            int code1, code2;
            if (codeN == 0) { code1 = 1; code2 = 2; }
            else if (codeN == 1) { code1 = 0; code2 = 2; }
            else { code1 = 0; code2 = 1; }
            /* col_dotv / col_dot with the columns picked first: the same products and sums in the same order */
            const v3 ra1 = colsel(Ra, code1), ra2 = colsel(Ra, code2), rb1 = colsel(Rb, a1), rb2 = colsel(Rb, a2);
            const double c1 = vdot(ra1, center), c2 = vdot(ra2, center);
            double m11 = vdot(ra1, rb1), m12 = vdot(ra1, rb2);
            double m21 = vdot(ra2, rb1), m22 = vdot(ra2, rb2);
            const double Sba1 = sel3(Sb, a1), Sba2 = sel3(Sb, a2);
            /* the quad, vertex per lane (lanes 0..3) */
            double qx, qy;
            {
                const double k1 = m11 * Sba1, k2 = m21 * Sba1, k3 = m12 * Sba2, k4 = m22 * Sba2;
                const double x0 = c1 - k1 - k3, y0 = c2 - k2 - k4, x1 = c1 - k1 + k3, y1 = c2 - k2 + k4;
                const double x2q = c1 + k1 + k3, y2q = c2 + k2 + k4, x3 = c1 + k1 - k3, y3 = c2 + k2 - k4;
                qx = lane == 0 ? x0 : lane == 1 ? x1 : lane == 2 ? x2q : x3;
                qy = lane == 0 ? y0 : lane == 1 ? y1 : lane == 2 ? y2q : y3;
            }
            const double rect0 = sel3(Sa, code1), rect1 = sel3(Sa, code2);
            ldouble* buf = (ldouble*)&sh.bs[0].buffer[0]; /* one pass's output points (x, y), at most 8 */
            int nq = 4;
            bool capped = false;
            for (int pass = 0; pass < 4 && !capped; pass++) {
                const int dir = pass >> 1;
                const double sgn = (pass & 1) ? 1.0 : -1.0, hd = dir ? rect1 : rect0;
                const int nj = lane + 1 < nq ? lane + 1 : 0;
                const double nx = __shfl(qx, nj), ny = __shfl(qy, nj);
                const bool live = lane < nq;
                const double qd = dir ? qy : qx, qo = dir ? qx : qy, nd = dir ? ny : nx, no = dir ? nx : ny;
                const bool in = live && sgn * qd < hd;
                const bool cross = live && ((sgn * qd < hd) ^ (sgn * nd < hd));
                const unsigned long long bi = ballot(in), bc = ballot(cross);
                const unsigned long long below = (1ull << lane) - 1ull;
                const int pin = __popcll(bi & below) + __popcll(bc & below), pcr = pin + (in ? 1 : 0);
                const int total = __popcll(bi) + __popcll(bc);
                __builtin_amdgcn_wave_barrier();
                if (in && pin < 8) { buf[2 * pin] = qx; buf[2 * pin + 1] = qy; }
                if (cross && pcr < 8) {
                    const double ix = qo + (no - qo) / (nd - qd) * (sgn * hd - qd);
                    buf[2 * pcr + 1 - dir] = ix;
                    buf[2 * pcr + dir] = sgn * hd;
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_wave_barrier();
                nq = total < 8 ? total : 8;
                capped = total >= 8;
                qx = lane < nq ? buf[2 * lane] : 0.0;
                qy = lane < nq ? buf[2 * lane + 1] : 0.0;
                __builtin_amdgcn_wave_barrier();
            }
            if (nq >= 1) {
                const double det1 = 1.0 / (m11 * m22 - m12 * m21);
                m11 *= det1; m12 *= det1; m21 *= det1; m22 *= det1;
                const v3 rba1 = rb1, rba2 = rb2;
                const bool live = lane < nq;
                const double k1 = m22 * (qx - c1) - m12 * (qy - c2);
                const double k2 = -m21 * (qx - c1) + m11 * (qy - c2);
                const v3 pc = vadd(vadd(center, vscale(rba1, k1)), vscale(rba2, k2));
                const double dep = sel3(Sa, codeN) - vdot(normal2, pc);
                const bool keep = live && dep >= 0;
                const unsigned long long km = ballot(keep);
                const int cnum = __popcll(km), cpos = __popcll(km & ((1ull << lane) - 1ull));
                v3 pw = vadd(pc, pa);
                if (code >= 4) pw = vsub(pw, vscale(normal, dep));
                if (cnum >= 1 && cnum <= 4) {
                    if (keep) {
                        Cand c;
                        c.n = vneg(normal);
                        c.pB = pw;
                        c.d = -dep;
                        sh.u.cand.c[k][cpos] = c;
                    }
                    nout = cnum;
                } else if (cnum > 4) { /* cullPoints to 4, starting from the deepest */
                    double dv = keep ? dep : 0.0;
                    int di = keep ? cpos : 0x7fffffff;
                    wave_best(dv, di, true);
                    const int i0 = di;
                    ldouble* kp = (ldouble*)&sh.bs[0].ret[0]; /* the kept clip points (x, y) in order */
                    __builtin_amdgcn_wave_barrier();
                    if (keep) { kp[2 * cpos] = qx; kp[2 * cpos + 1] = qy; }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    __builtin_amdgcn_wave_barrier();
                    const int n = cnum;
                    double a = 0, cx = 0, cy = 0, qq;
                    for (int i = 0; i < n - 1; i++) {
                        qq = kp[i * 2] * kp[i * 2 + 3] - kp[i * 2 + 2] * kp[i * 2 + 1];
                        a += qq;
                        cx += qq * (kp[i * 2] + kp[i * 2 + 2]);
                        cy += qq * (kp[i * 2 + 1] + kp[i * 2 + 3]);
                    }
                    qq = kp[n * 2 - 2] * kp[1] - kp[0] * kp[n * 2 - 1];
                    if (ug_fabs(a + qq) > 2.220446049250313e-16) a = 1.0 / (3.0 * (a + qq));
                    else a = 1e30;
                    cx = a * (cx + qq * (kp[n * 2 - 2] + kp[0]));
                    cy = a * (cy + qq * (kp[n * 2 - 1] + kp[1]));
                    const double ang = keep ? ug_atan2(qy - cy, qx - cx) : 0.0;
                    /* the angles by kept index: lane cpos of the kept set holds point cpos */
                    ldouble* A = (ldouble*)&sh.bs[0].ang[0];
                    __builtin_amdgcn_wave_barrier();
                    if (keep) A[cpos] = ang;
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    __builtin_amdgcn_wave_barrier();
                    const double Ai = lane < n ? A[lane] : 0.0;
                    const double Ai0 = A[i0];
                    unsigned long long avail = (n == 64 ? ~0ull : ((1ull << n) - 1ull)) & ~(1ull << i0);
                    int iret[4];
                    iret[0] = i0;
                    const int m = 4;
                    for (int j = 1; j < m; j++) {
                        double aj = (double)j * (2.0 * UG_PI / m) + Ai0;
                        if (aj > UG_PI) aj -= 2.0 * UG_PI;
                        double diff = ug_fabs(Ai - aj);
                        if (diff > UG_PI) diff = 2.0 * UG_PI - diff;
                        const bool av = (avail >> lane) & 1ull;
                        int idx = av && diff < 1e9 ? lane : 0x7fffffff;
                        double dd = av ? diff : 0.0;
                        wave_best(dd, idx, false);
                        iret[j] = idx == 0x7fffffff ? i0 : idx;
                        avail &= ~(1ull << iret[j]);
                    }
                    if (keep) {
                        const int slot = cpos == iret[0] ? 0 : cpos == iret[1] ? 1 : cpos == iret[2] ? 2 : cpos == iret[3] ? 3 : -1;
                        if (slot >= 0) {
                            Cand c;
                            c.n = vneg(normal);
                            c.pB = pw;
                            c.d = -dep;
                            sh.u.cand.c[k][slot] = c;
                        }
                    }
                    nout = m;
                }
            }
        }
    }
    if (lane == 0) sh.u.cand.n[k] = nout;
#ifdef UG_BB_CHECK
    if (lane == 0) { g_bbdbg[0] = code; g_bbdbg[1] = tsel; g_bbdbg[2] = nR; }
#ifdef UG_BB_DYNIDX /* every lane's view of the picked values (a lane whose index disagrees would show here) */
    {
        const v3 n0 = nR >= 0 ? V((nR < 3 ? R1 : R2).m[nR % 3], (nR < 3 ? R1 : R2).m[3 + nR % 3], (nR < 3 ? R1 : R2).m[6 + nR % 3]) : V(0, 0, 0);
        const v3 n1 = nR >= 0 ? (nR % 3 == 0 ? V((nR < 3 ? R1 : R2).m[0], (nR < 3 ? R1 : R2).m[3], (nR < 3 ? R1 : R2).m[6])
                                : nR % 3 == 1 ? V((nR < 3 ? R1 : R2).m[1], (nR < 3 ? R1 : R2).m[4], (nR < 3 ? R1 : R2).m[7])
                                              : V((nR < 3 ? R1 : R2).m[2], (nR < 3 ? R1 : R2).m[5], (nR < 3 ? R1 : R2).m[8]))
                              : V(0, 0, 0);
        if (n0.x != n1.x || n0.y != n1.y || n0.z != n1.z)
            printf("BBIDX lane %d code %d nR %d tsel %d dyn (%.17g %.17g %.17g) sel (%.17g %.17g %.17g)\n", lane, code, nR,
                   tsel, n0.x, n0.y, n0.z, n1.x, n1.y, n1.z);
    }
#endif
#endif
    __syncthreads();
}

/* performDiscreteCollisionDetection (oracle collide()), team version.  ws: this env's global workspace. */
/* FULL: the full-geometry instantiation (UG_GEOM_FULL); the LOD one has no calls into the full-hull functions, so
 * its register allocation is that of the LOD path alone */
/* the convex-convex path: pairs without a dedicated Bullet algorithm (oracle pair_is_gjk) */
__device__ __forceinline__ static bool pair_is_gjk(const Collider& A, const Collider& B) {
    if (A.gjkbox || B.gjkbox) return true;
    const bool pa = A.kind == UG_SHAPE_SPHERE || A.kind == UG_SHAPE_BOX;
    const bool pb = B.kind == UG_SHAPE_SPHERE || B.kind == UG_SHAPE_BOX;
    return !(pa && pb);
}
__device__ __forceinline__ static ugk::GShape gshape_of(const Collider& c) {
    ugk::GShape g;
    g.kind = c.kind;
    g.v0 = c.v0;
    g.nv = c.kind == UG_SHAPE_HULL ? c.nv : 0;
    g.imp = ugk::V3(c.gimp.x, c.gimp.y, c.gimp.z);
    g.margin = c.gmargin;
    g.scb = c.kind == UG_SHAPE_HULL ? c.scb : -1;
    g.sck = c.sck;
    return g;
}
__device__ __forceinline__ static ugk::gx to_gx(const XF& T) {
    ugk::gx r;
#pragma unroll
    for (int i = 0; i < 9; i++) r.R.m[i] = T.R.m[i];
    r.p = ugk::V3(T.p.x, T.p.y, T.p.z);
    return r;
}
/* pair k of the pass (sh.pinfo[k]) through btGjkPairDetector on the whole wave (ug_gjk.h): at most one point, written
 * to cand k in this restatement's pair order (a sphere-first pair runs with the sphere as GJK's B, then flipped --
 * oracle nc_gjk) */
/* pair k of the pass (sh.pinfo[k]) through btGjkPairDetector on the whole wave (ug_gjk.h): at most one point, written
 * to cand k in this restatement's pair order (a sphere-first pair runs with the sphere as GJK's B, then flipped --
 * oracle nc_gjk).  A query that ends without a point the manifold keeps leaves a separation certificate: the
 * separating axis n (the reported normal, or the classic GJK's last axis) with both cores' extents along it, and the
 * relative pose; while the motion bound in team_collide proves that the margin-expanded shapes stay farther apart than
 * the contact threshold, the query would again add nothing, and the pair is skipped. */
__device__ __forceinline__ static void gjk_one(const Scene* s, int k, UGK_GMEM ugk::EpaMem* E, gdouble* gc) {
    Shared& sh = g_sh;
    const int a = sh.pinfo[k].a, b = sh.pinfo[k].b;
    const Collider& A = s->col[a];
    const Collider& B = s->col[b];
    const bool swap = A.kind == UG_SHAPE_SPHERE && B.kind != UG_SHAPE_SPHERE;
    const ugk::GShape g0 = gshape_of(swap ? B : A), g1 = gshape_of(swap ? A : B);
    const ugk::gx T0 = to_gx(swap ? sh.pinfo[k].TB : sh.pinfo[k].TA), T1 = to_gx(swap ? sh.pinfo[k].TA : sh.pinfo[k].TB);
    const double thr = sh.pinfo[k].thr;
    ugk::gv n, p, ax = ugk::V3(0, 0, 0);
    double d = 0.0;
    const bool lead = (threadIdx.x & (GJK_G - 1)) == 0; /* the group's writer */
    if (gc[0] > 0.0) {
        /* the pair's certificate failed team_collide's motion bound: test it exactly instead -- A's core extent along
         * the certified axis (fixed in B's frame) in the current pose, one support -- before the whole query.  The
         * cores are still apart by more than the margins and the threshold along it: GJK would keep no point, so
         * none is produced and the certificate moves to this pose. */
        const ugk::gv nb = ugk::V3(gc[1], gc[2], gc[3]);
        const ugk::gv uw = ugk::mv(T1.R, nb);
        const ugk::gv dA = ugk::mtv(T0.R, ugk::neg(uw));
        const double hA = ugk::dot(dA, ugk::support0(g0, dA));
        const ugk::gv pp = ugk::mtv(T1.R, ugk::sub(T0.p, T1.p));
        const double sep = ugk::dot(nb, pp) - hA - gc[5];
        if (sep - g0.margin - g1.margin - thr > 1e-9 * (1.0 + ug_fabs(sep))) {
            UGK_COUNT(PC_GJK_RECERT, 1);
            if (lead) {
                const ugk::gm R = ugk::mtm(T1.R, T0.R);
                gc[4] = hA;
                for (int i = 0; i < 9; i++) gc[6 + i] = R.m[i];
                gc[15] = pp.x; gc[16] = pp.y; gc[17] = pp.z;
                sh.u.cand.n[k] = 0;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            return;
        }
    }
    const bool ok = ugk::gjk_pair(E, g0, T0, g1, T1, thr, n, p, d, &ax);
    /* certificate (GJK's order): the axis of a dropped point or of the classic GJK */
    const bool kept = ok && !(d > thr);
    ugk::gv u = ok ? n : ax;
    const double ul = ugk::dot(u, u);
    bool cert = !kept && ul > 1e-24;
    if (cert) {
        u = ugk::mulinv(u, ug_sqrt(ul));
        const ugk::gv dA = ugk::mtv(T0.R, ugk::neg(u)), dB = ugk::mtv(T1.R, u);
        const double hA = ugk::dot(dA, ugk::support0(g0, dA)), hB = ugk::dot(dB, ugk::support0(g1, dB));
        if (lead) {
            const ugk::gm R = ugk::mtm(T1.R, T0.R);
            const ugk::gv pp = ugk::mtv(T1.R, ugk::sub(T0.p, T1.p));
            gc[0] = 1.0;
            gc[1] = dB.x; gc[2] = dB.y; gc[3] = dB.z;
            gc[4] = hA; gc[5] = hB;
            for (int i = 0; i < 9; i++) gc[6 + i] = R.m[i];
            gc[15] = pp.x; gc[16] = pp.y; gc[17] = pp.z;
        }
    } else if (lead) {
        gc[0] = 0.0;
    }
    v3 cn = V(n.x, n.y, n.z), cp = V(p.x, p.y, p.z);
    if (swap) {
        cp = vadd(cp, vscale(cn, d));
        cn = vneg(cn);
    }
    if (lead) {
        sh.u.cand.n[k] = ok ? 1 : 0;
        sh.u.cand.c[k][0].n = cn;
        sh.u.cand.c[k][0].pB = cp;
        sh.u.cand.c[k][0].d = d;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
}

/* the GJK pairs of a pair chunk (bits of hq), in rounds of GJK_NG: lane group g runs the round's g-th pair on its own
 * EPA store.  One call per chunk: the callee-saved registers this solver needs are saved once per substep with GJK
 * pairs, not once per pair (they were 441 dwords per lane per call, most of the k_step's HBM traffic). */
#ifdef UG_GJK_INLINE
__device__ __forceinline__
#else
__device__ __noinline__
#endif
static void team_gjk(const Scene* s, unsigned long long hq, int c0, double* ws) {
    PROF_ENTRY(CS_GJK);
    PROF_CALL(CALL_GJK);
    Shared& sh = g_sh;
    const int nq = __popcll(hq), g = threadIdx.x / GJK_G;
    for (int r0 = 0; r0 < nq; r0 += GJK_NG) {
        if (r0 + g < nq) {
            unsigned long long m = hq;
            for (int j = 0; j < r0 + g; j++) m &= m - 1ull;
            const int k = __builtin_ctzll(m);
            gjk_one(s, k, (UGK_GMEM ugk::EpaMem*)(ws + WS_EPA) + g, (gdouble*)(ws + WS_GC) + GC_DOUBLES * sh.ov[c0 + k]);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
    }
    PROF_EXIT();
}

template <bool FULL, bool GJK>
__device__ __noinline__ static void team_collide(const Scene* s, double* ws) {
    PROF_ENTRY(CS_COLLIDE);
    PROF_CALL(CALL_COLLIDE);
    Shared& sh = g_sh;
    const int lane = threadIdx.x;
    EnvState& e = sh.e;
    if (lane < s->ncol) {
        const Collider& c = s->col[lane];
        XF O = owner_xf(e, sh.kin, c.owner);
        v3 lo, hi;
        world_aabb(O, c, lo, hi);
        sh.O[lane] = O;
        sh.lo[lane] = vsub(lo, V(UG_AABB_PAD, UG_AABB_PAD, UG_AABB_PAD));
        sh.hi[lane] = vadd(hi, V(UG_AABB_PAD, UG_AABB_PAD, UG_AABB_PAD));
    }
    /* live manifolds -> global workspace (read back per pair below; LDS list is rebuilt in place) */
    int nold = (int)e.nman;
    const double* src = (const double*)e.man;
    gdouble* const gws = (gdouble*)ws; /* global-typed: a generic store here would make later loads wait for it */
    for (int i = lane; i < nold * UG_MAN_DOUBLES; i += TEAM) gws[i] = src[i];
    if (lane < nold) sh.oldp[lane] = (int)e.man[lane].pair;
    __threadfence_block();
    __syncthreads();
    /* broadphase: ordered list of overlapping pairs */
    PROF_T0(t_broad);
    int base = 0;
    gdouble* const qs = (gdouble*)(ws + WS_QS); /* the quiescent-collision reference (GJK, full geometry) */
    for (int p0 = 0; p0 < s->npair; p0 += TEAM) {
        int p = p0 + lane;
        int ovl = 0;
        if (p < s->npair) {
            const PairDef& P = s->pair[p];
            int a = P.a, b = P.b;
            const bool act = collider_active(e, s->col[a]) && collider_active(e, s->col[b]);
            ovl = act && !(sh.lo[a].x > sh.hi[b].x || sh.hi[a].x < sh.lo[b].x || sh.lo[a].y > sh.hi[b].y ||
                           sh.hi[a].y < sh.lo[b].y || sh.lo[a].z > sh.hi[b].z || sh.hi[a].z < sh.lo[b].z);
            if (GJK && FULL) {
                /* a separated pair's padded-AABB gap (each box moves by at most its collider's displacement);
                 * an overlapping one's slack comes from its certificate below (-1: none) */
                const double g = fmax(fmax(fmax(sh.lo[a].x - sh.hi[b].x, sh.lo[b].x - sh.hi[a].x),
                                           fmax(sh.lo[a].y - sh.hi[b].y, sh.lo[b].y - sh.hi[a].y)),
                                      fmax(sh.lo[a].z - sh.hi[b].z, sh.lo[b].z - sh.hi[a].z));
                qs[p] = !act ? 1e300 : (ovl ? -1.0 : g);
            }
        }
        unsigned long long m = ballot(ovl);
        if (ovl) sh.ov[base + lane_prefix(m)] = p;
        base += __popcll(m);
    }
    if (lane == 0) sh.nov = base;
    __syncthreads();
    PROF_ADD(PF_BROAD, t_broad);
    int nov = base;
    int nnew = 0;
    bool allcert = true; /* every overlapping pair skipped by its certificate */
    for (int c0 = 0; c0 < nov; c0 += MAXOV) {
        int cn = nov - c0 < MAXOV ? nov - c0 : MAXOV;
        /* hull-box pairs of this chunk: cooperative narrowphase */
        PROF_T0(t_hull);
        /* every pair's transforms and collider fields at once (lane per pair: one load latency for the pass),
         * then the hull pairs in pair order, each reading its record uniformly from LDS */
        int hk = 0;
        bool certd = false; /* this lane's pair skipped by its separation certificate */
        if (lane < cn) {
            const int p = sh.ov[c0 + lane];
            const PairDef& P = s->pair[p];
            const Collider& A = s->col[P.a];
            const Collider& B = s->col[P.b];
            PairInfo pi;
            pi.TA = shape_xf(sh.O[P.a], A);
            pi.TB = shape_xf(sh.O[P.b], B);
            pi.A = hull_arg(A);
            pi.B = hull_arg(B);
            pi.thr = P.thr;
            pi.a = P.a; pi.b = P.b; pi.ka = A.kind; pi.kb = B.kind;
            sh.pinfo[lane] = pi;
            hk = A.kind == UG_SHAPE_HULL && (B.kind == UG_SHAPE_BOX || B.kind == UG_SHAPE_HULL);
            if (GJK) hk = pair_is_gjk(A, B); /* the wave runs the pair's GJK / EPA */
            if (GJK && hk) {
                /* its separation certificate (team_gjk): with R_AB, p_AB now, A's extent along -n grows by at most
                 * ||(R_AB - R_AB0)^T n|| times A's support radius, B's along n (B-fixed) not at all, so the cores stay
                 * at least s = n . p_AB - hA - that - hB apart; past the margins and the threshold GJK adds no point */
                const gcdouble* gc = (gcdouble*)(ws + WS_GC) + GC_DOUBLES * p;
                if (gc[0] > 0.0) {
                    const bool sw = A.kind == UG_SHAPE_SPHERE && B.kind != UG_SHAPE_SPHERE;
                    const XF& G0 = sw ? pi.TB : pi.TA;
                    const XF& G1 = sw ? pi.TA : pi.TB;
                    const Collider& C0 = sw ? B : A;
                    const Collider& C1 = sw ? A : B;
                    const m3 R = mtm(G1.R, G0.R);
                    const v3 pp = mtv(G1.R, vsub(G0.p, G1.p));
                    const v3 nb = V(gc[1], gc[2], gc[3]);
                    v3 w = V(0, 0, 0);
#pragma unroll
                    for (int i = 0; i < 3; i++) {
                        const double ni = i == 0 ? nb.x : (i == 1 ? nb.y : nb.z);
                        w.x += (R.m[3 * i] - gc[6 + 3 * i]) * ni;
                        w.y += (R.m[3 * i + 1] - gc[7 + 3 * i]) * ni;
                        w.z += (R.m[3 * i + 2] - gc[8 + 3 * i]) * ni;
                    }
                    const double sep = vdot(nb, pp) - gc[4] - vlen(w) * C0.gradius - gc[5];
                    if (sep - C0.gmargin - C1.gmargin - P.thr > 1e-9 * (1.0 + ug_fabs(sep))) {
                        hk = 0;
                        certd = true;
                        sh.u.cand.n[lane] = 0;
                        /* the cores' separation along n may shrink by this much before GJK could keep a point */
                        if (FULL) qs[p] = sep - C0.gmargin - C1.gmargin - P.thr - 1e-9 * (1.0 + ug_fabs(sep));
                    }
                }
            }
            else if (FULL) /* the disc cylinder against a polytope, either side */
                hk = hk || (B.kind == UG_SHAPE_CYL && (A.kind == UG_SHAPE_HULL || A.kind == UG_SHAPE_BOX)) ||
                     (A.kind == UG_SHAPE_CYL && B.kind == UG_SHAPE_BOX);
            if (!GJK && FULL && A.kind == UG_SHAPE_HULL && (B.kind == UG_SHAPE_BOX || B.kind == UG_SHAPE_CYL) && A.nv > TEAM) {
                /* the pair's separation certificate (team_hull_box_full / team_poly_cyl): while no point of either
                 * shape can have moved by its slack since, the evaluation would find no candidate -- skip it.  Every
                 * A vertex lies within rA of A's origin and every point of B within rB of B's, so a point moves by at
                 * most |dp| + ||dR||_F r in the other frame. */
                gcdouble* pc = (gcdouble*)(ws + WS_PC) + PC_DOUBLES * p;
                double rec[PC_DOUBLES];
#pragma unroll
                for (int i = 0; i < PC_DOUBLES; i++) rec[i] = pc[i];
                const m3 RAB = mtm(pi.TB.R, pi.TA.R);
                const v3 pAB = mtv(pi.TB.R, vsub(pi.TA.p, pi.TB.p));
                const v3 pBA = mtv(pi.TA.R, vsub(pi.TB.p, pi.TA.p));
                double f2 = 0.0;
#pragma unroll
                for (int i = 0; i < 9; i++) {
                    const double d = RAB.m[i] - rec[1 + i];
                    f2 += d * d;
                }
                const double fr = ug_sqrt(f2);
                /* B's points (box corners / the cylinder) move by at most dB in A's frame; hull-box: the hull's
                 * extent along the certified box face normal n changes by at most |n . dp_AB| + |dR_AB^T n| rA */
                const double dB = vlen(vsub(pBA, V(rec[13], rec[14], rec[15]))) + fr * rec[17];
                bool ok = rec[0] > 0.0 && dB < rec[0];
                if (B.kind == UG_SHAPE_BOX) {
                    const int f = (int)rec[19], ax = f >> 1;
                    const double sg = (f & 1) ? 1.0 : -1.0;
                    const double dpa = ax == 0 ? pAB.x - rec[10] : (ax == 1 ? pAB.y - rec[11] : pAB.z - rec[12]);
                    const double r0 = ax == 0 ? RAB.m[0] - rec[1] : (ax == 1 ? RAB.m[3] - rec[4] : RAB.m[6] - rec[7]);
                    const double r1 = ax == 0 ? RAB.m[1] - rec[2] : (ax == 1 ? RAB.m[4] - rec[5] : RAB.m[7] - rec[8]);
                    const double r2 = ax == 0 ? RAB.m[2] - rec[3] : (ax == 1 ? RAB.m[5] - rec[6] : RAB.m[8] - rec[9]);
                    const double dV = ug_fabs(sg * dpa) + ug_sqrt(r0 * r0 + r1 * r1 + r2 * r2) * rec[16];
                    ok = ok && rec[18] > 0.0 && dV < rec[18];
                }
                if (ok) {
                    hk = 0;
                    certd = true;
                    sh.u.cand.n[lane] = 0;
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        allcert = allcert && ballot(lane < cn && !certd) == 0ull;
        if (lane == 0) sh.is[3] = c0; /* the pass's first pair (team_poly_cyl's certificate slot) */
        if (GJK) {
            const unsigned long long hq = ballot(hk);
            if (hq) {
                PROF_PRE_CALL();
                team_gjk(s, hq, c0, ws);
                PROF_POST_CALL(CS_GJK);
            }
            PROF_CNT(PC_HULL, __popcll(hq));
        }
        for (unsigned long long hm = GJK ? 0ull : ballot(hk); hm != 0ull; hm &= hm - 1ull) {
            const int k = __builtin_ctzll(hm);
            const PairInfo pi = sh.pinfo[k];
            if (FULL && (pi.kb == UG_SHAPE_CYL || pi.ka == UG_SHAPE_CYL))
                team_poly_cyl(k, pi.ka == UG_SHAPE_CYL, (gdouble*)(ws + WS_FC));
            else if (FULL && pi.A.nv > TEAM) { /* a full-geometry robot hull (every full hull has more than 64 vertices) */
                if (pi.kb == UG_SHAPE_BOX)
                    team_hull_box_full(pi.A, pi.B, pi.TA, pi.TB, pi.thr, k,
                                       (unsigned short*)(ws + WS_HC2) + 8 * sh.ov[c0 + k], (gdouble*)(ws + WS_FC),
                                       (gdouble*)(ws + WS_PC) + PC_DOUBLES * sh.ov[c0 + k]);
                else team_hull_hull_full(pi.A, pi.B, pi.TA, pi.TB, pi.thr, k, (gdouble*)(ws + WS_FC));
            } else if (pi.kb == UG_SHAPE_BOX)
                team_hull_box(pi.A, pi.B, pi.TA, pi.TB, pi.thr, k, (unsigned char*)(ws + WS_HC) + 8 * sh.ov[c0 + k]);
            else team_hull_hull(pi.A, pi.B, pi.TA, pi.TB, pi.thr, k, (unsigned char*)(ws + WS_HH) + 64 * sh.ov[c0 + k]);
            PROF_CNT(PC_HULL, 1);
        }
        PROF_ADD(PF_HULL, t_hull);
        if (nold == 0 && ballot(lane < cn && !certd) == 0ull) {
            /* every pair of the chunk certified separated and no manifold from the last substep: the stages below
             * would find no candidate and no old point, and store nothing (the contact-free substeps of a reset) */
            __builtin_amdgcn_wave_barrier();
            continue;
        }
        PROF_T0(t_pairs);
        /* lane per pair: remaining narrowphases, manifold update.  The working manifold (g_sh.pm[lane]) and the
         * candidate list (g_sh.u.cand.c[lane], where the hull pairs' candidates already are) live in LDS. */
        /* previous manifolds of this pass's pairs: index lookup per lane (pair ids in LDS), then one cooperative
         * copy of their points from the workspace into the working manifolds (all loads in flight together) */
        PROF_T0(t_pl);
        __builtin_amdgcn_wave_barrier(); /* the pair records (sh.pinfo) are dead from here: pm reuses their LDS */
        if (lane < cn) {
            const int p = sh.ov[c0 + lane];
            int mo = -1;
            for (int m = 0; m < nold; m++)
                if (sh.oldp[m] == p) { mo = m; break; }
            sh.pmo[lane] = mo;
            sh.pm[lane].pair = p;
            sh.pm[lane].npts = mo >= 0 ? (int)gws[mo * UG_MAN_DOUBLES + 1] : 0;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        for (int i = lane; i < cn * 4 * UG_PT_DOUBLES; i += TEAM) {
            const int k = i / (4 * UG_PT_DOUBLES), f = i - k * (4 * UG_PT_DOUBLES);
            const int mo = sh.pmo[k];
            if (mo >= 0) ((__attribute__((address_space(3))) double*)&sh.pm[k].pt[0].lpA.x)[f] = gws[mo * UG_MAN_DOUBLES + 2 + f];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        PROF_ADD(PF_PR_LOOK, t_pl);
        int has = 0;
        int isbb = 0; /* box-box pairs run below in rounds of NBOXSLOT lanes, each with an LDS clip-buffer slot */
        if (lane < cn) {
            int p = sh.ov[c0 + lane];
            const PairDef& P = s->pair[p];
            const Collider& A = s->col[P.a];
            const Collider& B = s->col[P.b];
            PROF_T0(t_pn);
            XF TA = shape_xf(sh.O[P.a], A), TB = shape_xf(sh.O[P.b], B);
            CandList L;
            L.n = 0;
            L.c = (LCand*)&sh.u.cand.c[lane][0];
            const bool gj = GJK && pair_is_gjk(A, B);
            isbb = A.kind == UG_SHAPE_BOX && B.kind == UG_SHAPE_BOX && !gj;
            if (gj) {
                L.n = sh.u.cand.n[lane]; /* team_gjk wrote it */
            } else if ((A.kind == UG_SHAPE_HULL && (B.kind == UG_SHAPE_BOX || B.kind == UG_SHAPE_HULL)) ||
                (FULL && ((B.kind == UG_SHAPE_CYL && A.kind != UG_SHAPE_SPHERE) || A.kind == UG_SHAPE_CYL))) {
                L.n = sh.u.cand.n[lane]; /* team_hull_box / team_hull_hull / team_poly_cyl wrote them */
            } else if (FULL && A.kind == UG_SHAPE_SPHERE && B.kind == UG_SHAPE_CYL) {
                nc_sphere_cyl(TA, A, TB, B, P.thr, L);
            } else if (A.kind == UG_SHAPE_SPHERE && B.kind == UG_SHAPE_HULL) {
                nc_hull_sphere(TB, B, TA, A, P.thr, L);
                for (int i = 0; i < L.n; i++) { /* swapped roles: flip the normal, move the point onto the sphere */
                    const v3 cn = ldv(L.c[i].n), cp = ldv(L.c[i].pB);
                    stv(L.c[i].n, vneg(cn));
                    stv(L.c[i].pB, vadd(cp, vscale(cn, L.c[i].d)));
                }
            } else if (A.kind == UG_SHAPE_SPHERE && B.kind == UG_SHAPE_BOX) nc_sphere_box(TA, A, TB, B, P.thr, L);
            else if (A.kind == UG_SHAPE_SPHERE && B.kind == UG_SHAPE_SPHERE) nc_sphere_sphere(TA, A, TB, B, P.thr, L);
            else if (A.kind == UG_SHAPE_HULL && B.kind == UG_SHAPE_SPHERE) nc_hull_sphere(TA, A, TB, B, P.thr, L);
            else if (A.kind == UG_SHAPE_BOX && B.kind == UG_SHAPE_SPHERE) {
                nc_sphere_box(TB, B, TA, A, P.thr, L);
                for (int i = 0; i < L.n; i++) {
                    const v3 cn = ldv(L.c[i].n), cp = ldv(L.c[i].pB);
                    stv(L.c[i].n, vneg(cn));
                    stv(L.c[i].pB, vadd(cp, vscale(cn, L.c[i].d)));
                }
            }
            sh.u.cand.n[lane] = L.n;
            PROF_ADD(PF_PR_NP, t_pn);
        }
        PROF_T0(t_bb);
        /* box-box pairs: the whole wave per pair (team_box_box) */
        for (unsigned long long bbm = ballot(isbb); bbm != 0ull; bbm &= bbm - 1ull) {
            const int kb = __builtin_ctzll(bbm);
            const PairDef& P = s->pair[sh.ov[c0 + kb]];
            const Collider& A = s->col[P.a];
            const Collider& B = s->col[P.b];
            const XF TA = shape_xf(sh.O[P.a], A), TB = shape_xf(sh.O[P.b], B);
            const double Ah[3] = {A.half[0], A.half[1], A.half[2]}, Bh[3] = {B.half[0], B.half[1], B.half[2]};
            team_box_box(TA, Ah, TB, Bh, kb);
#ifdef UG_BB_CHECK /* development aid: the serial routine beside the team one, mismatches printed */
            if (lane == 0) {
                CandList L;
                L.n = 0;
                L.c = (LCand*)&sh.bs[2];
                nc_box_box(TA, A, TB, B, P.thr, L, *(LBoxScratch*)&sh.bs[1]);
                int same = L.n == sh.u.cand.n[kb];
                for (int i = 0; same && i < L.n; i++) {
                    const v3 an = ldv(L.c[i].n), ap = ldv(L.c[i].pB), bn = sh.u.cand.c[kb][i].n, bp = sh.u.cand.c[kb][i].pB;
                    same = an.x == bn.x && an.y == bn.y && an.z == bn.z && ap.x == bp.x && ap.y == bp.y && ap.z == bp.z &&
                           L.c[i].d == sh.u.cand.c[kb][i].d;
                }
                if (!same) {
                    printf("BBCHK pair %d-%d serial n %d team n %d code %d tsel %d nR %d | s0 %.17g %.17g %.17g d %.17g | t0 %.17g %.17g %.17g d %.17g\n",
                           P.a, P.b, L.n, sh.u.cand.n[kb], g_bbdbg[0], g_bbdbg[1], g_bbdbg[2],
                           L.n ? ldv(L.c[0].pB).x : 0.0, L.n ? ldv(L.c[0].pB).y : 0.0, L.n ? ldv(L.c[0].pB).z : 0.0, L.n ? L.c[0].d : 0.0,
                           sh.u.cand.c[kb][0].pB.x, sh.u.cand.c[kb][0].pB.y, sh.u.cand.c[kb][0].pB.z, sh.u.cand.c[kb][0].d);
                }
            }
            __syncthreads();
#endif
        }
        PROF_ADD(PF_PR_NP, t_bb);
        PROF_ADD(PF_PR_BB, t_bb);
        if (lane < cn) {
            const PairDef& P = s->pair[sh.ov[c0 + lane]];
            LManifold& M = *(LManifold*)&sh.pm[lane];
            CandList L;
            L.n = sh.u.cand.n[lane];
            L.c = (LCand*)&sh.u.cand.c[lane][0];
            PROF_T0(t_pm);
            /* a compound collision object refreshes its child manifolds before the narrowphase (oracle collide) */
            if (GJK && (s->col[P.a].compound || s->col[P.b].compound) && M.npts)
                manifold_refresh(M, lxf(sh.O[P.a]), lxf(sh.O[P.b]), P.thr);
            for (int i = 0; i < L.n; i++) {
                Cand c;
                c.n = ldv(L.c[i].n);
                c.pB = ldv(L.c[i].pB);
                c.d = L.c[i].d;
                manifold_add(M, lxf(sh.O[P.a]), lxf(sh.O[P.b]), c, P.thr);
            }
            if (M.npts) manifold_refresh(M, lxf(sh.O[P.a]), lxf(sh.O[P.b]), P.thr);
            has = M.npts > 0;
            PROF_ADD(PF_PR_MAN, t_pm);
        }
        PROF_T0(t_ps);
        __syncthreads();
        unsigned long long hm = ballot(has);
        if (has) {
            int pos = nnew + lane_prefix(hm);
            if (pos < MAXMAN) man_to_st(e.man[pos], *(const LManifold*)&sh.pm[lane]);
        }
        nnew += __popcll(hm);
        __syncthreads();
        PROF_ADD(PF_PR_ST, t_ps);
        PROF_ADD(PF_PAIRS, t_pairs);
    }
    if (lane == 0) {
        if (nnew > MAXMAN) e.overflow += (double)(nnew - MAXMAN);
        e.nman = (double)(nnew < MAXMAN ? nnew : MAXMAN);
    }
    if (GJK && FULL) {
        /* a quiescent-collision reference: no manifold, every overlapping pair certified, no free object (their
         * motion is not bounded here) -- the robot's q now, with the slacks written above */
        bool still = nnew == 0 && allcert;
        for (int o = 0; o < s->nobj; o++) still = still && e.oactive[o] == 0.0;
        if (still && lane < NB) qs[MAXPAIR + lane] = e.q[lane];
        if (lane == 0) sh.qsvalid = still ? 1 : 0;
    }
    __syncthreads();
    PROF_EXIT();
}

