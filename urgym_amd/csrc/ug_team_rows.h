/* ug_team_rows.h -- part of ug_team.h: constraint rows: enumeration, unit solves, the row build.
 * Included by ug_team.h inside namespace ugd, in this order (the kernel is one translation unit); not self-contained. */
/* ---------------- rows ---------------- */
__device__ static inline int ent_dofs(int ent) { return ent == 0 ? NB : 6; }
__device__ static inline int ent_off(int ent) { return ent == 0 ? 0 : NB + 6 * (ent - 1); }
__device__ static inline double ent_dot(int ent, const double* J, const double* v) {
    int n = ent_dofs(ent), o = ent_off(ent);
    double s = 0.0;
    for (int i = 0; i < n; i++) s += J[i] * v[o + i];
    return s;
}
__device__ static inline double ent_dot_local(int ent, const double* a, const double* b) {
    int n = ent_dofs(ent);
    double s = 0.0;
    for (int i = 0; i < n; i++) s += a[i] * b[i];
    return s;
}
__device__ static void point_jac(const Scene* sc, const EnvState& e, const Kin& k, int ent, int body, v3 p, v3 d,
                                 double* J, double* MiJ, const double* LDL) {
    if (ent == 0) {
        for (int i = 0; i < NB; i++) {
            J[i] = moves(i, body) ? vdot(d, vcross(k.a[i], vsub(p, k.p[i]))) : 0.0;
            MiJ[i] = J[i];
        }
        ldlt_solve(LDL, NB, MiJ);
    } else {
        int o = ent - 1;
        v3 r = vsub(p, e.obj[o].pos);
        v3 rn = vcross(r, d);
        J[0] = d.x; J[1] = d.y; J[2] = d.z; J[3] = rn.x; J[4] = rn.y; J[5] = rn.z;
        double im = 1.0 / sc->omass[o];
        m3 R = qmat(e.obj[o].quat);
        v3 ir = mtv(R, rn);
        ir = V(ir.x / sc->oinertia[o].x, ir.y / sc->oinertia[o].y, ir.z / sc->oinertia[o].z);
        ir = mv(R, ir);
        MiJ[0] = d.x * im; MiJ[1] = d.y * im; MiJ[2] = d.z * im; MiJ[3] = ir.x; MiJ[4] = ir.y; MiJ[5] = ir.z;
    }
}
__device__ static void ang_jac(const Scene* sc, const EnvState& e, const Kin& k, int ent, int body, v3 u, double* J,
                               double* MiJ, const double* LDL) {
    if (ent == 0) {
        for (int i = 0; i < NB; i++) {
            J[i] = moves(i, body) ? vdot(u, k.a[i]) : 0.0;
            MiJ[i] = J[i];
        }
        ldlt_solve(LDL, NB, MiJ);
    } else {
        int o = ent - 1;
        J[0] = 0.0; J[1] = 0.0; J[2] = 0.0; J[3] = u.x; J[4] = u.y; J[5] = u.z;
        m3 R = qmat(e.obj[o].quat);
        v3 ir = mtv(R, u);
        ir = V(ir.x / sc->oinertia[o].x, ir.y / sc->oinertia[o].y, ir.z / sc->oinertia[o].z);
        ir = mv(R, ir);
        MiJ[0] = 0.0; MiJ[1] = 0.0; MiJ[2] = 0.0; MiJ[3] = ir.x; MiJ[4] = ir.y; MiJ[5] = ir.z;
    }
}
__device__ static inline int ent_of_collider(const Collider& c, int& body) {
    body = -1;
    if (c.owner >= 0) { body = c.owner; return 0; }
    if (c.owner == -1) return -1;
    if (c.owner > -100) return -1 - c.owner;
    return -1;
}
__device__ static inline void put_seg(int ent, const double* src, double* dst) {
    int n = ent_dofs(ent), o = ent_off(ent);
    for (int i = 0; i < n; i++) dst[o + i] = src[i];
}
/* enumerate rows in solve order (lane 0): nc rows, then normals, then frictions */
__device__ static void enumerate_rows(Shared& sh, const Scene* s) {
    EnvState& e = sh.e;
    int n = 0, nnc = 0, nn = 0, nf = 0;
    /* first pass: counts and capacity decisions in the oracle's enumeration order */
    int ncnt = 0;
    for (int d = 0; d < NB; d++)
        for (int side = 0; side < 2; side++) {
            double pen = side == 0 ? e.q[d] - UG_DOF_LOWER[d] : UG_DOF_UPPER[d] - e.q[d];
            if (pen > 0) continue;
            if (ncnt >= MAXROWS) { e.overflow += 1.0; continue; }
            RowS& r = sh.rs[nnc];
            r.kind = 0; r.a = d; r.b = side;
            nnc++; ncnt++;
        }
    for (int m = 0; m < 7; m++) {
        if (e.mon[m] == 0.0) continue;
        if (ncnt >= MAXROWS) { e.overflow += 1.0; continue; }
        RowS& r = sh.rs[nnc];
        r.kind = 1; r.a = m;
        nnc++; ncnt++;
    }
    for (int g = 0; g < 5; g++) {
        if (ncnt >= MAXROWS) { e.overflow += 1.0; continue; }
        RowS& r = sh.rs[nnc];
        r.kind = 2; r.a = g;
        nnc++; ncnt++;
    }
    /* the box's joint limits in joint order, then the button's motor (oracle build_rows) */
    for (int jj = 0; jj < s->njoint; jj++) {
        const int o = s->jorder[jj];
        if (e.oactive[o] == 0.0) continue;
        const UgJoint& J = s->ojoint[o];
        const double qj = e.obj[o].w.x;
        for (int side = 0; side < 2; side++) {
            double pen = side == 0 ? qj - J.lower : J.upper - qj;
            if (pen > 0) continue;
            if (ncnt >= MAXROWS) { e.overflow += 1.0; continue; }
            RowS& r = sh.rs[nnc];
            r.kind = 8; r.a = o; r.b = side;
            nnc++; ncnt++;
        }
    }
    if (s->task == UG_TASK_BOX && e.oactive[1] != 0.0) {
        if (ncnt >= MAXROWS) e.overflow += 1.0;
        else {
            RowS& r = sh.rs[nnc];
            r.kind = 9; r.a = 1;
            nnc++; ncnt++;
        }
    }
    int nman = (int)e.nman;
    /* contact points kept (capacity: 3 rows each) */
    /* accepted points (capacity: 3 rows each, 5 with rolling friction), as the oracle's running count */
    int npt = 0, nroll = 0, cnt = ncnt;
    for (int m = 0; m < nman; m++) {
        const PairDef& P = s->pair[(int)e.man[m].pair];
        int bA, bB;
        int eA = ent_of_collider(s->col[P.a], bA), eB = ent_of_collider(s->col[P.b], bB);
        if (eA < 0 && eB < 0) continue;
        int need = P.rolling > 0.0 ? 5 : 3;
        for (int j = 0; j < (int)e.man[m].npts; j++) {
            if (cnt + need > MAXROWS) { e.overflow += 1.0; continue; }
            cnt += need;
            npt++;
            nroll += need == 5;
        }
    }
    nn = npt;
    nf = 2 * npt;
    /* positions in solve order: normals, frictions, rolling-friction rows */
    int pn = nnc, pf = nnc + nn, pr = nnc + nn + nf;
    cnt = ncnt;
    for (int m = 0; m < nman; m++) {
        const PairDef& P = s->pair[(int)e.man[m].pair];
        int bA, bB;
        int eA = ent_of_collider(s->col[P.a], bA), eB = ent_of_collider(s->col[P.b], bB);
        if (eA < 0 && eB < 0) continue;
        int need = P.rolling > 0.0 ? 5 : 3;
        for (int j = 0; j < (int)e.man[m].npts; j++) {
            if (cnt + need > MAXROWS) continue;
            cnt += need;
            RowS& r = sh.rs[pn];
            r.kind = 3; r.a = m; r.b = j; r.nrow = pn;
            for (int f = 0; f < 2; f++) {
                RowS& q = sh.rs[pf + f];
                q.kind = 4 + f; q.a = m; q.b = j; q.nrow = pn;
            }
            pf += 2;
            if (need == 5) {
                for (int f = 0; f < 2; f++) {
                    RowS& q = sh.rs[pr + f];
                    q.kind = 6 + f; q.a = m; q.b = j; q.nrow = pn;
                }
                pr += 2;
            }
            pn++;
        }
    }
    n = nnc + nn + nf + 2 * nroll;
    sh.nrows = n; sh.nnc = nnc; sh.nn = nn; sh.nf = nf;
}
/* enumerate_rows, wave-parallel: lane per limit side / motor / gear / manifold, positions by prefix
 * counts.  Identical output when every contact point fits (the usual case); when the capacity check
 * of the serial code would reject points, the serial enumeration runs instead. */
__device__ __noinline__ static void team_enumerate(const Scene* s) {
    PROF_ENTRY(CS_ENUM);
    PROF_CALL(CALL_ENUM);
    Shared& sh = g_sh;
    EnvState& e = sh.e;
    const int lane = threadIdx.x;
    /* non-contact rows: limits (dof, side) in index order, enabled motors, the 5 gears (<= NCMAX rows) */
    const bool lim = lane < 2 * NB && ([&] {
        const int d = lane >> 1, side = lane & 1;
        double pen = side == 0 ? e.q[d] - UG_DOF_LOWER[d] : UG_DOF_UPPER[d] - e.q[d];
        return !(pen > 0);
    })();
    const unsigned long long mlim = ballot(lim);
    const int nlim = __popcll(mlim);
    if (lim) {
        RowS& r = sh.rs[lane_prefix(mlim)];
        r.kind = 0; r.a = lane >> 1; r.b = lane & 1;
    }
    const bool mot = lane < 7 && e.mon[lane < 7 ? lane : 0] != 0.0;
    const unsigned long long mmot = ballot(mot);
    const int nmot = __popcll(mmot);
    if (mot) {
        RowS& r = sh.rs[nlim + lane_prefix(mmot)];
        r.kind = 1; r.a = lane;
    }
    if (lane < 5) {
        RowS& r = sh.rs[nlim + nmot + lane];
        r.kind = 2; r.a = lane;
    }
    /* the box's joint limits (lane 2 k + side: joint k in joint order) and the button's motor */
    int nbx = 0;
    if (s->njoint > 0) {
        const int side = lane & 1;
        int o = 0;
        bool jl = false;
        if (lane < 2 * s->njoint) {
            o = s->jorder[lane >> 1];
            const UgJoint& J = s->ojoint[o];
            const double qj = e.obj[o].w.x;
            const double pen = side == 0 ? qj - J.lower : J.upper - qj;
            jl = e.oactive[o] != 0.0 && !(pen > 0);
        }
        const unsigned long long mj = ballot(jl);
        nbx = __popcll(mj);
        if (jl) {
            RowS& r = sh.rs[nlim + nmot + 5 + lane_prefix(mj)];
            r.kind = 8; r.a = o; r.b = side;
        }
        if (s->task == UG_TASK_BOX && e.oactive[1] != 0.0) {
            if (lane == 0) {
                RowS& r = sh.rs[nlim + nmot + 5 + nbx];
                r.kind = 9; r.a = 1;
            }
            nbx++;
        }
    }
    const int nnc = nlim + nmot + 5 + nbx;
    /* contact points per manifold (lane m) */
    const int nman = (int)e.nman;
    int npt = 0, nroll = 0;
    if (lane < nman) {
        const PairDef& P = s->pair[(int)e.man[lane].pair];
        int bA, bB;
        int eA = ent_of_collider(s->col[P.a], bA), eB = ent_of_collider(s->col[P.b], bB);
        if (!(eA < 0 && eB < 0)) {
            npt = (int)e.man[lane].npts;
            nroll = P.rolling > 0.0 ? npt : 0;
        }
        sh.ecnt[lane] = npt;
        sh.ecnt[MAXMAN + lane] = nroll;
    }
    __builtin_amdgcn_wave_barrier();
    int pbase = 0, rbase = 0, tp = 0, tr = 0;
    for (int m = 0; m < nman; m++) {
        const int a = sh.ecnt[m], r = sh.ecnt[MAXMAN + m];
        if (m < lane) { pbase += a; rbase += r; }
        tp += a;
        tr += r;
    }
    __builtin_amdgcn_wave_barrier();
    const int total = nnc + 3 * tp + 2 * tr;
    if (total > MAXROWS) { /* the serial code's capacity checks decide which points are kept */
        if (lane == 0) enumerate_rows(sh, s);
        { PROF_EXIT(); return; }
    }
    const int nn = tp, nf = 2 * tp;
    if (lane < nman) {
        for (int j = 0; j < npt; j++) {
            const int pn = nnc + pbase + j;
            RowS& r = sh.rs[pn];
            r.kind = 3; r.a = lane; r.b = j; r.nrow = pn;
#pragma unroll
            for (int f = 0; f < 2; f++) {
                RowS& q = sh.rs[nnc + nn + 2 * (pbase + j) + f];
                q.kind = 4 + f; q.a = lane; q.b = j; q.nrow = pn;
            }
            if (nroll) {
#pragma unroll
                for (int f = 0; f < 2; f++) {
                    RowS& q = sh.rs[nnc + nn + nf + 2 * (rbase + j) + f];
                    q.kind = 6 + f; q.a = lane; q.b = j; q.nrow = pn;
                }
            }
        }
    }
    if (lane == 0) {
        sh.nrows = nnc + nn + nf + 2 * tr;
        sh.nnc = nnc;
        sh.nn = nn;
        sh.nf = nf;
    }
    PROF_EXIT();
}
/* ---- register-resident row build: every array index below is a compile-time constant (fully unrolled
 * loops, selects instead of dynamic stores), so the per-lane arrays stay in VGPRs instead of scratch.
 * Same operations in the same order as the oracle's build_rows (contact_row / dof_row / point_jac). */
/* ldlt() with compile-time indices */
__device__ __forceinline__ void ldlt_r(double (&A)[NB * NB]) {
#pragma unroll
    for (int j = 0; j < NB; j++) {
        double d = A[j * NB + j];
#pragma unroll
        for (int k2 = 0; k2 < j; k2++) d -= A[j * NB + k2] * A[j * NB + k2] * A[k2 * NB + k2];
        A[j * NB + j] = d;
#pragma unroll
        for (int i = j + 1; i < NB; i++) {
            double s = A[i * NB + j];
#pragma unroll
            for (int k2 = 0; k2 < j; k2++) s -= A[i * NB + k2] * A[j * NB + k2] * A[k2 * NB + k2];
            A[i * NB + j] = s / d;
        }
    }
}
template <typename M>
__device__ __forceinline__ void ldlt_solve_r(const M& A, double (&x)[NB]) {
#pragma unroll
    for (int i = 0; i < NB; i++)
#pragma unroll
        for (int k2 = 0; k2 < i; k2++) x[i] -= A[i * NB + k2] * x[k2];
#pragma unroll
    for (int i = 0; i < NB; i++) x[i] = x[i] / A[i * NB + i];
#pragma unroll
    for (int i = NB - 1; i >= 0; i--)
#pragma unroll
        for (int k2 = i + 1; k2 < NB; k2++) x[i] -= A[k2 * NB + i] * x[k2];
}
/* sum over the entity's dofs (12 robot / 6 object) of a[i] * b(i), in index order */
__device__ __forceinline__ double ent_dot_r(int ent, const double (&a)[NB], const double (&b)[NB]) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < NB; i++)
        if (i < 6 || ent == 0) s += a[i] * b[i];
    return s;
}
__device__ __forceinline__ double ent_dot_v0(int ent, const double (&a)[NB], const double* v0) {
    const int o = ent_off(ent);
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < NB; i++)
        if (i < 6 || ent == 0) s += a[i] * v0[o + i];
    return s;
}
/* Jacobian of a point p on entity ent along d (ANG: angular component along d, rolling rows) and
 * M^-1 J^T of it; for an object only [0, 6) is set */
template <bool ANG>
__device__ __forceinline__ void ent_jac_r(const Scene* sc, const EnvState& e, const Kin& k, int ent, int body, v3 p, v3 d,
                                          double (&J)[NB], double (&MiJ)[NB], const double* LDL) {
    if (ent == 0) {
#pragma unroll
        for (int i = 0; i < NB; i++) {
            double x;
            if (ANG) x = vdot(d, k.a[i]);
            else x = vdot(d, vcross(k.a[i], vsub(p, k.p[i])));
            J[i] = moves(i, body) ? x : 0.0;
            MiJ[i] = J[i];
        }
        ldlt_solve_r(LDL, MiJ);
    } else {
        const int o = ent - 1;
        m3 R = qmat(e.obj[o].quat);
        if (ANG) {
            J[0] = 0.0; J[1] = 0.0; J[2] = 0.0; J[3] = d.x; J[4] = d.y; J[5] = d.z;
            v3 ir = mtv(R, d);
            ir = V(ir.x / sc->oinertia[o].x, ir.y / sc->oinertia[o].y, ir.z / sc->oinertia[o].z);
            ir = mv(R, ir);
            MiJ[0] = 0.0; MiJ[1] = 0.0; MiJ[2] = 0.0; MiJ[3] = ir.x; MiJ[4] = ir.y; MiJ[5] = ir.z;
        } else {
            v3 r = vsub(p, e.obj[o].pos);
            v3 rn = vcross(r, d);
            J[0] = d.x; J[1] = d.y; J[2] = d.z; J[3] = rn.x; J[4] = rn.y; J[5] = rn.z;
            double im = 1.0 / sc->omass[o];
            v3 ir = mtv(R, rn);
            ir = V(ir.x / sc->oinertia[o].x, ir.y / sc->oinertia[o].y, ir.z / sc->oinertia[o].z);
            ir = mv(R, ir);
            MiJ[0] = d.x * im; MiJ[1] = d.y * im; MiJ[2] = d.z * im; MiJ[3] = ir.x; MiJ[4] = ir.y; MiJ[5] = ir.z;
        }
#pragma unroll
        for (int i = 6; i < NB; i++) { J[i] = 0.0; MiJ[i] = 0.0; }
    }
}
/* build row at position pos (one lane): J | M^-1 J^T into the workspace row, scalars into rs[pos] */
/* the LDL solves every limit / motor / gear row would repeat, once per substep: lane d < NB solves for the
 * unit vector e_d, lane NB + g for gear g's ratio * e_child (the same computation as the row's own) */
__device__ __noinline__ static void team_unit_solves() {
    PROF_ENTRY(CS_UNIT);
    PROF_CALL(CALL_UNIT);
    const int lane = threadIdx.x;
    if (lane < NB + 5) {
        const int g = lane - NB;
        const int c = g < 0 ? lane : UG_GEAR_CHILD[g < 0 ? 0 : g];
        const double v = g < 0 ? 1.0 : UG_GEAR_RATIO[g < 0 ? 0 : g];
        double x[NB];
#pragma unroll
        for (int i = 0; i < NB; i++) x[i] = i == c ? v : 0.0;
        ldlt_solve_r(g_sh.LDL, x);
#pragma unroll
        for (int i = 0; i < NB; i++) g_sh.u.mcol[lane][i] = x[i];
    }
    __syncthreads();
    PROF_EXIT();
}
/* robot part of a point Jacobian along d (ANG: angular rows) -- ent_jac_r's robot branch without the
 * solve, with the row kind's ANG as a runtime select so that every contact lane runs the same code */
__device__ __forceinline__ void robot_jac_sel(const Kin& k, bool ang, int body, v3 p, v3 d, double (&J)[NB]) {
    const int am = g_sh.anc[body]; /* the dofs that move the body (moves(), one LDS read) */
#pragma unroll
    for (int i = 0; i < NB; i++) {
        const double xa = vdot(d, k.a[i]);
        const double xl = vdot(d, vcross(k.a[i], vsub(p, k.p[i])));
        const double x = ang ? xa : xl;
        J[i] = ((am >> i) & 1) ? x : 0.0;
    }
}
/* object part of a point Jacobian and its M^-1 J^T (ent_jac_r's object branch, ANG as a select) */
__device__ __forceinline__ void object_jac_sel(const Scene* sc, const EnvState& e, bool ang, int ent, v3 p, v3 d,
                                               double (&J)[NB], double (&MiJ)[NB]) {
    const int o = ent - 1;
    if (sc->ojoint[o].kind != UGJ_FREE) { /* a one-dof link (ug_joint.h): its slot 0 only */
        const double pp[3] = {p.x, p.y, p.z}, dd[3] = {d.x, d.y, d.z};
        const double j = ang ? ugj_ang_jac(&sc->ojoint[o], dd) : ugj_point_jac(&sc->ojoint[o], pp, dd);
#pragma unroll
        for (int i = 0; i < NB; i++) { J[i] = 0.0; MiJ[i] = 0.0; }
        J[0] = j;
        MiJ[0] = j / g_sh.jM[o];
        return;
    }
    const m3 R = qmat(e.obj[o].quat);
    const v3 r = vsub(p, e.obj[o].pos);
    const v3 rn = vcross(r, d);
    const v3 w = ang ? d : rn; /* the angular part of J */
    v3 ir = mtv(R, w);
    ir = V(ir.x / sc->oinertia[o].x, ir.y / sc->oinertia[o].y, ir.z / sc->oinertia[o].z);
    ir = mv(R, ir);
    const double im = 1.0 / sc->omass[o];
    J[0] = ang ? 0.0 : d.x; J[1] = ang ? 0.0 : d.y; J[2] = ang ? 0.0 : d.z;
    J[3] = w.x; J[4] = w.y; J[5] = w.z;
    MiJ[0] = ang ? 0.0 : d.x * im; MiJ[1] = ang ? 0.0 : d.y * im; MiJ[2] = ang ? 0.0 : d.z * im;
    MiJ[3] = ir.x; MiJ[4] = ir.y; MiJ[5] = ir.z;
#pragma unroll
    for (int i = 6; i < NB; i++) { J[i] = 0.0; MiJ[i] = 0.0; }
}
/* Build the row at position pos (one lane): J | M^-1 J^T into the workspace row, scalars into rs[pos].
 * Three phases so that the expensive part is convergent across the wave: (1) per kind, the entity
 * Jacobians (robot parts unsolved; limit / motor / gear rows take the shared unit solves), (2) the LDL
 * solves of the robot parts, once for all lanes that need one, (3) per kind, dots, rhs and bounds.  Every
 * row's arithmetic is the oracle's (build_rows in oracle/ug_oracle.c). */
__device__ __forceinline__ static void build_row(const Scene* s, int pos, double* wrow, bool store_j = true) {
    Shared& sh = g_sh;
    const EnvState& e = sh.e;
    const double dt = UG_DT;
    RowS& r = sh.rs[pos];
    const int kind = r.kind;
    double invD = 0.0, rhs = 0.0, rhsPen = 0.0, lo = 0.0, hi = 0.0, imp = 0.0, fric = 0.0;
    /* ---- phase 1: Jacobians ---- */
    PROF_T0(t_rb1);
    double JA[NB], MA[NB], JB[NB], MB[NB];
#pragma unroll
    for (int i = 0; i < NB; i++) { JA[i] = 0.0; MA[i] = 0.0; JB[i] = 0.0; MB[i] = 0.0; }
    bool solA = false, solB = false;
    int dof = 0;
    double sgn = 1.0;
    int entA = -1, entB = -1;
    const StPt* cp = nullptr;
    const PairDef* PP = nullptr;
    bool ang = false;
    if (kind <= 1) {
        dof = kind == 0 ? r.a : (r.a < 6 ? r.a : UG_FINGER_DOF);
        sgn = (kind == 0 && r.b == 1) ? -1.0 : 1.0;
#pragma unroll
        for (int i = 0; i < NB; i++) {
            JA[i] = i == dof ? sgn : 0.0;
            MA[i] = sgn > 0.0 ? sh.u.mcol[dof][i] : JA[i]; /* the shared solve of e_dof (team_unit_solves) */
        }
        solA = !(sgn > 0.0);
    } else if (kind == 2) {
        const int pa = UG_FINGER_DOF, cb = UG_GEAR_CHILD[r.a];
        const double ratio = UG_GEAR_RATIO[r.a];
#pragma unroll
        for (int i = 0; i < NB; i++) {
            JA[i] = i == pa ? 1.0 : 0.0;
            JB[i] = i == cb ? ratio : 0.0;
            MA[i] = sh.u.mcol[pa][i];      /* = ldlt_solve(JA) */
            MB[i] = sh.u.mcol[NB + r.a][i]; /* = ldlt_solve(JB) */
        }
    } else if (kind >= 8) { /* a jointed object's limit / the button's motor: slot 0 of object r.a (oracle jdof_row) */
        sgn = (kind == 8 && r.b == 1) ? -1.0 : 1.0;
        JA[0] = sgn;
        MA[0] = sgn / sh.jM[r.a];
        entA = 1 + r.a;
    } else {
        const StMan& M = e.man[r.a];
        PP = &s->pair[(int)M.pair];
        int bodyA, bodyB;
        entA = ent_of_collider(s->col[PP->a], bodyA);
        entB = ent_of_collider(s->col[PP->b], bodyB);
        XF OA = owner_xf(e, sh.kin, s->col[PP->a].owner), OB = owner_xf(e, sh.kin, s->col[PP->b].owner);
        cp = &M.pt[r.b];
        v3 pA = xf_apply(OA, cp->lpA), pB = xf_apply(OB, cp->lpB);
        v3 n = cp->n;
        v3 d = n;
        ang = kind >= 6; /* rolling friction: angular rows about the friction axes */
        if (kind >= 4) {
            v3 t1, t2;
            if (ug_fabs(n.z) > 0.7071067811865475244) {
                double a = n.y * n.y + n.z * n.z, kk = 1.0 / ug_sqrt(a);
                t1 = V(0, -n.z * kk, n.y * kk);
                t2 = V(a * kk, -n.x * t1.z, n.x * t1.y);
            } else {
                double a = n.x * n.x + n.y * n.y, kk = 1.0 / ug_sqrt(a);
                t1 = V(-n.y * kk, n.x * kk, 0);
                t2 = V(-n.z * t1.y, n.z * t1.x, a * kk);
            }
            d = (kind == 4 || kind == 6) ? t1 : t2;
        }
        if (entA == 0) {
            robot_jac_sel(sh.kin, ang, bodyA, pA, d, JA);
            solA = true;
        } else if (entA > 0) {
            object_jac_sel(s, e, ang, entA, pA, d, JA, MA);
        }
        const v3 dB = vneg(d);
        if (entB == 0) {
            robot_jac_sel(sh.kin, ang, bodyB, pB, dB, JB);
            solB = true;
        } else if (entB > 0) {
            object_jac_sel(s, e, ang, entB, pB, dB, JB, MB);
        }
    }
    PROF_ADD(PF_RB1, t_rb1);
    PROF_T0(t_rb2);
    /* ---- phase 2: M^-1 J^T of the robot parts, one solve for every lane that needs it ---- */
    if (ballot(solA) != 0ull) {
        double x[NB];
#pragma unroll
        for (int i = 0; i < NB; i++) x[i] = JA[i];
        ldlt_solve_r(sh.LDL, x);
#pragma unroll
        for (int i = 0; i < NB; i++) MA[i] = solA ? x[i] : MA[i];
    }
    if (ballot(solB) != 0ull) {
        double x[NB];
#pragma unroll
        for (int i = 0; i < NB; i++) x[i] = JB[i];
        ldlt_solve_r(sh.LDL, x);
#pragma unroll
        for (int i = 0; i < NB; i++) MB[i] = solB ? x[i] : MB[i];
    }
    PROF_ADD(PF_RB2, t_rb2);
    PROF_T0(t_rb3);
    /* ---- phase 3: dots, rhs, bounds ---- */
    if (kind <= 1) {
        const int d = dof;
        double den = ent_dot_r(0, JA, MA);
        invD = den > 2.220446049250313e-16 ? 1.0 / den : 0.0;
        double relv = ent_dot_v0(0, JA, sh.v0);
        if (kind == 0) {
            double pen = r.b == 0 ? e.q[d] - UG_DOF_LOWER[d] : UG_DOF_UPPER[d] - e.q[d];
            double erp = (pen > UG_SPLIT_PEN_THR) ? UG_ERP : UG_ERP2;
            double perr = -pen * erp / dt, verr = -relv;
            double pimp = perr * invD, vimp = verr * invD;
            rhs = (pen > UG_SPLIT_PEN_THR) ? pimp + vimp : vimp;
            lo = 0.0; hi = UG_LIMIT_MAXIMP;
        } else {
            int m = r.a;
            double maxImp = UG_DOF_MAXFORCE[d] * dt;
            double qd = sh.v0[d];
            double pst = 1.0 * (e.mtarget[m] - e.q[d]) / dt;
            double verr = 0.0 - qd;
            double des = UG_MOTOR_KP * pst + qd + UG_MOTOR_KD * verr;
            double clamp = UG_DOF_MAXVEL[d];
            if (des > clamp) des = clamp;
            if (des < -clamp) des = -clamp;
            rhs = 0.0 * invD + (des - relv) * invD;
            lo = -maxImp; hi = maxImp;
        }
    } else if (kind == 2) {
        const int pa = UG_FINGER_DOF, cb = UG_GEAR_CHILD[r.a];
        double ratio = UG_GEAR_RATIO[r.a];
        double den = ent_dot_r(0, JA, MA) + ent_dot_r(0, JB, MB);
        invD = den > 2.220446049250313e-16 ? 1.0 / den : 0.0;
        double relv = ent_dot_v0(0, JA, sh.v0) + ent_dot_v0(0, JB, sh.v0);
        double diff = e.q[cb] * ratio + e.q[pa];
        double pen = -UG_GEAR_ERP * (0.0 - diff);
        double perr = -pen * UG_ERP / dt, verr = 0.0 - relv;
        rhs = perr * invD + verr * invD;
        double maxImp = UG_GEAR_MAXF * dt;
        lo = -maxImp; hi = maxImp;
    } else if (kind >= 8) {
        const int o = r.a;
        double den = sgn * MA[0];
        invD = den > 2.220446049250313e-16 ? 1.0 / den : 0.0;
        double relv = sgn * sh.v0[NB + 6 * o];
        if (kind == 8) {
            const UgJoint& J = s->ojoint[o];
            const double qj = e.obj[o].w.x;
            double pen = r.b == 0 ? qj - J.lower : J.upper - qj;
            double erp = (pen > UG_SPLIT_PEN_THR) ? UG_ERP : UG_ERP2;
            double perr = -pen * erp / dt, verr = -relv;
            double pimp = perr * invD, vimp = verr * invD;
            rhs = (pen > UG_SPLIT_PEN_THR) ? pimp + vimp : vimp;
            lo = 0.0; hi = UG_LIMIT_MAXIMP;
        } else { /* reset_box: position control, force 1, target 0, no velocity clamp */
            double qd = sh.v0[NB + 6 * o];
            double pst = 1.0 * (0.0 - e.obj[o].w.x) / dt;
            double verr = 0.0 - qd;
            double des = UG_MOTOR_KP * pst + qd + UG_MOTOR_KD * verr;
            double maxImp = UG_BX_BUTTON_FORCE * dt;
            rhs = 0.0 * invD + (des - relv) * invD;
            lo = -maxImp; hi = maxImp;
        }
    } else {
        const PairDef& P = *PP;
        double dA = 0.0, dB = 0.0, relv = 0.0;
        if (entA >= 0) {
            dA = ent_dot_r(entA, JA, MA);
            relv += ent_dot_v0(entA, JA, sh.v0);
        }
        if (entB >= 0) {
            dB = ent_dot_r(entB, JB, MB);
            relv += ent_dot_v0(entB, JB, sh.v0);
        }
        double den = dA + dB;
        invD = den > 2.220446049250313e-16 ? 1.0 / den : 0.0;
        if (kind == 3) {
            double pen = cp->dist + UG_LINEAR_SLOP;
            double rest = 0.0;
            if (!(ug_fabs(relv) < UG_REST_VEL_THR)) rest = P.restitution * -relv;
            if (rest <= 0.0) rest = 0.0;
            double verr = rest - relv, perr;
            double erp = (pen > UG_SPLIT_PEN_THR) ? UG_ERP : UG_ERP2;
            if (pen > 0) { perr = 0.0; verr -= pen / UG_DT; }
            else perr = -pen * erp / UG_DT;
            double pimp = perr * invD, vimp = verr * invD;
            if (pen > UG_SPLIT_PEN_THR) { rhs = pimp + vimp; rhsPen = 0.0; }
            else { rhs = vimp; rhsPen = pimp; }
            lo = 0.0; hi = 1e10;
            imp = cp->imp * UG_WARMSTART;
        } else {
            rhs = 0.0 * invD + (0.0 - relv) * invD;
            fric = ang ? P.rolling : P.friction;
        }
    }
    r.invD = invD; r.rinv = invD == 0.0 ? 0.0 : 1.0 / invD; r.rhs = rhs; r.rhsPen = rhsPen; r.lo = lo; r.hi = hi; r.imp = imp; r.impPen = 0.0; r.fric = fric;
    /* J | M^-1 J^T over the NVP dof slots: limit / motor rows their robot part, gear rows the sum of both
     * robot parts, contact rows each side's entity segment (zero elsewhere, pads included) */
    const int eA = kind <= 2 ? 0 : entA, eB = kind == 2 ? 0 : (kind <= 1 ? -1 : entB);
    if (store_j) {
#pragma unroll
    for (int i = 0; i < NVP; i++) {
        const int ent = i < NB ? 0 : (i < NV ? 1 + (i - NB) / 6 : -2);
        const int k = i < NB ? i : (i - NB) % 6;
        double j = 0.0, m = 0.0;
        if (kind == 2) {
            if (i < NB) { j = JA[i] + JB[i]; m = MA[i] + MB[i]; }
        } else {
            if (eA == ent) { j = JA[k]; m = MA[k]; }
            if (eB == ent) { j = JB[k]; m = MB[k]; }
        }
        wrow[i] = j;
        wrow[RJ + i] = m;
    }
    }
    PROF_ADD(PF_RB3, t_rb3);
}
/* the substep's rows, lane per row: outlined, so the row build's registers are its own and not live kernel state
 * (inline, its loop spilled 31 / reloaded 80 kernel registers per substep) */
__device__ __noinline__ static void team_build_rows(const Scene* s, int n, double* ws, bool store_j) {
    for (int p = threadIdx.x; p < n; p += TEAM) build_row(s, p, ws + WS_ROWS + p * RS, store_j);
}

