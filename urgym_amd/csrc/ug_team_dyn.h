/* ug_team_dyn.h -- part of ug_team.h: FK, CRBA / RNEA robot dynamics, LDL^T, integration (serial_pre / serial_post / serial_fk).
 * Included by ug_team.h inside namespace ugd, in this order (the kernel is one translation unit); not self-contained. */
/* ---- robot dynamics, wave-parallel (same operations and order as robot_dynamics / the oracle) ----
 * lane b < NB owns body b (inertias, spatial axis, mass-matrix column, RNEA forward step, forces); the
 * tree accumulations (composite inertia, force back-propagation) run component-parallel: lane c owns
 * one scalar component and walks the bodies in the serial code's descending order.  The RNEA forward
 * pass goes level by level down the (compile-time) tree.  Results: M -> LDL (LDS), C -> w.C. */
/* the kinematic tree as compile-time data (same initializer as UG_BODY_PARENT): tree loops with constant
 * parents keep their per-body arrays in registers */
constexpr int kParent[NB] = UG_BODY_PARENT_INIT;
__device__ __forceinline__ int body_depth(int b) {
    int d = 0;
    for (int j = UG_BODY_PARENT[b]; j >= 0; j = UG_BODY_PARENT[j]) d++;
    return d;
}
__device__ __noinline__ static void team_robot_dynamics(double g_) {
    PROF_ENTRY(CS_RDYN);
    PROF_CALL(CALL_RDYN);
    /* the LDS image is addressed directly (pointer arguments would turn every access into a flat one) */
    const double* qd = g_sh.e.qd;
    const Kin& k = g_sh.kin;
    double* M = g_sh.LDL;
    DynWork& w = g_sh.u.dyn;
    const double g = g_;
    const int lane = threadIdx.x;
    const bool own = lane < NB;
    const int b = own ? lane : 0;
    /* 1. per body: mass, first moment, world inertia about the origin, spatial axis */
    double m = 0.0;
    v3 h = V(0, 0, 0);
    m3 Jb;
    if (own) {
        m = UG_BODY_MASS[b];
        v3 c = k.c[b];
        h = vscale(c, m);
        m3 Iw = inertia_world(k.R[b], &UG_BODY_I[6 * b]);
        double cc = vdot(c, c);
        Jb.m[0] = Iw.m[0] + m * (cc - c.x * c.x); Jb.m[1] = Iw.m[1] - m * (c.x * c.y); Jb.m[2] = Iw.m[2] - m * (c.x * c.z);
        Jb.m[3] = Iw.m[3] - m * (c.y * c.x); Jb.m[4] = Iw.m[4] + m * (cc - c.y * c.y); Jb.m[5] = Iw.m[5] - m * (c.y * c.z);
        Jb.m[6] = Iw.m[6] - m * (c.z * c.x); Jb.m[7] = Iw.m[7] - m * (c.z * c.y); Jb.m[8] = Iw.m[8] + m * (cc - c.z * c.z);
        w.m[b] = m; w.h[b] = h; w.J[b] = Jb;
        w.cm[b] = m; w.ch[b] = h; w.cJ[b] = Jb;
        w.S[b].w = k.a[b];
        w.S[b].v = vcross(k.p[b], k.a[b]);
    }
    for (int i = lane; i < NB * NB; i += TEAM) M[i] = 0.0;
    __syncthreads();
    /* 2. composite inertias: cm[p] += cm[b], ch[p] += ch[b], cJ[p] += cJ[b] for b = NB-1 .. 0 (13 components) */
    if (lane < 13) {
        double* base = lane == 0 ? w.cm : (lane < 4 ? &w.ch[0].x + (lane - 1) : &w.cJ[0].m[0] + (lane - 4));
        const int stride = lane == 0 ? 1 : (lane < 4 ? 3 : 9);
        double v[NB];
#pragma unroll
        for (int i = 0; i < NB; i++) v[i] = base[i * stride];
#pragma unroll
        for (int i = NB - 1; i >= 0; i--) {
            const int p = kParent[i]; /* a constant after unrolling */
            if (p >= 0) v[p] = v[p] + v[i];
        }
#pragma unroll
        for (int i = 0; i < NB; i++) base[i * stride] = v[i];
    }
    __syncthreads();
    /* 3. mass matrix column of body b: M[b][b] and M[j][b] = M[b][j] for its ancestors j */
    if (own) {
        SV F = spatial_inertia_mul(w.cm[b], w.ch[b], w.cJ[b], w.S[b]);
        const SV Sb = w.S[b];
        M[b * NB + b] = vdot(Sb.w, F.w) + vdot(Sb.v, F.v);
        const int am = g_sh.anc[b]; /* ancestors j of b (the parent walk, from the LDS mask) */
#pragma unroll
        for (int j = NB - 1; j >= 0; j--) {
            if (j != b && ((am >> j) & 1)) {
                double x = vdot(w.S[j].w, F.w) + vdot(w.S[j].v, F.v);
                M[j * NB + b] = x;
                M[b * NB + j] = x;
            }
        }
    }
    /* 4. RNEA forward, one tree level at a time; then the body's force (independent of the others) */
    const int depth = own ? g_sh.bdepth[b] : -1; /* body_depth(b), cached in LDS */
    SV f;
    f.w = V(0, 0, 0);
    f.v = V(0, 0, 0);
    SV Vbb;
    Vbb.w = V(0, 0, 0);
    Vbb.v = V(0, 0, 0);
    /* the damping inertia in world axes does not depend on the parent: formed up front */
    const m3 Dw = inertia_world(k.R[b], &UG_BODY_DAMPI[6 * b]);
    /* RNEA forward as a per-lane ancestor walk: lane b recomputes the velocity / acceleration recursion
     * along its own root-to-b path (ancestor indices ascend with depth), the same operations on the same
     * inputs as the body-by-body pass, without a barrier per tree level */
    (void)depth;
    if (own) {
        const int am = g_sh.anc[b];
        SV Vp, Ap;
        Vp.w = V(0, 0, 0); Vp.v = V(0, 0, 0); Ap.w = V(0, 0, 0); Ap.v = V(0, 0, -g);
#pragma unroll
        for (int j = 0; j < NB; j++) {
            if ((am >> j) & 1) {
                const SV Sj = w.S[j];
                SV vj; vj.w = vscale(Sj.w, qd[j]); vj.v = vscale(Sj.v, qd[j]);
                SV Vj, Aj;
                Vj.w = vadd(Vp.w, vj.w); Vj.v = vadd(Vp.v, vj.v);
                Aj.w = vadd(Ap.w, vcross(Vj.w, vj.w));
                Aj.v = vadd(Ap.v, vadd(vcross(Vj.w, vj.v), vcross(Vj.v, vj.w)));
                Vp = Vj;
                Ap = Aj;
            }
        }
        const SV Vb = Vp, Ab = Ap;
        w.Vb[b] = Vb;
        w.Ab[b] = Ab;
        SV IA = spatial_inertia_mul(m, h, Jb, Ab);
        SV IV = spatial_inertia_mul(m, h, Jb, Vb);
        f.w = vadd(IA.w, vadd(vcross(Vb.w, IV.w), vcross(Vb.v, IV.v)));
        f.v = vadd(IA.v, vcross(Vb.w, IV.v));
        double wn = vlen(Vb.w);
        v3 tau = vscale(mv(Dw, Vb.w), UG_ANG_DAMP + UG_ANG_DAMP * wn);
        f.w = vadd(f.w, tau);
        Vbb = Vb;
    }
    __syncthreads();
    /* 5. link damping: lane l computes link l's force and torque; body b adds its links in link order */
    if (lane >= 1 && lane < UG_NL) {
        const int l = lane, bl = UG_LINK_BODY[l];
        if (bl >= 0) {
            v3 cl = vadd(k.p[bl], mv(k.R[bl], V(UG_LINK_COMP[3 * l], UG_LINK_COMP[3 * l + 1], UG_LINK_COMP[3 * l + 2])));
            const SV Vl = w.Vb[bl];
            v3 vl = vadd(Vl.v, vcross(Vl.w, cl));
            double vn = vlen(vl);
            v3 fd = vscale(vl, UG_LINK_MASS[l] * (UG_LIN_DAMP + UG_LIN_DAMP * vn));
            w.fdl[l] = fd;
            w.tl[l] = vcross(cl, fd);
        }
    }
    __syncthreads();
    if (own) {
        for (int l = 1; l < UG_NL; l++) {
            if (UG_LINK_BODY[l] != b) continue;
            f.v = vadd(f.v, w.fdl[l]);
            f.w = vadd(f.w, w.tl[l]);
        }
        w.f[b] = f;
    }
    __syncthreads();
    /* 6. forces back up the tree (6 components, descending bodies), then C[b] = S_b . f_b */
    if (lane < 6) {
        double* base = (lane < 3 ? &w.f[0].w.x : &w.f[0].v.x) + (lane % 3);
        const int stride = sizeof(SV) / sizeof(double);
        double v[NB];
#pragma unroll
        for (int i = 0; i < NB; i++) v[i] = base[i * stride];
#pragma unroll
        for (int i = NB - 1; i >= 0; i--) {
            const int p = kParent[i]; /* a constant after unrolling */
            if (p >= 0) v[p] = v[p] + v[i];
        }
#pragma unroll
        for (int i = 0; i < NB; i++) base[i * stride] = v[i];
    }
    __syncthreads();
    if (own) {
        const SV Sb = w.S[b], fb = w.f[b];
        w.C[b] = vdot(Sb.w, fb.w) + vdot(Sb.v, fb.v);
    }
    __syncthreads();
    (void)Vbb;
    PROF_EXIT();
}
/* lane 0: external forces (robot gravity/gyroscopic/damping via CRBA + RNEA, free objects), the LDL^T of
 * the mass matrix, and the row enumeration */
__device__ __noinline__ static void serial_pre(const Scene* s) {
    PROF_ENTRY(CS_PRE);
    PROF_CALL(CALL_PRE);
    Shared& sh = g_sh;
    EnvState& e = sh.e;
    const double dt = UG_DT;
    const int lane = threadIdx.x;
    PROF_T0(t_rd);
    PROF_PRE_CALL();
    team_robot_dynamics(s->gravity);
    PROF_POST_CALL(CS_RDYN);
    PROF_ADD(PF_RDYN, t_rd);
    PROF_T0(t_ldl);
    {
        /* LDL^T of the mass matrix, wave-parallel: lane i < NB owns row i.  Step j: every lane forms
         * t = a[j] - sum_k (a[k] * L_jk) * D_k (k ascending; L_jk broadcast from lane j), which on lane j is
         * ldlt()'s diagonal d and on lanes i > j its s; then a[j] = d (lane j) or s / d (i > j).  The same
         * operations in the same order as ldlt_r() / the oracle's ldlt(), one division per step instead of
         * one per element. */
        const bool own = lane < NB;
        double a[NB], D[NB];
#pragma unroll
        for (int c = 0; c < NB; c++) a[c] = own ? sh.LDL[lane * NB + c] : 0.0;
#pragma unroll
        for (int j = 0; j < NB; j++) {
            double t = a[j];
#pragma unroll
            for (int k2 = 0; k2 < j; k2++) t -= a[k2] * readlane_d(a[k2], j) * D[k2];
            const double d = readlane_d(t, j);
            D[j] = d;
            a[j] = lane == j ? d : (lane > j ? t / d : a[j]);
        }
        if (own) {
#pragma unroll
            for (int c = 0; c < NB; c++) sh.LDL[lane * NB + c] = a[c];
        }
        if (lane < NVP) sh.v0[lane] = 0.0; /* inactive objects' and padding slots stay 0 */
        __syncthreads();
    }
    if (lane == 0) {
        double C[NB];
#pragma unroll
        for (int i = 0; i < NB; i++) C[i] = sh.u.dyn.C[i];
        /* the qdd solve with the factored matrix in registers (compile-time indices, same order) */
        double A[NB * NB];
#pragma unroll
        for (int i = 0; i < NB * NB; i++) A[i] = sh.LDL[i];
        double qdd[NB];
#pragma unroll
        for (int i = 0; i < NB; i++) qdd[i] = -C[i];
        ldlt_solve_r(A, qdd);
        /* every dof velocity clamped to +-m_maxCoordinateVelocity (oracle substep) */
        for (int i = 0; i < NB; i++) { e.qd[i] = ug_vclamp(e.qd[i] + qdd[i] * dt, UG_MAX_COORD_VEL); sh.v0[i] = e.qd[i]; }
    } else if (lane <= s->nobj) { /* free bodies, one lane each (independent of the robot solve) */
        const int o = lane - 1;
        if (e.oactive[o] != 0.0 && s->ojoint[o].kind != UGJ_FREE) {
            /* a one-dof link on a fixed base (oracle substep, ug_joint.h): joint velocity in v.x, position in w.x */
            StObj& ob = e.obj[o];
            const double qt[4] = {ob.quat.x, ob.quat.y, ob.quat.z, ob.quat.w};
            double Mj, Cj;
            ugj_dynamics(&s->ojoint[o], qt, ob.v.x, s->gravity, &Mj, &Cj);
            sh.jM[o] = Mj;
            const double qdd = -Cj / Mj;
            ob.v.x = ug_vclamp(ob.v.x + qdd * dt, UG_MAX_COORD_VEL);
            sh.v0[NB + 6 * o] = ob.v.x;
        } else if (e.oactive[o] != 0.0) {
            StObj& ob = e.obj[o];
            v3 v = ob.v;
            double vn = vlen(v);
            v3 a = vsub(V(0, 0, s->gravity), vscale(v, UG_LIN_DAMP + UG_LIN_DAMP * vn));
            ob.v = vclamp_coord(vadd(v, vscale(a, dt)));
            m3 R = qmat(ob.quat);
            v3 wl = mtv(R, ob.w);
            v3 I = s->oinertia[o];
            v3 Iw = V(I.x * wl.x, I.y * wl.y, I.z * wl.z);
            double wn = vlen(wl);
            v3 z = vadd(vscale(Iw, UG_ANG_DAMP + UG_ANG_DAMP * wn), vcross(wl, Iw));
            v3 al = V(-z.x / I.x, -z.y / I.y, -z.z / I.z);
            ob.w = vclamp_coord(vadd(ob.w, vscale(mv(R, al), dt)));
            int off = NB + 6 * o;
            sh.v0[off] = ob.v.x; sh.v0[off + 1] = ob.v.y; sh.v0[off + 2] = ob.v.z;
            sh.v0[off + 3] = ob.w.x; sh.v0[off + 4] = ob.w.y; sh.v0[off + 5] = ob.w.z;
        }
    }
    __syncthreads();
    PROF_ADD(PF_LDL, t_ldl);
    PROF_T0(t_en);
    PROF_PRE_CALL();
    team_enumerate(s);
    PROF_POST_CALL(CS_ENUM);
    PROF_ADD(PF_ENUM, t_en);
    PROF_EXIT();
}
/* velocities += solver delta, positions integrate (v + split velocity): lane i < NB dof i, lane NB + o object o (each
 * element's operations as the oracle's serial loops; no element reads another) */
__device__ __noinline__ static void serial_post(const Scene* s, int split) {
    PROF_ENTRY(CS_POST);
    PROF_CALL(CALL_POST);
    Shared& sh = g_sh;
    EnvState& e = sh.e;
    const double dt = UG_DT;
    const int lane = threadIdx.x;
    const double* DV = sh.dvout;
    const double* DVS = sh.dvsout;
    if (lane < NB) {
        const int i = lane;
        /* the pose this substep's narrowphase saw, before it moves (the contact query's world positions) */
        e.prevq[i] = e.q[i];
        e.qd[i] = ug_vclamp(e.qd[i] + DV[i], UG_MAX_COORD_VEL);
        double vi = split ? e.qd[i] + DVS[i] : e.qd[i];
        e.q[i] = e.q[i] + vi * dt;
    } else if (lane < NB + MAXOBJ) {
        const int o = lane - NB;
        {
            const StObj& ob = e.obj[o];
            e.prevpose[o][0] = ob.pos.x; e.prevpose[o][1] = ob.pos.y; e.prevpose[o][2] = ob.pos.z;
            e.prevpose[o][3] = ob.quat.x; e.prevpose[o][4] = ob.quat.y; e.prevpose[o][5] = ob.quat.z;
            e.prevpose[o][6] = ob.quat.w;
        }
        if (o < s->nobj && e.oactive[o] != 0.0) {
            StObj& ob = e.obj[o];
            int off = NB + 6 * o;
            if (s->ojoint[o].kind != UGJ_FREE) {
                ob.v.x = ug_vclamp(ob.v.x + DV[off], UG_MAX_COORD_VEL);
                double vi = split ? ob.v.x + DVS[off] : ob.v.x;
                ob.w.x = ob.w.x + vi * dt;
                double qt[4], pt[3];
                ugj_frame(&s->ojoint[o], ob.w.x, qt, pt);
                ob.quat = Q(qt[0], qt[1], qt[2], qt[3]);
                ob.pos = V(pt[0], pt[1], pt[2]);
            } else {
                ob.v = vclamp_coord(vadd(ob.v, V(DV[off], DV[off + 1], DV[off + 2])));
                ob.w = vclamp_coord(vadd(ob.w, V(DV[off + 3], DV[off + 4], DV[off + 5])));
                v3 vl = ob.v, wa = ob.w;
                if (split) {
                    vl = vadd(vl, V(DVS[off], DVS[off + 1], DVS[off + 2]));
                    wa = vadd(wa, V(DVS[off + 3], DVS[off + 4], DVS[off + 5]));
                }
                ob.pos = vadd(ob.pos, vscale(vl, dt));
                double ang = vlen(wa);
                if (ang * dt > UG_ANGULAR_MOTION_THR) ang = UG_ANGULAR_MOTION_THR / dt;
                v3 ax;
                if (ang < 0.001) ax = vscale(wa, 0.5 * dt - (dt * dt * dt) * 0.020833333333 * ang * ang);
                else ax = vscale(wa, ug_sin(0.5 * ang * dt) / ang);
                q4 dq = Q(ax.x, ax.y, ax.z, ug_cos(0.5 * ang * dt));
                ob.quat = qnormalize(qmul(dq, ob.quat));
            }
        }
    }
    PROF_EXIT();
}
/* fk() wave-parallel: lane b < NB forms its joint rotation, then composes its own root-to-body chain
 * (same operations and order as fk() along that path) */
__device__ __noinline__ static void serial_fk() {
    PROF_ENTRY(CS_FK);
    PROF_CALL(CALL_FK);
    Kin& k = g_sh.kin;
    const int lane = threadIdx.x;
    const bool own = lane < NB;
    const int b = own ? lane : 0;
    /* each body's joint rotation once (lane per body), shared through LDS; then every lane walks its own
     * root-to-body path (ancestor indices ascend with depth) with fk()'s operations, no barrier per level */
    if (own) {
        const v3 ax = V(UG_BODY_AXIS[3 * b], UG_BODY_AXIS[3 * b + 1], UG_BODY_AXIS[3 * b + 2]);
        g_sh.u.rj[b] = axis_angle(ax, g_sh.e.q[b]);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    if (own) {
        const int am = g_sh.anc[b];
        m3 Rp = mident();
        v3 pp = V(0, 0, 0);
        m3 Rtmp = Rp;
#pragma unroll
        for (int j = 0; j < NB; j++) {
            if ((am >> j) & 1) {
                const m3 Rpb = mload(&UG_BODY_R[9 * j]);
                const v3 Ppb = V(UG_BODY_P[3 * j], UG_BODY_P[3 * j + 1], UG_BODY_P[3 * j + 2]);
                Rtmp = mm(Rp, Rpb);
                const m3 R = mm(Rtmp, g_sh.u.rj[j]);
                pp = vadd(pp, mv(Rp, Ppb));
                Rp = R;
            }
        }
        const v3 ax = V(UG_BODY_AXIS[3 * b], UG_BODY_AXIS[3 * b + 1], UG_BODY_AXIS[3 * b + 2]);
        const v3 com = V(UG_BODY_COM[3 * b], UG_BODY_COM[3 * b + 1], UG_BODY_COM[3 * b + 2]);
        k.R[b] = Rp;
        k.p[b] = pp;
        k.a[b] = mv(Rtmp, ax);
        k.c[b] = vadd(pp, mv(Rp, com));
    }
    __syncthreads();
    PROF_EXIT();
}

