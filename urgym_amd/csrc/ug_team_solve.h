/* ug_team_solve.h -- part of ug_team.h: the PGS solve (team_pgs: fixed layouts, contact-free and general sweeps) and the quiescent-collision test.
 * Included by ug_team.h inside namespace ugd, in this order (the kernel is one translation unit); not self-contained. */
#ifdef UG_DEBUG_DUMP
template <int J>
__device__ __forceinline__ void dump_A(const double (&A0)[PREG], const double (&A1)[PREG], double* dbg, int n, int lane) {
    if constexpr (J < PREG) {
        if (J < n) {
            dbg[J * MAXROWS + lane] = A0[J];
            dbg[J * MAXROWS + 64 + lane] = A1[J];
            dump_A<J + 1>(A0, A1, dbg, n, lane);
        }
    }
}
#endif
/* PGS: Delassus rows, warm start (normals), sweeps (residual early-out), the split-impulse pass; returns
 * whether the split pass ran (dvs valid).  Impulses are written back to sh.rs[].imp.  Its own function:
 * the 2 x PREG register rows of A get a register allocation of their own. */
/* a[i] of a small constant table by an unrolled select (immediates, no constant-memory load) */
template <typename T, int N>
__device__ __forceinline__ T csel(const T (&a)[N], int i) {
    T v = a[0];
#pragma unroll
    for (int g = 1; g < N; g++) v = i == g ? a[g] : v;
    return v;
}
/* the scaled Delassus rows of a motor / gear solve (n = nnc = 12): A[i][P] = the k-ordered fma chain of J_i . M^-1 J_P^T
 * over the dof slots (what the matrix cores compute, mfma_block), with J_i's one or two non-zero entries
 * (motor: 1 at its dof; gear: 1 at the finger dof, the ratio at the child dof) -- the zero terms of the chain
 * leave it unchanged -- then scaled -(A / D_i).  Branch-free, every LDS read independent. */
__device__ __forceinline__ void nc_direct_A(double (&A0)[PREG], int lane) {
    const int i = lane < 12 ? lane : 0;
    const RowS& r = g_sh.rs[i];
    const bool gear = r.kind == 2;
    const int ra = r.a;
    const int k1 = gear ? UG_FINGER_DOF : (ra < 6 ? ra : UG_FINGER_DOF);
    const int k2 = gear ? csel(UG_GEAR_CHILD, ra) : k1;
    const double j2 = gear ? csel(UG_GEAR_RATIO, ra) : 0.0;
    const double invD = lane < 12 ? r.invD : 0.0;
    int kP[12], aP[12];
#pragma unroll
    for (int P = 0; P < 12; P++) {
        kP[P] = __builtin_amdgcn_readfirstlane(g_sh.rs[P].kind);
        aP[P] = __builtin_amdgcn_readfirstlane(g_sh.rs[P].a);
    }
#pragma unroll
    for (int P = 0; P < PREG; P++) {
        if (P < 12) {
            const bool gP = kP[P] == 2;
            const int r1 = gP ? UG_FINGER_DOF : (aP[P] < 6 ? aP[P] : UG_FINGER_DOF);
            const int r2 = gP ? NB + aP[P] : r1;
            const double x11 = g_sh.u.mcol[r1][k1], x21 = g_sh.u.mcol[r2][k1];
            const double x12 = g_sh.u.mcol[r1][k2], x22 = g_sh.u.mcol[r2][k2];
            const double m1 = gP ? x11 + x21 : x11, m2 = gP ? x12 + x22 : x12;
            const double c1 = __builtin_fma(1.0, m1, 0.0), c2 = __builtin_fma(j2, m2, 0.0);
            const double raw = !gear ? c1 : (k1 < k2 ? __builtin_fma(j2, m2, c1) : __builtin_fma(1.0, m1, c2));
            const double x = -(raw * invD);
            A0[P] = lane < 12 ? x : 0.0;
        }
    }
}
/* A call site that never runs, to make a large function non-leaf.  LLVM's AMDGPU branch relaxation expands an
 * out-of-range branch (beyond +-32 Ki instructions) into s_getpc_b64 / s_add / s_setpc_b64 through a scavenged SGPR
 * pair, and in a leaf function it took s[30:31] -- the return address, which a leaf function never saves: team_pgs'
 * return then jumped back into its own body and the kernel never finished (measured on MI355X: Box-v0's reset hung
 * once team_pgs grew to ~56 k lines).  A non-leaf function keeps its return address in a VGPR lane from the prologue,
 * so the pair is free.  tests/test_isa_audit.py fails the build if any function writes s[30:31] without saving it. */
__device__ __noinline__ void ug_nonleaf_guard() { __asm__ volatile(""); }
__device__ __noinline__ static int team_pgs(double* ws_, int n_, int nnc_, int nn_, int nobj_, double& dv, double& dvs) {
    PROF_ENTRY(CS_PGS);
    PROF_CALL(CALL_PGS);
    if (__builtin_expect(n_ < 0, 0)) ug_nonleaf_guard(); /* never: n_ >= 0 (see ug_nonleaf_guard) */
    Shared& sh = g_sh;
    const int lane = threadIdx.x;
    /* arguments of a non-kernel function arrive in VGPRs: make the uniform ones scalar again */
    const int n = uniform(n_), nnc = uniform(nnc_), nn = uniform(nn_), nobj = uniform(nobj_);
    double* ws = uniform_ptr(ws_);
    const int fb = nnc + nn;
    PROF_T0(t_setup);
    gcdouble* rows = (gcdouble*)(ws + WS_ROWS);
    gdouble* wsA = (gdouble*)(ws + WS_A);
    double A0[PREG], A1[PREG];
    /* scaled Delassus rows on the matrix cores (mfma_block); slot 1 only when rows >= 64 exist */
    PROF_T0(t_mf);
    /* the fixed layout: 12 non-contact rows, 16..28 normals, at most 56 friction rows (BallBalance's contact
     * solves, in steps and in resets) */
#ifdef UG_DEBUG_DUMP
    const PosMap pm{n, fb, 0, nnc, nnc, n};
#else
    const bool flok = nnc == FL_NNC && nn >= 16 && fb <= FL_F0 && n - fb <= FL_NF;
    /* the narrowest fixed layout that holds the solve: friction from F0, at most 2 (F0 - 12) friction rows */
    const int flf0 = (fb <= FL_F020 && n - fb <= 2 * (FL_F020 - FL_NNC))   ? FL_F020
                     : (fb <= FL_F022 && n - fb <= 2 * (FL_F022 - FL_NNC)) ? FL_F022
                     : (fb <= FL_F0S && n - fb <= FL_NFS)                  ? FL_F0S
                                                                           : FL_F0;
    /* the single-slot layout: few normals (CubesPush 8, CubesGrasp 4-6), up to 20 non-contact rows */
    const bool fsb = !flok && nnc <= FSB_NC && nn >= 1 && nn <= FSB_F0 - FSB_NC && n - fb <= FSB_NF;
    const bool fs14ok = !flok && nnc <= FS14_NC && nn >= 3;
    const bool fs14g = fs14ok && nn <= FS14G_F0 - FS14_NC && n - fb <= FS14G_NF;
    const bool fs14p = fs14ok && !fs14g && nn <= FS14P_F0 - FS14_NC && n - fb <= FS14P_NF;
    const bool fs14w = fs14ok && !fs14g && !fs14p && nn <= FS14W_F0 - FS14_NC && n - fb <= FS14W_NF;
    const bool fs14h = fs14ok && !fs14g && !fs14p && !fs14w && nn <= FS14H_F0 - FS14_NC && n - fb <= FS14H_NF;
    const bool fs6ok = !flok && nnc <= FS_NC && nn >= 3 && nn <= FS6_F0 - FS_NC && n - fb <= FS6_NF;
    const bool fsok = !flok && nnc <= FS_NC && nn >= 3 && nn <= FS_F0 - FS_NC && n - fb <= FS_NF;
    const bool g12ok = !flok && !fsok && nnc <= FG12_NC && nn >= 3 && nn <= FG12_F0 - FG12_NC && n - fb <= FG12_NF;
    const bool g18ok = !flok && !fsok && !g12ok && nnc <= FG18_NC && nn >= 3 && nn <= FG18_F0 - FG18_NC &&
                       n - fb <= FG18_NF;
    const bool fgok = !flok && !fsok && !g12ok && !g18ok && nnc <= FG_NC && nn >= 16 && nn <= FG_F0 - FG_NC &&
                      n - fb <= FG_NF;
    const PosMap pm = flok ? PosMap{n, fb, flf0, nnc, nnc, flf0 + 2 * (flf0 - FL_NNC)}
                      : fsb ? PosMap{n, fb, FSB_F0, nnc, FSB_NC, FSB_F0 + FSB_NF}
                      : fs14g ? PosMap{n, fb, FS14G_F0, nnc, FS14_NC, FS14G_F0 + FS14G_NF}
                      : fs14p ? PosMap{n, fb, FS14P_F0, nnc, FS14_NC, FS14P_F0 + FS14P_NF}
                      : fs14w ? PosMap{n, fb, FS14W_F0, nnc, FS14_NC, FS14W_F0 + FS14W_NF}
                      : fs6ok ? PosMap{n, fb, FS6_F0, nnc, FS_NC, FS6_F0 + FS6_NF}
                      : fsok ? PosMap{n, fb, FS_F0, nnc, FS_NC, FS_F0 + FS_NF}
                      : fs14h ? PosMap{n, fb, FS14H_F0, nnc, FS14_NC, FS14H_F0 + FS14H_NF}
                      : g12ok ? PosMap{n, fb, FG12_F0, nnc, FG12_NC, FG12_F0 + FG12_NF}
                      : g18ok ? PosMap{n, fb, FG18_F0, nnc, FG18_NC, FG18_F0 + FG18_NF}
                      : fgok ? PosMap{n, fb, FG_F0, nnc, FG_NC, FG_F0 + FG_NF}
                             : PosMap{n, fb, 0, nnc, nnc, n};
#endif
    const int npos = pm.npos();
    /* the contact-free solve of 7 motor + 5 gear rows: its Delassus rows straight from the shared unit solves
     * in LDS (team_unit_solves), no workspace round trip */
#ifdef UG_DEBUG_DUMP
    const bool direct = false; /* the dump reads every column */
#else
    const bool direct = n == 12 && nnc == 12 && ballot(lane < 12 && sh.rs[lane].kind == 0) == 0ull;
#endif
    if (direct) {
        nc_direct_A(A0, lane); /* columns 0..11 only: the 12-row sweeps read nothing else of A0 / A1 */
    } else {
        const int q0 = pm.q(lane), q1 = pm.q(lane + 64);
        const double i0 = q0 >= 0 ? sh.rs[q0].invD : 0.0, i1 = q1 >= 0 ? sh.rs[q1].invD : 0.0;
        const bool k6 = nobj <= (4 * 6 - NB) / 6; /* the object dofs end within k-step 5 */
        if (k6) mfma_slot<0, 6>(rows, i0, A0, wsA, pm, lane);
        else mfma_slot<0, KS>(rows, i0, A0, wsA, pm, lane);
        if (npos > 64) {
            if (pm.fl && k6) mfma_slot<1, 6, 2>(rows, i1, A1, wsA, pm, lane);
            else if (pm.fl) mfma_slot<1, KS, 2>(rows, i1, A1, wsA, pm, lane);
            else if (k6) mfma_slot<1, 6>(rows, i1, A1, wsA, pm, lane);
            else mfma_slot<1, KS>(rows, i1, A1, wsA, pm, lane);
        } else {
#pragma unroll
            for (int j = 0; j < PREG; j++) A1[j] = 0.0;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    PROF_ADD(PF_MFMA, t_mf);
    gcdouble* wsAr = (gcdouble*)wsA;
    Lrow L;
    double fric[2], rhsPen[2];
    int nrow[2];
#pragma unroll
    for (int s = 0; s < 2; s++) {
        const int q = pm.q(lane + 64 * s);
        const bool in = q >= 0;
        const RowS& r = sh.rs[in ? q : 0];
        L.rhs[s] = in ? r.rhs : 0.0;
        L.invD[s] = in ? r.invD : 0.0;
        L.rinv[s] = in ? r.rinv : 0.0;
        L.lo[s] = in ? r.lo : 0.0;
        L.hi[s] = in ? r.hi : 0.0;
        L.imp[s] = in ? r.imp : 0.0;
        L.dsv[s] = 0.0;
        fric[s] = in ? r.fric : 0.0;
        nrow[s] = in ? r.nrow : 0;
        rhsPen[s] = in ? r.rhsPen : 0.0;
    }
    double W[2] = {L.rhs[0], L.rhs[1]}; /* u */
    PROF_T0(t_wm);
    if (nn > 0) { /* the normals' positions: [nnc, fb), or [FS_NC, FS_NC + nn) in the single-slot layout */
        const int wb = pm.fl ? pm.nb : nnc;
        sweep_warm<0>(A0, A1, wsAr, lane, wb, wb + nn, L, W);
    }
    PROF_ADD(PF_WARM, t_wm);
    PROF_ADD(PF_SPLIT, t_setup);
#ifdef UG_DEBUG_DUMP
    double* dbg = ws + WS_DBG;
    dump_A<0>(A0, A1, dbg, n, lane);
    dbg[MAXROWS * MAXROWS + lane] = W[0];
    dbg[MAXROWS * MAXROWS + 64 + lane] = W[1];
#endif
    /* the sweeps, specialised on whether slot 1 (rows 64..127) exists: with <= 64 rows the second u
     * register, its fma and its bookkeeping drop out of every row */
    auto passes = [&](auto span_tag) -> int {
        /* SPAN: the row positions the sweep code covers (32, 64 or 128); every chunk position of a section
         * costs one scalar test per sweep, so few-row solves (the resets' settling) get the short code */
        constexpr int SPAN = decltype(span_tag)::value;
        constexpr bool TWO = SPAN > 64;
        constexpr int NCH_NC = (NCMAX + CHUNK - 1) / CHUNK < SPAN / CHUNK ? (NCMAX + CHUNK - 1) / CHUNK : SPAN / CHUNK;
        int split = 0;
        PROF_T0(t_sw);
        /* pass 0: the velocity solve; pass 1: the split-impulse pass (normals only, from zero) */
    #pragma nounroll
        for (int pass = 0; pass < 2; pass++) {
            const int pen = pass;
            if (pen) {
                int anypen = 0;
    #pragma unroll
                for (int s = 0; s < 2; s++) {
                    const int p = lane + 64 * s;
                    anypen |= p >= nnc && p < fb && rhsPen[s] != 0.0;
                }
                split = ballot(anypen) != 0ull;
                if (!split) break;
    #pragma unroll
                for (int s = 0; s < 2; s++) {
                    L.rhs[s] = rhsPen[s];
                    L.imp[s] = 0.0;
                }
                W[0] = L.rhs[0];
                W[1] = L.rhs[1];
            }
    #pragma unroll
            for (int s = 0; s < 2; s++) {
                L.dlo[s] = L.lo[s] - L.imp[s];
                L.dhi[s] = L.hi[s] - L.imp[s];
            }
            for (int it = 0; it < UG_PGS_ITERS; it++) {
                bool bad = false;
                /* opaque per-sweep copies: keeps the per-chunk scalar tests inside the loop */
                int o_n = n, o_nnc = nnc, o_fb = fb;
                gcdouble* o_wsA = wsAr;
                asm volatile("" : "+s"(o_n), "+s"(o_nnc), "+s"(o_fb), "+s"(o_wsA));
                /* (even sweeps) non-contact rows reversed, then [s0, fb) */
                PROF_T0(t_s1);
                if (!pen && !(it & 1) && o_nnc > 0)
                    sweep_section<true, NCH_NC, TWO>(A0, A1, o_wsA, lane, 0, o_nnc, 0ull, 0ull, L, W);
                PROF_ADD(PF_SW_NC, t_s1);
                PROF_T0(t_s2);
                const int s0 = (pen || !(it & 1)) ? o_nnc : 0;
                if (s0 < o_fb) sweep_section<false, SPAN / CHUNK, TWO>(A0, A1, o_wsA, lane, s0, o_fb, 0ull, 0ull, L, W);
                PROF_ADD(PF_SW_CT, t_s2);
                PROF_T0(t_s3);
                const int f0 = pen ? o_nnc : 0;
                row_finish<TWO>(L, pos_mask(0, f0, o_fb, 0ull), pos_mask(1, f0, o_fb, 0ull), lane, bad);
                PROF_ADD(PF_SW_FIN, t_s3);
                /* friction and rolling rows: bounds +-mu * (their normal's impulse, final for this sweep),
                 * skipped while it is not positive.  A skipped row is made neutral (sweep_section):
                 * increment bounds [0, 0] give a delta of +-0, and u + a * (+-0) == u up to the sign of a
                 * zero u (which never reaches a non-zero result). */
                PROF_T0(t_s4);
                if (!pen && o_fb < o_n) {
                    g_sh.u.impx[lane] = L.imp[0];
                    g_sh.u.impx[64 + lane] = L.imp[1];
                    __builtin_amdgcn_wave_barrier();
                    unsigned long long sk[2] = {0ull, 0ull};
    #pragma unroll
                    for (int s = 0; s < (TWO ? 2 : 1); s++) {
                        const int p = lane + 64 * s;
                        const bool isf = p >= o_fb && p < o_n;
                        double tot = g_sh.u.impx[isf ? nrow[s] : 0];
                        const bool skip = isf && !(tot > 0.0);
                        L.lo[s] = isf ? -(fric[s] * tot) : L.lo[s];
                        L.hi[s] = isf ? fric[s] * tot : L.hi[s];
                        L.dlo[s] = L.lo[s] - L.imp[s];
                        L.dhi[s] = L.hi[s] - L.imp[s];
                        sk[s] = ballot(skip);
                    }
                    __builtin_amdgcn_wave_barrier();
                    PROF_ADD(PF_SW_FPREP, t_s4);
                    PROF_T0(t_s5);
                    sweep_section<false, SPAN / CHUNK, TWO>(A0, A1, o_wsA, lane, o_fb, o_n, sk[0], sk[1], L, W);
                    row_finish<TWO>(L, pos_mask(0, o_fb, o_n, sk[0]), pos_mask(1, o_fb, o_n, sk[1]), lane, bad);
                    PROF_ADD(PF_SW_FR, t_s5);
                }
                PROF_CNT(PC_ITERS, 1);
                PROF_T0(t_s6);
                if (ballot(bad) == 0ull || it >= UG_PGS_ITERS - 1) break;
                PROF_ADD(PF_SW_RES, t_s6);
            }
            if (!pen) {
                PROF_ADD(PF_SWEEPS, t_sw);
    #pragma unroll
                for (int s = 0; s < 2; s++)
                    if (lane + 64 * s < n) g_sh.rs[lane + 64 * s].imp = L.imp[s];
    #ifdef UG_DEBUG_DUMP
                dbg[MAXROWS * MAXROWS + 128 + lane] = W[0];
                dbg[MAXROWS * MAXROWS + 192 + lane] = W[1];
                dbg[MAXROWS * MAXROWS + 256 + lane] = L.imp[0];
                dbg[MAXROWS * MAXROWS + 320 + lane] = L.imp[1];
    #endif
            }
        }
        return split;
    };
    /* contact-free solve of the 7 motor + 5 gear rows (free-space motion: most of a reset's settling): the
     * sweeps as straight 12-row sequences, reversed on even sweeps, forward on odd ones -- the general
     * path's order without chunk tests or neutral rows; no normal rows, so no warm start and no split pass */
    auto passes_free12 = [&]() -> int {
        PROF_CNT(PF_FREE_PSETUP, __builtin_readcyclecounter() - t_setup);
        PROF_T0(t_sw);
#pragma unroll
        for (int s = 0; s < 2; s++) {
            L.dlo[s] = L.lo[s] - L.imp[s];
            L.dhi[s] = L.hi[s] - L.imp[s];
        }
        for (int it = 0; it < UG_PGS_ITERS; it++) {
            bool bad = false;
            gcdouble* o_wsA = wsAr;
            asm volatile("" : "+s"(o_wsA));
            /* 12 lane masks stay in SGPRs: the records by lane select (the fixed layout's 64 would spill) */
            if (!(it & 1)) straight_rows<11, -1, 12, false, true>(A0, A1, o_wsA, lane, L, W);
            else straight_rows<0, 1, 12, false, true>(A0, A1, o_wsA, lane, L, W);
            row_finish<false>(L, pos_mask(0, 0, 12, 0ull), 0ull, lane, bad);
            PROF_CNT(PC_ITERS, 1);
            if (ballot(bad) == 0ull || it >= UG_PGS_ITERS - 1) break;
        }
        PROF_ADD(PF_SWEEPS, t_sw);
        PROF_ADD(PF_FREE_PSWEEP, t_sw);
        if (lane < 12) g_sh.rs[lane].imp = L.imp[0];
        return 0;
    };
    /* the fixed layout's sweeps as straight row sequences (no chunk tests, no section copies): even sweeps the
     * non-contact rows reversed then the normal positions [12, 40), odd sweeps [0, 40) forward; then the friction
     * positions [40, 96).  Pads are neutral (zero bounds and column); only the section's own rows finish. */
    auto passes_fl = [&](auto shape) -> int {
        constexpr int NC = decltype(shape)::NC, F0 = decltype(shape)::F0, NF = decltype(shape)::NF;
        static_assert(F0 <= NF && F0 + NF - 64 <= 32, "slot 1 must fit a half-wave for the packing");
        const int nf = n - fb;
        int split = 0;
        PROF_T0(t_sw);
        /* slot 1 holds at most 32 rows (positions 64 .. F0 + NF - 1): the first part's slot-1 columns A1[k]
         * (k < F0) move into the upper half-wave of the friction columns' registers A1[F0 + k], halving the
         * slot-1 registers.  u of slot 1 then lives in two half-wave copies: the lower one is current during
         * the friction rows, the upper one (lanes 32..63 = rows 64..95) during the first part; each section
         * starts by copying the current one over the other (v_permlane32_swap), so every element still sees
         * the same fma chain in the same order. */
#pragma unroll
        for (int k = 0; k < F0; k++) {
            double x = A1[F0 + k], y = A1[k];
            swap32_d(x, y); /* x: lower half its own column, upper half column k's lower half */
            A1[F0 + k] = x;
        }
#pragma nounroll
        for (int pass = 0; pass < 2; pass++) {
            const int pen = pass;
            if (pen) {
                int anypen = 0;
#pragma unroll
                for (int s = 0; s < 2; s++) {
                    const int p = lane + 64 * s;
                    anypen |= p >= pm.nb && p < pm.nb + nn && rhsPen[s] != 0.0;
                }
                split = ballot(anypen) != 0ull;
                if (!split) break;
#pragma unroll
                for (int s = 0; s < 2; s++) {
                    L.rhs[s] = rhsPen[s];
                    L.imp[s] = 0.0;
                }
                W[0] = L.rhs[0];
                W[1] = L.rhs[1];
            }
#pragma unroll
            for (int s = 0; s < 2; s++) {
                L.dlo[s] = L.lo[s] - L.imp[s];
                L.dhi[s] = L.hi[s] - L.imp[s];
            }
            for (int it = 0; it < UG_PGS_ITERS; it++) {
                bool bad = false;
                {
                    double x = W[1], y = W[1];
                    swap32_d(x, y); /* upper copy := lower */
                    W[1] = x;
                }
                if (pen || !(it & 1)) {
                    if (!pen) straight_rows_fl<NC - 1, -1, NC, F0>(A0, A1, L, W);
                    straight_rows_fl<NC, 1, F0 - NC, F0>(A0, A1, L, W);
                } else {
                    straight_rows_fl<0, 1, F0, F0>(A0, A1, L, W);
                }
                {
                    double x = W[1], y = W[1];
                    swap32_d(x, y); /* lower copy := upper */
                    W[1] = y;
                }
                row_finish<false>(L, pos_mask(0, pen ? pm.nb : 0, pm.nb + nn, 0ull), 0ull, lane, bad);
                if (!pen && nf > 0) {
                    g_sh.u.impx[lane] = L.imp[0];
                    __builtin_amdgcn_wave_barrier();
                    unsigned long long sk[2];
#pragma unroll
                    for (int s = 0; s < 2; s++) {
                        const int p = lane + 64 * s;
                        const bool isf = p >= F0 && p < F0 + nf;
                        const double tot = g_sh.u.impx[isf ? pm.nb + (nrow[s] - nnc) : 0]; /* the normal's position */
                        const bool skip = isf && !(tot > 0.0);
                        L.lo[s] = isf ? -(fric[s] * tot) : L.lo[s];
                        L.hi[s] = isf ? fric[s] * tot : L.hi[s];
                        L.dlo[s] = skip ? 0.0 : L.lo[s] - L.imp[s];
                        L.dhi[s] = skip ? 0.0 : L.hi[s] - L.imp[s];
                        sk[s] = ballot(skip);
                    }
                    __builtin_amdgcn_wave_barrier();
                    straight_rows_fl<F0, 1, NF, 0>(A0, A1, L, W);
                    row_finish<true>(L, pos_mask(0, F0, F0 + nf, sk[0]), pos_mask(1, F0, F0 + nf, sk[1]),
                                     lane, bad);
                }
                PROF_CNT(PC_ITERS, 1);
                if (ballot(bad) == 0ull || it >= UG_PGS_ITERS - 1) break;
            }
            if (!pen) {
                PROF_ADD(PF_SWEEPS, t_sw);
#pragma unroll
                for (int s = 0; s < 2; s++) {
                    const int q = pm.q(lane + 64 * s);
                    if (q >= 0) g_sh.rs[q].imp = L.imp[s];
                }
            }
        }
        return split;
    };
    /* the single-slot fixed layouts (FS_*, FG12_*): even sweeps the non-contact positions reversed then the normal
     * positions, odd sweeps [0, F0) forward, then the friction positions -- the general path's row order with
     * neutral pads and no chunk tests; one u register (all positions < 64) */
    auto passes_fs = [&](auto shape) -> int {
        constexpr int NC = decltype(shape)::NC, F0 = decltype(shape)::F0, NF = decltype(shape)::NF;
        static_assert(F0 + NF <= 64, "a single-slot layout");
        const int nf = n - fb;
        int split = 0;
        PROF_T0(t_sw);
#pragma nounroll
        for (int pass = 0; pass < 2; pass++) {
            const int pen = pass;
            if (pen) {
                const int anypen = lane >= NC && lane < F0 && rhsPen[0] != 0.0;
                split = ballot(anypen) != 0ull;
                if (!split) break;
#pragma unroll
                for (int s = 0; s < 2; s++) {
                    L.rhs[s] = rhsPen[s];
                    L.imp[s] = 0.0;
                }
                W[0] = L.rhs[0];
                W[1] = L.rhs[1];
            }
#pragma unroll
            for (int s = 0; s < 2; s++) {
                L.dlo[s] = L.lo[s] - L.imp[s];
                L.dhi[s] = L.hi[s] - L.imp[s];
            }
            for (int it = 0; it < UG_PGS_ITERS; it++) {
                bool bad = false;
                gcdouble* o_wsA = wsAr;
                asm volatile("" : "+s"(o_wsA));
                if (pen || !(it & 1)) {
                    if (!pen) straight_rows<NC - 1, -1, NC>(A0, A1, o_wsA, lane, L, W);
                    straight_rows<NC, 1, F0 - NC>(A0, A1, o_wsA, lane, L, W);
                } else {
                    straight_rows<0, 1, F0>(A0, A1, o_wsA, lane, L, W);
                }
                row_finish<false>(L, pos_mask(0, pen ? NC : 0, F0, 0ull), 0ull, lane, bad);
                if (!pen && nf > 0) {
                    g_sh.u.impx[lane] = L.imp[0];
                    __builtin_amdgcn_wave_barrier();
                    const bool isf = lane >= F0 && lane < F0 + nf;
                    /* the friction row's normal: row nrow sits at position NC + (nrow - nnc) */
                    const double tot = g_sh.u.impx[isf ? NC + (nrow[0] - nnc) : 0];
                    const bool skip = isf && !(tot > 0.0);
                    L.lo[0] = isf ? -(fric[0] * tot) : L.lo[0];
                    L.hi[0] = isf ? fric[0] * tot : L.hi[0];
                    L.dlo[0] = skip ? 0.0 : L.lo[0] - L.imp[0];
                    L.dhi[0] = skip ? 0.0 : L.hi[0] - L.imp[0];
                    const unsigned long long sk = ballot(skip);
                    __builtin_amdgcn_wave_barrier();
                    straight_rows<F0, 1, NF>(A0, A1, o_wsA, lane, L, W);
                    row_finish<false>(L, pos_mask(0, F0, F0 + nf, sk), 0ull, lane, bad);
                }
                PROF_CNT(PC_ITERS, 1);
                if (ballot(bad) == 0ull || it >= UG_PGS_ITERS - 1) break;
            }
            if (!pen) {
                PROF_ADD(PF_SWEEPS, t_sw);
                const int q = pm.q(lane);
                if (q >= 0) g_sh.rs[q].imp = L.imp[0];
            }
        }
        return split;
    };
    PROF_T0(t_post);
    const int split = pm.fl == FSB_F0 && pm.nb == FSB_NC ? passes_fs(FLShape<FSB_NC, FSB_F0, FSB_NF>{})
                      : pm.fl == FS14G_F0       ? passes_fs(FLShape<FS14_NC, FS14G_F0, FS14G_NF>{})
                      : pm.fl == FS14P_F0     ? passes_fs(FLShape<FS14_NC, FS14P_F0, FS14P_NF>{})
                      : pm.fl == FS14W_F0     ? passes_fs(FLShape<FS14_NC, FS14W_F0, FS14W_NF>{})
                      : pm.fl == FS14H_F0     ? passes_fs(FLShape<FS14_NC, FS14H_F0, FS14H_NF>{})
                      : pm.fl == FS6_F0       ? passes_fs(FLShape<FS_NC, FS6_F0, FS6_NF>{})
                      : pm.fl == FS_F0        ? passes_fs(FLShape<FS_NC, FS_F0, FS_NF>{})
                      : pm.fl == FG12_F0      ? passes_fs(FLShape<FG12_NC, FG12_F0, FG12_NF>{})
                      : pm.fl == FG18_F0 && pm.nb == FG18_NC ? passes_fl(FLShape<FG18_NC, FG18_F0, FG18_NF>{})
                      : pm.fl == FG_F0        ? passes_fl(FLShape<FG_NC, FG_F0, FG_NF>{})
                      : pm.fl == FL_F020      ? passes_fl(FLShape<FL_NNC, FL_F020, 2 * (FL_F020 - FL_NNC)>{})
                      : pm.fl == FL_F022      ? passes_fl(FLShape<FL_NNC, FL_F022, 2 * (FL_F022 - FL_NNC)>{})
                      : pm.fl == FL_F0S       ? passes_fl(FLShape<FL_NNC, FL_F0S, FL_NFS>{})
                      : pm.fl                 ? passes_fl(FLShape<FL_NNC, FL_F0, FL_NF>{})
                      : (n == 12 && nnc == 12) ? passes_free12()
                      : n > 96             ? passes(std::integral_constant<int, 128>{})
                      : n > 64             ? passes(std::integral_constant<int, 96>{})
                      : n > 32             ? passes(std::integral_constant<int, 64>{})
                                           : passes(std::integral_constant<int, 32>{});
    /* dv[d] (dvs[d]) = fma chain over positions k of M^-1J_k[d] * impulse_k (lane d < NV) */
    __builtin_amdgcn_wave_barrier();
    if (split) { /* the split impulses by row (the accumulation below reads rows [nnc, fb)) */
        const int q0 = pm.q(lane), q1 = pm.q(64 + lane);
        if (q0 >= 0) sh.u.impx[q0] = L.imp[0];
        if (q1 >= 0) sh.u.impx[q1] = L.imp[1];
    }
    __builtin_amdgcn_wave_barrier();
    const int d = lane < NV ? lane : 0;
    double acc = 0.0, accs = 0.0;
    if (direct) { /* the 12 rows' M^-1 J^T at dof slot d from the unit solves, every LDS read up front */
        double m[12], im[12];
#pragma unroll
        for (int k = 0; k < 12; k++) {
            const int kk = __builtin_amdgcn_readfirstlane(sh.rs[k].kind), ka = __builtin_amdgcn_readfirstlane(sh.rs[k].a);
            const bool g = kk == 2;
            const int r1 = g ? UG_FINGER_DOF : (ka < 6 ? ka : UG_FINGER_DOF), r2 = g ? NB + ka : r1;
            const int dd = lane < NB ? lane : 0;
            const double x1 = sh.u.mcol[r1][dd], x2 = sh.u.mcol[r2][dd];
            m[k] = lane < NB ? (g ? x1 + x2 : x1) : 0.0;
            im[k] = sh.rs[k].imp;
        }
#pragma unroll
        for (int k = 0; k < 12; k++) acc = __builtin_fma(m[k], im[k], acc);
    } else {
        for (int k = 0; k < n; k++) acc = __builtin_fma(rows[k * RS + RJ + d], sh.rs[k].imp, acc);
    }
    if (split)
        for (int k = nnc; k < fb; k++) accs = __builtin_fma(rows[k * RS + RJ + d], sh.u.impx[k], accs);
    dv = lane < NV ? acc : 0.0;
    dvs = lane < NV ? accs : 0.0;
    __builtin_amdgcn_wave_barrier();
    if (direct) PROF_ADD(PF_FREE_PPOST, t_post);
    PROF_EXIT();
    return split;
}

/* The collision stage of a substep with nothing to find (the contact-free stretches of a reset, the arm moving in
 * free space): after a full pass that kept no manifold, certified every overlapping pair and saw no free object, each
 * pair's slack -- how far its colliders may still close before GJK could keep a point (its certificate's margin
 * beyond the contact threshold) or before its padded AABBs overlap (their gap) -- is in the workspace with the robot's
 * q.  While every pair's colliders have moved less than that since (a robot collider's points by at most
 * sum_j |q_j - q_ref_j| Scene::qsw[c][j], static ones not at all) and no glue ran (team_run clears the reference),
 * the full pass would find exactly that again: no pair overlaps that did not, every certificate still holds, no
 * manifold, nothing stored.  So it is skipped -- the same state, the same result bit for bit. */
__device__ static bool quiescent_ok(const Scene* s, const double* ws) {
    Shared& sh = g_sh;
    const int lane = threadIdx.x;
    const gcdouble* qs = (const gcdouble*)(ws + WS_QS);
    if (lane < s->ncol) {
        double D = 0.0;
        for (int j = 0; j < NB; j++) D += ug_fabs(sh.e.q[j] - qs[MAXPAIR + j]) * s->qsw[lane][j];
        sh.lo[lane].x = D; /* the collision stage's AABB scratch, unused until it runs */
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    bool bad = false;
    for (int p = lane; p < s->npair; p += TEAM) {
        const PairDef& P = s->pair[p];
        bad = bad || !((sh.lo[P.a].x + sh.lo[P.b].x) * (1.0 + 1e-12) + 1e-12 < qs[p]); /* NaN: not quiet */
    }
    __builtin_amdgcn_wave_barrier();
    return ballot(bad) == 0ull;
}

