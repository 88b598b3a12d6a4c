/* ug_team_pgs.h -- part of ug_team.h: PGS row-update primitives and the Delassus rows on the matrix cores.
 * Included by ug_team.h inside namespace ugd, in this order (the kernel is one translation unit); not self-contained. */
/* ---------------- PGS (btMultiBodyConstraintSolver), row space ----------------
 * The solver keeps u = rhs - (J dv) / D (each row's unclamped increment, one entry per row) instead of
 * dv: lane l owns the rows at positions l and l + 64 (slot 0 / slot 1) -- their scalars, their impulse and
 * their u -- and holds its rows of the scaled Delassus matrix NB = -diag(1/D) J M^-1 J^T in VGPRs
 * (A0[P] / A1[P] = NB[l][P], NB[l+64][P]).  Updating row P is lane-parallel arithmetic on every lane's
 * own row (only lane P's result is used), one broadcast of the impulse change (two v_readlane) and one
 * fma per slot: u += NB[:, P] * delta.  No cross-lane reduction and no LDS traffic inside a sweep.  The
 * owner lane records the increment; its impulse and residual are advanced after the section.  Row
 * positions are template parameters, so A0[P] / A1[P] are compile-time register names and every
 * row-range test is a scalar branch (one per CHUNK rows).  Columns P >= PREG come from the global workspace.  Arithmetic
 * order is the oracle's pgs() (oracle/ug_oracle.c). */
#define NCMAX (2 * NB + 12) /* limits (both sides) + 7 motors + 5 gears */
#define CHUNK 8             /* rows per branch-free sweep chunk (one scalar test per chunk; 4 measured slower) */
struct Lrow { /* the two rows this lane owns (slot s: position lane + 64 s) */
    double rhs[2], invD[2], rinv[2], lo[2], hi[2], imp[2];
    double dlo[2], dhi[2]; /* lo - imp, hi - imp */
    double dsv[2];         /* the increment applied when the row was solved in this section */
};

/* branch-free select on the bit patterns (keeps the clamp out of control flow) */
__device__ __forceinline__ double bsel(bool c, double a, double b) {
    unsigned long long m = 0ull - (unsigned long long)c;
    unsigned long long r = (__double_as_longlong(a) & m) | (__double_as_longlong(b) & ~m);
    return __longlong_as_double(r);
}
template <int P>
__device__ __forceinline__ void colA(const double (&A0)[PREG], const double (&A1)[PREG], gcdouble* wsA, int lane,
                                     double& a0, double& a1) {
    if constexpr (P < PREG) {
        a0 = A0[P];
        a1 = A1[P];
    } else {
        a0 = wsA[(P - PREG) * MAXROWS + lane];
        a1 = wsA[(P - PREG) * MAXROWS + 64 + lane];
    }
}
/* lane L of the result := x (uniform), other lanes keep old: two v_writelane_b32 */
template <int L>
__device__ __forceinline__ double writelane_d(double old, double x) {
    int lo = __double2loint(old), hi = __double2hiint(old);
    const int xl = __builtin_amdgcn_readfirstlane(__double2loint(x)), xh = __builtin_amdgcn_readfirstlane(__double2hiint(x));
    asm("v_writelane_b32 %0, %1, %2" : "+v"(lo) : "s"(xl), "i"(L));
    asm("v_writelane_b32 %0, %1, %2" : "+v"(hi) : "s"(xh), "i"(L));
    return __hiloint2double(hi, lo);
}
/* resolveSingleConstraintRowGeneric [ext] (oracle solve_row_w) for the row at position P: every lane
 * forms the clamped increment of its own row, lane (P & 63)'s is broadcast, applied to w and recorded in
 * that lane (the impulse itself is advanced after the section).  W holds each row's unclamped increment
 * u = rhs - (J dv) / D and A0 / A1 the negated, 1/D-scaled Delassus rows.  Chain: max, min, readlane, fma. */
/* lane L of the result := x (that lane's own value), other lanes keep old: a row's record by a select on a
 * constant lane mask (inverse ballot), since lane L's own clamped value is the broadcast one -- cheaper than
 * v_writelane of the broadcast value where the masks stay in SGPRs (tools/micro/pgs3.hip) */
template <int L>
__device__ __forceinline__ double own_lane_sel(double old, double x) {
    return __builtin_amdgcn_inverse_ballot_w64(1ull << L) ? x : old;
}
/* w + a * (lane O's x) with the broadcast folded into the fma: DP-ALU DPP row_newbcast (gfx90a+) hands every
 * 16-lane row the value of its own lane O, so it serves rows held in lanes 0..15 (the contact-free 12-row
 * solve) and takes the two v_readlane and the SGPR hop off the row chain.  s_nop 1: the two wait states a DPP
 * read of a VGPR the previous VALU op wrote needs. */
template <int O>
__device__ __forceinline__ double clamp_fma_bcast16(double a, double dlo, double dhi, double& w) {
    static_assert(O >= 0 && O < 16, "row_newbcast reaches the lanes of one 16-lane row");
    double dn;
    /* the clamp in the same block: v_max_f64 / v_min_f64 are what fmax / fmin compile to, and an fmax of an
     * asm result would cost a canonicalising v_max first */
    asm("v_max_f64 %0, %1, %2\n\t"
        "v_min_f64 %0, %0, %3\n\t"
        "s_nop 1\n\t"
        "v_fmac_f64_dpp %1, %0, %4 row_newbcast:%5 row_mask:0xf bank_mask:0xf"
        : "=&v"(dn), "+v"(w)
        : "v"(dlo), "v"(dhi), "v"(a), "i"(O));
    return dn;
}
template <int P, bool TWO, bool SEL = false>
__device__ __forceinline__ void row_upd(const double (&A0)[PREG], const double (&A1)[PREG], gcdouble* wsA, int lane,
                                        Lrow& L, double (&W)[2]) {
    constexpr int s = P >> 6, O = P & 63;
    double a0, a1;
    colA<P>(A0, A1, wsA, lane, a0, a1);
    if constexpr (SEL) { /* rows in lanes 0..15, one slot: broadcast inside the fma, record by lane select */
        static_assert(!TWO && P < 16, "the DPP row update serves one slot of at most 16 rows");
        const double dn = clamp_fma_bcast16<O>(a0, L.dlo[0], L.dhi[0], W[0]);
        L.dsv[s] = own_lane_sel<O>(L.dsv[s], dn);
    } else {
        double dn = __builtin_fmin(__builtin_fmax(W[s], L.dlo[s]), L.dhi[s]);
        double d = readlane_d(dn, O);
        W[0] = __builtin_fma(a0, d, W[0]);
        if (TWO) W[1] = __builtin_fma(a1, d, W[1]); /* slot 1 exists only with more than 64 rows */
        L.dsv[s] = writelane_d<O>(L.dsv[s], d);
    }
}
/* the fixed layout's row update: the slot-1 column of row P is read from A1[P + OFS] (passes_fl packs the
 * first part's slot-1 columns into the upper half-wave of the friction columns' registers) */
template <int P, int OFS>
__device__ __forceinline__ void row_upd_fl(const double (&A0)[PREG], const double (&A1)[PREG], Lrow& L,
                                           double (&W)[2]) {
    constexpr int s = P >> 6, O = P & 63;
    const double a0 = A0[P], a1 = A1[P + OFS];
    double dn = __builtin_fmin(__builtin_fmax(W[s], L.dlo[s]), L.dhi[s]);
    double d = readlane_d(dn, O);
    W[0] = __builtin_fma(a0, d, W[0]);
    W[1] = __builtin_fma(a1, d, W[1]);
    L.dsv[s] = writelane_d<O>(L.dsv[s], d);
}
template <int P, int STEP, int K, int OFS>
__device__ __forceinline__ void straight_rows_fl(const double (&A0)[PREG], const double (&A1)[PREG], Lrow& L,
                                                 double (&W)[2]) {
    if constexpr (K > 0) {
        row_upd_fl<P, OFS>(A0, A1, L, W);
        straight_rows_fl<P + STEP, STEP, K - 1, OFS>(A0, A1, L, W);
    }
}
/* after a section: the lanes whose row was solved advance their impulse by the recorded increment and
 * flag a (delta / D)^2 above the residual threshold.  The sweep's convergence test (the largest (delta / D)^2
 * of the sweep <= threshold, oracle pgs()) is then "no row flagged": the same decision as folding a running
 * max and comparing it (NaN included: a NaN square is flagged, as a NaN max fails the test), without the
 * max / select chain in front of the wave-wide test. */
template <bool TWO>
__device__ __forceinline__ void row_finish(Lrow& L, unsigned long long m0, unsigned long long m1, int lane,
                                           bool& bad) {
#pragma unroll
    for (int s = 0; s < (TWO ? 2 : 1); s++) {
        const bool did = (((s ? m1 : m0) >> lane) & 1ull) != 0ull;
        const double dn = L.dsv[s];
        double x = dn * L.rinv[s];
        x = x * x;
        bad = bad | (did & !(x <= UG_RESIDUAL_THR));
        L.imp[s] = did ? L.imp[s] + dn : L.imp[s];
        L.dlo[s] = L.lo[s] - L.imp[s];
        L.dhi[s] = L.hi[s] - L.imp[s];
    }
}
/* lanes whose slot-s row position lies in [a, b), minus skip */
__device__ __forceinline__ unsigned long long pos_mask(int s, int a, int b, unsigned long long skip) {
    const int lo = a - 64 * s, hi = b - 64 * s; /* lane range */
    const int l0 = lo < 0 ? 0 : (lo > 64 ? 64 : lo), l1 = hi < 0 ? 0 : (hi > 64 ? 64 : hi);
    if (l1 <= l0) return 0ull;
    unsigned long long m = (l1 - l0 == 64) ? ~0ull : (((1ull << (l1 - l0)) - 1ull) << l0);
    return m & ~skip;
}
/* one CHUNK-row chunk, rows in increasing (REV: decreasing) position, no per-row tests */
template <int C, bool REV, int K, bool TWO>
__device__ __forceinline__ void chunk_rows(const double (&A0)[PREG], const double (&A1)[PREG], gcdouble* wsA, int lane,
                                           Lrow& L, double (&W)[2]) {
    if constexpr (K < CHUNK) {
        row_upd<REV ? CHUNK * C + CHUNK - 1 - K : CHUNK * C + K, TWO>(A0, A1, wsA, lane, L, W);
        chunk_rows<C, REV, K + 1, TWO>(A0, A1, wsA, lane, L, W);
    }
}
/* the chunks [c_lo, c_hi] of a section, in increasing (REV: decreasing) order.  Rows of those chunks
 * outside the section are neutral: the caller zeroes their increment bounds, so they broadcast +-0 and
 * leave u unchanged.  One scalar test per chunk instead of per row. */
template <int I, bool REV, int NCH, bool TWO>
__device__ __forceinline__ void sweep_chunks(const double (&A0)[PREG], const double (&A1)[PREG], gcdouble* wsA,
                                             int lane, int c_lo, int c_hi, Lrow& L, double (&W)[2]) {
    if constexpr (I < NCH) {
        constexpr int C = REV ? NCH - 1 - I : I;
        if (__builtin_expect(C >= c_lo && C <= c_hi, 1)) { /* likely: the chunk body stays on the fall-through path */
            chunk_rows<C, REV, 0, TWO>(A0, A1, wsA, lane, L, W);
            PROF_CNT(PC_CHUNKS, 1);
        }
        sweep_chunks<I + 1, REV, NCH, TWO>(A0, A1, wsA, lane, c_lo, c_hi, L, W);
    }
}
/* the section [a, b) (a < b): a copy of the lane rows with zero increment bounds outside it (and on the
 * rows set in skip), swept chunk-wise; the recorded increments come back in L.dsv */
template <bool REV, int NCH, bool TWO>
__device__ __forceinline__ void sweep_section(const double (&A0)[PREG], const double (&A1)[PREG], gcdouble* wsA,
                                              int lane, int a, int b, unsigned long long sk0, unsigned long long sk1,
                                              Lrow& L, double (&W)[2]) {
    Lrow F = L;
    bool in[2] = {false, false};
#pragma unroll
    for (int s = 0; s < (TWO ? 2 : 1); s++) {
        const int p = lane + 64 * s;
        const bool skip = (((s ? sk1 : sk0) >> lane) & 1ull) != 0ull;
        in[s] = p >= a && p < b && !skip;
        F.dlo[s] = in[s] ? L.dlo[s] : 0.0;
        F.dhi[s] = in[s] ? L.dhi[s] : 0.0;
    }
    sweep_chunks<0, REV, NCH, TWO>(A0, A1, wsA, lane, a / CHUNK, (b - 1) / CHUNK, F, W);
    /* only the section's own records: a neutral row's record would clobber one still to be finished */
#pragma unroll
    for (int s = 0; s < (TWO ? 2 : 1); s++) L.dsv[s] = in[s] ? F.dsv[s] : L.dsv[s];
}
/* rows P0, P0 + STEP, ... (NR of them) straight, no chunk tests and no neutral rows (the contact-free solve) */
template <int P, int STEP, int K, bool TWO = false, bool SEL = false>
__device__ __forceinline__ void straight_rows(const double (&A0)[PREG], const double (&A1)[PREG], gcdouble* wsA,
                                              int lane, Lrow& L, double (&W)[2]) {
    if constexpr (K > 0) {
        row_upd<P, TWO, SEL>(A0, A1, wsA, lane, L, W);
        straight_rows<P + STEP, STEP, K - 1, TWO, SEL>(A0, A1, wsA, lane, L, W);
    }
}
/* warm start: normal rows [nnc, fb) with a carried impulse, w += A[:, P] * impulse */
template <int P>
__device__ __forceinline__ void sweep_warm(const double (&A0)[PREG], const double (&A1)[PREG], gcdouble* wsA,
                                           int lane, int nnc, int fb, const Lrow& L, double (&W)[2]) {
    if constexpr (P < MAXROWS) {
        if (P < fb) {
            if (P >= nnc) {
                double imp = readlane_d(L.imp[P >> 6], P & 63);
                if (imp != 0.0) {
                    double a0, a1;
                    colA<P>(A0, A1, wsA, lane, a0, a1);
                    W[0] = __builtin_fma(a0, imp, W[0]);
                    W[1] = __builtin_fma(a1, imp, W[1]);
                }
            }
            sweep_warm<P + 1>(A0, A1, wsA, lane, nnc, fb, L, W);
        }
    }
}
/* ---- Delassus rows on the matrix cores ----
 * A[i][p] = fma chain over the 32 (padded) dof slots of J_i[d] * M^-1J_p[d] is a 32-deep dot product, so a
 * 16x16 tile of A is KS = 8 chained v_mfma_f64_16x16x4_f64: their numerics are a k-ordered fma chain, bit-identical
 * to the oracle's rdot() (checked on MI355X: tools/micro/mfma64.hip, mfma_build.hip).  For the column
 * block PB (columns p = 16 PB + 0..15) the four row tiles of slot S are computed with the columns on the
 * A operand, so tile g leaves A[64 S + 16 g + m][16 PB + h + 4 r] in lane 16 h + m, register r; a 4x4
 * transpose of (tile, lane row) with permlane32_swap / permlane16_swap then hands lane l its own row:
 * A[64 S + l][16 PB + h + 4 r] in W[h][r].  Rows and columns beyond n are zero. */
typedef double d4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void swap32_d(double& x, double& y) {
    auto l = __builtin_amdgcn_permlane32_swap((unsigned)__double2loint(x), (unsigned)__double2loint(y), false, false);
    auto h = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(x), (unsigned)__double2hiint(y), false, false);
    x = __hiloint2double(h[0], l[0]);
    y = __hiloint2double(h[1], l[1]);
}
__device__ __forceinline__ void swap16_d(double& x, double& y) {
    auto l = __builtin_amdgcn_permlane16_swap((unsigned)__double2loint(x), (unsigned)__double2loint(y), false, false);
    auto h = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(x), (unsigned)__double2hiint(y), false, false);
    x = __hiloint2double(h[0], l[0]);
    y = __hiloint2double(h[1], l[1]);
}
/* solve position -> row index.  The general layout is the identity over [0, n).  The fixed layout (team_pgs
 * passes_fl) keeps the non-contact and normal rows at [0, fb) and moves the friction rows to [f0, f0 + n - fb),
 * so that every section starts at a compile-time position; the positions in between are pads (-1: zero J, zero
 * bounds, so a zero column and a neutral row). */
#define FL_NNC 12 /* non-contact rows of the fixed layout (7 motors + 5 gears) */
#define FL_F0 40  /* first friction position: normals at [12, 40) (at most 28) */
#define FL_NF 56  /* friction positions [40, 96): at most 56 rows */
#define FL_F0S 36 /* the short variant (at most 24 normals): friction at [36, 84) */
#define FL_NFS 48
/* narrower variants for BallBalance's common solves (tools/row_hist.py: 19-25 normals, 2 friction rows each; 71 % with
 * at most 20 normals, 81 % with at most 22): friction at [32, 72) and at [34, 78) -- each pad position costs a row
 * update in every sweep */
#define FL_F020 32
#define FL_F022 34
/* the single-slot fixed layout (CubesPush / CubesGrasp contact solves, BallBalance's early reset contacts): at
 * most FS_NC non-contact rows (motors, gears, violated limits) at [0, nnc), pads to FS_NC, at most
 * FS_F0 - FS_NC normals, pads to FS_F0, at most FS_NF friction rows; 50 positions, all in slot 0 */
#define FS_NC 20
#define FS_F0 30
#define FS_NF 20
/* its narrow variant for CubesGrasp's common solves (12-18 non-contact rows, 4-6 normals, 2 friction rows each):
 * normals from 20, friction from 26, 38 positions */
#define FS6_F0 26
#define FS6_NF 12
/* narrower single-slot layouts for at most 14 non-contact rows (tools/row_hist.py, round 6): CubesPush's common solves
 * (12-13 non-contact rows, 8 normals, 16 friction rows: 86 % of its step solves) at 38 positions instead of FS's 50
 * (normals from 14, friction from 22), its 9-10-normal solves at 44, and CubesGrasp's (12-14 non-contact rows, 4-6
 * normals) at 32 instead of FS6's 38 (normals from 14, friction from 20) -- every pad position costs a row update
 * in each of the 50 sweeps */
#define FS14_NC 14
#define FS14G_F0 20
#define FS14G_NF 12
#define FS14P_F0 22
#define FS14P_NF 16
#define FS14W_F0 24
#define FS14W_NF 20
/* and Golf's 11-15-normal solves (12-13 non-contact rows, friction + rolling rows 2 nn + 2): single-slot at 61 positions
 * (normals from 14, friction + rolling from 29) instead of FG12's 64 (<= 12 normals) or FG18's two-slot 74 */
#define FS14H_F0 29
#define FS14H_NF 32
/* solves with one or two normals and up to 22 non-contact rows (Box-v0's: 15-21 non-contact rows -- the box's joint
 * limits and button motor beside the arm's 12 -- and one normal, 91 % of its step solves; BallBalance's first reset
 * contacts): 28 positions (normals from 22, friction from 24) instead of the general path's chunked 32-span */
#define FSB_NC 22
#define FSB_F0 24
#define FSB_NF 4
/* the two-slot layout for Golf's contact solves (13 non-contact rows with the club's limit row, up to 28
 * normals, friction + rolling rows up to 52): non-contact rows at [0, nnc), pads to 16, normals from 16,
 * friction from 44, 96 positions */
#define FG_NC 16
#define FG_F0 44
#define FG_NF 52
/* Golf's narrower solves (tools/row_hist.py UG_TASK=3: 12-13 non-contact rows, 4-17 normals, 2 friction rows per
 * normal + 2 rolling rows, all 50 sweeps): a single-slot layout for up to 12 normals (friction + rolling from 28,
 * 64 positions) and a two-slot one for up to 18 (friction + rolling from 34, 74 positions), so a solve's pads stay
 * a fraction of its rows instead of filling FG's 96 positions or taking the chunked general path */
#define FG12_NC 16
#define FG12_F0 28
#define FG12_NF 36
#define FG18_NC 16
#define FG18_F0 34
#define FG18_NF 40
template <int NC_, int F0_, int NF_>
struct FLShape {
    static constexpr int NC = NC_, F0 = F0_, NF = NF_;
};
struct PosMap {
    int n, fb, fl; /* fl: the fixed layout's first friction position (FL_F0, FL_F0S or FS_F0), 0 for the identity */
    int nc, nb;    /* the fixed layouts: non-contact rows [0, nc) at positions [0, nc), normals from position nb */
    int np;        /* positions the sweeps cover */
    __device__ __forceinline__ int q(int p) const {
        if (!fl) return p < n ? p : -1;
        if (p < nb) return p < nc ? p : -1;
        if (p < fl) {
            const int r = nc + (p - nb);
            return r < fb ? r : -1;
        }
        const int r = fb + (p - fl);
        return r < n ? r : -1;
    }
    /* positions the Delassus build covers: the fixed layouts' straight sweeps read every column they span,
     * so all of them are built (pad columns zero) */
    __device__ __forceinline__ int npos() const { return fl ? np : n; }
};
/* the slot's row operands (J of rows 64 S + 16 g + (lane & 15), dof slots 4 ks + (lane >> 4)) are the same
 * for every column block: loaded once per slot into B; each block then loads only its 6 column operands */
template <int PB, int K>
__device__ __forceinline__ void mfma_cols(gcdouble* rows, const PosMap& pm, int lane, double (&a)[KS]) {
    const int q = pm.q(16 * PB + (lane & 15));
#pragma unroll
    for (int ks = 0; ks < K; ks++) a[ks] = q >= 0 ? rows[q * RS + RJ + 4 * ks + (lane >> 4)] : 0.0;
}
template <int PB, int S, int K, int G>
__device__ __forceinline__ void mfma_block(gcdouble* rows, const double (&B)[KS][4], const double (&a)[KS], double invDr,
                                           double (&A)[PREG], gdouble* wsA, const PosMap& pm, int n, int lane) {
    if constexpr (16 * PB < MAXROWS) {
        if (16 * PB < n) {
            double an[KS]; /* the next block's column operands, in flight during this block */
            if (16 * PB + 16 < n) mfma_cols<PB + 1, K>(rows, pm, lane, an);
            d4v acc[4];
#pragma unroll
            for (int g = 0; g < 4; g++) acc[g] = d4v{0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int ks = 0; ks < K; ks++)
#pragma unroll
                for (int g = 0; g < G; g++) acc[g] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ks], B[ks][g], acc[g], 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 4; r++) {
                double v[4] = {acc[0][r], acc[1][r], acc[2][r], acc[3][r]};
                swap32_d(v[0], v[2]);
                swap32_d(v[1], v[3]);
                swap16_d(v[0], v[1]);
                swap16_d(v[2], v[3]);
#pragma unroll
                for (int h = 0; h < 4; h++) {
                    constexpr int base = 16 * PB;
                    double x = -(v[h] * invDr);      /* NB = -(A / D) of this lane's row */
                    asm volatile("" : "+v"(x));      /* materialise here (no sinking into the sweeps) */
                    const int P = base + h + 4 * r;  /* compile-time after unrolling */
                    if (P < PREG) A[P < PREG ? P : 0] = x;
                    else wsA[(P - PREG) * MAXROWS + 64 * S + lane] = x;
                }
            }
            mfma_block<PB + 1, S, K, G>(rows, B, an, invDr, A, wsA, pm, n, lane);
        }
    }
}
/* K: the k-steps that can hold a non-zero (4 K >= NB + 6 nobj; the dof slots beyond are zero in every row,
 * and a chain of exact zero terms on an accumulator that is never -0 changes nothing) */
/* G: the row tiles of the slot that can hold a row (the fixed layout's slot 1 has at most 32 rows: tiles 2
 * and 3 are pads, their accumulators stay zero) */
template <int S, int K, int G = 4>
__device__ __forceinline__ void mfma_slot(gcdouble* rows, double invDr, double (&A)[PREG], gdouble* wsA,
                                          const PosMap& pm, int lane) {
    const int n = pm.npos();
    double B[KS][4];
#pragma unroll
    for (int ks = 0; ks < K; ks++)
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int q = pm.q(64 * S + 16 * g + (lane & 15));
            B[ks][g] = q >= 0 ? rows[q * RS + 4 * ks + (lane >> 4)] : 0.0;
        }
    double a[KS];
    mfma_cols<0, K>(rows, pm, lane, a);
    mfma_block<0, S, K, G>(rows, B, a, invDr, A, wsA, pm, n, lane);
}
__device__ __forceinline__ int uniform(int x) { return __builtin_amdgcn_readfirstlane(x); }
template <typename T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
    unsigned long long u = (unsigned long long)p;
    unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u), hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
    return (T*)(((unsigned long long)hi << 32) | lo);
}

