/* ug_team.h -- one wavefront per environment ("team") implementation of the hot path.
 *
 * Why: the env-step is a long sequential chain (<=480 substeps, each a projected
 * Gauss-Seidel over ~90 constraint rows x 50 iterations).  One env per lane left
 * the PGS rows (48 doubles each) streaming through scratch and used 64 of the
 * chip's 1024 SIMDs at 4096 envs.  Here a 64-lane wavefront owns one env:
 *
 *  - the env state (canonical layout, ug_layout.h) lives in LDS for the whole launch;
 *  - collision: lane per collider (transforms, AABBs), lane per pair (broadphase,
 *    box/sphere narrowphase, manifold update), the whole wave per hull-box pair
 *    (lane per hull vertex, 8 lanes per box corner over the hull's face planes,
 *    wave-wide arg-min/arg-max for the 4-point reduction);
 *  - constraint rows: lane per row (Jacobian, M^-1 J^T, rhs), staged through LDS;
 *  - PGS: row p lives in the VGPRs of half (p & 1) of the wave (lane d holds
 *    J[d], M^-1J[d] of that row, d = dof slot 0..31), the velocity delta is
 *    replicated in both halves; a row update is a 16-lane DPP tree reduction,
 *    two readlanes, the clamp, and a permlane32 broadcast of M^-1J * delta;
 *  - the remaining sequential pieces (FK, CRBA/RNEA/LDL^T, IK, integration,
 *    task glue) run on lane 0 with their data in LDS.
 * Arithmetic order is that of oracle/ug_oracle.c (the pairwise tree of the DPP
 * reduction included), so results stay bit-identical to the CPU restatement.
 */
#ifndef UG_TEAM_H
#define UG_TEAM_H

#include <type_traits>
#include <utility>

#include "ug_device.h"
#include "prio_model.h"
#include "prio_model_tb.h"
#include "prio_model_cp.h"
#include "prio_model_cg.h"
#include "prio_model_gf.h"
#include "prio_model_tbt.h"
#include "prio_model_gj.h"
#include "prio_model_cgt.h"
#include "ug_glue.h"

namespace ugd {

#define TEAM 64
typedef __attribute__((address_space(1))) const double gcdouble;
typedef __attribute__((address_space(1))) double gdouble;
#define UG_NPROF 134 /* phase accumulators of the -DUG_PROF build */
#define NVP 32
#define PREG 96             /* Delassus columns held in VGPRs; columns beyond stream from the global workspace */
/* a row's J and M^-1 J^T over the NVP = 32 dof slots (robot 12, objects 3 x 6, 2 zero pads) */
#define RJ NVP              /* offset of M^-1 J^T in a workspace row */
#define RS (2 * NVP)        /* workspace row stride (doubles) */
#define KS (NVP / 4)        /* k-steps of the 16x16x4 MFMA Delassus tiles */
static_assert(NV <= NVP, "dof slots exceed the padded row");
/* per-env global workspace (L2-resident): old manifolds (collision), every row's J | M^-1 J^T (32 + 32
 * doubles, written lane-per-row by the row build), then the Delassus columns >= PREG (column-major) */
#define WS_ROWS (UG_MAXMAN * UG_MAN_DOUBLES)
#define WS_A (WS_ROWS + MAXROWS * RS)
/* hull-box pairs' corner certificates: per pair, the face that last maximised each box corner's plane
 * distance (8 bytes; a hint only -- team_hull_box proves with it or scans every face) */
#define WS_HC (WS_A + (MAXROWS - PREG) * MAXROWS)
/* full-geometry mode (UG_GEOM_FULL): a hull pair's candidates (FC_MAX x 7 doubles: n, pB, d), and the corner
 * certificates as 16-bit face indices (the full hulls have up to UG_FULL_HULL_MAXF faces) */
#define FC_MAX 1024
static_assert(UG_FULL_HULL_MAXV + 64 + 8 <= FC_MAX, "a full hull pair's candidates must fit the workspace list");
/* hull-hull pairs (LOD): per pair and per B vertex, the A face that last maximised its plane distance (a hint, as
 * the corner certificates) */
#define WS_HH (WS_HC + MAXPAIR)
#define WS_FC (WS_HH + 8 * MAXPAIR)
#define WS_HC2 (WS_FC + 7 * FC_MAX)
/* per-env workspace stride: the LOD geometry ends at WS_FC, the full geometry adds its candidate list and 16-bit
 * certificates (a handle allocates only what its mode uses) */
#define WS_LOD_DOUBLES WS_FC
#define WS_SV (WS_HC2 + 2 * MAXPAIR) /* the cylinder pass's surviving support points (4 x UG_FULL_HULL_MAXF ints) */
/* full-geometry separation certificates of hull-box and hull-cylinder pairs (team_hull_box_full, team_poly_cyl): per
 * pair, the relative pose of the last candidate-free evaluation and the margins by which it cleared the contact
 * threshold: [0] the box corners' (hull-box) / the separating face's (hull-cylinder) margin, [1..9] R_AB,
 * [10..12] p_AB, [13..15] p_BA, [16] the hull's vertex radius, [17] B's point radius (box corner / cylinder),
 * hull-box: [18] the margin by which every hull vertex lies beyond the box face [19] (0..5 = -x, +x, -y, +y, -z, +z).
 * Zeroed at creation (margin 0: no certificate). */
#define PC_DOUBLES 20
#define WS_PC (WS_SV + 2 * UG_FULL_HULL_MAXF)
#define WS_FULL_DOUBLES (WS_PC + PC_DOUBLES * MAXPAIR)
#ifdef UG_DEBUG_DUMP /* development aid: team_pgs dumps A, w and impulses after the workspace proper */
#define WS_DBG WS_FULL_DOUBLES
#define WS_DOUBLES (WS_DBG + MAXROWS * MAXROWS + 8 * MAXROWS)
#define WS_STRIDE_VIH(full) ((size_t)WS_DOUBLES)
#else
#define WS_DOUBLES WS_FULL_DOUBLES
#define WS_STRIDE_VIH(full) ((size_t)((full) ? WS_FULL_DOUBLES : WS_LOD_DOUBLES))
#endif
/* the convex-convex path (UG_CONTACT_GJK): the penetration solver's store (ug_gjk.h EpaMem: btGjkEpa2's 132 support
 * vertices, 256 faces and their lists, the horizon walk's stack) after everything else */
#define WS_EPA WS_DOUBLES
#ifndef UG_GJK_G
#define UG_GJK_G 16 /* lanes per GJK pair (ugd::GJK_G): the wave runs 64 / UG_GJK_G pairs at once, one store each */
#endif
#define EPA_DOUBLES ((sizeof(ugk::EpaMem) + sizeof(double) - 1) / sizeof(double))
/* the convex-convex path's separation certificates, per pair: [0] valid, [1..3] the separating axis n in B's frame,
 * [4] A's core extent along -n at the evaluation, [5] B's core extent along n, [6..14] R_AB, [15..17] p_AB (A's pose in
 * B's frame then); GJK's (A, B) order (a sphere-first pair swapped) */
#define GC_DOUBLES 18
#define WS_GC (WS_EPA + EPA_DOUBLES * (64 / UG_GJK_G)) /* one EPA store per GJK lane group */
/* the quiescent-collision reference (team_collide / quiescent_ok): per pair the distance its colliders may still close
 * without a contact (a certificate's slack, a padded-AABB gap; 1e300 for a pair with an inactive collider), then the
 * robot's q when it was taken */
#define WS_QS (WS_GC + GC_DOUBLES * MAXPAIR)
#define WS_STRIDE(full, gjk) ((gjk) ? (size_t)(WS_QS + MAXPAIR + NB) : WS_STRIDE_VIH(full))

#define MAXOV 26 /* pairs per lane-per-pair pass: their working manifolds share LDS with the rows (Shared::pm) */
#define NBOXSLOT 5 /* box-box pairs run per round, one LDS clip-buffer slot each (they share the hull candidates' LDS) */

/* ---------------- env state (canonical layout) ---------------- */
struct StObj { v3 pos; q4 quat; v3 v, w; };
struct StPt { v3 lpA, lpB, n; double dist, imp, imp1, imp2; };
struct StMan { double pair, npts; StPt pt[4]; };
struct EnvState {
    double q[NB], qd[NB], mtarget[7], mon[7], oactive[MAXOBJ];
    StObj obj[MAXOBJ];
    double nman;
    StMan man[MAXMAN];
    double goal_approached, goal_grasped, overflow, spare;
    double prevq[NB], prevpose[MAXOBJ][7]; /* the last substep's narrowphase poses (ug_layout.h UG_F_PREV) */
};
static_assert(sizeof(EnvState) == UG_STATE_DIM * sizeof(double), "EnvState must match ug_layout.h");
static_assert(sizeof(Manifold) * MAXOV <= 88 * MAXROWS, "working manifolds must fit in the rows' LDS");

/* the collider fields the wave narrowphases read, and a pair's shape transforms: formed lane-per-pair once
 * per collision pass (team_collide), read back uniformly by the hull pair loop */
struct HullArg { int nv, v0, nf, f0, c0; double margin; double half[3]; };
struct PairInfo { XF TA, TB; HullArg A, B; double thr; int a, b, ka, kb; };
__device__ __forceinline__ static HullArg hull_arg(const Collider& c) {
    HullArg h;
    h.nv = c.nv; h.v0 = c.v0; h.nf = c.nf; h.f0 = c.f0; h.c0 = c.c0; h.margin = c.margin;
    h.half[0] = c.half[0]; h.half[1] = c.half[1]; h.half[2] = c.half[2];
    return h;
}

struct RowS {
    double invD, rinv, rhs, rhsPen, lo, hi, imp, impPen, fric; /* rinv = invD == 0 ? 0 : 1 / invD */
    int kind; /* 0 limit, 1 motor, 2 gear, 3 normal, 4/5 friction dir 1/2, 6/7 rolling axis 1/2,
               * 8 a jointed object's limit, 9 the Box button's motor */
    int a, b; /* limit: dof, side | motor: m | gear: g | contact: manifold, point | 8: object, side | 9: object */
    int nrow; /* friction: position of its normal row */
};

struct Shared {
    EnvState e;
    Kin kin;
    double LDL[NB * NB];
    double v0[NVP];
    double dvout[NVP], dvsout[NVP];
    XF O[MAXCOL];
    v3 lo[MAXCOL], hi[MAXCOL];
    int nov, ov[MAXPAIR];
    int nrows, nnc, nn, nf, split;
    union {
        RowS rs[MAXROWS];        /* row build .. impulse write-back */
        Manifold pm[MAXOV];      /* collision: lane k's working manifold (rows are dead until the row build) */
        PairInfo pinfo[MAXOV];   /* collision: pair k's transforms and collider fields (before pm is written) */
    };
    union {
        double mcol[NB + 5][NB]; /* row build: M^-1 e_d (d < NB) and M^-1 (ratio_g e_child_g) of gear g */
        struct { Cand c[MAXOV][4]; int n[MAXOV]; } cand;
        double impx[MAXROWS]; /* PGS: row impulses gathered through LDS (after the Delassus build) */
        m3 rj[NB];            /* FK: each body's joint rotation (axis_angle), shared for the ancestor walks */
        DynWork dyn;          /* serial_pre: robot_dynamics work arrays */
    } u;
    union {
        Cand hc[64];              /* hull narrowphase candidates */
        BoxScratch bs[NBOXSLOT];  /* lane-per-pair box-box clip buffers (after the hull pairs of the pass) */
        /* 8-lane GJK groups (UG_GJK_G 8): per group the btGjkEpa2 GJK's four-vertex store (4 x 6 doubles) and the EPA's
         * hull-slot table (256 bytes), during team_gjk only (16-lane groups keep them in v0 | dvout | dvsout and LDL) */
        double gjk_lds[(64 / UG_GJK_G) * (4 * 6 + 32)];
    };
    double a12[NB];
    double jM[MAXOBJ];    /* effective inertia of the jointed objects in this substep (serial_pre; ug_joint.h) */
    double fs[8];
    int is[8];
    int ecnt[2 * MAXMAN]; /* team_enumerate: accepted points / rolling points per manifold */
    int oldp[MAXMAN];     /* collision: pair ids of the previous manifolds (their records are in the workspace) */
    int pmo[MAXOV];       /* collision: previous-manifold index of lane k's pair in this pass, -1 if none */
    int anc[NB];          /* bit d set: dof d moves body b (moves(d, b)); filled by team_load */
    int flags;            /* UG_FLAG_* of this launch (lane 0) */
    int stats[UG_NSTAT];  /* the env's UG_STAT_* counters (lane 0), loaded / stored with the state */
    int bdepth[NB];       /* tree depth of body b (body_depth); filled by team_load */
    int qsvalid;          /* the workspace holds a quiescent-collision reference (WS_QS) for the current program point */
#ifdef UG_PROF
    unsigned long long prof[UG_NPROF];
    unsigned long long tcall, tret; /* PROF_PRE_CALL / PROF_EXIT stamps (lane 0) */
#endif
};

/* the env's LDS image: one per workgroup; a namespace-scope object gives every access a constant address */
static __shared__ Shared g_sh;

/* phase timers (build with -DUG_PROF; read back with urgym_debug_prof) */
#ifdef UG_PROF
__device__ unsigned long long g_prof[UG_NPROF];
#define UG_BT_MAX 8192
__device__ unsigned long long g_btime[4 * UG_BT_MAX]; /* k_step block timeline (urgym_debug_prof reset == 2) */
#define PROF_T0(v) unsigned long long v = __builtin_readcyclecounter()
#define PROF_ADD(k, v)                                                   \
    do {                                                                 \
        if (threadIdx.x == 0) g_sh.prof[k] += __builtin_readcyclecounter() - (v); \
    } while (0)
#define PROF_CNT(k, val)                                 \
    do {                                               \
        if (threadIdx.x == 0) g_sh.prof[k] += (unsigned long long)(val); \
    } while (0)
#else
#define PROF_T0(v)
#define PROF_ADD(k, v)
#define PROF_CNT(k, x)
#endif
enum { PF_COLLIDE = 0, PF_DYN, PF_ROWS, PF_PGS, PF_SPLIT, PF_INTEG, PF_GLUE, PF_TOTAL,
       PC_SUBSTEPS = 8, PC_ROWS, PC_ITERS, PC_OVL, PC_HULL, PC_NMAN, PF_SWEEPS, PF_HULL,
       PF_RDYN, PF_ENUM, PF_BROAD, PF_PAIRS, PF_HB_VERT, PF_HB_CORNER, PF_HB_REDUCE, PF_FK, PF_LDL, PF_UNIT, PF_ROWB, PF_RB1, PF_RB2, PF_RB3, PF_MFMA, PF_WARM, PF_SW_NC, PF_SW_CT, PF_SW_FIN, PF_SW_FPREP, PF_SW_FR,
       PF_SW_RES, PF_PR_LOOK, PF_PR_NP, PF_PR_MAN, PF_PR_ST, PC_CHUNKS, PC_NNC, PC_NN, PC_N64, PC_N80, PC_N96,
       PC_FREE, PF_FREE_COL, PF_FREE_DYN, PF_FREE_ROWS, PF_FREE_PGS, PF_FREE_INT,
       PF_FREE_PSETUP, PF_FREE_PSWEEP, PF_FREE_PPOST, PF_PR_BB, PF_HS, PC_CYPAIR, PF_CY1, PF_CY2, PC_CYSV, PC_CYIT,
       /* the contact-free substeps' share of these sub-phase counters (UG_FREE_SPLIT below) */
       PF_FREE_SUB0 = 64,
       /* the convex-convex path (ug_gjk.h): queries, penetration-path queries, classic GJK / libccd iterations, hull
        * support queries and their cycles */
       PC_GJK = 80, PC_GJK_EPA, PC_GJK_IT, PC_GJK_CCD, PC_GJK_SUP, PF_GJK_SUP,
       /* EPA iterations, cycles: the whole query, the penetration path, the libccd test, the classic GJK */
       PC_EPA_IT, PF_GJK_ALL, PF_GJK_PEN, PF_GJK_CCD, PF_GJK_CLASSIC,
       /* inside the penetration path: btGjkEpa2's GJK, the EPA setup (enclose + tetrahedron), its iterations' support,
        * horizon walk and findbest, the witnesses */
       PF_EPA_GJK, PF_EPA_SETUP, PF_EPA_SUP, PF_EPA_EXPAND, PF_EPA_BEST,
       /* inside the libccd test and the classic GJK: the support pairs, the simplex work */
       PF_CCD_SUP, PF_CCD_DO, PF_CLS_SUP, PF_CLS_VS,
       PC_GJK_RECERT, /* GJK pairs skipped by the exact certificate re-test (gjk_one) */
       /* inside the hull support: the cycles until its cell is known, until its loads have landed (a forced wait,
        * profiling build only), and the supports that took a cell (not the whole scan) */
       PF_SUP_CELL, PF_SUP_MEM, PC_SUP_CELLS,
       /* calls of the __noinline__ phases (tools/scratch_attr.py: their callee-saved saves and spills x calls) */
       PC_CALL0 = 104, PC_QUIET = 115, /* substeps whose collision stage quiescent_ok proved empty */
       /* the calling-convention cost of the big __noinline__ phases: per phase, cycles from the
        * caller's last instruction before the call to the callee's first statement (call + prologue: the callee-saved
        * VGPR saves), and from the callee's last statement to the caller's first instruction after it (epilogue: the
        * restores, the wait for them, the return) */
       PF_CS0 = 116 /* [PF_CS0 + 2 k] prologue, [PF_CS0 + 2 k + 1] epilogue of CS_* */ };
enum { CS_GJK = 0, CS_COLLIDE, CS_PGS, CS_FK, CS_PRE, CS_POST, CS_UNIT, CS_RDYN, CS_ENUM, CS_N };
enum { CALL_GJK = 0, CALL_COLLIDE, CALL_ENUM, CALL_UNIT, CALL_RDYN, CALL_PRE, CALL_POST, CALL_FK, CALL_PGS, CALL_GLUE,
       CALL_REDUCE4, CALL_N };
#define PROF_CALL(k) PROF_CNT(PC_CALL0 + (k), 1)
#ifdef UG_PROF
#define PROF_PRE_CALL() do { if (threadIdx.x == 0) g_sh.tcall = __builtin_readcyclecounter(); } while (0)
#define PROF_ENTRY(k)                                                                              \
    do {                                                                                           \
        const unsigned long long t_ = __builtin_readcyclecounter();                                \
        if (threadIdx.x == 0) g_sh.prof[PF_CS0 + 2 * (k)] += t_ - g_sh.tcall;                      \
    } while (0)
#define PROF_EXIT() do { if (threadIdx.x == 0) g_sh.tret = __builtin_readcyclecounter(); } while (0)
#define PROF_POST_CALL(k)                                                                          \
    do {                                                                                           \
        const unsigned long long t_ = __builtin_readcyclecounter();                                \
        if (threadIdx.x == 0) g_sh.prof[PF_CS0 + 2 * (k) + 1] += t_ - g_sh.tret;                   \
    } while (0)
#else
#define PROF_PRE_CALL()
#define PROF_ENTRY(k)
#define PROF_EXIT()
#define PROF_POST_CALL(k)
#endif
#define UG_FREE_SPLIT_N 14
#ifdef UG_PROF
__device__ static const int kFreeSplit[UG_FREE_SPLIT_N] = {PF_FK, PF_BROAD, PF_HULL, PF_PR_LOOK, PF_PR_NP, PF_PR_MAN, PF_PR_ST,
                                                           PF_PAIRS, PC_OVL, PC_HULL, PF_RDYN, PF_LDL, PF_ENUM, PF_UNIT};
#endif

} /* namespace ugd */
/* the convex-convex narrowphase (Bullet's GJK / EPA pair detector), run by the whole wave per pair */
#define UGK_FN __device__ static inline
/* gjk_pair is forced inline into team_gjk, which becomes a leaf (measured round 6): as a call inside
 * team_gjk it left team_gjk's callee-saved SGPRs no free VGPR lane, so its prologue and epilogue saved and restored 34
 * SGPRs each through scratch one at a time with a full memory wait per register -- 17 k + 52 k cycles per call, 7.5 %
 * of a BallBalance substep (profiles/round6_phase_ballbalance_callsave_before.txt; after: 3.6 k + 7.0 k,
 * round6_phase_ballbalance_callsave_after.txt) */
#define UGK_FN_PAIR __device__ static __forceinline__
#define UGK_GMEM __attribute__((address_space(1)))
#define UGK_LMEM __attribute__((address_space(3)))
#define UGK_OPAQUE(x) __asm__ volatile("" : "+v"(x))
#define UGK_GROUP_PARALLEL 1
#ifdef UG_PROF /* its event counters (PC_GJK_*) and phase timers, lane 0 of the env's wave */
/* summed over the lane groups that run pairs at once (LDS atomics): work, not wall time */
#define UGK_COUNT(k, v) do { if ((threadIdx.x & (UG_GJK_G - 1)) == 0) atomicAdd(&ugd::g_sh.prof[ugd::k], (unsigned long long)(v)); } while (0)
#define UGK_T0(v) const unsigned long long v = __builtin_readcyclecounter()
#define UGK_ADD(k, v) UGK_COUNT(k, __builtin_readcyclecounter() - (v))
#endif
#include "ug_gjk.h"
namespace ugd {

/* ---------------- wave helpers ---------------- */
template <int CTRL>
__device__ __forceinline__ double dpp(double x) {
    int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), CTRL, 0xF, 0xF, false);
    int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
template <int CTRL>
__device__ __forceinline__ int dppi(int x) { return __builtin_amdgcn_mov_dpp(x, CTRL, 0xF, 0xF, false); }
/* pairwise tree over each 16-lane row: quad xor1, quad xor2, half-row mirror, row mirror.
 * Every lane of the row ends with ((x0+x1)+(x2+x3))+... -- oracle tree16(). */
__device__ __forceinline__ double reduce16(double x) {
    x = x + dpp<0xB1>(x);
    x = x + dpp<0x4E>(x);
    x = x + dpp<0x141>(x);
    x = x + dpp<0x140>(x);
    return x;
}
__device__ __forceinline__ double readlane_d(double x, int l) {
    int lo = __builtin_amdgcn_readlane(__double2loint(x), l);
    int hi = __builtin_amdgcn_readlane(__double2hiint(x), l);
    return __hiloint2double(hi, lo);
}
/* every lane l receives x from lane (32*h + (l & 31)) */
__device__ __forceinline__ double half_bcast(double x, int h) {
    int lo = __double2loint(x), hi = __double2hiint(x);
    auto plo = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    auto phi = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    return h == 0 ? __hiloint2double(phi[0], plo[0]) : __hiloint2double(phi[1], plo[1]);
}
__device__ __forceinline__ unsigned long long ballot(int p) { return __ballot(p); }
/* wave-wide min / max of a double (rows of 16 by DPP, then the four rows), uniform result */
__device__ __forceinline__ double wave_min_d(double x) {
    x = ug_min(x, dpp<0xB1>(x)); x = ug_min(x, dpp<0x4E>(x)); x = ug_min(x, dpp<0x141>(x)); x = ug_min(x, dpp<0x140>(x));
    return ug_min(ug_min(readlane_d(x, 0), readlane_d(x, 16)), ug_min(readlane_d(x, 32), readlane_d(x, 48)));
}
__device__ __forceinline__ double wave_max_d(double x) {
    x = ug_max(x, dpp<0xB1>(x)); x = ug_max(x, dpp<0x4E>(x)); x = ug_max(x, dpp<0x141>(x)); x = ug_max(x, dpp<0x140>(x));
    return ug_max(ug_max(readlane_d(x, 0), readlane_d(x, 16)), ug_max(readlane_d(x, 32), readlane_d(x, 48)));
}
__device__ __forceinline__ int lane_prefix(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0));
}
/* wave-wide best (value, index): want_max picks the larger value, else the smaller; ties -> lower index;
 * invalid lanes pass idx = 0x7fffffff.  Result is uniform. */
__device__ __forceinline__ bool better(double v, int i, double w, int j, bool want_max) {
    if (j == 0x7fffffff) return true;
    if (i == 0x7fffffff) return false;
    if (v != w) return want_max ? v > w : v < w;
    return i < j;
}
__device__ __forceinline__ void wave_best(double& v, int& idx, bool want_max) {
#define STEP(CTRL)                                             \
    {                                                          \
        double w = dpp<CTRL>(v);                               \
        int j = dppi<CTRL>(idx);                               \
        if (!better(v, idx, w, j, want_max)) { v = w; idx = j; } \
    }
    STEP(0xB1) STEP(0x4E) STEP(0x141) STEP(0x140)
#undef STEP
    double bv = readlane_d(v, 0);
    int bi = __builtin_amdgcn_readlane(idx, 0);
    for (int r = 16; r < 64; r += 16) {
        double w = readlane_d(v, r);
        int j = __builtin_amdgcn_readlane(idx, r);
        if (!better(bv, bi, w, j, want_max)) { bv = w; bi = j; }
    }
    v = bv;
    idx = bi;
}

/* The GJK / EPA of one pair runs on a group of GJK_G lanes (one DPP row): the wave runs up to GJK_NG pairs at once,
 * each group uniform within itself (every lane of it computes the same values), the groups diverging as their pairs'
 * iterations differ.  group_best is wave_best over the group's row. */
constexpr int GJK_G = UG_GJK_G, GJK_NG = TEAM / GJK_G;
static_assert(TEAM == 64, "WS_GC counts 64 lanes");
static_assert(GJK_G == 16 || GJK_G == 8, "a GJK lane group is one DPP row or half-row (the reductions below)");
__device__ __forceinline__ void group_best(double& v, int& idx, bool want_max) {
#define STEP(CTRL)                                               \
    {                                                            \
        double w = dpp<CTRL>(v);                                 \
        int j = dppi<CTRL>(idx);                                 \
        if (!better(v, idx, w, j, want_max)) { v = w; idx = j; } \
    }
    STEP(0xB1) STEP(0x4E) STEP(0x141) /* quad xor 1, quad xor 2, half-row mirror: 8 lanes */
    if constexpr (GJK_G == 16) STEP(0x140) /* row mirror: 16 */
#undef STEP
}

} /* namespace ugd */
/* ug_gjk.h's hull support on the lane group: btVector3::maxDot's first maximum (the largest dot product, on a tie the
 * lowest vertex index) over the whole hull, called by every lane of the group (its GJK runs uniformly).  Lane l of the
 * group dots vertices l, l + G, ... of a vertex range keeping its first maximum, and the DPP arg-max keeps the larger
 * value and, on a tie, the lower index.  (Culling a full hull's 64-vertex chunks by their bounding spheres -- the
 * best-bound chunk first, then every chunk whose bound reaches its maximum -- measured 2.2x slower per support on
 * BallBalance: the spheres overlap, most chunks pass, and each pass is a serial load + reduction.) */
__device__ __forceinline__ void hs_scan(int v0, int nv, ugk::gv d, int gl, double& best, int& bi, ugk::gv& bv) {
    constexpr int G = ugd::GJK_G, U = G == TEAM ? 4 : 8; /* 16 measured the same (r4l) */
    /* U vertices per trip: their loads in flight together (the hull is cache-resident, the latency is the cost) */
    for (int i0 = gl; i0 < nv; i0 += U * G) {
        double x[U], y[U], z[U];
#pragma unroll
        for (int k = 0; k < U; k++) {
            const int i = i0 + k * G < nv ? i0 + k * G : i0;
            const double* p = &UG_HULL_V[3 * (v0 + i)];
            x[k] = p[0]; y[k] = p[1]; z[k] = p[2];
        }
#pragma unroll
        for (int k = 0; k < U; k++) {
            const double dd = x[k] * d.x + y[k] * d.y + z[k] * d.z;
            const int i = i0 + k * G;
            if (i < nv && (dd > best || (dd == best && i < bi))) { /* maxDot's test: a NaN never wins */
                best = dd;
                bi = i;
                bv = ugk::V3(x[k], y[k], z[k]);
            }
        }
    }
}
#define UGK_RCPF(x) __builtin_amdgcn_rcpf(x)
#include "ug_supcell.h"
/* the direction cell's candidates (supcell_data.h).  Lane l of the group dots candidate l of the cell, its coordinates
 * read straight from the cell's slot (one memory round).  The list ascends, so the first maximal dot product over it
 * is the lowest lane holding the group's maximum: a DPP max of the dot products (all finite on this path), then the
 * lowest lane of the group whose product equals it (a ballot), whose coordinates the group reads.  A cell with a
 * longer list (UG_SC_OVF, tied flat faces) walks it in trips of G through the vertex indices instead, keeping each
 * lane's first maximum keyed by vertex index x G + lane, and takes the group's arg-max. */
__device__ __forceinline__ double group_max(double x) {
    x = ug_max(x, ugd::dpp<0xB1>(x));
    x = ug_max(x, ugd::dpp<0x4E>(x));
    x = ug_max(x, ugd::dpp<0x141>(x));
    if constexpr (ugd::GJK_G == 16) x = ug_max(x, ugd::dpp<0x140>(x));
    return x;
}
__device__ __forceinline__ ugk::gv hs_cells(int v0, int scb, int cell, ugk::gv d, int gl) {
    constexpr int G = ugd::GJK_G, K = UG_SC_SLOTS / G; /* candidates per lane: lane l holds slots l, l + G */
    static_assert(UG_SC_SLOTS % G == 0 && K <= 2, "a cell's slots over the lanes of a GJK group");
    const int c = scb + cell;
    const unsigned short* L = &UG_SC_IDX[c * UG_SC_SLOTS];
    const double* P = &UG_SC_XYZ[(c * UG_SC_SLOTS + gl) * 3];
    const int s0 = L[0];
    /* loaded with the list head: the common case needs nothing else */
    ugk::gv bv = ugk::V3(P[0], P[1], P[2]);
    ugk::gv bv2 = bv;
    if constexpr (K == 2) bv2 = ugk::V3(P[3 * G], P[3 * G + 1], P[3 * G + 2]);
    const int base = (int)(threadIdx.x & ~(G - 1));
    int src;
    if (s0 != UG_SC_OVF) {
        const double dd = bv.x * d.x + bv.y * d.y + bv.z * d.z;
        if constexpr (K == 1) {
            const double M = group_max(dd);
            const unsigned long long hit = ugd::ballot(dd == M);
            src = base + __builtin_ctzll((hit >> base) & ((1ull << G) - 1ull));
        } else {
            /* the first maximum over the ascending list: slots l (< G) before slots G + l */
            const double dd2 = bv2.x * d.x + bv2.y * d.y + bv2.z * d.z;
            const double M = group_max(ug_max(dd, dd2));
            const unsigned long long h1 = (ugd::ballot(dd == M) >> base) & ((1ull << G) - 1ull);
            const unsigned long long h2 = (ugd::ballot(dd2 == M) >> base) & ((1ull << G) - 1ull);
            src = base + __builtin_ctzll(h1 ? h1 : h2);
            if (!h1) bv = bv2;
        }
    } else {
        double best = -__builtin_inf();
        int key = 0x7fffffff;
        const int cnt = L[1], off = L[2] | (L[3] << 16);
        for (int t = 0; t < cnt; t += G) { /* the list is padded to whole trips */
            const int i = UG_SC_IDX[off + t + gl];
            const double* p = &UG_HULL_V[3 * (v0 + i)];
            const double x = p[0], y = p[1], z = p[2];
            const double e = x * d.x + y * d.y + z * d.z;
            const int k = i * G + gl;
            if (e > best || (e == best && k < key)) {
                best = e;
                key = k;
                bv = ugk::V3(x, y, z);
            }
        }
        ugd::group_best(best, key, true);
        src = base + (key & (G - 1));
    }
    return ugk::V3(__shfl(bv.x, src, TEAM), __shfl(bv.y, src, TEAM), __shfl(bv.z, src, TEAM));
}
UGK_FN ugk::gv ugk_hull_support(const ugk::GShape& sh, ugk::gv d) {
    constexpr int G = ugd::GJK_G;
    const int gl = threadIdx.x & (G - 1);
    PROF_T0(t_sup);
    const int cell = sh.scb >= 0 ? ugk_sc_cell(d.x, d.y, d.z, sh.sck) : -1;
    ugk::gv r;
#ifdef UG_PROF
    if (gl == 0) atomicAdd(&ugd::g_sh.prof[ugd::PF_SUP_CELL], __builtin_readcyclecounter() - t_sup);
#endif
    if (cell >= 0) { /* a finite direction: its cell holds every vertex that can win the full scan (build_supcells.py) */
        r = hs_cells(sh.v0, sh.scb, cell, d, gl);
#ifdef UG_PROF
        if (gl == 0) {
            atomicAdd(&ugd::g_sh.prof[ugd::PF_SUP_MEM], __builtin_readcyclecounter() - t_sup);
            atomicAdd(&ugd::g_sh.prof[ugd::PC_SUP_CELLS], 1ull);
        }
#endif
    } else {
        double best = -__builtin_inf();
        int bi = 0x7fffffff;
        ugk::gv bv = ugk::V3(0.0, 0.0, 0.0);
        hs_scan(sh.v0, sh.nv, d, gl, best, bi, bv);
        ugd::group_best(best, bi, true);
        if (bi == 0x7fffffff) { /* no comparable dot product (a NaN direction): vertex 0, as maxDot leaves it */
            const double* p = &UG_HULL_V[3 * sh.v0];
            r = ugk::V3(p[0], p[1], p[2]);
        } else { /* the winner's coordinates from the lane that dotted it (vertex i sits in lane i mod G) */
            const int src = (int)(threadIdx.x & ~(G - 1)) + (bi & (G - 1));
            r = ugk::V3(__shfl(bv.x, src, TEAM), __shfl(bv.y, src, TEAM), __shfl(bv.z, src, TEAM));
        }
    }
#ifdef UG_PROF
    if (gl == 0) {
        atomicAdd(&ugd::g_sh.prof[ugd::PF_GJK_SUP], __builtin_readcyclecounter() - t_sup);
        atomicAdd(&ugd::g_sh.prof[ugd::PC_GJK_SUP], 1ull);
    }
#endif
    return r;
}

/* The EPA / btGjkEpa2 records.  The btGjkEpa2 GJK's four-vertex store and the EPA's hull-slot table live in LDS the
 * collision stage leaves unused (v0 | dvout | dvsout, written by serial_pre and after the PGS; LDL, written by
 * serial_pre), one slice per lane group, reached through LDS-typed pointers (ds_* instructions); the faces, hull slots
 * and EPA vertices stay in the group's workspace store, reached through global-typed pointers (global_*).  A record
 * that may sit in either space would need a generic pointer, and every flat access waits for all outstanding memory
 * operations of the wave (measured: 308 full waits in the solver with LDS / workspace tiers for the faces). */
#define UG_LDS __attribute__((address_space(3)))
#if UG_GJK_G == 16
static_assert(ugd::GJK_NG * 4 * sizeof(ugk::ESv) <= 3 * sizeof(double) * NVP, "the GJK stores in v0 | dvout | dvsout");
static_assert(offsetof(ugd::Shared, dvsout) == offsetof(ugd::Shared, v0) + 2 * sizeof(double) * NVP, "v0, dvout, dvsout adjacent");
static_assert(ugd::GJK_NG * ugk::kEpaMaxFaces <= sizeof(double) * NB * NB, "EPA hull-slot tables in LDL");
#define UG_GJK_SV_BASE (&ugd::g_sh.v0[0])
#define UG_GJK_HPOS_BASE (&ugd::g_sh.LDL[0])
#else
static_assert(sizeof(ugk::ESv) == 6 * sizeof(double) && ugk::kEpaMaxFaces == 256, "Shared::gjk_lds's sizing");
#define UG_GJK_SV_BASE (&ugd::g_sh.gjk_lds[0])
#define UG_GJK_HPOS_BASE (&ugd::g_sh.gjk_lds[ugd::GJK_NG * 4 * 6])
#endif
__device__ __forceinline__ int gjk_grp() { return (int)(threadIdx.x / ugd::GJK_G); }
__device__ __forceinline__ UG_LDS ugk::ESv* lds_sv() { return (UG_LDS ugk::ESv*)(UG_LDS void*)UG_GJK_SV_BASE + gjk_grp() * 4; }
UGK_FN ugk::ESv ugk_svl_get(UGK_GMEM ugk::EpaMem*, int i) {
    const UG_LDS ugk::ESv& s = lds_sv()[i];
    ugk::ESv v;
    v.d = ugk::V3(s.d.x, s.d.y, s.d.z);
    v.w = ugk::V3(s.w.x, s.w.y, s.w.z);
    return v;
}
UGK_FN void ugk_svl_put(UGK_GMEM ugk::EpaMem*, int i, const ugk::ESv& v) {
    UG_LDS ugk::ESv& s = lds_sv()[i];
    s.d.x = v.d.x; s.d.y = v.d.y; s.d.z = v.d.z;
    s.w.x = v.w.x; s.w.y = v.w.y; s.w.z = v.w.z;
}
UGK_FN UGK_LMEM unsigned char* ugk_hpos(UGK_GMEM ugk::EpaMem*) {
    return (UGK_LMEM unsigned char*)(UGK_LMEM void*)UG_GJK_HPOS_BASE + gjk_grp() * ugk::kEpaMaxFaces;
}
UGK_FN ugk::EFace ugk_face_get(UGK_GMEM ugk::EpaMem* E, int f) {
    const UGK_GMEM ugk::EFace& G = E->fc[f];
    ugk::EFace F;
    F.n = ugk::V3(G.n.x, G.n.y, G.n.z);
    F.d = G.d;
    for (int j = 0; j < 3; j++) { F.c[j] = G.c[j]; F.f[j] = G.f[j]; F.e[j] = G.e[j]; }
    F.pass = G.pass;
    return F;
}
UGK_FN void ugk_face_put(UGK_GMEM ugk::EpaMem* E, int f, const ugk::EFace& F) {
    UGK_GMEM ugk::EFace& G = E->fc[f];
    G.n.x = F.n.x; G.n.y = F.n.y; G.n.z = F.n.z;
    G.d = F.d;
    for (int j = 0; j < 3; j++) { G.c[j] = F.c[j]; G.f[j] = F.f[j]; G.e[j] = F.e[j]; }
    G.pass = F.pass;
}
UGK_FN void ugk_face_pass(UGK_GMEM ugk::EpaMem* E, int f, int pass) { E->fc[f].pass = (unsigned char)pass; }
UGK_FN void ugk_face_link(UGK_GMEM ugk::EpaMem* E, int f, int j, int nf, int ne) {
    E->fc[f].f[j] = (unsigned char)nf;
    E->fc[f].e[j] = (unsigned char)ne;
}
UGK_FN ugk::EHull ugk_hull_get(UGK_GMEM ugk::EpaMem* E, int i) {
    ugk::EHull h;
    h.d = E->hl[i].d; h.stamp = E->hl[i].stamp; h.f = E->hl[i].f;
    return h;
}
UGK_FN void ugk_hull_put(UGK_GMEM ugk::EpaMem* E, int i, const ugk::EHull& h) {
    E->hl[i].d = h.d; E->hl[i].stamp = h.stamp; E->hl[i].f = h.f;
}

/* ug_gjk.h's lane-group hooks: the lane's index in its group, a value as another lane of the group holds it */
UGK_FN int ugk_glane() { return (int)(threadIdx.x & (ugd::GJK_G - 1)); }
UGK_FN double ugk_gread(double v, int j) { return __shfl(v, (int)(threadIdx.x & ~(ugd::GJK_G - 1)) + j, TEAM); }
UGK_FN int ugk_greadi(int v, int j) { return __shfl(v, (int)(threadIdx.x & ~(ugd::GJK_G - 1)) + j, TEAM); }
UGK_FN bool ugk_gany(bool p) {
    return ((ugd::ballot(p) >> (threadIdx.x & ~(ugd::GJK_G - 1))) & ((1ull << ugd::GJK_G) - 1ull)) != 0ull;
}
UGK_FN int ugk_gsize() { return ugd::GJK_G; }

/* ug_gjk.h's small stacks on the lane group: slots [0, GJK_G) in one register, lane i of the group holding slot i
 * (read back through ds_bpermute, an LDS-crossbar hop instead of a workspace round trip), deeper slots in memory */
UGK_FN void ugk_ls_put(UGK_GMEM int* mem, ugk::LStack& s, int i, int v) {
    if (i < ugd::GJK_G) {
        if ((int)(threadIdx.x & (ugd::GJK_G - 1)) == i) s.reg = v;
    } else {
        mem[i] = v;
    }
}
UGK_FN int ugk_ls_get(const UGK_GMEM int* mem, const ugk::LStack& s, int i) {
    if (i < ugd::GJK_G) return __shfl(s.reg, (int)(threadIdx.x & ~(ugd::GJK_G - 1)) + i, TEAM);
    return mem[i];
}
/* ug_gjk.h's EPA hook on the lane group: m_hull's first minimum (smallest d * d, ties to the largest append stamp; a
 * NaN at the root -- the largest stamp -- keeps the root) as a lane-strided scan of the hull array + a DPP arg-min of
 * the key (d * d, (2^20 - stamp) * 256 + face); the root is looked up only when some face of the hull has a NaN plane */
UGK_FN int ugk_epa_findbest(const UGK_GMEM ugk::EpaMem* E, int hcount) {
    constexpr int G = ugd::GJK_G;
    const int gl = threadIdx.x & (G - 1);
    double bv = 0.0, rs = -1.0;
    int bi = 0x7fffffff, ri = 0x7fffffff;
    bool nan = false;
    for (int i = gl; i < hcount; i += G) {
        const ugk::EHull h = ugk_hull_get(const_cast<UGK_GMEM ugk::EpaMem*>(E), i);
        const double sqd = h.d * h.d;
        if (ri == 0x7fffffff || (double)h.stamp > rs) { rs = (double)h.stamp; ri = i; }
        if (sqd != sqd) { nan = true; continue; }
        const int key = ((1 << 20) - h.stamp) * ugk::kEpaMaxFaces + h.f; /* lower key = larger stamp */
        if (bi == 0x7fffffff || sqd < bv || (sqd == bv && key < bi)) { bv = sqd; bi = key; }
    }
    if ((ugd::ballot(nan) >> (threadIdx.x & ~(G - 1))) & ((1ull << G) - 1ull)) {
        ugd::group_best(rs, ri, true); /* the root: the largest stamp */
        const ugk::EHull h = ugk_hull_get(const_cast<UGK_GMEM ugk::EpaMem*>(E), ri);
        if ((h.d * h.d) != (h.d * h.d)) return h.f;
    }
    ugd::group_best(bv, bi, false);
    return bi & (ugk::kEpaMaxFaces - 1);
}
namespace ugd {

/* ---------------- env-state helpers (lane-serial) ---------------- */
__device__ static XF owner_xf(const EnvState& e, const Kin& k, int owner) {
    XF T;
    if (owner >= 0) { T.R = k.R[owner]; T.p = k.p[owner]; }
    else if (owner <= -2 && owner > -100) { int o = -2 - owner; T.R = qmat(e.obj[o].quat); T.p = e.obj[o].pos; }
    else { T.R = mident(); T.p = V(0, 0, 0); }
    return T;
}
__device__ static inline int collider_active(const EnvState& e, const Collider& c) {
    if (c.owner <= -2 && c.owner > -100) return e.oactive[-2 - c.owner] != 0.0;
    return 1;
}
__device__ static inline void man_to_st(StMan& S, const LManifold& M) {
    S.pair = (double)M.pair;
    S.npts = (double)M.npts;
    for (int p = 0; p < 4; p++) {
        StPt& s = S.pt[p];
        bool live = p < M.npts;
        const v3 a = ldv(M.pt[p].lpA), b = ldv(M.pt[p].lpB), n = ldv(M.pt[p].n);
        s.lpA = live ? a : V(0, 0, 0);
        s.lpB = live ? b : V(0, 0, 0);
        s.n = live ? n : V(0, 0, 0);
        s.dist = live ? M.pt[p].dist : 0.0;
        s.imp = live ? M.pt[p].imp : 0.0;
        s.imp1 = live ? M.pt[p].imp1 : 0.0;
        s.imp2 = live ? M.pt[p].imp2 : 0.0;
    }
}

#include "ug_team_collide.h"
#include "ug_team_rows.h"
#include "ug_team_pgs.h"
#include "ug_team_dyn.h"
#include "ug_team_solve.h"
#include "ug_team_run.h"

}  // namespace ugd
#endif
