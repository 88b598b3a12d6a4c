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
#include "ug_glue.h"

namespace ugd {

#define TEAM 64
typedef __attribute__((address_space(1))) const double gcdouble;
typedef __attribute__((address_space(1))) double gdouble;
#define UG_NPROF 116 /* phase accumulators of the -DUG_PROF build */
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
#define UG_GJK_G 16 /* lanes per GJK pair (ugd::GJK_G): the wave runs 64 / UG_GJK_G pairs at once, one store each */
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
       PC_CALL0 = 104, PC_QUIET = 115 /* substeps whose collision stage quiescent_ok proved empty */ };
enum { CALL_GJK = 0, CALL_COLLIDE, CALL_ENUM, CALL_UNIT, CALL_RDYN, CALL_PRE, CALL_POST, CALL_FK, CALL_PGS, CALL_GLUE,
       CALL_REDUCE4, CALL_N };
#define PROF_CALL(k) PROF_CNT(PC_CALL0 + (k), 1)
#define UG_FREE_SPLIT_N 14
#ifdef UG_PROF
__device__ static const int kFreeSplit[UG_FREE_SPLIT_N] = {PF_FK, PF_BROAD, PF_HULL, PF_PR_LOOK, PF_PR_NP, PF_PR_MAN, PF_PR_ST,
                                                           PF_PAIRS, PC_OVL, PC_HULL, PF_RDYN, PF_LDL, PF_ENUM, PF_UNIT};
#endif

} /* namespace ugd */
/* the convex-convex narrowphase (Bullet's GJK / EPA pair detector), run by the whole wave per pair */
#define UGK_FN __device__ static inline
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
static_assert(GJK_G == 16, "a GJK lane group is one DPP row (the group masks and ds_bpermute reads assume it)");
__device__ __forceinline__ void group_best(double& v, int& idx, bool want_max) {
    if (GJK_G == TEAM) {
        wave_best(v, idx, want_max);
        return;
    }
#define STEP(CTRL)                                               \
    {                                                            \
        double w = dpp<CTRL>(v);                                 \
        int j = dppi<CTRL>(idx);                                 \
        if (!better(v, idx, w, j, want_max)) { v = w; idx = j; } \
    }
    STEP(0xB1) STEP(0x4E) STEP(0x141) STEP(0x140)
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
    return ug_max(x, ugd::dpp<0x140>(x));
}
__device__ __forceinline__ ugk::gv hs_cells(int v0, int scb, int cell, ugk::gv d, int gl) {
    constexpr int G = ugd::GJK_G;
    static_assert(UG_SC_SLOTS == G, "one cell slot per lane of a GJK group");
    const int c = scb + cell;
    const unsigned short* L = &UG_SC_IDX[c * UG_SC_SLOTS];
    const double* P = &UG_SC_XYZ[(c * UG_SC_SLOTS + gl) * 3];
    const int s0 = L[0];
    ugk::gv bv = ugk::V3(P[0], P[1], P[2]); /* loaded with the list head: the common case needs nothing else */
    const int base = (int)(threadIdx.x & ~(G - 1));
    int src;
    if (s0 != UG_SC_OVF) {
        const double dd = bv.x * d.x + bv.y * d.y + bv.z * d.z;
        const double M = group_max(dd);
        const unsigned long long hit = ugd::ballot(dd == M);
        src = base + __builtin_ctzll((hit >> base) & ((1ull << G) - 1ull));
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
static_assert(ugd::GJK_NG * 4 * sizeof(ugk::ESv) <= 3 * sizeof(double) * NVP, "the GJK stores in v0 | dvout | dvsout");
static_assert(offsetof(ugd::Shared, dvsout) == offsetof(ugd::Shared, v0) + 2 * sizeof(double) * NVP, "v0, dvout, dvsout adjacent");
static_assert(ugd::GJK_NG * ugk::kEpaMaxFaces <= sizeof(double) * NB * NB, "EPA hull-slot tables in LDL");
__device__ __forceinline__ int gjk_grp() { return (int)(threadIdx.x / ugd::GJK_G); }
__device__ __forceinline__ UG_LDS ugk::ESv* lds_sv() { return (UG_LDS ugk::ESv*)(UG_LDS void*)&ugd::g_sh.v0[0] + gjk_grp() * 4; }
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
    return (UGK_LMEM unsigned char*)(UGK_LMEM void*)&ugd::g_sh.LDL[0] + gjk_grp() * ugk::kEpaMaxFaces;
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
__device__ __noinline__ static void team_gjk(const Scene* s, unsigned long long hq, int c0, double* ws) {
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
}

template <bool FULL, bool GJK>
__device__ __noinline__ static void team_collide(const Scene* s, double* ws) {
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
            if (hq) team_gjk(s, hq, c0, ws);
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
}

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
        return;
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
}
/* lane 0: external forces (robot gravity/gyroscopic/damping via CRBA + RNEA, free objects), the LDL^T of
 * the mass matrix, and the row enumeration */
__device__ __noinline__ static void serial_pre(const Scene* s) {
    PROF_CALL(CALL_PRE);
    Shared& sh = g_sh;
    EnvState& e = sh.e;
    const double dt = UG_DT;
    const int lane = threadIdx.x;
    PROF_T0(t_rd);
    team_robot_dynamics(s->gravity);
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
    team_enumerate(s);
    PROF_ADD(PF_ENUM, t_en);
}
/* lane 0: velocities += solver delta, positions integrate (v + split velocity) */
__device__ __noinline__ static void serial_post(const Scene* s, int split) {
    PROF_CALL(CALL_POST);
    Shared& sh = g_sh;
    EnvState& e = sh.e;
    const double dt = UG_DT;
    const int lane = threadIdx.x;
    if (lane == 0) {
        const double* DV = sh.dvout;
        const double* DVS = sh.dvsout;
        /* the poses this substep's narrowphase saw, before they move (the contact query's world positions) */
        for (int i = 0; i < NB; i++) e.prevq[i] = e.q[i];
        for (int o = 0; o < MAXOBJ; o++) {
            const StObj& ob = e.obj[o];
            e.prevpose[o][0] = ob.pos.x; e.prevpose[o][1] = ob.pos.y; e.prevpose[o][2] = ob.pos.z;
            e.prevpose[o][3] = ob.quat.x; e.prevpose[o][4] = ob.quat.y; e.prevpose[o][5] = ob.quat.z;
            e.prevpose[o][6] = ob.quat.w;
        }
        for (int i = 0; i < NB; i++) {
            e.qd[i] = ug_vclamp(e.qd[i] + DV[i], UG_MAX_COORD_VEL);
            double vi = split ? e.qd[i] + DVS[i] : e.qd[i];
            e.q[i] = e.q[i] + vi * dt;
        }
        for (int o = 0; o < s->nobj; o++) {
            if (e.oactive[o] == 0.0) continue;
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
                continue;
            }
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
/* fk() wave-parallel: lane b < NB forms its joint rotation, then composes its own root-to-body chain
 * (same operations and order as fk() along that path) */
__device__ __noinline__ static void serial_fk() {
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
}

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
    const bool fs6ok = !flok && nnc <= FS_NC && nn >= 3 && nn <= FS6_F0 - FS_NC && n - fb <= FS6_NF;
    const bool fsok = !flok && nnc <= FS_NC && nn >= 3 && nn <= FS_F0 - FS_NC && n - fb <= FS_NF;
    const bool g12ok = !flok && !fsok && nnc <= FG12_NC && nn >= 3 && nn <= FG12_F0 - FG12_NC && n - fb <= FG12_NF;
    const bool g18ok = !flok && !fsok && !g12ok && nnc <= FG18_NC && nn >= 3 && nn <= FG18_F0 - FG18_NC &&
                       n - fb <= FG18_NF;
    const bool fgok = !flok && !fsok && !g12ok && !g18ok && nnc <= FG_NC && nn >= 16 && nn <= FG_F0 - FG_NC &&
                      n - fb <= FG_NF;
    const PosMap pm = flok ? PosMap{n, fb, flf0, nnc, nnc, flf0 + 2 * (flf0 - FL_NNC)}
                      : fs6ok ? PosMap{n, fb, FS6_F0, nnc, FS_NC, FS6_F0 + FS6_NF}
                      : fsok ? PosMap{n, fb, FS_F0, nnc, FS_NC, FS_F0 + FS_NF}
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
    const int split = pm.fl == FS6_F0         ? passes_fs(FLShape<FS_NC, FS6_F0, FS6_NF>{})
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

/* ---------------- one p.stepSimulation() (oracle substep()) ---------------- */
__device__ __forceinline__ static void team_substep(const Scene* s, double* ws) {
    Shared& sh = g_sh;
    const int lane = threadIdx.x;
    EnvState& e = sh.e;
#ifdef UG_PROF
    unsigned long long fsnap = lane < UG_FREE_SPLIT_N ? sh.prof[kFreeSplit[lane]] : 0ull; /* lane i: counter i */
#endif
    PROF_T0(t_col);
    serial_fk();
    __syncthreads();
    PROF_ADD(PF_FK, t_col);
    const double ov0 = e.overflow;
    if (s->gjk) {
        if (s->full) {
            if (!(uniform(sh.qsvalid) && quiescent_ok(s, ws))) team_collide<true, true>(s, ws);
            else PROF_CNT(PC_QUIET, 1);
        } else team_collide<false, true>(s, ws);
    } else {
        if (s->full) team_collide<true, false>(s, ws);
        else team_collide<false, false>(s, ws);
    }
    const double ov1 = e.overflow;
    if (lane == 0) {
        sh.stats[UG_STAT_SUBSTEPS]++;
        if (ov1 != ov0) { sh.stats[UG_STAT_MANCAP]++; sh.flags |= UG_FLAG_DROPPED; }
    }
    PROF_ADD(PF_COLLIDE, t_col);
    PROF_T0(t_dyn);
    serial_pre(s);
    __syncthreads();
    if (lane == 0 && e.overflow != ov1) { sh.stats[UG_STAT_ROWCAP]++; sh.flags |= UG_FLAG_DROPPED; }
    PROF_ADD(PF_DYN, t_dyn);
    PROF_T0(t_rows);
    const int n = uniform(sh.nrows), nnc = uniform(sh.nnc), nn = uniform(sh.nn);
    PROF_CNT(PC_SUBSTEPS, 1);
    PROF_CNT(PC_ROWS, n);
    PROF_CNT(PC_NNC, nnc);
    PROF_CNT(PC_NN, nn);
    PROF_CNT(PC_N64, n <= 64);
    PROF_CNT(PC_N80, n > 64 && n <= 80);
    PROF_CNT(PC_N96, n > 80 && n <= 96);
    PROF_CNT(PC_OVL, sh.nov);
    PROF_CNT(PC_NMAN, (int)e.nman);
    /* rows: built lane-per-row into the workspace (J | M^-1 J^T) and LDS (scalars) */
    PROF_T0(t_unit);
    team_unit_solves();
    PROF_ADD(PF_UNIT, t_unit);
    PROF_T0(t_rowb);
    /* the motor / gear solve (team_pgs's direct path) reads its Delassus rows and M^-1 J^T from the unit
     * solves in LDS: its J | M^-1 J^T stay out of the workspace */
#ifdef UG_DEBUG_DUMP
    const bool nc_direct = false;
#else
    const bool nc_direct = n == 12 && nnc == 12 && ballot(lane < 12 && sh.rs[lane].kind == 0) == 0ull;
#endif
    for (int p = lane; p < n; p += TEAM) build_row(s, p, ws + WS_ROWS + p * RS, !nc_direct);
    PROF_ADD(PF_ROWB, t_rowb);
    __threadfence_block();
    __syncthreads();
    PROF_ADD(PF_ROWS, t_rows);
    PROF_T0(t_pgs);
    double dv, dvs;
    int split = team_pgs(ws, n, nnc, nn, s->nobj, dv, dvs);
    if (lane == 0 && split) sh.stats[UG_STAT_SPLIT]++;
    PROF_ADD(PF_PGS, t_pgs);
    PROF_T0(t_int);
    if (lane < NVP) { sh.dvout[lane] = dv; sh.dvsout[lane] = dvs; }
    /* impulses back into the manifold points (lane per row) */
    for (int p = nnc + lane; p < n; p += TEAM) {
        const RowS& r = sh.rs[p];
        StPt& pt = e.man[r.a].pt[r.b];
        if (r.kind == 3) pt.imp = r.imp;
        else if (r.kind == 4) pt.imp1 = r.imp;
        else if (r.kind == 5) pt.imp2 = r.imp;
    }
    __syncthreads();
    serial_post(s, split);
    __syncthreads();
    PROF_ADD(PF_INTEG, t_int);
#ifdef UG_PROF
    if (n == 12 && nnc == 12) { /* contact-free substeps (most of a reset's settling) on their own */
        PROF_CNT(PC_FREE, 1);
        PROF_CNT(PF_FREE_COL, t_dyn - t_col);
        PROF_CNT(PF_FREE_DYN, t_rows - t_dyn);
        PROF_CNT(PF_FREE_ROWS, t_pgs - t_rows);
        PROF_CNT(PF_FREE_PGS, t_int - t_pgs);
        PROF_ADD(PF_FREE_INT, t_int);
    }
    __syncthreads();
    if (n == 12 && nnc == 12 && lane < UG_FREE_SPLIT_N) sh.prof[PF_FREE_SUB0 + lane] += sh.prof[kFreeSplit[lane]] - fsnap;
    __syncthreads();
#endif
}

/* ---------------- robot control + BallBalance glue (lane 0 unless noted) ---------------- */
__device__ static inline void set_gripper(EnvState& e, double L) {
    e.mtarget[6] = gripper_angle(L);
    e.mon[6] = 1.0;
}
__device__ static inline void open_gripper(EnvState& e, double pct) {
    set_gripper(e, UG_GRIP_MIN + (UG_GRIP_MAX - UG_GRIP_MIN) * (pct / 100.0));
}
__device__ static inline void close_gripper(EnvState& e, double pct) {
    set_gripper(e, UG_GRIP_MAX - (UG_GRIP_MAX - UG_GRIP_MIN) * (pct / 100.0));
}
__device__ static void move_ee_end(EnvState& e, v3 pos, q4 orn) {
    double qt[NB];
    ik_solve(e.q, pos, orn, qt);
    for (int i = 0; i < 6; i++) { e.mtarget[i] = qt[i]; e.mon[i] = 1.0; }
}
__device__ static void link_state_of(const double* q, int l, v3& p, q4& o) {
    Kin k;
    fk(q, k);
    m3 R;
    link_frame(k, l, 1, R, p);
    o = mquat(R);
}
__device__ static v3 gripper_center(const double* q) {
    Kin k;
    fk(q, k);
    v3 lo = V(1e300, 1e300, 1e300), hi = V(-1e300, -1e300, -1e300);
    const int links[2] = {11, 16};
    for (int i = 0; i < 2; i++) {
        int l = links[i];
        m3 R;
        v3 p;
        link_frame(k, l, 1, R, p);
        v3 c = vadd(mv(R, V(UG_LINK_AABB_C[3 * l], UG_LINK_AABB_C[3 * l + 1], UG_LINK_AABB_C[3 * l + 2])), p);
        v3 hh = V(UG_LINK_AABB_H[3 * l], UG_LINK_AABB_H[3 * l + 1], UG_LINK_AABB_H[3 * l + 2]);
        const double* r = R.m;
        v3 ext = V(ug_fabs(r[0]) * hh.x + ug_fabs(r[1]) * hh.y + ug_fabs(r[2]) * hh.z,
                   ug_fabs(r[3]) * hh.x + ug_fabs(r[4]) * hh.y + ug_fabs(r[5]) * hh.z,
                   ug_fabs(r[6]) * hh.x + ug_fabs(r[7]) * hh.y + ug_fabs(r[8]) * hh.z);
        v3 mn = vsub(c, ext), mx = vadd(c, ext);
        lo = V(ug_min(lo.x, mn.x), ug_min(lo.y, mn.y), ug_min(lo.z, mn.z));
        hi = V(ug_max(hi.x, mx.x), ug_max(hi.y, mx.y), ug_max(hi.z, mx.z));
    }
    return V((hi.x + lo.x) / 2.0, (hi.y + lo.y) / 2.0, (hi.z + lo.z) / 2.0);
}
__device__ static void drop_manifolds_of(EnvState& e, const Scene* s, int c0, int c1) {
    int k = 0, nm = (int)e.nman;
    for (int m = 0; m < nm; m++) {
        const PairDef& P = s->pair[(int)e.man[m].pair];
        if ((P.a >= c0 && P.a < c1) || (P.b >= c0 && P.b < c1)) continue;
        if (k != m) e.man[k] = e.man[m];
        k++;
    }
    e.nman = (double)k;
}
__device__ static void remove_object(EnvState& e, const Scene* s, int o) {
    e.oactive[o] = 0.0;
    int c0 = s->ocol[o], c1 = c0 + s->oncol[o];
    int k = 0, nm = (int)e.nman;
    for (int m = 0; m < nm; m++) {
        const PairDef& P = s->pair[(int)e.man[m].pair];
        if ((P.a >= c0 && P.a < c1) || (P.b >= c0 && P.b < c1)) continue;
        if (k != m) e.man[k] = e.man[m];
        k++;
    }
    e.nman = (double)k;
}
__device__ static void place_object(EnvState& e, int o, v3 pos, q4 orn) {
    e.oactive[o] = 1.0;
    e.obj[o].pos = pos;
    e.obj[o].quat = orn;
    e.obj[o].v = V(0, 0, 0);
    e.obj[o].w = V(0, 0, 0);
}
/* random.uniform(a, b) from the env's stream, or from a caller-supplied draw in [0,1) */
struct Draws {
    Rng rng;
    const double* given;
    int k;
    /* one random.random(): the caller's reset draw when given, else the env's MT19937 stream */
    __device__ double next() { return given ? given[k++] : mt_random(rng); }
    __device__ double uniform(double a, double b) { return ugg_uniform(a, b, next()); }
};
__device__ static void bb_obs(const EnvState& e, double* obs) {
    v3 eu = euler_from_quat(e.obj[0].quat);
    obs[0] = eu.x; obs[1] = eu.y; obs[2] = eu.z;
    obs[3] = e.obj[0].pos.x - e.obj[1].pos.x;
    obs[4] = e.obj[0].pos.y - e.obj[1].pos.y;
    obs[5] = e.obj[0].pos.z - e.obj[1].pos.z;
}
/* p.getContactPoints existence: a manifold point between a robot link in [lmin, lmax]
 * and collider cb (robot colliders are always side A of their pairs) */
__device__ static int robot_contact(const EnvState& e, const Scene* s, int cb, int lmin, int lmax) {
    int nm = (int)e.nman;
    for (int m = 0; m < nm; m++) {
        const PairDef& P = s->pair[(int)e.man[m].pair];
        if (e.man[m].npts <= 0.0 || P.b != cb) continue;
        int l = s->col[P.a].link;
        if (l >= lmin && l <= lmax) return 1;
    }
    return 0;
}
__device__ static int static_collider(const Scene* s, int ent) {
    for (int i = 0; i < s->ncol; i++)
        if (s->col[i].ent == ent) return i;
    return -1;
}
__device__ static void move_ee_joint(EnvState& e, const double* q6) {
    for (int i = 0; i < 6; i++) { e.mtarget[i] = q6[i]; e.mon[i] = 1.0; }
}
/* CubesPush obs (env_cubes_push_v0.py:196-205) */
__device__ static void cp_obs(const EnvState& e, double* obs) {
    v3 pe;
    q4 oe;
    link_state_of(e.q, UG_EE_LINK, pe, oe);
    obs[0] = pe.x; obs[1] = pe.y; obs[2] = pe.z;
    for (int o = 0; o < 2; o++) { obs[3 + 3 * o] = e.obj[o].pos.x; obs[4 + 3 * o] = e.obj[o].pos.y; obs[5 + 3 * o] = e.obj[o].pos.z; }
}
/* CubesGrasp: opening from link frames 11/16 (env_cubes_grasp_v0.py:349-376) */
__device__ static double cg_opening(const EnvState& e) {
    Kin k;
    fk(e.q, k);
    m3 R1, R2;
    v3 p1, p2;
    link_frame(k, 11, 0, R1, p1);
    link_frame(k, 16, 0, R2, p2);
    return ugg_cg_opening(ug_norm3(p2.x - p1.x, p2.y - p1.y, p2.z - p1.z));
}
__device__ static void cg_obs(const EnvState& e, double* obs) {
    /* :268-287 */
    v3 pe;
    q4 oe;
    link_state_of(e.q, UG_EE_LINK, pe, oe);
    obs[0] = e.goal_approached; obs[1] = e.goal_grasped;
    obs[2] = pe.x; obs[3] = pe.y; obs[4] = pe.z; obs[5] = oe.x; obs[6] = oe.y; obs[7] = oe.z; obs[8] = oe.w;
    obs[9] = cg_opening(e);
    obs[10] = e.obj[0].pos.x; obs[11] = e.obj[0].pos.y; obs[12] = e.obj[0].pos.z;
    obs[13] = e.obj[0].quat.x; obs[14] = e.obj[0].quat.y; obs[15] = e.obj[0].quat.z; obs[16] = e.obj[0].quat.w;
}
/* Golf: any manifold point between colliders [a0, a1) and [b0, b1) (either side of the pair) */
__device__ static int pair_contact(const EnvState& e, const Scene* s, int a0, int a1, int b0, int b1) {
    int nm = (int)e.nman;
    for (int m = 0; m < nm; m++) {
        const PairDef& P = s->pair[(int)e.man[m].pair];
        if (e.man[m].npts <= 0.0) continue;
        if ((P.a >= a0 && P.a < a1 && P.b >= b0 && P.b < b1) || (P.b >= a0 && P.b < a1 && P.a >= b0 && P.a < b1))
            return 1;
    }
    return 0;
}
/* club reference point at base-frame height zoff: composite COM + R (0, 0, zoff - zc) */
__device__ static v3 club_point(const EnvState& e, double zoff) {
    m3 R = qmat(e.obj[0].quat);
    return vadd(e.obj[0].pos, mv(R, V(0.0, 0.0, zoff - UG_GF_ZC)));
}
__device__ static void gf_obs(const EnvState& e, double* obs) {
    v3 st = club_point(e, UG_GF_FOOT_Z);
    double stick[3] = {st.x, st.y, st.z}, ball[3] = {e.obj[1].pos.x, e.obj[1].pos.y, e.obj[1].pos.z};
    double hole[3] = {UG_GF_PITCH_X, UG_GF_PITCH_Y, UG_GF_PITCH_Z};
    ugg_gf_obs(stick, ball, hole, obs);
}
/* CubesPushDiff obs (env_cubes_push_diff_v0.py:202-212): ee position, each cube minus the ee position */
__device__ static void cpd_obs(const EnvState& e, double* obs) {
    v3 pe;
    q4 oe;
    link_state_of(e.q, UG_EE_LINK, pe, oe);
    obs[0] = pe.x; obs[1] = pe.y; obs[2] = pe.z;
    for (int o = 0; o < 2; o++) {
        obs[3 + 3 * o] = e.obj[o].pos.x - pe.x; obs[4 + 3 * o] = e.obj[o].pos.y - pe.y; obs[5 + 3 * o] = e.obj[o].pos.z - pe.z;
    }
}
/* TwoBallsBalance obs (env_two_balls_balance_v0.py:157-163): paddle euler, paddle - ball 1, paddle - ball 2 */
__device__ static void tb_obs(const EnvState& e, double* obs) {
    v3 eu = euler_from_quat(e.obj[0].quat);
    obs[0] = eu.x; obs[1] = eu.y; obs[2] = eu.z;
    for (int b = 0; b < 2; b++) {
        obs[3 + 3 * b] = e.obj[0].pos.x - e.obj[1 + b].pos.x;
        obs[4 + 3 * b] = e.obj[0].pos.y - e.obj[1 + b].pos.y;
        obs[5 + 3 * b] = e.obj[0].pos.z - e.obj[1 + b].pos.z;
    }
}
/* non-finite state guard (oracle state_finite): q, qd and the active objects' state */
__device__ static int state_finite(const Scene* s, const EnvState& e) {
    for (int i = 0; i < NB; i++)
        if (!__builtin_isfinite(e.q[i]) || !__builtin_isfinite(e.qd[i])) return 0;
    for (int o = 0; o < s->nobj; o++) {
        if (e.oactive[o] == 0.0) continue;
        const double* v = &e.obj[o].pos.x;
        for (int j = 0; j < UG_OBJ_DOUBLES; j++)
            if (!__builtin_isfinite(v[j])) return 0;
    }
    return 1;
}
/* a reset of a non-finite state starts from a clean robot (oracle sanitize) */
__device__ static void sanitize(const Scene* s, EnvState& e) {
    if (state_finite(s, e)) return;
    for (int i = 0; i < NB; i++) { e.q[i] = 0.0; e.qd[i] = 0.0; }
    for (int m = 0; m < 7; m++) { e.mtarget[m] = 0.0; e.mon[m] = 0.0; }
    for (int o = 0; o < MAXOBJ; o++) {
        e.oactive[o] = 0.0;
        e.obj[o].pos = V(0, 0, 0); e.obj[o].quat = Q(0, 0, 0, 0); e.obj[o].v = V(0, 0, 0); e.obj[o].w = V(0, 0, 0);
    }
    e.nman = 0.0;
}
/* ---- Box (env_box_v0.py; oracle bx_*) ---- */
/* get_ee_pose() in world coordinates: the robot base stands at (0, UG_BX_ROBOT_Y, 0) */
__device__ __forceinline__ static void bx_ee_world(const EnvState& e, double* w7) {
    v3 pe;
    q4 oe;
    link_state_of(e.q, UG_EE_LINK, pe, oe);
    w7[0] = pe.x; w7[1] = pe.y + UG_BX_ROBOT_Y; w7[2] = pe.z;
    w7[3] = oe.x; w7[4] = oe.y; w7[5] = oe.z; w7[6] = oe.w;
}
/* move_ee(world pose, 'end'): the target taken into the base frame (position shifted back, orientation through
 * btMatrix3x3 setRotation / getRotation) */
__device__ static void bx_move_ee(EnvState& e, const double* w7) {
    const m3 R = qmat(Q(w7[3], w7[4], w7[5], w7[6]));
    move_ee_end(e, V(w7[0], w7[1] - UG_BX_ROBOT_Y, w7[2]), mquat(R));
}
/* reset_box (:172-177): both joints to 0 at rest, the link frames follow */
__device__ static void bx_place(const Scene* s, EnvState& e) {
    for (int o = 0; o < 2; o++) {
        e.oactive[o] = 1.0;
        e.obj[o].v = V(0, 0, 0);
        e.obj[o].w = V(0, 0, 0);
        double qt[4], pt[3];
        ugj_frame(&s->ojoint[o], 0.0, qt, pt);
        e.obj[o].quat = Q(qt[0], qt[1], qt[2], qt[3]);
        e.obj[o].pos = V(pt[0], pt[1], pt[2]);
    }
}
__device__ static void task_obs(const Scene* s, const EnvState& e, double* obs) {
    if (s->task == UG_TASK_BOX) bx_ee_world(e, obs); /* :161-170 np.array(ee_pos) */
    else if (s->variant == UG_TASK_TWOBALLS) tb_obs(e, obs);
    else if (s->variant == UG_TASK_CUBESPUSHDIFF) cpd_obs(e, obs);
    else if (s->task == UG_TASK_CUBESPUSH) cp_obs(e, obs);
    else if (s->task == UG_TASK_CUBESGRASP) cg_obs(e, obs);
    else if (s->variant == UG_TASK_GOLFJOINTS) { /* env_golf_joints_v0.py:228-235: arm joints, then the Golf obs */
        for (int i = 0; i < 6; i++) obs[i] = e.q[i];
        gf_obs(e, obs + 6);
    } else if (s->task == UG_TASK_GOLF) gf_obs(e, obs);
    else bb_obs(e, obs);
}
/* ---------------- the env program: step / reset as one substep loop ----------------
 * The reference's control flow (env_ball_balance_v0.py: step 105-134, reset 145-170, wait_until_stable
 * 94-103, robot.reset 89-106) is a sequence of glue actions separated by physics loops.  It runs here as
 * a small state machine around a single inlined team_substep(), so the PGS register slots exist once. */
enum { G_STEP = 0, G_STEP_DONE, G_RESET, G_RESET_ROBOT, G_RESET_PLACE, G_RESET_DONE, G_END };
enum { L_NONE = 0, L_FIXED10, L_WAIT, L_FIXED120 };
struct RunIO {
    const float* act;    /* step action (task act_dim floats) */
    double* obs;         /* obs row */
    double* final_obs;   /* final obs row (autoreset) or null */
    Draws dr;            /* reset draws */
    int autoreset, trunc;
    double rew;
    int term, succ, reset_done;
};
/* lane-0 glue of one program point; returns the physics loop to run next and sets *next */
__device__ __noinline__ static int glue(const Scene* s, int pc, RunIO& io, int* next) {
    PROF_CALL(CALL_GLUE);
    EnvState& e = g_sh.e;
    const int task = s->task;
    const int O = UG_OBS_DIM(s->variant);
    switch (pc) {
        case G_STEP: {
            v3 pe;
            q4 oe;
            if (task == UG_TASK_BOX) { /* env_box_v0.py:125-129: ee pose + action, the gripper, 120 substeps */
                double w7[7], t7[7];
                bx_ee_world(e, w7);
                ugg_box_target(w7, io.act, t7);
                bx_move_ee(e, t7);
                e.mtarget[6] = gripper_angle((double)io.act[7]); /* move_gripper(action[-1]) */
                e.mon[6] = 1.0;
                *next = G_STEP_DONE;
                return L_FIXED120;
            }
            if (task == UG_TASK_CUBESGRASP) {
                /* env_cubes_grasp_v0.py:132-158: random.choices picks joint move or gripper command */
                int sel = ugg_cg_choose(io.act[0], io.act[1], io.dr.next());
                if (sel == 0) {
                    double q6[6];
                    for (int i = 0; i < 6; i++) q6[i] = (double)io.act[2 + i];
                    move_ee_joint(e, q6);
                } else if (io.act[8] < 0.5f) {
                    open_gripper(e, 100.0);
                } else {
                    close_gripper(e, 100.0);
                }
            } else if (task == UG_TASK_CUBESPUSH) {
                /* env_cubes_push_v0.py:115-127: EE position + action, vertical orientation */
                link_state_of(e.q, UG_EE_LINK, pe, oe);
                move_ee_end(e, V(pe.x + (double)io.act[0], pe.y + (double)io.act[1], pe.z + (double)io.act[2]),
                            Q(0.0, UG_VQ_S, 0.0, UG_VQ_C));
            } else if (s->variant == UG_TASK_GOLFJOINTS) {
                /* env_golf_joints_v0.py:122-124: arm joint positions + action (float64 + float32 -> float64),
                 * move_ee(..., 'joint') */
                double q6[6];
                for (int i = 0; i < 6; i++) q6[i] = e.q[i] + (double)io.act[i];
                move_ee_joint(e, q6);
            } else if (task == UG_TASK_GOLF) {
                /* env_golf_v0.py:115-127: EE position + action, the reset orientation (0, 0, -0.7, 0.7) */
                link_state_of(e.q, UG_EE_LINK, pe, oe);
                move_ee_end(e, V(pe.x + (double)io.act[0], pe.y + (double)io.act[1], pe.z + (double)io.act[2]),
                            Q(0.0, 0.0, -0.70, 0.70));
            } else {
                /* env_ball_balance_v0.py:105-118: move_ee(end pose + action on the euler angles) */
                link_state_of(e.q, UG_EE_LINK, pe, oe);
                v3 eu = euler_from_quat(oe);
                eu.x += (double)io.act[0]; eu.y += (double)io.act[1]; eu.z += (double)io.act[2];
                move_ee_end(e, pe, quat_from_euler(eu));
            }
            *next = G_STEP_DONE;
            return L_WAIT;
        }
        case G_STEP_DONE:
            if (task == UG_TASK_CUBESPUSH) { /* :129-150 */
                int table = robot_contact(e, s, static_collider(s, 10), 1, UG_NL - 1);
                int touched = robot_contact(e, s, s->ocol[1], 9, 18);
                io.succ = ugg_cp_reward(table, touched, e.obj[0].pos.x, e.obj[0].pos.y, e.obj[0].pos.z, e.obj[1].pos.x,
                                        e.obj[1].pos.y, e.obj[1].pos.z, s->sparse, &io.rew);
                io.term = io.succ;
            } else if (task == UG_TASK_CUBESGRASP) { /* :160-192 */
                v3 gc = gripper_center(e.q);
                double d = ug_norm3(gc.x - e.obj[0].pos.x, gc.y - e.obj[0].pos.y, gc.z - e.obj[0].pos.z);
                int grasp = robot_contact(e, s, s->ocol[0], 11, 13) && robot_contact(e, s, s->ocol[0], 16, 18);
                int app = (int)e.goal_approached, gr = (int)e.goal_grasped;
                io.succ = ugg_cg_reward(&app, &gr, d, cg_opening(e), grasp, e.obj[0].pos.z, &io.rew);
                e.goal_approached = (double)app;
                e.goal_grasped = (double)gr;
                io.term = io.succ;
            } else if (task == UG_TASK_GOLF) { /* env_golf_v0.py:129-183 */
                int c0 = s->ocol[0], c1 = c0 + s->oncol[0], cb = s->ocol[1], cp = static_collider(s, 12);
                int in_fingers = 0;
                for (int c = c0; c < c1; c++) in_fingers |= robot_contact(e, s, c, 9, 18);
                int floor = robot_contact(e, s, cp, 0, UG_NL - 1) || pair_contact(e, s, c0, c1, cp, cp + 1);
                int touched = pair_contact(e, s, cb, cb + 1, c0, c1);
                v3 st = club_point(e, UG_GF_FOOT_Z);
                double stick[3] = {st.x, st.y, st.z}, ball[3] = {e.obj[1].pos.x, e.obj[1].pos.y, e.obj[1].pos.z};
                double hole[3] = {UG_GF_PITCH_X, UG_GF_PITCH_Y, UG_GF_PITCH_Z};
                io.succ = ugg_gf_reward(ball, hole, stick, in_fingers, floor, touched, s->sparse, &io.rew, &io.term);
            } else if (task == UG_TASK_BOX) { /* env_box_v0.py:131-139, update_reward :141-159 */
                const int bc = s->ocol[1];
                int press = ugg_box_press(e.obj[1].w.x, s->button_mode, robot_contact(e, s, bc, 0, UG_NL - 1),
                                          robot_contact(e, s, bc, 9, 18));
                int op = (int)e.goal_approached, pr = (int)e.goal_grasped, cl = (int)e.spare;
                io.term = ugg_box_reward(&op, &pr, &cl, e.obj[0].w.x, press, &io.rew);
                e.goal_approached = (double)op;
                e.goal_grasped = (double)pr;
                e.spare = (double)cl;
                io.succ = io.term;
            } else if (s->variant == UG_TASK_TWOBALLS) { /* env_two_balls_balance_v0.py:110-146 */
                double b1[3] = {e.obj[1].pos.x, e.obj[1].pos.y, e.obj[1].pos.z};
                double b2[3] = {e.obj[2].pos.x, e.obj[2].pos.y, e.obj[2].pos.z};
                io.term = ugg_tb_reward(io.act, b1, b2, e.obj[0].pos.z, &io.rew);
                io.succ = 0;
            } else { /* env_ball_balance_v0.py:119-134: reward 1, terminated when the ball falls below the paddle */
                io.rew = 1.0;
                io.term = e.obj[1].pos.z < e.obj[0].pos.z;
                io.succ = 0;
            }
            if (!state_finite(s, e)) { /* end the episode, zero reward; the autoreset restarts from a clean state */
                io.term = 1;
                io.succ = 0;
                io.rew = 0.0;
                g_sh.flags |= UG_FLAG_NONFINITE;
                g_sh.stats[UG_STAT_NONFINITE]++;
            }
            task_obs(s, e, io.obs);
            if (io.autoreset && (io.term || io.trunc)) {
                if (io.final_obs)
                    for (int j = 0; j < O; j++) io.final_obs[j] = io.obs[j];
                *next = G_RESET;
                return L_NONE;
            }
            *next = G_END;
            return L_NONE;
        case G_RESET: /* robot.reset(): reset_arm (rest pose) + 10 substeps */
            sanitize(s, e);
            e.goal_approached = 0.0;
            e.goal_grasped = 0.0;
            e.spare = 0.0; /* Box: box_closed */
            for (int i = 0; i < 6; i++) { e.q[i] = UG_ARM_REST[i]; e.qd[i] = 0.0; }
            *next = G_RESET_ROBOT;
            return L_FIXED10;
        case G_RESET_ROBOT: /* reset_gripper (open 100), then the task's scene and start pose */
            open_gripper(e, 100.0);
            if (task == UG_TASK_BOX) { /* env_box_v0.py:181-184: move_ee(get_ee_pose(), 'end'), reset_box(); no settling */
                double w7[7];
                bx_ee_world(e, w7);
                bx_move_ee(e, w7);
                bx_place(s, e);
                *next = G_RESET_DONE;
                return L_NONE;
            }
            for (int o = 0; o < s->nobj; o++) remove_object(e, s, o);
            if (task == UG_TASK_CUBESPUSH) { /* env_cubes_push_v0.py:207-227, create_cubes :240-246 */
                place_object(e, 0, V(0.0, -0.5, 0.1), Q(0, 0, 0, 1));
                double x = ugg_cp_cube1_x(io.dr.next());
                place_object(e, 1, V(x, -0.7, 0.1), Q(0, 0, 0, 1));
                move_ee_end(e, V(x, -0.7, 0.1 + UG_CP_EE_DZ), Q(0.0, UG_VQ_S, 0.0, UG_VQ_C));
                close_gripper(e, 100.0);
                *next = G_RESET_DONE;
            } else if (task == UG_TASK_CUBESGRASP) { /* env_cubes_grasp_v0.py:289-307, create_cubes :310-330 */
                double u0 = io.dr.next(), u1 = io.dr.next(), x, y;
                ugg_cg_cube_xy(u0, u1, &x, &y);
                place_object(e, 0, V(x, y, 0.1), Q(0, 0, 0, 1));
                v3 pe;
                q4 oe;
                link_state_of(e.q, UG_EE_LINK, pe, oe);
                move_ee_end(e, pe, oe);
                *next = G_RESET_DONE;
            } else if (task == UG_TASK_GOLF) { /* env_golf_v0.py:238-252: pitch re-created, start pose, open 20% */
                int cp = static_collider(s, 12);
                drop_manifolds_of(e, s, cp, cp + 1);
                move_ee_end(e, V(0.0, -0.60, 0.40), Q(0.0, 0.0, -0.70, 0.70));
                open_gripper(e, 20.0);
                *next = G_RESET_PLACE;
            } else { /* env_ball_balance_v0.py:145-160: move_ee(start pose); open 20% */
                move_ee_end(e, V(0.0, -0.60, 0.60), Q(0.50, -0.50, -0.50, 0.50));
                open_gripper(e, 20.0);
                *next = G_RESET_PLACE;
            }
            return L_WAIT;
        case G_RESET_PLACE: { /* BallBalance: paddle between the fingers, ball above it; close gripper */
            if (task == UG_TASK_GOLF) { /* env_golf_v0.py:254-265: club under the gripper centre, ball; close */
                v3 gc = gripper_center(e.q);
                place_object(e, 0, V(gc.x, gc.y, gc.z - 0.05 + UG_GF_ZC), Q(0, 0, 0, 1));
                double u0 = io.dr.next(), u1 = io.dr.next(), bx, by;
                ugg_gf_ball_xy(u0, u1, &bx, &by);
                place_object(e, 1, V(bx, by, 0.1), Q(0, 0, 0, 1));
                close_gripper(e, 100.0);
                *next = G_RESET_DONE;
                return L_WAIT;
            }
            v3 pe;
            q4 oe;
            link_state_of(e.q, UG_EE_LINK, pe, oe);
            v3 gc = gripper_center(e.q);
            v3 pose = V(pe.x, pe.y - 0.2, gc.z);
            place_object(e, 0, pose, Q(0, 0, 0, 1));
            if (s->variant == UG_TASK_TWOBALLS) { /* create_balls(0.003) (env_two_balls_balance_v0.py:212-235) */
                double u[4], pd[3] = {pose.x, pose.y, pose.z}, b1[3], b2[3];
                for (int k = 0; k < 4; k++) u[k] = io.dr.next();
                ugg_tb_balls(pd, UG_TB_BALL_R, u, b1, b2);
                place_object(e, 1, V(b1[0], b1[1], b1[2]), e.obj[0].quat);
                place_object(e, 2, V(b2[0], b2[1], b2[2]), e.obj[0].quat);
            } else {
                v3 bp = V(pose.x, pose.y, pose.z + 0.2 + UG_BB_BALL_R);
                bp.x += io.dr.uniform(-0.03, 0.03);
                bp.y += io.dr.uniform(-0.08, 0.02);
                place_object(e, 1, bp, e.obj[0].quat);
            }
            close_gripper(e, 100.0);
            *next = G_RESET_DONE;
            return L_WAIT;
        }
        case G_RESET_DONE:
            e.goal_approached = 0.0;
            e.goal_grasped = 0.0;
            e.spare = 0.0;
            if (!state_finite(s, e)) { /* a reset that settled into a non-finite state: surfaced (oracle reset_impl) */
                g_sh.flags |= UG_FLAG_NONFINITE;
                g_sh.stats[UG_STAT_NONFINITE]++;
            }
            task_obs(s, e, io.obs);
            io.reset_done = 1;
            *next = G_END;
            return L_NONE;
    }
    *next = G_END;
    return L_NONE;
}
/* wave-wide state_finite(): lane l < NB tests q / qd of dof l, lane NB + j the j-th value of the objects' block
 * (active objects only); one ballot */
__device__ __forceinline__ static int team_nonfinite(const Scene* s) {
    const EnvState& e = g_sh.e;
    const int lane = threadIdx.x;
    bool bad = false;
    if (lane < NB) bad = !__builtin_isfinite(e.q[lane]) || !__builtin_isfinite(e.qd[lane]);
    const int j = lane - NB;
    if (j >= 0 && j < MAXOBJ * UG_OBJ_DOUBLES) {
        const int o = j / UG_OBJ_DOUBLES;
        bad = o < s->nobj && e.oactive[o] != 0.0 && !__builtin_isfinite((&e.obj[0].pos.x)[j]);
    }
    return ballot(bad) != 0ull;
}
/* the non-finite guard voids a runaway state (oracle poison): q, qd and the active objects' state NaN, no contacts */
__device__ __forceinline__ static void team_poison(const Scene* s) {
    EnvState& e = g_sh.e;
    const int lane = threadIdx.x;
    if (lane < NB) { e.q[lane] = __builtin_nan(""); e.qd[lane] = __builtin_nan(""); }
    const int j = lane - NB;
    if (j >= 0 && j < MAXOBJ * UG_OBJ_DOUBLES) {
        const int o = j / UG_OBJ_DOUBLES;
        if (o < s->nobj && e.oactive[o] != 0.0) (&e.obj[0].pos.x)[j] = __builtin_nan("");
    }
    if (lane == 0) e.nman = 0.0;
    __syncthreads();
}
/* runs the program from pc0 to the end; returns physics substeps taken */
__device__ __forceinline__ static int team_run(const Scene* s, double* ws, int pc0, RunIO& io) {
    Shared& sh = g_sh;
    const int lane = threadIdx.x;
    int pc = pc0, ns = 0;
    while (true) {
        PROF_T0(t_glue);
        if (lane == 0) {
            int next;
            sh.is[1] = glue(s, pc, io, &next);
            sh.is[2] = next;
            sh.qsvalid = 0; /* the glue may move, create or remove bodies: the next substep collides in full */
        }
        __syncthreads();
        PROF_ADD(PF_GLUE, t_glue);
        int loop = uniform(sh.is[1]);
        pc = uniform(sh.is[2]);
        if (loop == L_NONE) {
            if (pc == G_END) break;
            continue;
        }
        /* physics: 10 fixed substeps, or wait_until_stable (<= 480 substeps until sum|dq| < eps) */
        double pos = lane < NB ? sh.e.q[lane] : 0.0;
        for (int i = 0;; i++) {
            team_substep(s, ws);
            ns++;
            /* a non-finite state ends the loop at once (oracle wait_until_stable / robot_reset) */
            if (team_nonfinite(s)) {
                team_poison(s);
                break;
            }
            if (loop == L_FIXED10 || loop == L_FIXED120) { /* robot.reset's 10 substeps / Box's 120 per step */
                if (i + 1 == (loop == L_FIXED10 ? 10 : UG_BX_STEPS)) break;
                continue;
            }
            double qn = lane < NB ? sh.e.q[lane] : 0.0;
            if (lane < NB) sh.a12[lane] = ug_fabs(pos - qn);
            __syncthreads();
            if (lane == 0) sh.is[0] = np_sum12(sh.a12) < UG_STABLE_EPS;
            __syncthreads();
            const int stable = uniform(sh.is[0]);
            if (stable || i + 1 == UG_STABLE_STEPS) {
                /* "did not stabilize" (env_ball_balance_v0.py:102-103): surfaced as a flag and a counter */
                if (!stable && lane == 0) { sh.stats[UG_STAT_UNSTABLE]++; sh.flags |= UG_FLAG_UNSTABLE; }
                break;
            }
            pos = qn;
        }
    }
    return ns;
}

/* ---------------- state in/out (cooperative, canonical layout) ---------------- */
__device__ static void team_load(const double* S, const int* stats) {
    Shared& sh = g_sh;
    double* dst = (double*)&sh.e;
    for (int i = threadIdx.x; i < UG_STATE_DIM; i += TEAM) dst[i] = S[i];
    if (threadIdx.x < UG_NSTAT) sh.stats[threadIdx.x] = stats ? stats[threadIdx.x] : 0;
    if (threadIdx.x == 0) { sh.flags = 0; sh.qsvalid = 0; }
    if (threadIdx.x < NB) {
        int m = 0;
        for (int b = threadIdx.x; b >= 0; b = UG_BODY_PARENT[b]) m |= 1 << b;
        sh.anc[threadIdx.x] = m;
        sh.bdepth[threadIdx.x] = body_depth(threadIdx.x);
    }
#ifdef UG_PROF
    for (int i = threadIdx.x; i < UG_NPROF; i += TEAM) sh.prof[i] = 0;
#endif
    __syncthreads();
}
__device__ static void team_prof_flush() {
    Shared& sh = g_sh;
#ifdef UG_PROF
    __syncthreads();
    for (int i = threadIdx.x; i < UG_NPROF; i += TEAM) atomicAdd(&g_prof[i], sh.prof[i]);
#endif
}
/* BallBalance / TwoBalls reset predictor inputs (scheduling only): ball o in the paddle frame -> its paddle-frame
 * offset, velocities and in-plane gravity and the log times of an edge-roll + free-fall estimate (14 inputs,
 * tools/fit_priority.py features()) */
__device__ static void bb_ball_inputs(const EnvState& e, const m3& R, int o, double (&x)[UG_PM_IN]) {
    const v3 l = mtv(R, vsub(e.obj[o].pos, e.obj[0].pos));
    const v3 lv = mtv(R, vsub(e.obj[o].v, e.obj[0].v));
    const v3 gl = mtv(R, V(0.0, 0.0, -9.81));
    const double sx = l.x < 0.0 ? -1.0 : (l.x > 0.0 ? 1.0 : 0.0), sy = l.y < 0.0 ? -1.0 : (l.y > 0.0 ? 1.0 : 0.0);
    const double fx = fabs(l.x) / UG_BB_PADDLE_HX, fy = fabs(l.y) / UG_BB_PADDLE_HY;
    const double vx = lv.x * sx, vy = lv.y * sy;
    const double dz = e.obj[o].pos.z - e.obj[0].pos.z, bvz = e.obj[o].v.z;
    const double tf = dz < 0.0 ? 0.0 : (bvz + sqrt(bvz * bvz + 2.0 * 9.81 * dz)) / 9.81;
    const double tex = fx >= 1.0 ? 0.0 : (1.0 - fx) * UG_BB_PADDLE_HX / fmax(vx, 0.05);
    const double tey = fy >= 1.0 ? 0.0 : (1.0 - fy) * UG_BB_PADDLE_HY / fmax(vy, 0.05);
    const double v[UG_PM_IN] = {fx, fy, l.z, vx, vy, lv.z, dz, bvz, gl.x * sx, gl.y * sy,
                                log(fmin(tex, tey) + tf + 1e-3), log(tex + 1e-3), log(tey + 1e-3), log(tf + 1e-3)};
    for (int i = 0; i < UG_PM_IN; i++) x[i] = v[i];
}
/* a 1-hidden-layer ReLU MLP's logit over standardised inputs */
template <int IN, int HID>
__device__ static double mlp_logit(const double* x, const double* mu, const double* sd, const double* W1,
                                   const double* B1, const double* W2, double b2) {
    double z[IN];
    for (int i = 0; i < IN; i++) z[i] = (x[i] - mu[i]) / sd[i];
    double out = b2;
    for (int h = 0; h < HID; h++) {
        double a = B1[h];
        for (int i = 0; i < IN; i++) a += z[i] * W1[i * HID + h];
        out += fmax(a, 0.0) * W2[h];
    }
    return out;
}
/* BallBalance: the logit of "this env ends its episode in the next env-step" from one ball, a 14 -> 16 (ReLU) -> 1 MLP
 * (prio_model.h, tools/fit_priority.py) */
__device__ static double bb_reset_logit(const EnvState& e, const m3& R, int o) {
    double x[UG_PM_IN];
    bb_ball_inputs(e, R, o, x);
    return mlp_logit<UG_PM_IN, UG_PM_HID>(x, UG_PM_MU, UG_PM_SD, UG_PM_W1, UG_PM_B1, UG_PM_W2, UG_PM_B2);
}
/* TwoBallsBalance: one model over both balls' inputs, the episode's elapsed steps and the paddle's vertical velocity,
 * 31 -> 16 (ReLU) -> 1 (prio_model_tb.h, tools/fit_priority.py --task 6): the larger of two single-ball logits
 * ranked the resets where both balls hit the paddle together last (~55 per step, the launch 37 ms against 23.5 ms
 * for the longest-first order) */
__device__ static double tb_reset_logit(const EnvState& e, const m3& R, int el) {
    static_assert(UG_PT_IN == 2 * UG_PM_IN + 3, "two balls' inputs, elapsed (clipped, log) and the paddle's vz");
    double x[UG_PT_IN], b[UG_PM_IN];
    for (int o = 1; o <= 2; o++) {
        bb_ball_inputs(e, R, o, b);
        for (int i = 0; i < UG_PM_IN; i++) x[(o - 1) * UG_PM_IN + i] = b[i];
    }
    x[2 * UG_PM_IN] = fmin((double)el, 10.0);
    x[2 * UG_PM_IN + 1] = log((double)el + 1.0);
    x[2 * UG_PM_IN + 2] = e.obj[0].v.z;
    return mlp_logit<UG_PT_IN, UG_PT_HID>(x, UG_PT_MU, UG_PT_SD, UG_PT_W1, UG_PT_B1, UG_PT_W2, UG_PT_B2);
}
/* Launch-order priority of an env for the next k_step (0..255, higher runs first).  The launch time is the
 * longest env chain, and an env-step that ends its episode carries a ~170-substep autoreset: envs likely
 * to end next step are dispatched first so their reset overlaps the other envs' steps.  Scheduling only --
 * every env computes the same thing whatever its position in the launch.  Predicted truncation: 255;
 * TwoBalls: its own two-ball model (tb_reset_logit) in 255 levels; BallBalance: the reset predictor's logit in 255 levels
 * (held-out random-action BallBalance x 4096:
 * 0.44 of ~270 resets per step ranked outside the first 1024 launch slots, against 1.1 for an edge-roll +
 * free-fall time and 5.8 for a position-extrapolation score); otherwise the env's last substep count. */
#define UG_PM_FINE_L0 -12.0 /* BallBalance's logit in 255 launch levels: [-12, 5.78) in steps of 0.07 */
#define UG_PM_FINE_DL 0.07
__device__ static int logit_level(double lg, double l0, double dl) {
    const double b = floor((lg - l0) / dl);
    return b > 254.0 ? 254 : (b < 0.0 ? 0 : (int)b); /* a NaN logit: level 0 */
}
__device__ static int team_priority(const Scene* s, int nsub, int el_next, int max_steps, int autoreset) {
    const EnvState& e = g_sh.e;
    if (autoreset && max_steps > 0 && el_next >= max_steps) return 255;
    if (s->variant == UG_TASK_TWOBALLS && e.oactive[0] != 0.0 && e.oactive[1] != 0.0 && e.oactive[2] != 0.0)
        return logit_level(tb_reset_logit(e, qmat(e.obj[0].quat), el_next - 1), UG_PT_L0, UG_PT_DL);
    if (s->task == UG_TASK_BALLBALANCE && e.oactive[0] != 0.0) {
        const m3 R = qmat(e.obj[0].quat);
        double lg = -1e300;
        for (int o = 1; o < s->nobj; o++)
            if (e.oactive[o] != 0.0) lg = fmax(lg, bb_reset_logit(e, R, o));
        return logit_level(lg, UG_PM_FINE_L0, UG_PM_FINE_DL);
    }
    int b = 0;
    while (b < 14 && (2 << b) <= nsub) b++;
    return b;
}
/* manifold slots beyond nman are written as (pair -1, zeros), as ugo_get_state does */
__device__ static void team_store(double* S, int* stats, uint8_t* flags) {
    const Shared& sh = g_sh;
    __syncthreads();
    if (stats && threadIdx.x < UG_NSTAT) stats[threadIdx.x] = sh.stats[threadIdx.x];
    if (flags && threadIdx.x == 0) *flags = (uint8_t)sh.flags;
    const double* src = (const double*)&sh.e;
    int nm = (int)sh.e.nman;
    for (int i = threadIdx.x; i < UG_STATE_DIM; i += TEAM) {
        double v = src[i];
        if (i >= UG_F_MAN && i < UG_F_TASK) {
            int m = (i - UG_F_MAN) / UG_MAN_DOUBLES, f = (i - UG_F_MAN) % UG_MAN_DOUBLES;
            if (m >= nm) v = f == 0 ? -1.0 : 0.0;
        }
        S[i] = v;
    }
}

}  // namespace ugd
#endif
