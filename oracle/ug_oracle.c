/* ug_oracle.c -- CPU restatement of URGym's hot path (TEST INFRASTRUCTURE ONLY).
 *
 * Plain C99, one environment at a time, array-of-structs, no vectorisation:
 * the readable statement of the algorithm that the HIP kernels in
 * urgym_amd/csrc must reproduce bit-for-bit (same operation order, no FMA
 * contraction: build with -ffp-contract=off; transcendentals from
 * urgym_amd/csrc/ug_detmath.h).  See ug_oracle.h for scope and DESIGN.md for
 * the Bullet behaviours restated here ([ext] = from Bullet/PyBullet, not
 * checkable in this build).
 */
#include "ug_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifdef UG_MODEL_DATA /* collision-fidelity builds (tools/collision_fidelity.py) swap in their model header */
#include UG_MODEL_DATA
#elif defined(UG_ROBOT_R140) /* the UR5Robotiq140 restatement (libugoracle_r140.so, robot.py:221-240) */
#include "../urgym_amd/csrc/model_data_r140.h"
#else
#include "../urgym_amd/csrc/model_data.h"
#endif
#include "../urgym_amd/csrc/scene_data.h"
#include "../urgym_amd/csrc/ug_detmath.h"
#include "../urgym_amd/csrc/ug_glue.h"
#include "../urgym_amd/csrc/ug_joint.h"
#include "../urgym_amd/csrc/ug_layout.h"
#include "../urgym_amd/csrc/ug_render.h"

#define NB UG_NB
#define MAXOBJ UG_MAXOBJ
#define NV (NB + 6 * MAXOBJ)
#define MAXMAN UG_MAXMAN
#define MAXROWS 128
#define MAXCOL 28
#define MAXPAIR 192
#ifndef MAXCAND
#define MAXCAND 1024 /* candidate storage: a full hull's vertices + the box corners (UG_FULL_HULL_MAXV + 8) */
#endif
#ifndef LOD_MAXCAND
#define LOD_MAXCAND 64 /* candidates a hull pair keeps with the LOD hulls (the kernels' LDS list) */
#endif
#define PT_DOUBLES UG_PT_DOUBLES
#define MAN_DOUBLES UG_MAN_DOUBLES
#define STATE_DIM UG_STATE_DIM

/* ======================================================================== */
/* small linear algebra (fixed evaluation order, mirrored by the HIP side)   */
/* ======================================================================== */
typedef struct { double x, y, z; } v3;
typedef struct { double m[9]; } m3; /* row-major */
typedef struct { double x, y, z, w; } q4;

static v3 V(double x, double y, double z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
static v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static v3 vscale(v3 a, double s) { return V(a.x * s, a.y * s, a.z * s); }
static v3 vneg(v3 a) { return V(-a.x, -a.y, -a.z); }
static double vdot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static v3 vcross(v3 a, v3 b) { return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
static double vlen(v3 a) { return ug_sqrt(vdot(a, a)); }
static v3 mv(const m3* M, v3 v) {
    const double* m = M->m;
    return V(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[3] * v.x + m[4] * v.y + m[5] * v.z,
             m[6] * v.x + m[7] * v.y + m[8] * v.z);
}
static v3 mtv(const m3* M, v3 v) { /* M^T v */
    const double* m = M->m;
    return V(m[0] * v.x + m[3] * v.y + m[6] * v.z, m[1] * v.x + m[4] * v.y + m[7] * v.z,
             m[2] * v.x + m[5] * v.y + m[8] * v.z);
}
static m3 mm(const m3* A, const m3* B) {
    m3 C;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            C.m[3 * i + j] = A->m[3 * i] * B->m[j] + A->m[3 * i + 1] * B->m[3 + j] + A->m[3 * i + 2] * B->m[6 + j];
    return C;
}
static m3 mtm(const m3* A, const m3* B) { /* A^T B */
    m3 C;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            C.m[3 * i + j] = A->m[i] * B->m[j] + A->m[3 + i] * B->m[3 + j] + A->m[6 + i] * B->m[6 + j];
    return C;
}
static m3 mload(const double* p) { m3 r; memcpy(r.m, p, sizeof(r.m)); return r; }
static m3 mident(void) { m3 r; memset(r.m, 0, sizeof(r.m)); r.m[0] = r.m[4] = r.m[8] = 1.0; return r; }
/* symmetric inertia (xx,yy,zz,xy,xz,yz) in frame R -> world: R I R^T */
static m3 inertia_world(const m3* R, const double* I6) {
    m3 I;
    I.m[0] = I6[0]; I.m[4] = I6[1]; I.m[8] = I6[2];
    I.m[1] = I.m[3] = I6[3]; I.m[2] = I.m[6] = I6[4]; I.m[5] = I.m[7] = I6[5];
    m3 T = mm(R, &I);
    m3 C;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            C.m[3 * i + j] = T.m[3 * i] * R->m[3 * j] + T.m[3 * i + 1] * R->m[3 * j + 1] + T.m[3 * i + 2] * R->m[3 * j + 2];
    return C;
}
/* Rodrigues rotation about unit axis a by angle q */
static m3 axis_angle(v3 a, double q) {
    double c = ug_cos(q), s = ug_sin(q), t = 1.0 - c;
    m3 R;
    R.m[0] = t * a.x * a.x + c;       R.m[1] = t * a.x * a.y - s * a.z; R.m[2] = t * a.x * a.z + s * a.y;
    R.m[3] = t * a.x * a.y + s * a.z; R.m[4] = t * a.y * a.y + c;       R.m[5] = t * a.y * a.z - s * a.x;
    R.m[6] = t * a.x * a.z - s * a.y; R.m[7] = t * a.y * a.z + s * a.x; R.m[8] = t * a.z * a.z + c;
    return R;
}
static q4 Q(double x, double y, double z, double w) { q4 r; r.x = x; r.y = y; r.z = z; r.w = w; return r; }
/* btQuaternion operator* (Hamilton product, (x,y,z,w)) */
static q4 qmul(q4 a, q4 b) {
    return Q(a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z,
             a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z);
}
static q4 qnormalize(q4 a) {
    double l = ug_sqrt(a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w);
    return Q(a.x / l, a.y / l, a.z / l, a.w / l);
}
/* btMatrix3x3::setRotation */
static m3 qmat(q4 q) {
    double d = q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w;
    double s = 2.0 / d;
    double xs = q.x * s, ys = q.y * s, zs = q.z * s;
    double wx = q.w * xs, wy = q.w * ys, wz = q.w * zs;
    double xx = q.x * xs, xy = q.x * ys, xz = q.x * zs;
    double yy = q.y * ys, yz = q.y * zs, zz = q.z * zs;
    m3 R;
    R.m[0] = 1.0 - (yy + zz); R.m[1] = xy - wz; R.m[2] = xz + wy;
    R.m[3] = xy + wz; R.m[4] = 1.0 - (xx + zz); R.m[5] = yz - wx;
    R.m[6] = xz - wy; R.m[7] = yz + wx; R.m[8] = 1.0 - (xx + yy);
    return R;
}
/* btMatrix3x3::getRotation */
static q4 mquat(const m3* M) {
    const double* m = M->m;
    double trace = m[0] + m[4] + m[8];
    double t[4];
    if (trace > 0.0) {
        double s = ug_sqrt(trace + 1.0);
        t[3] = s * 0.5;
        s = 0.5 / s;
        t[0] = (m[7] - m[5]) * s;
        t[1] = (m[2] - m[6]) * s;
        t[2] = (m[3] - m[1]) * s;
    } else {
        int i = m[0] < m[4] ? (m[4] < m[8] ? 2 : 1) : (m[0] < m[8] ? 2 : 0);
        int j = (i + 1) % 3, k = (i + 2) % 3;
        double s = ug_sqrt(m[4 * i] - m[4 * j] - m[4 * k] + 1.0);
        t[i] = s * 0.5;
        s = 0.5 / s;
        t[3] = (m[3 * k + j] - m[3 * j + k]) * s;
        t[j] = (m[3 * j + i] + m[3 * i + j]) * s;
        t[k] = (m[3 * k + i] + m[3 * i + k]) * s;
    }
    return Q(t[0], t[1], t[2], t[3]);
}

/* pybullet.c getEulerFromQuaternion / getQuaternionFromEuler [ext] (used by env_ball_balance_v0.py:114-116,139) */
static v3 euler_from_quat(q4 q) {
    double sqx = q.x * q.x, sqy = q.y * q.y, sqz = q.z * q.z, squ = q.w * q.w;
    double sarg = -2.0 * (q.x * q.z - q.w * q.y);
    v3 r;
    if (sarg <= -0.99999) {
        r.x = 0.0; r.y = -0.5 * UG_PI; r.z = 2.0 * ug_atan2(q.x, -q.y);
    } else if (sarg >= 0.99999) {
        r.x = 0.0; r.y = 0.5 * UG_PI; r.z = 2.0 * ug_atan2(-q.x, q.y);
    } else {
        r.x = ug_atan2(2.0 * (q.y * q.z + q.w * q.x), squ - sqx - sqy + sqz);
        r.y = ug_asin(sarg);
        r.z = ug_atan2(2.0 * (q.x * q.y + q.w * q.z), squ + sqx - sqy - sqz);
    }
    return r;
}
static q4 quat_from_euler(v3 rpy) {
    double phi = rpy.x / 2.0, the = rpy.y / 2.0, psi = rpy.z / 2.0;
    double sp = ug_sin(phi), cp = ug_cos(phi), st = ug_sin(the), ct = ug_cos(the), ss = ug_sin(psi), cs = ug_cos(psi);
    q4 q = Q(sp * ct * cs - cp * st * ss, cp * st * cs + sp * ct * ss, cp * ct * ss - sp * st * cs,
             cp * ct * cs + sp * st * ss);
    double len = ug_sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    return Q(q.x / len, q.y / len, q.z / len, q.w / len);
}

/* ======================================================================== */
/* Python `random` (MT19937) -- reset draws, env_*:create_ball/create_cube   */
/* ======================================================================== */
typedef struct { uint32_t mt[624]; int idx; } mt19937;
static void mt_init_genrand(mt19937* r, uint32_t s) {
    r->mt[0] = s;
    for (int i = 1; i < 624; i++) r->mt[i] = 1812433253u * (r->mt[i - 1] ^ (r->mt[i - 1] >> 30)) + (uint32_t)i;
    r->idx = 624;
}
/* CPython random.seed(int) -> init_by_array([seed]) for 0 <= seed < 2^32 */
static void mt_seed(mt19937* r, uint32_t seed) {
    uint32_t key[1] = {seed};
    int klen = 1;
    mt_init_genrand(r, 19650218u);
    int i = 1, j = 0;
    for (int k = 624 > klen ? 624 : klen; k; k--) {
        r->mt[i] = (r->mt[i] ^ ((r->mt[i - 1] ^ (r->mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
        i++; j++;
        if (i >= 624) { r->mt[0] = r->mt[623]; i = 1; }
        if (j >= klen) j = 0;
    }
    for (int k = 623; k; k--) {
        r->mt[i] = (r->mt[i] ^ ((r->mt[i - 1] ^ (r->mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
        i++;
        if (i >= 624) { r->mt[0] = r->mt[623]; i = 1; }
    }
    r->mt[0] = 0x80000000u;
    r->idx = 624;
}
static uint32_t mt_next(mt19937* r) {
    if (r->idx >= 624) {
        for (int k = 0; k < 624; k++) {
            uint32_t y = (r->mt[k] & 0x80000000u) | (r->mt[(k + 1) % 624] & 0x7fffffffu);
            r->mt[k] = r->mt[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        r->idx = 0;
    }
    uint32_t y = r->mt[r->idx++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}
static double mt_random(mt19937* r) {
    uint32_t a = mt_next(r) >> 5, b = mt_next(r) >> 6;
    return ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);
}
static double mt_uniform(mt19937* r, double a, double b) { return a + (b - a) * mt_random(r); }

/* ======================================================================== */
/* scene description                                                         */
/* ======================================================================== */
typedef struct {
    int kind;
    double half[3];   /* box half extents (margin inside) / sphere radius in half[0] */
    double margin;    /* box: inner margin; hull: outer margin; sphere: radius */
    int v0, nv, f0, nf;
    m3 R; v3 P;       /* shape frame in owner frame */
    m3 aR; v3 aP;     /* AABB frame in owner frame */
    v3 ac, ah;        /* AABB centre / half extents in the AABB frame */
    double disc;      /* angular motion disc */
    double friction, restitution, rolling;
    int owner;        /* >=0 robot body, -1 fixed robot base, -2-i object i, -100 static */
    int ent;          /* 0 robot, 1+i object i, 10+s static s */
    int link;         /* pybullet link index for robot colliders, -1 otherwise */
    int full;         /* full-geometry mode (URGYM_FLAG_FULL_GEOMETRY): hull pairs keep every candidate */
    /* the convex-convex path (UG_CONTACT_GJK, ug_gjk_ref.h): Bullet's shape as GJK sees it */
    v3 gimp;          /* box / cylinder implicit dimensions (outer minus margin) */
    double gmargin;   /* getMargin(): box / hull / cylinder collision margin, sphere radius */
    int gjkbox;       /* a convex mesh PyBullet holds as btConvexHullShape, kept here as its box (the Golf pitch): its
                       * pairs take the convex-convex path whatever the other shape */
    int compound;     /* the collision object's shape is a btCompoundShape (a URDF link whose collision frame is not its
                       * inertial frame, a multi-shape body): btCompoundCollisionAlgorithm refreshes the child manifold
                       * before the child narrowphase */
} collider;

typedef struct { int a, b; double thr, friction, restitution, rolling; } pairdef;

typedef struct {
    int task;    /* base task: scene and physics */
    int variant; /* the env id's task (a variant shares its base task's scene) */
    int full;    /* full-geometry mode: robot hulls with every vertex and face of the mesh's convex hull */
    int gjk;     /* contact generation: 1 Bullet's convex-convex GJK / EPA (the default), 0 vertex-in-hull (UG_CONTACT_VIH) */
    double gravity;
    int nobj;
    double omass[MAXOBJ];
    v3 oinertia[MAXOBJ];
    int ncol;
    collider col[MAXCOL];
    int ocol[MAXOBJ]; /* first collider of each object */
    int oncol[MAXOBJ]; /* colliders of each object (consecutive) */
    UgJoint ojoint[MAXOBJ]; /* one-dof links on a fixed base (Box: door, button; ug_joint.h); kind UGJ_FREE otherwise */
    int njoint, jorder[MAXOBJ]; /* the jointed objects in the multibody's joint order (Box: button = joint 0, door = 1) */
    int npair;
    pairdef pair[MAXPAIR];
} scene;

typedef struct { v3 lpA, lpB, n; double dist, imp, imp1, imp2; } cpoint;
typedef struct { int pair, npts; cpoint pt[4]; } manifold;

struct ugo_env {
    scene sc;
    double q[NB], qd[NB];
    double mtarget[7];
    int mon[7];
    int oactive[MAXOBJ];
    v3 opos[MAXOBJ];
    q4 oquat[MAXOBJ];
    v3 ov[MAXOBJ], ow[MAXOBJ];
    int nman;
    manifold man[MAXMAN];
    int goal_approached, goal_grasped;
    int goal_closed;       /* Box: box_closed (env_box_v0.py:90); goal_approached / goal_grasped = box_opened / button_pressed */
    int button_mode;       /* Box: button_touch_mode (UG_BX_TOUCH_*, env_box_v0.py:20) */
    double jM[MAXOBJ];     /* effective inertia of the jointed objects in the current substep (not state) */
    int overflow;
    mt19937 rng;
    int sparse;            /* reward_type != 'dense' (ctor kwarg of every env, env_cubes_push_v0.py:42) */
    int pgs_bullet;        /* tests only: solve with the velocity-space Bullet-shaped PGS (pgs_bullet) */
    int flags;             /* UG_FLAG_* of the last step / reset call */
    int stats[UG_NSTAT];   /* UG_STAT_* counters */
    double prevq[NB];      /* the last substep's narrowphase poses (ug_layout.h UG_F_PREV): the contact query's */
    v3 prevpos[MAXOBJ];    /* world positions are the points' anchors under these, as Bullet's refreshContactPoints */
    q4 prevquat[MAXOBJ];   /* leaves m_positionWorldOnA/B */
};

static void box_collider(collider* c, double hx, double hy, double hz, double margin, double friction) {
    memset(c, 0, sizeof(*c));
    c->kind = UG_SHAPE_BOX;
    c->half[0] = hx; c->half[1] = hy; c->half[2] = hz;
    c->margin = margin;
    c->R = mident(); c->P = V(0, 0, 0);
    c->aR = mident(); c->aP = V(0, 0, 0);
    c->ac = V(0, 0, 0); c->ah = V(hx, hy, hz);
    c->disc = ug_sqrt(hx * hx + hy * hy + hz * hz);
    c->friction = friction;
    c->link = -1;
}
/* btBoxShape::setSafeMargin for createCollisionShape(GEOM_BOX) [ext] */
static double safe_margin(double hx, double hy, double hz) {
    double m = hx < hy ? hx : hy;
    m = m < hz ? m : hz;
    m = 0.1 * m;
    return m < 0.04 ? m : 0.04;
}

/* Bullet's shape parameters for GJK: a box / cylinder keeps its implicit dimensions inside the margin
 * (btBoxShape / btCylinderShape ctor + setMargin keep the outer extents); a sphere's margin is its radius.  The
 * full-geometry cylinder (createCollisionShape(GEOM_CYLINDER) -> btCylinderShapeZ) carries the safe margin of its
 * constructor, min(0.04, 0.1 min(r, h/2)) [ext]. */
static void gjk_params(collider* c) {
    c->gimp = V(0, 0, 0);
    c->gmargin = c->margin;
    if (c->kind == UG_SHAPE_SPHERE) c->gmargin = c->half[0];
    else if (c->kind == UG_SHAPE_BOX) c->gimp = V(c->half[0] - c->margin, c->half[1] - c->margin, c->half[2] - c->margin);
    else if (c->kind == UG_SHAPE_CYL) {
        const double r = c->half[0], hh = c->half[2];
        double m = 0.1 * (r < hh ? r : hh);
        if (m > 0.04) m = 0.04;
        c->gmargin = m;
        c->gimp = V(r - m, r - m, hh - m);
    }
}
static void add_pair(scene* s, int a, int b) {
    pairdef* p = &s->pair[s->npair++];
    p->a = a; p->b = b;
    double d = s->col[a].disc < s->col[b].disc ? s->col[a].disc : s->col[b].disc;
    p->thr = d * UG_CONTACT_BREAK;
    double f = s->col[a].friction * s->col[b].friction;
    if (f < -UG_MAX_FRICTION) f = -UG_MAX_FRICTION;
    if (f > UG_MAX_FRICTION) f = UG_MAX_FRICTION;
    p->friction = f;
    p->restitution = s->col[a].restitution * s->col[b].restitution;
    /* btManifoldResult::calculateCombinedRollingFriction [ext] */
    double r = s->col[a].rolling * s->col[b].friction + s->col[a].friction * s->col[b].rolling;
    if (r < -UG_MAX_FRICTION) r = -UG_MAX_FRICTION;
    if (r > UG_MAX_FRICTION) r = UG_MAX_FRICTION;
    p->rolling = r;
}

static void build_scene(scene* s, int variant, int flags) {
    memset(s, 0, sizeof(*s));
    const int task = UG_BASE_TASK(variant);
    s->full = UG_GEOM_IS_FULL(flags);
    s->task = task;
    s->variant = variant;
    s->gravity = task == UG_TASK_CUBESGRASP || task == UG_TASK_BOX ? -10.0 : -9.8; /* env_cubes_grasp_v0.py:43,
                                                                                   * env_box_v0.py:60 vs :59 */
    /* robot links 1..18 (link 0 is welded to the fixed base: its contacts carry no dynamics and no
     * reward predicate reads them -- env_cubes_push_v0.py:180 excludes it) */
    for (int l = 1; l < UG_NL; l++) {
        collider* c = &s->col[s->ncol++];
        memset(c, 0, sizeof(*c));
        int si = -1;
        for (int k = 0; k < UG_NSHAPE; k++)
            if (UG_SHAPE_LINK[k] == l) si = k;
        c->kind = UG_SHAPE_KIND[si] == 0 ? UG_SHAPE_BOX : UG_SHAPE_HULL;
        c->half[0] = UG_SHAPE_HALF[3 * si]; c->half[1] = UG_SHAPE_HALF[3 * si + 1]; c->half[2] = UG_SHAPE_HALF[3 * si + 2];
        c->margin = UG_URDF_MARGIN;
        c->v0 = UG_SHAPE_V0[si]; c->nv = UG_SHAPE_NV[si]; c->f0 = UG_SHAPE_F0[si]; c->nf = UG_SHAPE_NF[si];
        if (s->full) { /* PyBullet's hull of all mesh vertices instead of the collision LOD */
            c->v0 = UG_SHAPE_FV0[si]; c->nv = UG_SHAPE_FNV[si]; c->f0 = UG_SHAPE_FF0[si]; c->nf = UG_SHAPE_FNF[si];
        }
        c->R = mload(&UG_SHAPE_R[9 * si]);
        c->P = V(UG_SHAPE_P[3 * si], UG_SHAPE_P[3 * si + 1], UG_SHAPE_P[3 * si + 2]);
        c->aR = mload(&UG_LINK_COMR[9 * l]);
        c->aP = V(UG_LINK_COMP[3 * l], UG_LINK_COMP[3 * l + 1], UG_LINK_COMP[3 * l + 2]);
        c->ac = V(UG_LINK_AABB_C[3 * l], UG_LINK_AABB_C[3 * l + 1], UG_LINK_AABB_C[3 * l + 2]);
        c->ah = V(UG_LINK_AABB_H[3 * l], UG_LINK_AABB_H[3 * l + 1], UG_LINK_AABB_H[3 * l + 2]);
        c->disc = UG_LINK_DISC[l];
        c->friction = UG_DEFAULT_FRICTION;
        c->owner = UG_LINK_BODY[l];
        c->ent = 0;
        c->link = l;
        c->full = s->full;
        /* URDF2Bullet keeps a link's single collision shape bare only when its frame is the link's inertial frame
         * (child transform identity); otherwise the link collides through a btCompoundShape [ext] */
        int same = c->P.x == c->aP.x && c->P.y == c->aP.y && c->P.z == c->aP.z;
        for (int i = 0; i < 9; i++) same = same && c->R.m[i] == c->aR.m[i];
        c->compound = !same;
    }
    int nrobot = s->ncol;
    int statics[8], nstat = 0;
    if (task == UG_TASK_BALLBALANCE) {
        /* paddle (env_ball_balance_v0.py:175-184), ball (:186-205); TwoBallsBalance: two balls of radius 0.003
         * (env_two_balls_balance_v0.py:187, 212-235) */
        const int two = variant == UG_TASK_TWOBALLS;
        s->nobj = two ? 3 : 2;
        double hx = UG_BB_PADDLE_HX, hy = UG_BB_PADDLE_HY, hz = UG_BB_PADDLE_HZ, m = UG_BB_PADDLE_MASS;
        s->omass[0] = m;
        s->oinertia[0] = V(m / 12.0 * (4.0 * hy * hy + 4.0 * hz * hz), m / 12.0 * (4.0 * hx * hx + 4.0 * hz * hz),
                           m / 12.0 * (4.0 * hx * hx + 4.0 * hy * hy));
        collider* c = &s->col[s->ncol];
        box_collider(c, hx, hy, hz, safe_margin(hx, hy, hz), UG_DEFAULT_FRICTION);
        c->owner = -2; c->ent = 1;
        s->ocol[0] = s->ncol++;
        double r = two ? UG_TB_BALL_R : UG_BB_BALL_R, mb = UG_BB_BALL_MASS;
        for (int o = 1; o < s->nobj; o++) {
            s->omass[o] = mb;
            double ib = 0.4 * mb * r * r; /* btSphereShape::calculateLocalInertia [ext] */
            s->oinertia[o] = V(ib, ib, ib);
            c = &s->col[s->ncol];
            box_collider(c, r, r, r, r, UG_DEFAULT_FRICTION);
            c->kind = UG_SHAPE_SPHERE;
            c->half[1] = c->half[2] = 0.0;
            c->disc = ug_sqrt(3.0) * r;
            c->owner = -2 - o; c->ent = 1 + o;
            s->ocol[o] = s->ncol++;
        }
    }
    if (task == UG_TASK_CUBESPUSH || task == UG_TASK_CUBESGRASP) {
        /* cube.urdf x 0.04 (env_cubes_push_v0.py:232-246: two; env_cubes_grasp_v0.py:300-330: one):
         * URDF box, default URDF margin, inertia from the shape's box [ext] */
        s->nobj = task == UG_TASK_CUBESPUSH ? 2 : 1;
        for (int o = 0; o < s->nobj; o++) {
            double h = UG_CUBE_HALF, m = UG_CUBE_MASS;
            s->omass[o] = m;
            double ii = m / 12.0 * (4.0 * h * h + 4.0 * h * h);
            s->oinertia[o] = V(ii, ii, ii);
            collider* c = &s->col[s->ncol];
            box_collider(c, h, h, h, UG_URDF_MARGIN, UG_CUBE_FRICTION);
            c->owner = -2 - o; c->ent = 1 + o;
            s->ocol[o] = s->ncol++;
        }
    }
    if (task == UG_TASK_CUBESGRASP) {
        /* plane.urdf at the origin, no table (env_cubes_grasp_v0.py:48) */
        collider* c = &s->col[s->ncol];
        box_collider(c, UG_PLANE_HALF_XY, UG_PLANE_HALF_XY, UG_PLANE_HALF_Z, UG_URDF_MARGIN, UG_PLANE_FRICTION);
        c->P = V(0.0, 0.0, -UG_PLANE_HALF_Z); c->aP = c->P;
        c->disc = ug_sqrt(15.0 * 15.0 * 2.0 + 25.0) + 5.0;
        c->owner = -100; c->ent = 11;
        c->compound = 1;
        statics[nstat++] = s->ncol++;
    }
    if (task == UG_TASK_GOLF) {
        /* club (env_golf_v0.py:289-332): one rigid body at the composite COM of its three 1 kg parts */
        s->nobj = 2;
        double m = UG_GF_PART_MASS, zc = UG_GF_ZC;
        double bx = UG_GF_BASE_HX, bz = UG_GF_BASE_HZ, fx = UG_GF_FOOT_HX, fy = UG_GF_FOOT_HY;
        double r = UG_CYL_R, hh = UG_CYL_HH;
        /* part inertias: btBoxShape / btCylinderShapeZ calculateLocalInertia [ext] */
        v3 Ib = V(m / 12.0 * (4.0 * bx * bx + 4.0 * bz * bz), m / 12.0 * (4.0 * bx * bx + 4.0 * bz * bz),
                  m / 12.0 * (4.0 * bx * bx + 4.0 * bx * bx));
        v3 If = V(m / 12.0 * (4.0 * fy * fy + 4.0 * fy * fy), m / 12.0 * (4.0 * fx * fx + 4.0 * fy * fy),
                  m / 12.0 * (4.0 * fx * fx + 4.0 * fy * fy));
        double ic = m / 12.0 * (4.0 * hh * hh) + m / 4.0 * (r * r);
        v3 Ic = V(ic, ic, m / 2.0 * (r * r));
        double d0 = 0.0 - zc, d1 = UG_GF_FOOT_Z - zc, d2 = UG_GF_DISC_Z - zc; /* offsets along z */
        s->omass[0] = 3.0 * m;
        s->oinertia[0] = V(Ib.x + m * d0 * d0 + If.x + m * d1 * d1 + Ic.x + m * d2 * d2,
                           Ib.y + m * d0 * d0 + If.y + m * d1 * d1 + Ic.y + m * d2 * d2, Ib.z + If.z + Ic.z);
        s->ocol[0] = s->ncol;
        collider* c = &s->col[s->ncol++];
        box_collider(c, bx, bx, bz, safe_margin(bx, bx, bz), UG_GF_BASE_FRICTION);
        c->restitution = UG_GF_BASE_RESTITUTION;
        c->P = V(0.0, 0.0, d0); c->aP = c->P;
        c->owner = -2; c->ent = 1;
        c = &s->col[s->ncol++];
        box_collider(c, fx, fy, fy, safe_margin(fx, fy, fy), UG_DEFAULT_FRICTION);
        c->P = V(0.0, 0.0, d1); c->aP = c->P;
        c->owner = -2; c->ent = 1;
        c = &s->col[s->ncol++];
        box_collider(c, r, r, hh, UG_CYL_MARGIN, UG_DEFAULT_FRICTION);
        c->kind = UG_SHAPE_HULL;
        c->margin = UG_CYL_MARGIN;
        if (s->full) { /* GEOM_CYLINDER (env_golf_v0.py:305) as a cylinder, not the 16-gon prism */
            c->kind = UG_SHAPE_CYL;
            c->margin = 0.0;
        }
        c->v0 = UG_CYL_V0; c->nv = UG_CYL_NV; c->f0 = UG_CYL_F0; c->nf = UG_CYL_NF;
        c->P = V(0.0, 0.0, d2); c->aP = c->P;
        c->owner = -2; c->ent = 1;
        s->oncol[0] = 3;
        /* ball (:335-358) */
        double rb = UG_GF_BALL_R, mb = UG_GF_BALL_MASS;
        s->omass[1] = mb;
        double ib = 0.4 * mb * rb * rb;
        s->oinertia[1] = V(ib, ib, ib);
        c = &s->col[s->ncol];
        box_collider(c, rb, rb, rb, rb, UG_DEFAULT_FRICTION);
        c->kind = UG_SHAPE_SPHERE;
        c->half[1] = c->half[2] = 0.0;
        c->disc = ug_sqrt(3.0) * rb;
        c->restitution = UG_GF_BALL_RESTITUTION;
        c->rolling = UG_GF_BALL_ROLLING;
        c->owner = -3; c->ent = 2;
        s->ocol[1] = s->ncol++;
        s->oncol[1] = 1;
    }
    if (task == UG_TASK_BALLBALANCE || task == UG_TASK_CUBESPUSH || task == UG_TASK_GOLF) {
        /* table (env_ball_balance_v0.py:71,216-247) and plane at z=-0.5 (:70) */
        collider* c = &s->col[s->ncol];
        box_collider(c, 0.5, 1.0, 0.25, safe_margin(0.5, 1.0, 0.25), UG_DEFAULT_FRICTION);
        c->P = V(0.0, 0.0, -0.25); c->aP = c->P;
        c->owner = -100; c->ent = 10;
        statics[nstat++] = s->ncol++;
        c = &s->col[s->ncol];
        box_collider(c, UG_PLANE_HALF_XY, UG_PLANE_HALF_XY, UG_PLANE_HALF_Z, UG_URDF_MARGIN, UG_PLANE_FRICTION);
        c->P = V(0.0, 0.0, -0.5 - UG_PLANE_HALF_Z); c->aP = c->P;
        c->disc = ug_sqrt(15.0 * 15.0 * 2.0 + 25.0) + 5.0;
        c->owner = -100; c->ent = 11;
        c->compound = 1;
        statics[nstat++] = s->ncol++;
    }
    if (task == UG_TASK_GOLF) {
        /* pitch: static convex hull of golf_pitch.obj (a slab), margin outside (env_golf_v0.py:428-446) */
        collider* c = &s->col[s->ncol];
        box_collider(c, UG_GF_PITCH_HX + UG_URDF_MARGIN, UG_GF_PITCH_HX + UG_URDF_MARGIN,
                     UG_GF_PITCH_HZ + UG_URDF_MARGIN, UG_URDF_MARGIN, UG_DEFAULT_FRICTION);
        c->P = V(UG_GF_PITCH_X, UG_GF_PITCH_Y, UG_GF_PITCH_Z); c->aP = c->P;
        c->owner = -100; c->ent = 12;
        c->gjkbox = 1; /* createCollisionShape(GEOM_MESH): a btConvexHullShape, so every pair is convex-convex */
        statics[nstat++] = s->ncol++;
    }
    if (task == UG_TASK_BOX) {
        /* skew-box-button.urdf (env_box_v0.py:80-85), fixed base at the world origin = (0, -UG_BX_ROBOT_Y, 0) here:
         * object 0 = the door link (revolute, the handles merged in: a box and three cylinders), object 1 = the
         * button (prismatic cylinder), the merged base's four walls static (entity 13), plane.urdf at z = 0 (11).
         * Each link is one collision object whose compound shape sets the breaking threshold (its angular motion
         * disc); URDF primitives keep their URDF extents as the outer surface, default lateral friction (the
         * <contact_coefficients> tag of h3 is not read by PyBullet's URDF parser [ext]). */
        const double by = -UG_BX_ROBOT_Y;
        s->nobj = 2;
        ugj_box_links(&s->ojoint[0], &s->ojoint[1]);
        s->njoint = 2;
        s->jorder[0] = 1; /* joint 0: the button (env_box_v0.py:173-175, :193) */
        s->jorder[1] = 0; /* joint 1: the door (:144, :155, :174-176) */
        /* door compound AABB in its inertial frame (COM origin) -> disc */
        const double* B = UG_BX_DOOR_BOX;
        const UgJoint* D = &s->ojoint[0];
        double lo[3] = {B[0] - B[3], B[1] - B[4], B[2] - B[5]}, hi[3] = {B[0] + B[3], B[1] + B[4], B[2] + B[5]};
        for (int i = 0; i < 3; i++) {
            const double* H = &UG_BX_HANDLE[4 * i];
            double e3[3] = {H[3], i == 2 ? UG_BX_HANDLE_HH[i] : H[3], i == 2 ? H[3] : UG_BX_HANDLE_HH[i]};
            for (int k = 0; k < 3; k++) {
                double l = H[k] - e3[k], u = H[k] + e3[k];
                lo[k] = l < lo[k] ? l : lo[k];
                hi[k] = u > hi[k] ? u : hi[k];
            }
        }
        for (int k = 0; k < 3; k++) { lo[k] = lo[k] - D->com[k]; hi[k] = hi[k] - D->com[k]; }
        double ddisc = ugj_disc(lo, hi);
        collider* c = &s->col[s->ncol];
        box_collider(c, B[3], B[4], B[5], UG_URDF_MARGIN, UG_DEFAULT_FRICTION);
        c->P = V(B[0], B[1], B[2]); c->aP = c->P;
        c->disc = ddisc;
        c->owner = -2; c->ent = 1;
        c->compound = 1; /* URDF_MERGE_FIXED_LINKS: door + h1 h2 h3 */
        s->ocol[0] = s->ncol++;
        for (int i = 0; i < 3; i++) {
            const double* H = &UG_BX_HANDLE[4 * i];
            c = &s->col[s->ncol++];
            box_collider(c, H[3], H[3], UG_BX_HANDLE_HH[i], 0.0, UG_DEFAULT_FRICTION);
            c->kind = UG_SHAPE_CYL;
            c->P = V(H[0], H[1], H[2]); c->aP = c->P;
            if (i == 2) { q4 qh; ugj_box_h3_quat(&qh.x); c->R = qmat(qh); c->aR = c->R; }
            c->disc = ddisc;
            c->owner = -2; c->ent = 1;
            c->compound = 1;
        }
        s->oncol[0] = 4;
        c = &s->col[s->ncol];
        box_collider(c, UG_BX_BUTTON_R, UG_BX_BUTTON_R, UG_BX_BUTTON_HH, 0.0, UG_DEFAULT_FRICTION);
        c->kind = UG_SHAPE_CYL;
        {
            double blo[3] = {-UG_BX_BUTTON_R, -UG_BX_BUTTON_R, -UG_BX_BUTTON_HH}, bhi[3] = {UG_BX_BUTTON_R, UG_BX_BUTTON_R, UG_BX_BUTTON_HH};
            c->disc = ugj_disc(blo, bhi);
        }
        c->owner = -3; c->ent = 2;
        s->ocol[1] = s->ncol++;
        s->oncol[1] = 1;
        /* walls: the fixed base's compound (box1..box4) */
        double wlo[3] = {1e30, 1e30, 1e30}, whi[3] = {-1e30, -1e30, -1e30};
        for (int w = 0; w < 4; w++)
            for (int k = 0; k < 3; k++) {
                double l = UG_BX_WALL_POS[3 * w + k] - UG_BX_WALL_HALF[3 * w + k], u = UG_BX_WALL_POS[3 * w + k] + UG_BX_WALL_HALF[3 * w + k];
                wlo[k] = l < wlo[k] ? l : wlo[k];
                whi[k] = u > whi[k] ? u : whi[k];
            }
        double wdisc = ugj_disc(wlo, whi);
        for (int w = 0; w < 4; w++) {
            c = &s->col[s->ncol];
            box_collider(c, UG_BX_WALL_HALF[3 * w], UG_BX_WALL_HALF[3 * w + 1], UG_BX_WALL_HALF[3 * w + 2], UG_URDF_MARGIN,
                         UG_DEFAULT_FRICTION);
            c->P = V(UG_BX_WALL_POS[3 * w], UG_BX_WALL_POS[3 * w + 1] + by, UG_BX_WALL_POS[3 * w + 2]); c->aP = c->P;
            c->disc = wdisc;
            c->owner = -100; c->ent = 13;
            c->compound = 1; /* the merged base: box1..box4 */
            statics[nstat++] = s->ncol++;
        }
        c = &s->col[s->ncol];
        box_collider(c, UG_PLANE_HALF_XY, UG_PLANE_HALF_XY, UG_PLANE_HALF_Z, UG_URDF_MARGIN, UG_PLANE_FRICTION);
        c->P = V(0.0, by, -UG_PLANE_HALF_Z); c->aP = c->P;
        c->disc = ug_sqrt(15.0 * 15.0 * 2.0 + 25.0) + 5.0;
        c->owner = -100; c->ent = 11;
        c->compound = 1;
        statics[nstat++] = s->ncol++;
    }
    for (int o = 0; o < s->nobj; o++)
        if (s->oncol[o] == 0) s->oncol[o] = 1;
    /* pairs: robot x objects, robot x statics, object x object, object x static (objects: each collider).  Box:
     * the door's box against the button (URDF_USE_SELF_COLLISION: siblings collide, a link and its parent -- the
     * walls -- do not); the handle cylinders never reach the button (they sit on the door's top face, which
     * rotates away from it over the joint range [0, 2]) and carry no pair; of the statics only the plane can meet
     * the button (fully pressed its bottom reaches z = -0.005), the door cannot reach the plane. */
    for (int o = 0; o < s->nobj; o++)
        for (int c = s->ocol[o]; c < s->ocol[o] + s->oncol[o]; c++)
            for (int l = 0; l < nrobot; l++) add_pair(s, l, c);
    for (int t = 0; t < nstat; t++)
        for (int l = 0; l < nrobot; l++) add_pair(s, l, statics[t]);
    for (int o = 0; o < s->nobj; o++)
        for (int p = o + 1; p < s->nobj; p++)
            for (int ca = s->ocol[o]; ca < s->ocol[o] + s->oncol[o]; ca++)
                for (int cb = s->ocol[p]; cb < s->ocol[p] + s->oncol[p]; cb++) {
                    int a = ca, b = cb;
                    if (task == UG_TASK_BOX && s->col[a].kind == UG_SHAPE_CYL) continue;
                    /* canonical order for the narrowphase: sphere first */
                    if (s->col[b].kind == UG_SHAPE_SPHERE && s->col[a].kind != UG_SHAPE_SPHERE) { int t = a; a = b; b = t; }
                    add_pair(s, a, b);
                }
    for (int o = 0; o < s->nobj; o++)
        for (int c = s->ocol[o]; c < s->ocol[o] + s->oncol[o]; c++)
            for (int t = 0; t < nstat; t++) {
                if (task == UG_TASK_BOX && !(o == 1 && s->col[statics[t]].ent == 11)) continue;
                add_pair(s, c, statics[t]);
            }
    /* contact generation and each collider as the convex-convex path sees it (ug_gjk_ref.h) */
    s->gjk = UG_CONTACT_IS_GJK(flags);
    for (int i = 0; i < s->ncol; i++) gjk_params(&s->col[i]);
}

/* ======================================================================== */
/* kinematics                                                                */
/* ======================================================================== */
typedef struct {
    m3 R[NB];
    v3 p[NB];
    v3 a[NB];  /* joint axis, world */
    v3 c[NB];  /* body COM, world */
} kin;

static void fk(const double* q, kin* k) {
    for (int b = 0; b < NB; b++) {
        int pb = UG_BODY_PARENT[b];
        m3 Rpb = mload(&UG_BODY_R[9 * b]);
        v3 Ppb = V(UG_BODY_P[3 * b], UG_BODY_P[3 * b + 1], UG_BODY_P[3 * b + 2]);
        v3 ax = V(UG_BODY_AXIS[3 * b], UG_BODY_AXIS[3 * b + 1], UG_BODY_AXIS[3 * b + 2]);
        m3 Rj = axis_angle(ax, q[b]);
        m3 Rp, Rtmp;
        v3 pp;
        if (pb < 0) { Rp = mident(); pp = V(0, 0, 0); }
        else { Rp = k->R[pb]; pp = k->p[pb]; }
        Rtmp = mm(&Rp, &Rpb);
        k->R[b] = mm(&Rtmp, &Rj);
        k->p[b] = vadd(pp, mv(&Rp, Ppb));
        k->a[b] = mv(&Rtmp, ax);
        v3 com = V(UG_BODY_COM[3 * b], UG_BODY_COM[3 * b + 1], UG_BODY_COM[3 * b + 2]);
        k->c[b] = vadd(k->p[b], mv(&k->R[b], com));
    }
}
/* link frame (URDF link frame) or link COM frame (getLinkState[0:2], collision object frame) */
static void link_frame(const kin* k, int l, int com, m3* R, v3* p) {
    int b = UG_LINK_BODY[l];
    m3 Rl = mload(com ? &UG_LINK_COMR[9 * l] : &UG_LINK_R[9 * l]);
    const double* P = com ? &UG_LINK_COMP[3 * l] : &UG_LINK_P[3 * l];
    v3 Pl = V(P[0], P[1], P[2]);
    if (b < 0) { *R = Rl; *p = Pl; return; }
    *R = mm(&k->R[b], &Rl);
    *p = vadd(k->p[b], mv(&k->R[b], Pl));
}
/* does dof d move body b? */
static int moves(int d, int b) {
    while (b >= 0) {
        if (b == d) return 1;
        b = UG_BODY_PARENT[b];
    }
    return 0;
}

/* ======================================================================== */
/* robot dynamics: CRBA mass matrix + RNEA bias forces in world-frame        */
/* spatial coordinates (Featherstone).  Equivalent to btMultiBody's ABA      */
/* (computeAccelerationsArticulatedBodyAlgorithmMultiDof [ext]) with gravity, */
/* gyroscopic terms and the default quadratic link damping.                  */
/* ======================================================================== */
typedef struct { v3 w, v; } sv; /* spatial vector (angular, linear at world origin) */

static sv spatial_inertia_mul(double m, v3 h, const m3* J, sv x) {
    sv r;
    r.w = vadd(mv(J, x.w), vcross(h, x.v));
    r.v = vsub(vscale(x.v, m), vcross(h, x.w));
    return r;
}

/* returns M (row-major NBxNB) and bias C (generalised force with qdd = 0) */
static void robot_dynamics(const double* qd, const kin* k, double g, double* M, double* C) {
    double m[NB];
    v3 h[NB];
    m3 J[NB];
    double cm[NB];
    v3 ch[NB];
    m3 cJ[NB];
    for (int b = 0; b < NB; b++) {
        m[b] = UG_BODY_MASS[b];
        v3 c = k->c[b];
        h[b] = vscale(c, m[b]);
        m3 Iw = inertia_world(&k->R[b], &UG_BODY_I[6 * b]);
        double cc = vdot(c, c);
        m3 Jb;
        Jb.m[0] = Iw.m[0] + m[b] * (cc - c.x * c.x); Jb.m[1] = Iw.m[1] - m[b] * (c.x * c.y); Jb.m[2] = Iw.m[2] - m[b] * (c.x * c.z);
        Jb.m[3] = Iw.m[3] - m[b] * (c.y * c.x); Jb.m[4] = Iw.m[4] + m[b] * (cc - c.y * c.y); Jb.m[5] = Iw.m[5] - m[b] * (c.y * c.z);
        Jb.m[6] = Iw.m[6] - m[b] * (c.z * c.x); Jb.m[7] = Iw.m[7] - m[b] * (c.z * c.y); Jb.m[8] = Iw.m[8] + m[b] * (cc - c.z * c.z);
        J[b] = Jb;
        cm[b] = m[b]; ch[b] = h[b]; cJ[b] = Jb;
    }
    /* composite inertias, leaves to root (parents have lower index) */
    for (int b = NB - 1; b >= 0; b--) {
        int p = UG_BODY_PARENT[b];
        if (p < 0) continue;
        cm[p] += cm[b];
        ch[p] = vadd(ch[p], ch[b]);
        for (int i = 0; i < 9; i++) cJ[p].m[i] += cJ[b].m[i];
    }
    sv S[NB];
    for (int b = 0; b < NB; b++) { S[b].w = k->a[b]; S[b].v = vcross(k->p[b], k->a[b]); }
    memset(M, 0, sizeof(double) * NB * NB);
    for (int b = 0; b < NB; b++) {
        sv F = spatial_inertia_mul(cm[b], ch[b], &cJ[b], S[b]);
        M[b * NB + b] = vdot(S[b].w, F.w) + vdot(S[b].v, F.v);
        int j = UG_BODY_PARENT[b];
        while (j >= 0) {
            double x = vdot(S[j].w, F.w) + vdot(S[j].v, F.v);
            M[j * NB + b] = x;
            M[b * NB + j] = x;
            j = UG_BODY_PARENT[j];
        }
    }
    /* RNEA with qdd = 0: velocities, bias accelerations, forces */
    sv Vb[NB], Ab[NB], f[NB];
    for (int b = 0; b < NB; b++) {
        int p = UG_BODY_PARENT[b];
        sv Vp, Ap;
        if (p < 0) { Vp.w = V(0, 0, 0); Vp.v = V(0, 0, 0); Ap.w = V(0, 0, 0); Ap.v = V(0, 0, -g); }
        else { Vp = Vb[p]; Ap = Ab[p]; }
        sv vj; vj.w = vscale(S[b].w, qd[b]); vj.v = vscale(S[b].v, qd[b]);
        Vb[b].w = vadd(Vp.w, vj.w); Vb[b].v = vadd(Vp.v, vj.v);
        /* A = Ap + V x vj (motion cross product) */
        Ab[b].w = vadd(Ap.w, vcross(Vb[b].w, vj.w));
        Ab[b].v = vadd(Ap.v, vadd(vcross(Vb[b].w, vj.v), vcross(Vb[b].v, vj.w)));
        sv IA = spatial_inertia_mul(m[b], h[b], &J[b], Ab[b]);
        sv IV = spatial_inertia_mul(m[b], h[b], &J[b], Vb[b]);
        /* V x* IV  = (w x n + v x f, w x f) */
        f[b].w = vadd(IA.w, vadd(vcross(Vb[b].w, IV.w), vcross(Vb[b].v, IV.v)));
        f[b].v = vadd(IA.v, vcross(Vb[b].w, IV.v));
        /* damping (btMultiBody DAMPING_K1/K2 = 0.04), bias includes +damping */
        double wn = vlen(Vb[b].w);
        m3 D = inertia_world(&k->R[b], &UG_BODY_DAMPI[6 * b]);
        v3 tau = vscale(mv(&D, Vb[b].w), UG_ANG_DAMP + UG_ANG_DAMP * wn);
        f[b].w = vadd(f[b].w, tau);
    }
    for (int l = 1; l < UG_NL; l++) {
        int b = UG_LINK_BODY[l];
        if (b < 0) continue;
        v3 cl = vadd(k->p[b], mv(&k->R[b], V(UG_LINK_COMP[3 * l], UG_LINK_COMP[3 * l + 1], UG_LINK_COMP[3 * l + 2])));
        v3 vl = vadd(Vb[b].v, vcross(Vb[b].w, cl));
        double vn = vlen(vl);
        v3 fd = vscale(vl, UG_LINK_MASS[l] * (UG_LIN_DAMP + UG_LIN_DAMP * vn));
        f[b].v = vadd(f[b].v, fd);
        f[b].w = vadd(f[b].w, vcross(cl, fd));
    }
    for (int b = NB - 1; b >= 0; b--) {
        C[b] = vdot(S[b].w, f[b].w) + vdot(S[b].v, f[b].v);
        int p = UG_BODY_PARENT[b];
        if (p >= 0) { f[p].w = vadd(f[p].w, f[b].w); f[p].v = vadd(f[p].v, f[b].v); }
    }
}

/* dense LDL^T of the SPD mass matrix (in place: strict lower = L, diag = D) */
static void ldlt(double* A, int n) {
    for (int j = 0; j < n; j++) {
        double d = A[j * n + j];
        for (int k2 = 0; k2 < j; k2++) d -= A[j * n + k2] * A[j * n + k2] * A[k2 * n + k2];
        A[j * n + j] = d;
        for (int i = j + 1; i < n; i++) {
            double s = A[i * n + j];
            for (int k2 = 0; k2 < j; k2++) s -= A[i * n + k2] * A[j * n + k2] * A[k2 * n + k2];
            A[i * n + j] = s / d;
        }
    }
}
static void ldlt_solve(const double* A, int n, double* x) {
    for (int i = 0; i < n; i++)
        for (int k2 = 0; k2 < i; k2++) x[i] -= A[i * n + k2] * x[k2];
    for (int i = 0; i < n; i++) x[i] = x[i] / A[i * n + i];
    for (int i = n - 1; i >= 0; i--)
        for (int k2 = i + 1; k2 < n; k2++) x[i] -= A[k2 * n + i] * x[k2];
}

/* ======================================================================== */
/* collision: world transforms, broadphase, narrowphase, persistent manifolds */
/* ======================================================================== */
typedef struct { m3 R; v3 p; } xf;
static v3 xf_apply(const xf* T, v3 x) { return vadd(mv(&T->R, x), T->p); }
static v3 xf_inv_apply(const xf* T, v3 x) { return mtv(&T->R, vsub(x, T->p)); }

/* owner frame (robot body / object COM / world) */
static xf owner_xf(const ugo_env* e, const kin* k, int owner) {
    xf T;
    if (owner >= 0) { T.R = k->R[owner]; T.p = k->p[owner]; }
    else if (owner <= -2 && owner > -100) { int o = -2 - owner; T.R = qmat(e->oquat[o]); T.p = e->opos[o]; }
    else { T.R = mident(); T.p = V(0, 0, 0); }
    return T;
}
static xf shape_xf(const xf* O, const collider* c) {
    xf T;
    T.R = mm(&O->R, &c->R);
    T.p = vadd(O->p, mv(&O->R, c->P));
    return T;
}
static void world_aabb(const xf* O, const collider* c, v3* lo, v3* hi) {
    m3 Rw = mm(&O->R, &c->aR);
    v3 pw = vadd(O->p, mv(&O->R, c->aP));
    v3 ctr = vadd(mv(&Rw, c->ac), pw);
    const double* r = Rw.m;
    v3 ext = V(ug_fabs(r[0]) * c->ah.x + ug_fabs(r[1]) * c->ah.y + ug_fabs(r[2]) * c->ah.z,
               ug_fabs(r[3]) * c->ah.x + ug_fabs(r[4]) * c->ah.y + ug_fabs(r[5]) * c->ah.z,
               ug_fabs(r[6]) * c->ah.x + ug_fabs(r[7]) * c->ah.y + ug_fabs(r[8]) * c->ah.z);
    *lo = vsub(ctr, ext);
    *hi = vadd(ctr, ext);
}

/* contact candidate: normal on B (world, B->A), point on B (world), signed distance */
typedef struct { v3 n, pB; double d; } cand;
typedef struct { int n, cap; cand c[MAXCAND]; } candlist;
static void cand_init(candlist* L, int cap) {
    L->n = 0;
    L->cap = cap < MAXCAND ? cap : MAXCAND;
}
static void cand_add(candlist* L, v3 n, v3 pB, double d) {
    if (L->n < L->cap) { L->c[L->n].n = n; L->c[L->n].pB = pB; L->c[L->n].d = d; L->n++; }
}

#include "ug_gjk_ref.h"
/* the convex-convex path (scene gjk): Bullet's GJK / EPA pair detector, one point per pair and call */
static void gshape_of(const collider* c, gshape* g) {
    g->kind = c->kind;
    g->v = c->kind == UG_SHAPE_HULL ? &UG_HULL_V[3 * c->v0] : NULL;
    g->nv = c->kind == UG_SHAPE_HULL ? c->nv : 0;
    g->imp = c->gimp;
    g->margin = c->gmargin;
}
/* pairs with a dedicated Bullet algorithm keep it: sphere-sphere, sphere-box (btSphereBoxCollisionAlgorithm),
 * box-box (btBoxBoxCollisionAlgorithm); everything else is btConvexConvexAlgorithm */
static int pair_is_gjk(const collider* A, const collider* B) {
    if (A->gjkbox || B->gjkbox) return 1;
    const int pa = A->kind == UG_SHAPE_SPHERE || A->kind == UG_SHAPE_BOX;
    const int pb = B->kind == UG_SHAPE_SPHERE || B->kind == UG_SHAPE_BOX;
    return !(pa && pb);
}
/* test hook: one convex-convex query on explicit shapes and poses (tests/test_gjk.py) */
int ugo_gjk_pair(int kA, int v0A, int nvA, const double* impA, double mA, const double* RA, const double* pA, int kB, int v0B,
                 int nvB, const double* impB, double mB, const double* RB, const double* pB, double thr, double* out) {
    gshape A = {kA, kA == UG_SHAPE_HULL ? &UG_HULL_V[3 * v0A] : NULL, nvA, V(impA[0], impA[1], impA[2]), mA};
    gshape B = {kB, kB == UG_SHAPE_HULL ? &UG_HULL_V[3 * v0B] : NULL, nvB, V(impB[0], impB[1], impB[2]), mB};
    xf TA, TB;
    TA.R = mload(RA); TA.p = V(pA[0], pA[1], pA[2]);
    TB.R = mload(RB); TB.p = V(pB[0], pB[1], pB[2]);
    v3 n, p;
    double d;
    if (!gjk_pair(&A, &TA, &B, &TB, thr, &n, &p, &d)) return 0;
    out[0] = n.x; out[1] = n.y; out[2] = n.z;
    out[3] = p.x; out[4] = p.y; out[5] = p.z;
    out[6] = d;
    return 1;
}
/* test hook: the last ugo_gjk_pair query's exits (ug_gjk_ref.h g_gjk_dbg) */
void ugo_gjk_debug(int* out) {
    for (int i = 0; i < 4; i++) out[i] = g_gjk_dbg[i];
}
/* debug aid (tools/debug_gjk.py): the convex-convex queries of this thread, as urgym_debug_gjk packs them, with
 * their results (ok, normal, point, distance) */
#define GREC_MAX 8192
#define GREC_DOUBLES 47
static __thread int g_rec_on, g_rec_n;
static __thread double g_rec[GREC_MAX * GREC_DOUBLES];
void ugo_gjk_record(int on) {
    if (on) g_rec_n = 0;
    g_rec_on = on;
}
int ugo_gjk_records(double* out, int max) {
    const int n = g_rec_n < max ? g_rec_n : max;
    memcpy(out, g_rec, sizeof(double) * GREC_DOUBLES * (size_t)n);
    return g_rec_n;
}
static void grec_shape(double* q, const gshape* g, int v0, const xf* T) {
    q[0] = g->kind; q[1] = v0; q[2] = g->nv; q[3] = g->imp.x; q[4] = g->imp.y; q[5] = g->imp.z; q[6] = g->margin;
    for (int i = 0; i < 9; i++) q[7 + i] = T->R.m[i];
    q[16] = T->p.x; q[17] = T->p.y; q[18] = T->p.z;
}
static int gjk_pair_rec(const gshape* A, int va, const xf* TA, const gshape* B, int vb, const xf* TB, double thr, v3* n,
                        v3* p, double* d) {
    const int ok = gjk_pair(A, TA, B, TB, thr, n, p, d);
    if (g_rec_on && g_rec_n < GREC_MAX) {
        double* q = g_rec + GREC_DOUBLES * g_rec_n++;
        grec_shape(q, A, va, TA);
        grec_shape(q + 19, B, vb, TB);
        q[38] = thr;
        q[39] = ok;
        q[40] = n->x; q[41] = n->y; q[42] = n->z; q[43] = p->x; q[44] = p->y; q[45] = p->z; q[46] = *d;
    }
    return ok;
}
static void nc_gjk(const xf* TA, const collider* A, const xf* TB, const collider* B, double thr, candlist* out) {
    gshape ga, gb;
    gshape_of(A, &ga);
    gshape_of(B, &gb);
    v3 n = V(0, 0, 0), p = V(0, 0, 0);
    double d = 0.0;
    if (A->kind == UG_SHAPE_SPHERE && B->kind != UG_SHAPE_SPHERE) {
        /* the sphere-first pair order of this restatement: B is GJK's shape A, the result turned into (A, B) */
        if (gjk_pair_rec(&gb, B->v0, TB, &ga, A->v0, TA, thr, &n, &p, &d)) cand_add(out, vneg(n), vadd(p, vscale(n, d)), d);
        return;
    }
    if (gjk_pair_rec(&ga, A->v0, TA, &gb, B->v0, TB, thr, &n, &p, &d)) cand_add(out, n, p, d);
}

/* btSphereBoxCollisionAlgorithm::getSphereDistance [ext]: sphere A, box B */
static void nc_sphere_box(const xf* TA, const collider* A, const xf* TB, const collider* B, double thr, candlist* out) {
    double r = A->half[0];
    double bm = B->margin;
    v3 he = V(B->half[0] - bm, B->half[1] - bm, B->half[2] - bm);
    v3 rel = xf_inv_apply(TB, TA->p);
    v3 cp = rel;
    cp.x = ug_min(he.x, cp.x); cp.x = ug_max(-he.x, cp.x);
    cp.y = ug_min(he.y, cp.y); cp.y = ug_max(-he.y, cp.y);
    cp.z = ug_min(he.z, cp.z); cp.z = ug_max(-he.z, cp.z);
    double idist = r + bm;
    double cdist = idist + thr;
    v3 n = vsub(rel, cp);
    double d2 = vdot(n, n);
    if (d2 > cdist * cdist) return;
    double dist;
    if (d2 <= 2.220446049250313e-16) {
        /* getSpherePenetration: project onto the closest face */
        double fd = he.x - rel.x, mind = fd;
        cp.x = he.x; n = V(1, 0, 0);
        fd = he.x + rel.x; if (fd < mind) { mind = fd; cp = rel; cp.x = -he.x; n = V(-1, 0, 0); }
        fd = he.y - rel.y; if (fd < mind) { mind = fd; cp = rel; cp.y = he.y; n = V(0, 1, 0); }
        fd = he.y + rel.y; if (fd < mind) { mind = fd; cp = rel; cp.y = -he.y; n = V(0, -1, 0); }
        fd = he.z - rel.z; if (fd < mind) { mind = fd; cp = rel; cp.z = he.z; n = V(0, 0, 1); }
        fd = he.z + rel.z; if (fd < mind) { mind = fd; cp = rel; cp.z = -he.z; n = V(0, 0, -1); }
        dist = -mind;
    } else {
        dist = ug_sqrt(d2);
        n = vscale(n, 1.0 / dist);
    }
    v3 pb = vadd(cp, vscale(n, bm));
    double depth = dist - idist;
    cand_add(out, mv(&TB->R, n), xf_apply(TB, pb), depth);
}

static void nc_sphere_sphere(const xf* TA, const collider* A, const xf* TB, const collider* B, double thr, candlist* out) {
    v3 d = vsub(TA->p, TB->p);
    double len = vlen(d);
    double dist = len - (A->half[0] + B->half[0]);
    if (dist > thr) return;
    v3 n = len > 2.220446049250313e-16 ? vscale(d, 1.0 / len) : V(1, 0, 0);
    cand_add(out, n, vadd(TB->p, vscale(n, B->half[0])), dist);
}

/* --- box-box: ODE dBoxBox2 as used by btBoxBoxDetector [ext] --- */
static int intersect_rect_quad(const double h[2], double p[8], double ret[16]) {
    int nq = 4, nr = 0;
    double buffer[16];
    double* q = p;
    double* r = ret;
    for (int dir = 0; dir <= 1; dir++) {
        for (int sign = -1; sign <= 1; sign += 2) {
            double* pq = q;
            double* pr = r;
            nr = 0;
            for (int i = nq; i > 0; i--) {
                if (sign * pq[dir] < h[dir]) {
                    pr[0] = pq[0]; pr[1] = pq[1];
                    pr += 2; nr++;
                    if (nr & 8) { q = r; goto done; }
                }
                double* nextq = (i > 1) ? pq + 2 : q;
                if ((sign * pq[dir] < h[dir]) ^ (sign * nextq[dir] < h[dir])) {
                    pr[1 - dir] = pq[1 - dir] + (nextq[1 - dir] - pq[1 - dir]) / (nextq[dir] - pq[dir]) * (sign * h[dir] - pq[dir]);
                    pr[dir] = sign * h[dir];
                    pr += 2; nr++;
                    if (nr & 8) { q = r; goto done; }
                }
                pq += 2;
            }
            q = r;
            r = (q == ret) ? buffer : ret;
            nq = nr;
        }
    }
done:
    if (q != ret) memcpy(ret, q, (size_t)nr * 2 * sizeof(double));
    return nr;
}
static void cull_points(int n, const double p[], int m, int i0, int iret[]) {
    double a, cx, cy, qq;
    if (n == 1) { cx = p[0]; cy = p[1]; }
    else if (n == 2) { cx = 0.5 * (p[0] + p[2]); cy = 0.5 * (p[1] + p[3]); }
    else {
        a = 0; cx = 0; cy = 0;
        for (int i = 0; i < n - 1; i++) {
            qq = p[i * 2] * p[i * 2 + 3] - p[i * 2 + 2] * p[i * 2 + 1];
            a += qq;
            cx += qq * (p[i * 2] + p[i * 2 + 2]);
            cy += qq * (p[i * 2 + 1] + p[i * 2 + 3]);
        }
        qq = p[n * 2 - 2] * p[1] - p[0] * p[n * 2 - 1];
        if (ug_fabs(a + qq) > 2.220446049250313e-16) a = 1.0 / (3.0 * (a + qq));
        else a = 1e30;
        cx = a * (cx + qq * (p[n * 2 - 2] + p[0]));
        cy = a * (cy + qq * (p[n * 2 - 1] + p[1]));
    }
    double A[8];
    for (int i = 0; i < n; i++) A[i] = ug_atan2(p[i * 2 + 1] - cy, p[i * 2] - cx);
    int avail[8];
    for (int i = 0; i < n; i++) avail[i] = 1;
    avail[i0] = 0;
    iret[0] = i0;
    for (int j = 1; j < m; j++) {
        a = (double)j * (2.0 * UG_PI / m) + A[i0];
        if (a > UG_PI) a -= 2.0 * UG_PI;
        double maxdiff = 1e9, diff;
        iret[j] = i0;
        for (int i = 0; i < n; i++) {
            if (avail[i]) {
                diff = ug_fabs(A[i] - a);
                if (diff > UG_PI) diff = 2.0 * UG_PI - diff;
                if (diff < maxdiff) { maxdiff = diff; iret[j] = i; }
            }
        }
        avail[iret[j]] = 0;
    }
}
/* R[i*4+j] addressing of dMatrix3 replaced by m3 row-major: element (i,j) = m[3i+j]; column j = axis j */
static double col_dot(const m3* A, int i, const m3* B, int j) { /* column i of A . column j of B */
    return A->m[i] * B->m[j] + A->m[3 + i] * B->m[3 + j] + A->m[6 + i] * B->m[6 + j];
}
static double col_dotv(const m3* A, int i, v3 v) { return A->m[i] * v.x + A->m[3 + i] * v.y + A->m[6 + i] * v.z; }
static double vget(v3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
static void vsetc(v3* v, int i, double x) { if (i == 0) v->x = x; else if (i == 1) v->y = x; else v->z = x; }

static void nc_box_box(const xf* TA, const collider* A, const xf* TB, const collider* B, double thr, candlist* out) {
    (void)thr;
    const double fudge = 1.05;
    const m3* R1 = &TA->R;
    const m3* R2 = &TB->R;
    v3 p1 = TA->p, p2 = TB->p;
    v3 p = vsub(p2, p1);
    v3 pp = mtv(R1, p);
    double Ah[3] = {A->half[0], A->half[1], A->half[2]};
    double Bh[3] = {B->half[0], B->half[1], B->half[2]};
    double R11 = col_dot(R1, 0, R2, 0), R12 = col_dot(R1, 0, R2, 1), R13 = col_dot(R1, 0, R2, 2);
    double R21 = col_dot(R1, 1, R2, 0), R22 = col_dot(R1, 1, R2, 1), R23 = col_dot(R1, 1, R2, 2);
    double R31 = col_dot(R1, 2, R2, 0), R32 = col_dot(R1, 2, R2, 1), R33 = col_dot(R1, 2, R2, 2);
    double Q11 = ug_fabs(R11), Q12 = ug_fabs(R12), Q13 = ug_fabs(R13);
    double Q21 = ug_fabs(R21), Q22 = ug_fabs(R22), Q23 = ug_fabs(R23);
    double Q31 = ug_fabs(R31), Q32 = ug_fabs(R32), Q33 = ug_fabs(R33);
    double s = -1e300, s2, l, e1;
    int invert_normal = 0, code = 0;
    int nR = -1; /* 0..2 column of R1, 3..5 column of R2, -1 use normalC */
    v3 normalC = V(0, 0, 0);
#define TST(expr1, expr2, norm, cc)             \
    e1 = (expr1);                               \
    s2 = ug_fabs(e1) - (expr2);                 \
    if (s2 > 0) return;                         \
    if (s2 > s) { s = s2; nR = norm; invert_normal = (e1 < 0); code = (cc); }
    TST(pp.x, (Ah[0] + Bh[0] * Q11 + Bh[1] * Q12 + Bh[2] * Q13), 0, 1);
    TST(pp.y, (Ah[1] + Bh[0] * Q21 + Bh[1] * Q22 + Bh[2] * Q23), 1, 2);
    TST(pp.z, (Ah[2] + Bh[0] * Q31 + Bh[1] * Q32 + Bh[2] * Q33), 2, 3);
    TST(col_dotv(R2, 0, p), (Ah[0] * Q11 + Ah[1] * Q21 + Ah[2] * Q31 + Bh[0]), 3, 4);
    TST(col_dotv(R2, 1, p), (Ah[0] * Q12 + Ah[1] * Q22 + Ah[2] * Q32 + Bh[1]), 4, 5);
    TST(col_dotv(R2, 2, p), (Ah[0] * Q13 + Ah[1] * Q23 + Ah[2] * Q33 + Bh[2]), 5, 6);
#undef TST
#define TST(expr1, expr2, n1, n2, n3, cc)                                      \
    e1 = (expr1);                                                              \
    s2 = ug_fabs(e1) - (expr2);                                                \
    if (s2 > 0) return;                                                        \
    l = ug_sqrt((n1) * (n1) + (n2) * (n2) + (n3) * (n3));                      \
    if (l > 0) {                                                               \
        s2 /= l;                                                               \
        if (s2 * fudge > s) {                                                  \
            s = s2; nR = -1;                                                   \
            normalC = V((n1) / l, (n2) / l, (n3) / l);                         \
            invert_normal = (e1 < 0); code = (cc);                             \
        }                                                                      \
    }
    TST(pp.z * R21 - pp.y * R31, (Ah[1] * Q31 + Ah[2] * Q21 + Bh[1] * Q13 + Bh[2] * Q12), 0, -R31, R21, 7);
    TST(pp.z * R22 - pp.y * R32, (Ah[1] * Q32 + Ah[2] * Q22 + Bh[0] * Q13 + Bh[2] * Q11), 0, -R32, R22, 8);
    TST(pp.z * R23 - pp.y * R33, (Ah[1] * Q33 + Ah[2] * Q23 + Bh[0] * Q12 + Bh[1] * Q11), 0, -R33, R23, 9);
    TST(pp.x * R31 - pp.z * R11, (Ah[0] * Q31 + Ah[2] * Q11 + Bh[1] * Q23 + Bh[2] * Q22), R31, 0, -R11, 10);
    TST(pp.x * R32 - pp.z * R12, (Ah[0] * Q32 + Ah[2] * Q12 + Bh[0] * Q23 + Bh[2] * Q21), R32, 0, -R12, 11);
    TST(pp.x * R33 - pp.z * R13, (Ah[0] * Q33 + Ah[2] * Q13 + Bh[0] * Q22 + Bh[1] * Q21), R33, 0, -R13, 12);
    TST(pp.y * R11 - pp.x * R21, (Ah[0] * Q21 + Ah[1] * Q11 + Bh[1] * Q33 + Bh[2] * Q32), -R21, R11, 0, 13);
    TST(pp.y * R12 - pp.x * R22, (Ah[0] * Q22 + Ah[1] * Q12 + Bh[0] * Q33 + Bh[2] * Q31), -R22, R12, 0, 14);
    TST(pp.y * R13 - pp.x * R23, (Ah[0] * Q23 + Ah[1] * Q13 + Bh[0] * Q32 + Bh[1] * Q31), -R23, R13, 0, 15);
#undef TST
    if (!code) return;
    v3 normal;
    if (nR >= 0) {
        const m3* Rn = nR < 3 ? R1 : R2;
        int c = nR % 3;
        normal = V(Rn->m[c], Rn->m[3 + c], Rn->m[6 + c]);
    } else {
        normal = mv(R1, normalC);
    }
    if (invert_normal) normal = vneg(normal);
    double depth = -s;
    if (code > 6) {
        v3 pa = p1;
        for (int j = 0; j < 3; j++) {
            double sign = (col_dotv(R1, j, normal) > 0) ? 1.0 : -1.0;
            pa = vadd(pa, V(sign * Ah[j] * R1->m[j], sign * Ah[j] * R1->m[3 + j], sign * Ah[j] * R1->m[6 + j]));
        }
        v3 pb = p2;
        for (int j = 0; j < 3; j++) {
            double sign = (col_dotv(R2, j, normal) > 0) ? -1.0 : 1.0;
            pb = vadd(pb, V(sign * Bh[j] * R2->m[j], sign * Bh[j] * R2->m[3 + j], sign * Bh[j] * R2->m[6 + j]));
        }
        int ia = (code - 7) / 3, ib = (code - 7) % 3;
        v3 ua = V(R1->m[ia], R1->m[3 + ia], R1->m[6 + ia]);
        v3 ub = V(R2->m[ib], R2->m[3 + ib], R2->m[6 + ib]);
        /* dLineClosestApproach */
        v3 pd = vsub(pb, pa);
        double uaub = vdot(ua, ub), q1 = vdot(ua, pd), q2 = -vdot(ub, pd);
        double d = 1.0 - uaub * uaub, alpha, beta;
        if (d <= 0.0001) { alpha = 0; beta = 0; }
        else { d = 1.0 / d; alpha = (q1 + uaub * q2) * d; beta = (uaub * q1 + q2) * d; }
        (void)alpha;
        pb = vadd(pb, vscale(ub, beta));
        cand_add(out, vneg(normal), pb, -depth);
        return;
    }
    const m3 *Ra, *Rb;
    v3 pa, pb;
    const double *Sa, *Sb;
    if (code <= 3) { Ra = R1; Rb = R2; pa = p1; pb = p2; Sa = Ah; Sb = Bh; }
    else { Ra = R2; Rb = R1; pa = p2; pb = p1; Sa = Bh; Sb = Ah; }
    v3 normal2 = code <= 3 ? normal : vneg(normal);
    v3 nr = mtv(Rb, normal2);
    v3 anr = V(ug_fabs(nr.x), ug_fabs(nr.y), ug_fabs(nr.z));
    int lanr, a1, a2;
    if (anr.y > anr.x) {
        if (anr.y > anr.z) { a1 = 0; lanr = 1; a2 = 2; }
        else { a1 = 0; a2 = 1; lanr = 2; }
    } else {
        if (anr.x > anr.z) { lanr = 0; a1 = 1; a2 = 2; }
        else { a1 = 0; a2 = 1; lanr = 2; }
    }
    v3 center;
    v3 rbl = V(Rb->m[lanr], Rb->m[3 + lanr], Rb->m[6 + lanr]);
    if (vget(nr, lanr) < 0) center = vadd(vsub(pb, pa), vscale(rbl, Sb[lanr]));
    else center = vsub(vsub(pb, pa), vscale(rbl, Sb[lanr]));
    int codeN, code1, code2;
    codeN = code <= 3 ? code - 1 : code - 4;
    if (codeN == 0) { code1 = 1; code2 = 2; }
    else if (codeN == 1) { code1 = 0; code2 = 2; }
    else { code1 = 0; code2 = 1; }
    double quad[8];
    double c1 = col_dotv(Ra, code1, center), c2 = col_dotv(Ra, code2, center);
    double m11 = col_dot(Ra, code1, Rb, a1), m12 = col_dot(Ra, code1, Rb, a2);
    double m21 = col_dot(Ra, code2, Rb, a1), m22 = col_dot(Ra, code2, Rb, a2);
    {
        double k1 = m11 * Sb[a1], k2 = m21 * Sb[a1], k3 = m12 * Sb[a2], k4 = m22 * Sb[a2];
        quad[0] = c1 - k1 - k3; quad[1] = c2 - k2 - k4;
        quad[2] = c1 - k1 + k3; quad[3] = c2 - k2 + k4;
        quad[4] = c1 + k1 + k3; quad[5] = c2 + k2 + k4;
        quad[6] = c1 + k1 - k3; quad[7] = c2 + k2 - k4;
    }
    double rect[2] = {Sa[code1], Sa[code2]};
    double ret[16];
    int n = intersect_rect_quad(rect, quad, ret);
    if (n < 1) return;
    v3 point[8];
    double dep[8];
    double det1 = 1.0 / (m11 * m22 - m12 * m21);
    m11 *= det1; m12 *= det1; m21 *= det1; m22 *= det1;
    int cnum = 0;
    v3 rba1 = V(Rb->m[a1], Rb->m[3 + a1], Rb->m[6 + a1]);
    v3 rba2 = V(Rb->m[a2], Rb->m[3 + a2], Rb->m[6 + a2]);
    for (int j = 0; j < n; j++) {
        double k1 = m22 * (ret[j * 2] - c1) - m12 * (ret[j * 2 + 1] - c2);
        double k2 = -m21 * (ret[j * 2] - c1) + m11 * (ret[j * 2 + 1] - c2);
        point[cnum] = vadd(vadd(center, vscale(rba1, k1)), vscale(rba2, k2));
        dep[cnum] = Sa[codeN] - vdot(normal2, point[cnum]);
        if (dep[cnum] >= 0) {
            ret[cnum * 2] = ret[j * 2];
            ret[cnum * 2 + 1] = ret[j * 2 + 1];
            cnum++;
        }
    }
    if (cnum < 1) return;
    int maxc = 4;
    if (maxc > cnum) maxc = cnum;
    if (cnum <= maxc) {
        for (int j = 0; j < cnum; j++) {
            v3 pw = vadd(point[j], pa);
            if (code >= 4) pw = vsub(pw, vscale(normal, dep[j]));
            cand_add(out, vneg(normal), pw, -dep[j]);
        }
    } else {
        int i1 = 0;
        double maxdepth = dep[0];
        for (int i = 1; i < cnum; i++)
            if (dep[i] > maxdepth) { maxdepth = dep[i]; i1 = i; }
        int iret[8];
        cull_points(cnum, ret, maxc, i1, iret);
        for (int j = 0; j < maxc; j++) {
            v3 pw = vadd(point[iret[j]], pa);
            if (code >= 4) pw = vsub(pw, vscale(normal, dep[iret[j]]));
            cand_add(out, vneg(normal), pw, -dep[iret[j]]);
        }
    }
}

/* convex hull (robot link, A) vs box (B): vertex-in-box + corner-in-hull
 * (restated substitute for btConvexConvexAlgorithm GJK/EPA + polyhedral
 * clipping [ext]; see DESIGN.md "contact generation") */
static void reduce4(candlist* L) {
    if (L->n <= 4) return;
    cand sel[4];
    int used[MAXCAND];
    memset(used, 0, sizeof(used));
    int best = 0;
    for (int i = 1; i < L->n; i++)
        if (L->c[i].d < L->c[best].d) best = i;
    sel[0] = L->c[best];
    used[best] = 1;
    for (int s = 1; s < 4; s++) {
        int bi = -1;
        double bd = -1.0;
        for (int i = 0; i < L->n; i++) {
            if (used[i]) continue;
            double md = 1e300;
            for (int t = 0; t < s; t++) {
                v3 dd = vsub(L->c[i].pB, sel[t].pB);
                double x = vdot(dd, dd);
                if (x < md) md = x;
            }
            if (md > bd) { bd = md; bi = i; }
        }
        sel[s] = L->c[bi];
        used[bi] = 1;
    }
    for (int s = 0; s < 4; s++) L->c[s] = sel[s];
    L->n = 4;
}
#ifndef UG_FIDELITY
static void nc_hull_box(const xf* TA, const collider* A, const xf* TB, const collider* B, double thr, candlist* out) {
    m3 RAB = mtm(&TB->R, &TA->R);
    v3 pAB = mtv(&TB->R, vsub(TA->p, TB->p));
    v3 h = V(B->half[0], B->half[1], B->half[2]);
    double mA = A->margin;
    static _Thread_local candlist L;
    cand_init(&L, A->full ? MAXCAND : LOD_MAXCAND);
    for (int i = 0; i < A->nv; i++) {
        const double* vv = &UG_HULL_V[3 * (A->v0 + i)];
        v3 x = vadd(mv(&RAB, V(vv[0], vv[1], vv[2])), pAB);
        v3 d = V(ug_fabs(x.x) - h.x, ug_fabs(x.y) - h.y, ug_fabs(x.z) - h.z);
        double dist;
        v3 nl, pl;
        if (d.x < 0 && d.y < 0 && d.z < 0) {
            int k = 0;
            double dm = d.x;
            if (d.y > dm) { dm = d.y; k = 1; }
            if (d.z > dm) { dm = d.z; k = 2; }
            dist = dm;
            double sg = vget(x, k) < 0 ? -1.0 : 1.0;
            nl = V(0, 0, 0); vsetc(&nl, k, sg);
            pl = x; vsetc(&pl, k, sg * vget(h, k));
        } else {
            v3 q = V(ug_max(-h.x, ug_min(h.x, x.x)), ug_max(-h.y, ug_min(h.y, x.y)), ug_max(-h.z, ug_min(h.z, x.z)));
            v3 df = vsub(x, q);
            double dl = vlen(df);
            if (dl - mA >= thr) continue;
            dist = dl;
            nl = vscale(df, 1.0 / dl);
            pl = q;
        }
        double depth = dist - mA;
        if (depth < thr) cand_add(&L, mv(&TB->R, nl), xf_apply(TB, pl), depth);
    }
    m3 RBA = mtm(&TA->R, &TB->R);
    v3 pBA = mtv(&TA->R, vsub(TB->p, TA->p));
    for (int c = 0; c < 8; c++) {
        v3 cl = V((c & 1) ? h.x : -h.x, (c & 2) ? h.y : -h.y, (c & 4) ? h.z : -h.z);
        v3 y = vadd(mv(&RBA, cl), pBA);
        double smax = -1e300;
        int fm = -1;
        for (int f = 0; f < A->nf; f++) {
            const double* F = &UG_HULL_F[4 * (A->f0 + f)];
            double sd = F[0] * y.x + F[1] * y.y + F[2] * y.z - F[3];
            if (sd > smax) { smax = sd; fm = f; }
            if (sd - mA >= thr) break; /* outside this face: cannot be a contact */
        }
        double depth = smax - mA;
        if (depth < thr) {
            const double* F = &UG_HULL_F[4 * (A->f0 + fm)];
            v3 nw = mv(&TA->R, V(F[0], F[1], F[2]));
            cand_add(&L, vneg(nw), xf_apply(TB, cl), depth);
        }
    }
    reduce4(&L);
    for (int i = 0; i < L.n; i++) cand_add(out, L.c[i].n, L.c[i].pB, L.c[i].d);
}
/* hull (A, robot link) vs hull (B, club disc prism): vertex-in-hull both ways with the face planes
 * (restated substitute for GJK/EPA, as nc_hull_box): A's vertices against B's planes, then B's vertices
 * against A's planes, deepest + farthest-spread 4 points */
static void nc_hull_hull(const xf* TA, const collider* A, const xf* TB, const collider* B, double thr, candlist* out) {
    double mA = A->margin, mB = B->margin;
    static _Thread_local candlist L;
    cand_init(&L, A->full ? MAXCAND : LOD_MAXCAND);
    /* A vertex x in B's frame: max over B's faces of n.x - d */
    m3 RAB = mtm(&TB->R, &TA->R);
    v3 pAB = mtv(&TB->R, vsub(TA->p, TB->p));
    for (int i = 0; i < A->nv; i++) {
        const double* vv = &UG_HULL_V[3 * (A->v0 + i)];
        v3 x = vadd(mv(&RAB, V(vv[0], vv[1], vv[2])), pAB);
        double smax = -1e300;
        int fm = -1;
        for (int f = 0; f < B->nf; f++) {
            const double* F = &UG_HULL_F[4 * (B->f0 + f)];
            double sd = F[0] * x.x + F[1] * x.y + F[2] * x.z - F[3];
            if (sd > smax) { smax = sd; fm = f; }
        }
        double depth = smax - mA - mB;
        if (depth < thr) {
            const double* F = &UG_HULL_F[4 * (B->f0 + fm)];
            v3 nl = V(F[0], F[1], F[2]);
            v3 pl = vsub(x, vscale(nl, smax));
            cand_add(&L, mv(&TB->R, nl), xf_apply(TB, pl), depth);
        }
    }
    /* B vertex y in A's frame against A's faces */
    m3 RBA = mtm(&TA->R, &TB->R);
    v3 pBA = mtv(&TA->R, vsub(TB->p, TA->p));
    for (int i = 0; i < B->nv; i++) {
        const double* vv = &UG_HULL_V[3 * (B->v0 + i)];
        v3 yl = V(vv[0], vv[1], vv[2]);
        v3 y = vadd(mv(&RBA, yl), pBA);
        double smax = -1e300;
        int fm = -1;
        for (int f = 0; f < A->nf; f++) {
            const double* F = &UG_HULL_F[4 * (A->f0 + f)];
            double sd = F[0] * y.x + F[1] * y.y + F[2] * y.z - F[3];
            if (sd > smax) { smax = sd; fm = f; }
        }
        double depth = smax - mA - mB;
        if (depth < thr) {
            const double* F = &UG_HULL_F[4 * (A->f0 + fm)];
            v3 nw = mv(&TA->R, V(F[0], F[1], F[2]));
            cand_add(&L, vneg(nw), xf_apply(TB, yl), depth);
        }
    }
    reduce4(&L);
    for (int i = 0; i < L.n; i++) cand_add(out, L.c[i].n, L.c[i].pB, L.c[i].d);
}
/* hull (robot link, A) vs sphere (B): deepest face plane */
static void nc_hull_sphere(const xf* TA, const collider* A, const xf* TB, const collider* B, double thr, candlist* out) {
    v3 y = mtv(&TA->R, vsub(TB->p, TA->p));
    double r = B->half[0];
    double smax = -1e300;
    int fm = -1;
    for (int f = 0; f < A->nf; f++) {
        const double* F = &UG_HULL_F[4 * (A->f0 + f)];
        double sd = F[0] * y.x + F[1] * y.y + F[2] * y.z - F[3];
        if (sd > smax) { smax = sd; fm = f; }
    }
    double depth = smax - r - A->margin;
    if (depth >= thr) return;
    const double* F = &UG_HULL_F[4 * (A->f0 + fm)];
    v3 nw = vneg(mv(&TA->R, V(F[0], F[1], F[2])));
    cand_add(out, nw, vadd(TB->p, vscale(nw, r)), depth);
}

#else
#include "ug_fidelity.h"
#endif

/* ---- full geometry: the club disc as a true cylinder (UG_SHAPE_CYL) ----
 * btCylinderShapeZ [ext] (env_golf_v0.py:305: GEOM_CYLINDER radius 0.04, height 0.01) collides through GJK/EPA on its
 * analytic support map.  Restated here in the framework of the other convex pairs: exact point-to-cylinder distances
 * for the other shape's vertices (box corners / hull vertices / sphere centre), and the cylinder's support points
 * along the other shape's inward face normals tested against that shape's planes (as a box corner is against a
 * hull), deepest + farthest-spread 4.  The cylinder is its outer surface (radius r, half height hh, the safe margin
 * included); a support direction along the axis (a flat cap against a face) gives the cap's 4 rim points on the
 * shape frame's x / y axes.  Used with the full geometry (the default); UG_GEOM_LOD keeps the 16-gon prism. */
/* signed distance from x (cylinder frame) to the solid cylinder; nl: outward unit normal at the nearest surface point
 * pl (inside: the nearer of the side and the cap) */
static double cyl_point(double r, double hh, v3 x, v3* nl, v3* pl) {
    const double rho = ug_sqrt(x.x * x.x + x.y * x.y);
    const double dr = rho - r, dz = ug_fabs(x.z) - hh;
    const double sz = x.z < 0 ? -1.0 : 1.0;
    if (dr <= 0 && dz <= 0) {
        if (dr > dz && rho > 0) {
            *nl = V(x.x / rho, x.y / rho, 0.0);
            *pl = V(nl->x * r, nl->y * r, x.z);
            return dr;
        }
        *nl = V(0.0, 0.0, sz);
        *pl = V(x.x, x.y, sz * hh);
        return dz;
    }
    const double k = rho > r ? r / rho : 1.0;
    const v3 q = V(x.x * k, x.y * k, ug_max(-hh, ug_min(hh, x.z)));
    const v3 d = vsub(x, q);
    const double len = vlen(d);
    *nl = vscale(d, 1.0 / len);
    *pl = q;
    return len;
}
/* support points of the cylinder along u (cylinder frame): one rim point, or the cap's 4 rim points when u lies along
 * the axis */
static int cyl_support(double r, double hh, v3 u, v3* out) {
    const double sz = u.z < 0 ? -1.0 : 1.0;
    const double ur = ug_sqrt(u.x * u.x + u.y * u.y);
    if (ur > 1e-9) {
        out[0] = V(r * (u.x / ur), r * (u.y / ur), sz * hh);
        return 1;
    }
    out[0] = V(r, 0.0, sz * hh);
    out[1] = V(-r, 0.0, sz * hh);
    out[2] = V(0.0, r, sz * hh);
    out[3] = V(0.0, -r, sz * hh);
    return 4;
}
/* sphere (A) vs cylinder (B) */
static void nc_sphere_cyl(const xf* TA, const collider* A, const xf* TB, const collider* B, double thr, candlist* out) {
    const v3 x = xf_inv_apply(TB, TA->p);
    v3 nl, pl;
    const double d = cyl_point(B->half[0], B->half[2], x, &nl, &pl);
    const double depth = d - A->half[0];
    if (depth < thr) cand_add(out, mv(&TB->R, nl), xf_apply(TB, pl), depth);
}
/* face f of the polytope A (a box's 6 faces -x +x -y +y -z +z, or a hull's planes) as n.x <= off in A's frame */
static void poly_face(const collider* A, int f, v3* n, double* off) {
    if (A->kind == UG_SHAPE_BOX) {
        const int ax = f >> 1;
        const double sg = (f & 1) ? 1.0 : -1.0;
        *n = V(ax == 0 ? sg : 0.0, ax == 1 ? sg : 0.0, ax == 2 ? sg : 0.0);
        *off = A->half[ax];
        return;
    }
    const double* F = &UG_HULL_F[4 * (A->f0 + f)];
    *n = V(F[0], F[1], F[2]);
    *off = F[3];
}
/* polytope (A: robot hull or box) vs cylinder (B): A's vertices against the cylinder, then the cylinder's support
 * points along -n_f for every face f of A that has the cylinder's centre in front of it, each tested against all of
 * A's planes (the first maximum; the scan stops at a plane that already clears the threshold, as the corner test) */
static void nc_poly_cyl(const xf* TA, const collider* A, const xf* TB, const collider* B, double thr, candlist* out) {
    const double r = B->half[0], hh = B->half[2];
    const int hull = A->kind == UG_SHAPE_HULL;
    const double mA = hull ? A->margin : 0.0;
    const int nv = hull ? A->nv : 8, nf = hull ? A->nf : 6;
    static _Thread_local candlist L;
    cand_init(&L, A->full ? MAXCAND : LOD_MAXCAND);
    const m3 RAB = mtm(&TB->R, &TA->R);
    const v3 pAB = mtv(&TB->R, vsub(TA->p, TB->p));
    for (int i = 0; i < nv; i++) {
        v3 xa;
        if (hull) {
            const double* vv = &UG_HULL_V[3 * (A->v0 + i)];
            xa = V(vv[0], vv[1], vv[2]);
        } else {
            xa = V((i & 1) ? A->half[0] : -A->half[0], (i & 2) ? A->half[1] : -A->half[1], (i & 4) ? A->half[2] : -A->half[2]);
        }
        const v3 x = vadd(mv(&RAB, xa), pAB);
        v3 nl, pl;
        const double depth = cyl_point(r, hh, x, &nl, &pl) - mA;
        if (depth < thr) cand_add(&L, mv(&TB->R, nl), xf_apply(TB, pl), depth);
    }
    const m3 RBA = mtm(&TA->R, &TB->R);
    const v3 pBA = mtv(&TA->R, vsub(TB->p, TA->p));
    for (int f = 0; f < nf; f++) {
        v3 n;
        double off;
        poly_face(A, f, &n, &off);
        if (vdot(n, pBA) - off <= 0) continue; /* the cylinder's centre is not in front of face f */
        v3 sp[4];
        const int k = cyl_support(r, hh, mtv(&RBA, vneg(n)), sp);
        for (int j = 0; j < k; j++) {
            const v3 y = vadd(mv(&RBA, sp[j]), pBA);
            if (vdot(n, y) - off - mA >= thr) continue;
            double smax = -1e300;
            int fm = -1;
            for (int g = 0; g < nf; g++) {
                v3 ng;
                double og;
                poly_face(A, g, &ng, &og);
                const double sd = ng.x * y.x + ng.y * y.y + ng.z * y.z - og;
                if (sd > smax) { smax = sd; fm = g; }
                if (sd - mA >= thr) break;
            }
            const double depth = smax - mA;
            if (depth < thr) {
                v3 nm;
                double om;
                poly_face(A, fm, &nm, &om);
                cand_add(&L, vneg(mv(&TA->R, nm)), xf_apply(TB, sp[j]), depth);
            }
        }
    }
    reduce4(&L);
    for (int i = 0; i < L.n; i++) cand_add(out, L.c[i].n, L.c[i].pB, L.c[i].d);
}

/* btPersistentManifold [ext]: getCacheEntry / replaceContactPoint / addManifoldPoint / sortCachedPoints */
static int sort_cached(const manifold* M, const cpoint* pt) {
    int maxi = -1;
    double maxpen = pt->dist;
    for (int i = 0; i < 4; i++)
        if (M->pt[i].dist < maxpen) { maxi = i; maxpen = M->pt[i].dist; }
    double res[4] = {0, 0, 0, 0};
    if (maxi != 0) { v3 a = vsub(pt->lpA, M->pt[1].lpA), b = vsub(M->pt[3].lpA, M->pt[2].lpA); v3 c = vcross(a, b); res[0] = vdot(c, c); }
    if (maxi != 1) { v3 a = vsub(pt->lpA, M->pt[0].lpA), b = vsub(M->pt[3].lpA, M->pt[2].lpA); v3 c = vcross(a, b); res[1] = vdot(c, c); }
    if (maxi != 2) { v3 a = vsub(pt->lpA, M->pt[0].lpA), b = vsub(M->pt[3].lpA, M->pt[1].lpA); v3 c = vcross(a, b); res[2] = vdot(c, c); }
    if (maxi != 3) { v3 a = vsub(pt->lpA, M->pt[0].lpA), b = vsub(M->pt[2].lpA, M->pt[1].lpA); v3 c = vcross(a, b); res[3] = vdot(c, c); }
    int bi = -1;
    double bv = -1e300;
    for (int i = 0; i < 4; i++)
        if (ug_fabs(res[i]) > bv) { bv = ug_fabs(res[i]); bi = i; }
    return bi;
}
static void manifold_add(manifold* M, const xf* TA, const xf* TB, const cand* c, double thr) {
    if (c->d > thr) return;
    v3 pA = vadd(c->pB, vscale(c->n, c->d));
    cpoint np;
    np.lpA = xf_inv_apply(TA, pA);
    np.lpB = xf_inv_apply(TB, c->pB);
    np.n = c->n;
    np.dist = c->d;
    np.imp = np.imp1 = np.imp2 = 0.0;
    double shortest = thr * thr;
    int near = -1;
    for (int i = 0; i < M->npts; i++) {
        v3 d = vsub(M->pt[i].lpA, np.lpA);
        double x = vdot(d, d);
        if (x < shortest) { shortest = x; near = i; }
    }
    if (near >= 0) {
        np.imp = M->pt[near].imp; np.imp1 = M->pt[near].imp1; np.imp2 = M->pt[near].imp2;
        M->pt[near] = np;
        return;
    }
    int ins = M->npts;
    if (ins == 4) ins = sort_cached(M, &np);
    else M->npts++;
    if (ins < 0) ins = 0;
    M->pt[ins] = np;
}
/* test hook (tests/test_manifold_kat.py): manifold_add on a crafted manifold.  pts: npts x 13 doubles (lpA, lpB, n,
 * dist, imp, imp1, imp2); TA, TB: R (row-major 9) + p (3); c: n, pB, d.  Writes the manifold back (4 x 13) and returns
 * its point count. */
int ugo_manifold_add(double* pts, int npts, const double* TA12, const double* TB12, const double* c7, double thr) {
    manifold M;
    M.npts = npts;
    for (int i = 0; i < npts; i++) {
        const double* q = pts + 13 * i;
        M.pt[i].lpA = V(q[0], q[1], q[2]);
        M.pt[i].lpB = V(q[3], q[4], q[5]);
        M.pt[i].n = V(q[6], q[7], q[8]);
        M.pt[i].dist = q[9];
        M.pt[i].imp = q[10]; M.pt[i].imp1 = q[11]; M.pt[i].imp2 = q[12];
    }
    xf TA, TB;
    TA.R = mload(TA12); TA.p = V(TA12[9], TA12[10], TA12[11]);
    TB.R = mload(TB12); TB.p = V(TB12[9], TB12[10], TB12[11]);
    cand c;
    c.n = V(c7[0], c7[1], c7[2]);
    c.pB = V(c7[3], c7[4], c7[5]);
    c.d = c7[6];
    manifold_add(&M, &TA, &TB, &c, thr);
    for (int i = 0; i < M.npts; i++) {
        double* q = pts + 13 * i;
        q[0] = M.pt[i].lpA.x; q[1] = M.pt[i].lpA.y; q[2] = M.pt[i].lpA.z;
        q[3] = M.pt[i].lpB.x; q[4] = M.pt[i].lpB.y; q[5] = M.pt[i].lpB.z;
        q[6] = M.pt[i].n.x; q[7] = M.pt[i].n.y; q[8] = M.pt[i].n.z;
        q[9] = M.pt[i].dist; q[10] = M.pt[i].imp; q[11] = M.pt[i].imp1; q[12] = M.pt[i].imp2;
    }
    return M.npts;
}
static void manifold_refresh(manifold* M, const xf* TA, const xf* TB, double thr) {
    for (int i = M->npts - 1; i >= 0; i--) {
        cpoint* p = &M->pt[i];
        v3 pA = xf_apply(TA, p->lpA), pB = xf_apply(TB, p->lpB);
        p->dist = vdot(vsub(pA, pB), p->n);
    }
    for (int i = M->npts - 1; i >= 0; i--) {
        cpoint* p = &M->pt[i];
        int rm = 0;
        if (p->dist > thr) rm = 1;
        else {
            v3 pA = xf_apply(TA, p->lpA), pB = xf_apply(TB, p->lpB);
            v3 proj = vsub(pA, vscale(p->n, p->dist));
            v3 d = vsub(pB, proj);
            if (vdot(d, d) > thr * thr) rm = 1;
        }
        if (rm) {
            int last = M->npts - 1;
            if (i != last) M->pt[i] = M->pt[last];
            M->npts--;
        }
    }
}

static int collider_active(const ugo_env* e, const collider* c) {
    if (c->owner <= -2 && c->owner > -100) return e->oactive[-2 - c->owner];
    return 1;
}

/* performDiscreteCollisionDetection: broadphase + narrowphase + manifold update */
static void collide(ugo_env* e, const kin* k) {
    const scene* s = &e->sc;
    xf O[MAXCOL];
    v3 lo[MAXCOL], hi[MAXCOL];
    for (int i = 0; i < s->ncol; i++) {
        const collider* c = &s->col[i];
        O[i] = owner_xf(e, k, c->owner);
        world_aabb(&O[i], c, &lo[i], &hi[i]);
        lo[i] = vsub(lo[i], V(UG_AABB_PAD, UG_AABB_PAD, UG_AABB_PAD));
        hi[i] = vadd(hi[i], V(UG_AABB_PAD, UG_AABB_PAD, UG_AABB_PAD));
    }
    /* Narrowphase for every overlapping pair, in pair-table order.  The manifold list is kept
     * sorted by pair id and holds only pairs with contact points (an empty manifold carries neither
     * rows nor predicates); a pair whose AABBs stop overlapping loses its manifold (Bullet destroys
     * the algorithm with the broadphase pair).  Bullet's own manifold order (dispatcher array, then
     * island sort) is not reproducible, so the row order here is: by pair id, then point. */
    manifold nm[MAXMAN];
    int nn = 0, cursor = 0;
    for (int p = 0; p < s->npair; p++) {
        const pairdef* P = &s->pair[p];
        int a = P->a, b = P->b;
        manifold M;
        M.pair = p;
        M.npts = 0;
        while (cursor < e->nman && e->man[cursor].pair < p) cursor++;
        if (cursor < e->nman && e->man[cursor].pair == p) M = e->man[cursor];
        int ov = collider_active(e, &s->col[a]) && collider_active(e, &s->col[b]) &&
                 !(lo[a].x > hi[b].x || hi[a].x < lo[b].x || lo[a].y > hi[b].y || hi[a].y < lo[b].y ||
                   lo[a].z > hi[b].z || hi[a].z < lo[b].z);
        if (!ov) continue;
        const collider* A = &s->col[a];
        const collider* B = &s->col[b];
        xf TA = shape_xf(&O[a], A), TB = shape_xf(&O[b], B);
        candlist L;
        cand_init(&L, LOD_MAXCAND);
        if (s->gjk && pair_is_gjk(A, B)) nc_gjk(&TA, A, &TB, B, P->thr, &L);
        else if (A->kind == UG_SHAPE_SPHERE && B->kind == UG_SHAPE_BOX) nc_sphere_box(&TA, A, &TB, B, P->thr, &L);
        else if (A->kind == UG_SHAPE_SPHERE && B->kind == UG_SHAPE_SPHERE) nc_sphere_sphere(&TA, A, &TB, B, P->thr, &L);
        else if (A->kind == UG_SHAPE_BOX && B->kind == UG_SHAPE_BOX) nc_box_box(&TA, A, &TB, B, P->thr, &L);
        else if (A->kind == UG_SHAPE_HULL && B->kind == UG_SHAPE_BOX) nc_hull_box(&TA, A, &TB, B, P->thr, &L);
        else if (A->kind == UG_SHAPE_HULL && B->kind == UG_SHAPE_SPHERE) nc_hull_sphere(&TA, A, &TB, B, P->thr, &L);
        else if (A->kind == UG_SHAPE_HULL && B->kind == UG_SHAPE_HULL) nc_hull_hull(&TA, A, &TB, B, P->thr, &L);
        else if (A->kind == UG_SHAPE_SPHERE && B->kind == UG_SHAPE_CYL) nc_sphere_cyl(&TA, A, &TB, B, P->thr, &L);
        else if ((A->kind == UG_SHAPE_HULL || A->kind == UG_SHAPE_BOX) && B->kind == UG_SHAPE_CYL)
            nc_poly_cyl(&TA, A, &TB, B, P->thr, &L);
        else if (A->kind == UG_SHAPE_CYL && B->kind == UG_SHAPE_BOX) {
            /* cylinder-box with swapped roles: flip the normal, move the point onto the box */
            candlist L2;
            cand_init(&L2, LOD_MAXCAND);
            nc_poly_cyl(&TB, B, &TA, A, P->thr, &L2);
            for (int i = 0; i < L2.n; i++)
                cand_add(&L, vneg(L2.c[i].n), vadd(L2.c[i].pB, vscale(L2.c[i].n, L2.c[i].d)), L2.c[i].d);
        }
        else if (A->kind == UG_SHAPE_SPHERE && B->kind == UG_SHAPE_HULL) {
            /* hull-sphere with swapped roles: flip normal, move the point onto the sphere */
            candlist L2;
            cand_init(&L2, LOD_MAXCAND);
            nc_hull_sphere(&TB, B, &TA, A, P->thr, &L2);
            for (int i = 0; i < L2.n; i++)
                cand_add(&L, vneg(L2.c[i].n), vadd(L2.c[i].pB, vscale(L2.c[i].n, L2.c[i].d)), L2.c[i].d);
        }
        else if (A->kind == UG_SHAPE_BOX && B->kind == UG_SHAPE_SPHERE) {
            /* sphere-box with swapped roles: flip normal, move the point onto the sphere */
            candlist L2;
            cand_init(&L2, LOD_MAXCAND);
            nc_sphere_box(&TB, B, &TA, A, P->thr, &L2);
            for (int i = 0; i < L2.n; i++)
                cand_add(&L, vneg(L2.c[i].n), vadd(L2.c[i].pB, vscale(L2.c[i].n, L2.c[i].d)), L2.c[i].d);
        }
#ifdef UG_ROWHIST /* development aid (tools/row_hist.py): every overlapping pair, its candidates and the deepest */
        {
            extern int dprintf(int, const char*, ...);
            double dm = 1e9;
            for (int i = 0; i < L.n; i++) dm = L.c[i].d < dm ? L.c[i].d : dm;
            dprintf(2, "PAIR %d %d %d %d %d %d %.6f\n", p, a, b, A->kind, B->kind, L.n, dm);
        }
#endif
        /* manifold frames = owner frames.  A compound collision object refreshes its child manifolds before the
         * child narrowphases (btCompoundCollisionAlgorithm::processCollision), then the child's own algorithm
         * refreshes after its points (the convex-convex path; the vertex-in-hull mode keeps rounds 1-3's order) */
        if (s->gjk && (A->compound || B->compound) && M.npts) manifold_refresh(&M, &O[a], &O[b], P->thr);
        for (int i = 0; i < L.n; i++) manifold_add(&M, &O[a], &O[b], &L.c[i], P->thr);
        if (M.npts) manifold_refresh(&M, &O[a], &O[b], P->thr);
        if (M.npts == 0) continue;
        if (nn < MAXMAN) nm[nn++] = M;
        else e->overflow++;
    }
    for (int m = 0; m < nn; m++) e->man[m] = nm[m];
    e->nman = nn;
}

/* ======================================================================== */
/* constraint rows + projected Gauss-Seidel (btMultiBodyConstraintSolver)    */
/* ======================================================================== */
/* A row holds its Jacobian J and M^-1 J^T over the full generalized-velocity vector
 * (robot dofs 0..11, object o at 12 + 6 o .. 17 + 6 o, zero-padded to UG_NVP = 32 slots). */
#define UG_NVP 32
typedef struct {
    double J[UG_NVP], MiJ[UG_NVP];
    double invD, rhs, rhsPen, lo, hi, imp, impPen, fric;
    int man, pt, kind;         /* kind 0 non-contact, 1 normal, 2/3 friction dir 1/2, 4/5 rolling axis 1/2 */
    int nrow;                  /* friction rows: index of their normal row */
} row;

typedef struct {
    int n, nnc, nn, nf, nr;
    row r[MAXROWS];
    int idx_nc[MAXROWS], idx_n[MAXROWS], idx_f[MAXROWS], idx_r[MAXROWS];
} rowset;

static int ent_dofs(int ent) { return ent == 0 ? NB : 6; }
static int ent_off(int ent) { return ent == 0 ? 0 : NB + 6 * (ent - 1); }
static double ent_dot(int ent, const double* J, const double* v) {
    int n = ent_dofs(ent), o = ent_off(ent);
    double s = 0.0;
    for (int i = 0; i < n; i++) s += J[i] * v[o + i];
    return s;
}
static double ent_dot_local(int ent, const double* a, const double* b) {
    int n = ent_dofs(ent);
    double s = 0.0;
    for (int i = 0; i < n; i++) s += a[i] * b[i];
    return s;
}
static void scatter(int ent, const double* src, double* dst) {
    int n = ent_dofs(ent), o = ent_off(ent);
    for (int i = 0; i < n; i++) dst[o + i] = src[i];
}

/* Jacobian of a point p on entity ent along direction d (linear) */
static void point_jac(const ugo_env* e, const kin* k, int ent, int body, v3 p, v3 d, double* J, double* MiJ,
                      const double* LDL) {
    if (ent == 0) {
        for (int i = 0; i < NB; i++) {
            J[i] = moves(i, body) ? vdot(d, vcross(k->a[i], vsub(p, k->p[i]))) : 0.0;
            MiJ[i] = J[i];
        }
        ldlt_solve(LDL, NB, MiJ);
    } else {
        int o = ent - 1;
        const UgJoint* Jt = &e->sc.ojoint[o];
        if (Jt->kind != UGJ_FREE) { /* one-dof link (ug_joint.h): its slot 0 */
            double pp[3] = {p.x, p.y, p.z}, dd[3] = {d.x, d.y, d.z};
            double j = ugj_point_jac(Jt, pp, dd);
            J[0] = j; J[1] = 0.0; J[2] = 0.0; J[3] = 0.0; J[4] = 0.0; J[5] = 0.0;
            MiJ[0] = j / e->jM[o]; MiJ[1] = 0.0; MiJ[2] = 0.0; MiJ[3] = 0.0; MiJ[4] = 0.0; MiJ[5] = 0.0;
            return;
        }
        v3 r = vsub(p, e->opos[o]);
        v3 rn = vcross(r, d);
        J[0] = d.x; J[1] = d.y; J[2] = d.z; J[3] = rn.x; J[4] = rn.y; J[5] = rn.z;
        double im = 1.0 / e->sc.omass[o];
        m3 R = qmat(e->oquat[o]);
        v3 ir = mtv(&R, rn);
        ir = V(ir.x / e->sc.oinertia[o].x, ir.y / e->sc.oinertia[o].y, ir.z / e->sc.oinertia[o].z);
        ir = mv(&R, ir);
        MiJ[0] = d.x * im; MiJ[1] = d.y * im; MiJ[2] = d.z * im; MiJ[3] = ir.x; MiJ[4] = ir.y; MiJ[5] = ir.z;
    }
}

/* Jacobian of an angular velocity component along u on entity ent (rolling friction rows) */
static void ang_jac(const ugo_env* e, const kin* k, int ent, int body, v3 u, double* J, double* MiJ, const double* LDL) {
    if (ent == 0) {
        for (int i = 0; i < NB; i++) {
            J[i] = moves(i, body) ? vdot(u, k->a[i]) : 0.0;
            MiJ[i] = J[i];
        }
        ldlt_solve(LDL, NB, MiJ);
    } else {
        int o = ent - 1;
        const UgJoint* Jt = &e->sc.ojoint[o];
        if (Jt->kind != UGJ_FREE) {
            double uu[3] = {u.x, u.y, u.z};
            double j = ugj_ang_jac(Jt, uu);
            J[0] = j; J[1] = 0.0; J[2] = 0.0; J[3] = 0.0; J[4] = 0.0; J[5] = 0.0;
            MiJ[0] = j / e->jM[o]; MiJ[1] = 0.0; MiJ[2] = 0.0; MiJ[3] = 0.0; MiJ[4] = 0.0; MiJ[5] = 0.0;
            return;
        }
        J[0] = 0.0; J[1] = 0.0; J[2] = 0.0; J[3] = u.x; J[4] = u.y; J[5] = u.z;
        m3 R = qmat(e->oquat[o]);
        v3 ir = mtv(&R, u);
        ir = V(ir.x / e->sc.oinertia[o].x, ir.y / e->sc.oinertia[o].y, ir.z / e->sc.oinertia[o].z);
        ir = mv(&R, ir);
        MiJ[0] = 0.0; MiJ[1] = 0.0; MiJ[2] = 0.0; MiJ[3] = ir.x; MiJ[4] = ir.y; MiJ[5] = ir.z;
    }
}
static int ent_of_collider(const collider* c, int* body) {
    *body = -1;
    if (c->owner >= 0) { *body = c->owner; return 0; }
    if (c->owner == -1) return -1; /* fixed robot base */
    if (c->owner > -100) return -1 - c->owner; /* object i -> 1+i */
    return -1;
}

static void row_clear(row* r) { memset(r, 0, sizeof(*r)); }

/* contact-type row: J_A at pA along +d, J_B at pB along -d; returns relative velocity J.v0 */
static double contact_row(const ugo_env* e, const kin* k, const double* LDL, const double* v0, row* r, int entA,
                          int bodyA, int entB, int bodyB, v3 pA, v3 pB, v3 d, int ang) {
    double JA[NB], MiJA[NB], JB[NB], MiJB[NB];
    double dA = 0.0, dB = 0.0, relv = 0.0;
    if (entA >= 0) {
        if (ang) ang_jac(e, k, entA, bodyA, d, JA, MiJA, LDL);
        else point_jac(e, k, entA, bodyA, pA, d, JA, MiJA, LDL);
        dA = ent_dot_local(entA, JA, MiJA);
        relv += ent_dot(entA, JA, v0);
        scatter(entA, JA, r->J);
        scatter(entA, MiJA, r->MiJ);
    }
    if (entB >= 0) {
        if (ang) ang_jac(e, k, entB, bodyB, vneg(d), JB, MiJB, LDL);
        else point_jac(e, k, entB, bodyB, pB, vneg(d), JB, MiJB, LDL);
        dB = ent_dot_local(entB, JB, MiJB);
        relv += ent_dot(entB, JB, v0);
        scatter(entB, JB, r->J);
        scatter(entB, MiJB, r->MiJ);
    }
    double den = dA + dB;
    r->invD = den > 2.220446049250313e-16 ? 1.0 / den : 0.0;
    return relv;
}
/* single-dof row of a jointed object's slot (its limits and motor) */
static double jdof_row(const ugo_env* e, const double* v0, row* r, int o, double sgn) {
    int off = NB + 6 * o;
    r->J[off] = sgn;
    r->MiJ[off] = sgn / e->jM[o];
    double den = sgn * r->MiJ[off];
    r->invD = den > 2.220446049250313e-16 ? 1.0 / den : 0.0;
    return sgn * v0[off];
}
/* single-dof row (limit / motor): J = sgn * e_d */
static double dof_row(const double* LDL, const double* v0, row* r, int d, double sgn) {
    double J[NB], MiJ[NB];
    memset(J, 0, sizeof(J));
    J[d] = sgn;
    memcpy(MiJ, J, sizeof(J));
    ldlt_solve(LDL, NB, MiJ);
    double den = ent_dot_local(0, J, MiJ);
    r->invD = den > 2.220446049250313e-16 ? 1.0 / den : 0.0;
    scatter(0, J, r->J);
    scatter(0, MiJ, r->MiJ);
    return ent_dot(0, J, v0);
}

static void build_rows(ugo_env* e, const kin* k, const double* LDL, const double* v0, rowset* rs) {
    rs->n = rs->nnc = rs->nn = rs->nf = rs->nr = 0;
    const double dt = UG_DT;
    /* joint limits (btMultiBodyJointLimitConstraint, created at URDF load in link order) */
    for (int d = 0; d < NB; d++) {
        for (int side = 0; side < 2; side++) {
            double pen = side == 0 ? e->q[d] - UG_DOF_LOWER[d] : UG_DOF_UPPER[d] - e->q[d];
            if (pen > 0) continue;
            if (rs->n >= MAXROWS) { e->overflow++; continue; }
            row* r = &rs->r[rs->n];
            row_clear(r);
            double relv = dof_row(LDL, v0, r, d, side == 0 ? 1.0 : -1.0);
            double erp = (pen > UG_SPLIT_PEN_THR) ? UG_ERP : UG_ERP2;
            double perr = -pen * erp / dt, verr = -relv;
            double pimp = perr * r->invD, vimp = verr * r->invD;
            r->rhs = (pen > UG_SPLIT_PEN_THR) ? pimp + vimp : vimp;
            r->lo = 0.0; r->hi = UG_LIMIT_MAXIMP;
            r->kind = 0;
            rs->idx_nc[rs->nnc++] = rs->n++;
        }
    }
    /* position motors (btMultiBodyJointMotor, created per joint at load; zero-force ones carry no impulse) */
    for (int m = 0; m < 7; m++) {
        if (!e->mon[m]) continue;
        int d = m < 6 ? m : UG_FINGER_DOF;
        double maxImp = UG_DOF_MAXFORCE[d] * dt;
        if (rs->n >= MAXROWS) { e->overflow++; continue; }
        row* r = &rs->r[rs->n];
        row_clear(r);
        double relv = dof_row(LDL, v0, r, d, 1.0);
        double qd = v0[d];
        double pst = 1.0 * (e->mtarget[m] - e->q[d]) / dt;
        double verr = 0.0 - qd;
        double des = UG_MOTOR_KP * pst + qd + UG_MOTOR_KD * verr;
        double clamp = UG_DOF_MAXVEL[d];
        if (des > clamp) des = clamp;
        if (des < -clamp) des = -clamp;
        r->rhs = 0.0 * r->invD + (des - relv) * r->invD;
        r->lo = -maxImp; r->hi = maxImp;
        r->kind = 0;
        rs->idx_nc[rs->nnc++] = rs->n++;
    }
    /* mimic gears (robot.py:202-211): J_A = e_finger, J_B = ratio e_child (same multibody: Bullet's
     * diagonal omits the A/B cross term; J and M^-1 J^T of the two parts are summed) */
    for (int g = 0; g < 5; g++) {
        if (rs->n >= MAXROWS) { e->overflow++; continue; }
        int pa = UG_FINGER_DOF, cb = UG_GEAR_CHILD[g];
        double ratio = UG_GEAR_RATIO[g];
        row* r = &rs->r[rs->n];
        row_clear(r);
        double JA[NB], JB[NB], MiJA[NB], MiJB[NB];
        memset(JA, 0, sizeof(JA));
        memset(JB, 0, sizeof(JB));
        JA[pa] = 1.0;
        JB[cb] = ratio;
        memcpy(MiJA, JA, sizeof(JA));
        memcpy(MiJB, JB, sizeof(JB));
        ldlt_solve(LDL, NB, MiJA);
        ldlt_solve(LDL, NB, MiJB);
        double den = ent_dot_local(0, JA, MiJA) + ent_dot_local(0, JB, MiJB);
        r->invD = den > 2.220446049250313e-16 ? 1.0 / den : 0.0;
        for (int i = 0; i < NB; i++) { r->J[i] = JA[i] + JB[i]; r->MiJ[i] = MiJA[i] + MiJB[i]; }
        double relv = ent_dot(0, JA, v0) + ent_dot(0, JB, v0);
        double diff = e->q[cb] * ratio + e->q[pa];
        double pen = -UG_GEAR_ERP * (0.0 - diff);
        /* fillMultiBodyConstraint: split impulse not implemented for multibody rows -> always m_erp, combined */
        double perr = -pen * UG_ERP / dt, verr = 0.0 - relv;
        r->rhs = perr * r->invD + verr * r->invD;
        double maxImp = UG_GEAR_MAXF * dt;
        r->lo = -maxImp; r->hi = maxImp;
        r->kind = 0;
        rs->idx_nc[rs->nnc++] = rs->n++;
    }
    /* the box's joint limits (btMultiBodyJointLimitConstraint, created at its load after the robot's constraints,
     * joint order) and the button's position motor (reset_box, env_box_v0.py:175: force 1, target 0, default
     * gains, no maxVelocity -> no clamp [ext]; the door's motor has force 0 (:176) and carries no row) */
    const scene* s = &e->sc;
    for (int jj = 0; jj < s->njoint; jj++) {
        int o = s->jorder[jj];
        if (!e->oactive[o]) continue;
        const UgJoint* Jt = &s->ojoint[o];
        double qj = e->ow[o].x;
        for (int side = 0; side < 2; side++) {
            double pen = side == 0 ? qj - Jt->lower : Jt->upper - qj;
            if (pen > 0) continue;
            if (rs->n >= MAXROWS) { e->overflow++; continue; }
            row* r = &rs->r[rs->n];
            row_clear(r);
            double relv = jdof_row(e, v0, r, o, side == 0 ? 1.0 : -1.0);
            double erp = (pen > UG_SPLIT_PEN_THR) ? UG_ERP : UG_ERP2;
            double perr = -pen * erp / dt, verr = -relv;
            double pimp = perr * r->invD, vimp = verr * r->invD;
            r->rhs = (pen > UG_SPLIT_PEN_THR) ? pimp + vimp : vimp;
            r->lo = 0.0; r->hi = UG_LIMIT_MAXIMP;
            r->kind = 0;
            rs->idx_nc[rs->nnc++] = rs->n++;
        }
    }
    if (s->task == UG_TASK_BOX && e->oactive[1]) {
        if (rs->n >= MAXROWS) e->overflow++;
        else {
            row* r = &rs->r[rs->n];
            row_clear(r);
            double relv = jdof_row(e, v0, r, 1, 1.0);
            double qd = v0[NB + 6];
            double pst = 1.0 * (0.0 - e->ow[1].x) / dt;
            double verr = 0.0 - qd;
            double des = UG_MOTOR_KP * pst + qd + UG_MOTOR_KD * verr;
            double maxImp = UG_BX_BUTTON_FORCE * dt;
            r->rhs = 0.0 * r->invD + (des - relv) * r->invD;
            r->lo = -maxImp; r->hi = maxImp;
            r->kind = 0;
            rs->idx_nc[rs->nnc++] = rs->n++;
        }
    }
    /* contacts, manifold order: normal row + two friction rows per point */
    for (int m = 0; m < e->nman; m++) {
        const manifold* M = &e->man[m];
        const pairdef* P = &s->pair[M->pair];
        int bodyA, bodyB;
        int entA = ent_of_collider(&s->col[P->a], &bodyA);
        int entB = ent_of_collider(&s->col[P->b], &bodyB);
        if (entA < 0 && entB < 0) continue;
        xf OA = owner_xf(e, k, s->col[P->a].owner), OB = owner_xf(e, k, s->col[P->b].owner);
        int roll = P->rolling > 0.0; /* rolling friction: two more angular rows per point */
        for (int j = 0; j < M->npts; j++) {
            if (rs->n + (roll ? 5 : 3) > MAXROWS) { e->overflow++; continue; }
            const cpoint* cp = &M->pt[j];
            v3 pA = xf_apply(&OA, cp->lpA), pB = xf_apply(&OB, cp->lpB);
            v3 n = cp->n;
            int ni = rs->n;
            row* r = &rs->r[ni];
            row_clear(r);
            double relv = contact_row(e, k, LDL, v0, r, entA, bodyA, entB, bodyB, pA, pB, n, 0);
            /* a row with zero effective mass (e.g. a contact normal parallel to the only joint axis)
             * is kept as a no-op: rhs = 0, impulse stays 0, residual 0 (Bullet drops it) */
            double pen = cp->dist + UG_LINEAR_SLOP;
            double rest = 0.0;
            if (!(ug_fabs(relv) < UG_REST_VEL_THR)) rest = P->restitution * -relv;
            if (rest <= 0.0) rest = 0.0;
            double verr = rest - relv, perr;
            double erp = (pen > UG_SPLIT_PEN_THR) ? UG_ERP : UG_ERP2;
            if (pen > 0) { perr = 0.0; verr -= pen / UG_DT; }
            else perr = -pen * erp / UG_DT;
            double pimp = perr * r->invD, vimp = verr * r->invD;
            if (pen > UG_SPLIT_PEN_THR) { r->rhs = pimp + vimp; r->rhsPen = 0.0; }
            else { r->rhs = vimp; r->rhsPen = pimp; }
            r->lo = 0.0; r->hi = 1e10;
            r->imp = cp->imp * UG_WARMSTART;
            r->kind = 1; r->man = m; r->pt = j;
            rs->idx_n[rs->nn++] = rs->n++;
            /* btPlaneSpace1 friction directions */
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
            for (int fdir = 0; fdir < 2; fdir++) {
                row* f = &rs->r[rs->n];
                row_clear(f);
                double frel = contact_row(e, k, LDL, v0, f, entA, bodyA, entB, bodyB, pA, pB, fdir == 0 ? t1 : t2, 0);
                f->rhs = 0.0 * f->invD + (0.0 - frel) * f->invD;
                f->fric = P->friction;
                f->lo = 0.0; f->hi = 0.0;
                f->imp = 0.0;
                f->kind = 2 + fdir; f->man = m; f->pt = j; f->nrow = ni;
                rs->idx_f[rs->nf++] = rs->n++;
            }
            /* btMultiBodyConstraintSolver torsional (rolling) friction [ext]: angular rows about the two
             * btPlaneSpace1 axes, bounds +-rolling * the normal impulse (restated as pyramid rows) */
            for (int rdir = 0; roll && rdir < 2; rdir++) {
                row* f = &rs->r[rs->n];
                row_clear(f);
                double frel = contact_row(e, k, LDL, v0, f, entA, bodyA, entB, bodyB, pA, pB, rdir == 0 ? t1 : t2, 1);
                f->rhs = 0.0 * f->invD + (0.0 - frel) * f->invD;
                f->fric = P->rolling;
                f->lo = 0.0; f->hi = 0.0;
                f->imp = 0.0;
                f->kind = 4 + rdir; f->man = m; f->pt = j; f->nrow = ni;
                rs->idx_r[rs->nr++] = rs->n++;
            }
        }
    }
}

/* ---- projected Gauss-Seidel in row space ----
 * Bullet's btMultiBodyConstraintSolver keeps the solver's velocity delta dv and evaluates each row as
 * delta_r = rhs_r - (J_r . dv) / D_r.  The same iteration is written here in row space: the unclamped
 * increment u_r = rhs_r - (J_r . dv) / D_r of every row is kept instead of dv, so a row update reads u_r
 * and adds column r of the scaled Delassus matrix NB[i][j] = -(J_i M^-1 J_j^T) / D_i times the impulse
 * change to u.  Mathematically this is the identical sequence of Gauss-Seidel updates (same row order,
 * same clamps, same residual); only the floating-point rounding differs, and it is *defined* here so that
 * the HIP kernel (one lane per row) reproduces it bit for bit:
 *   NB[i][j] = -((fma chain over slots d = 0..UG_NVP-1 of J_i[d] * MiJ_j[d]) * invD_i)  (solve positions)
 *   u_i      = rhs_i, then u_i = fma(NB[i][r], delta_r, u_i) after each update of row r
 *   dv[d]    = fma chain over positions k = 0..n-1 of MiJ_k[d] * impulse_k   (after the iterations)
 * Solve positions: non-contact rows [0, nnc), normals [nnc, fb), frictions, then rolling-friction rows. */
static __thread double g_A[MAXROWS][MAXROWS]; /* NB */
static double rdot(const double* J, const double* MiJ) {
    double s = 0.0;
    for (int d = 0; d < UG_NVP; d++) s = fma(J[d], MiJ[d], s); /* padded slots are zero */
    return s;
}
/* resolveSingleConstraintRowGeneric [ext] (cfm = 0) for the row at position p, in its clamp-the-increment
 * form: delta = clamp(u_p, lo - imp, hi - imp), imp += delta.  (Bullet clamps imp + delta against
 * [lo, hi] and assigns the bound; the two agree up to the rounding of imp + (bound - imp), i.e. at most
 * one ulp on a clamped impulse.) */
static double solve_row_u(row* r, int p, int n, double* u, int pen) {
    double imp = pen ? r->impPen : r->imp;
    double dlo = r->lo - imp, dhi = r->hi - imp;
    double di = u[p];
    di = di < dlo ? dlo : di; /* v_max_f64 */
    di = di > dhi ? dhi : di; /* v_min_f64 */
    imp = imp + di;
    if (pen) r->impPen = imp; else r->imp = imp;
    for (int q = 0; q < n; q++) u[q] = fma(g_A[q][p], di, u[q]);
    double rinv = r->invD == 0.0 ? 0.0 : 1.0 / r->invD;
    return di * rinv;
}

/* debug record of the last PGS call (tests only): n, nnc, nn, nf, nr, sweeps, split sweeps */
static __thread int g_dbg[8];
void ugo_debug_rows(int* out) { memcpy(out, g_dbg, sizeof(g_dbg)); }
static __thread double g_dbg_w[4 * 128];
/* last PGS call: A (row-major [MAXROWS][MAXROWS]), w after the warm start, w and impulses after the sweeps */
void ugo_debug_pgs(double* A, double* w4) {
    memcpy(A, g_A, sizeof(g_A));
    memcpy(w4, g_dbg_w, sizeof(g_dbg_w));
}
static int pgs(rowset* rs, double* dv, double* dvs) {
    row* R[MAXROWS];
    int n = 0, pos_of[MAXROWS];
    for (int j = 0; j < rs->nnc; j++) R[n++] = &rs->r[rs->idx_nc[j]];
    for (int j = 0; j < rs->nn; j++) R[n++] = &rs->r[rs->idx_n[j]];
    for (int j = 0; j < rs->nf; j++) R[n++] = &rs->r[rs->idx_f[j]];
    for (int j = 0; j < rs->nr; j++) R[n++] = &rs->r[rs->idx_r[j]];
    for (int p = 0; p < n; p++) pos_of[R[p] - rs->r] = p;
    const int nnc = rs->nnc, fb = rs->nnc + rs->nn;
    g_dbg[0] = n; g_dbg[1] = nnc; g_dbg[2] = rs->nn; g_dbg[3] = rs->nf; g_dbg[4] = rs->nr; g_dbg[5] = 0; g_dbg[6] = 0;
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) g_A[i][j] = -(rdot(R[i]->J, R[j]->MiJ) * R[i]->invD);
    double w[MAXROWS]; /* u */
    for (int q = 0; q < n; q++) w[q] = R[q]->rhs;
    /* warm start (normal rows only; Bullet warm-starts friction with 0) */
    for (int p = nnc; p < fb; p++) {
        double imp = R[p]->imp;
        if (imp != 0.0)
            for (int q = 0; q < n; q++) w[q] = fma(g_A[q][p], imp, w[q]);
    }
    for (int q = 0; q < 128; q++) g_dbg_w[q] = q < n ? w[q] : 0.0;
    for (int it = 0; it < UG_PGS_ITERS; it++) {
        double res = 0.0;
        /* non-contact rows: alternate direction (reverse on even sweeps) */
        for (int j = 0; j < nnc; j++) {
            int p = (it & 1) ? j : nnc - 1 - j;
            double x = solve_row_u(R[p], p, n, w, 0);
            x = x * x;
            res = res > x ? res : x;
        }
        for (int p = nnc; p < fb; p++) {
            double x = solve_row_u(R[p], p, n, w, 0);
            x = x * x;
            res = res > x ? res : x;
        }
        /* friction / rolling rows: bounds +-mu * (their normal's impulse), skipped while it is not positive */
        for (int p = fb; p < n; p++) {
            row* f = R[p];
            double tot = R[pos_of[f->nrow]]->imp;
            if (tot > 0.0) {
                f->lo = -(f->fric * tot);
                f->hi = f->fric * tot;
                double x = solve_row_u(f, p, n, w, 0);
                x = x * x;
                res = res > x ? res : x;
            }
        }
        g_dbg[5] = it + 1;
        if (res <= UG_RESIDUAL_THR || it >= UG_PGS_ITERS - 1) break;
    }
    for (int q = 0; q < 128; q++) { g_dbg_w[128 + q] = q < n ? w[q] : 0.0; g_dbg_w[256 + q] = q < n ? R[q]->imp : 0.0; }
    for (int d = 0; d < NV; d++) {
        double s = 0.0;
        for (int k = 0; k < n; k++) s = fma(R[k]->MiJ[d], R[k]->imp, s);
        dv[d] = s;
    }
#ifdef UG_ROWHIST /* development aid (tools/row_hist.py): the row layout and sweep count of every solve */
    extern int dprintf(int, const char*, ...);
    dprintf(2, "ROWS %d %d %d %d %d %d\n", n, nnc, rs->nn, rs->nf, rs->nr, g_dbg[5]);
#endif
    /* split-impulse pass for deep penetrations (rhsPenetration rows, normals only, from zero) */
    int any = 0;
    for (int p = nnc; p < fb; p++)
        if (R[p]->rhsPen != 0.0) any = 1;
    if (!any) return 0;
    for (int q = 0; q < n; q++) w[q] = R[q]->rhsPen;
    for (int it = 0; it < UG_PGS_ITERS; it++) {
        double res = 0.0;
        for (int p = nnc; p < fb; p++) {
            double x = solve_row_u(R[p], p, n, w, 1);
            x = x * x;
            res = res > x ? res : x;
        }
        g_dbg[6] = it + 1;
        if (res <= UG_RESIDUAL_THR || it >= UG_PGS_ITERS - 1) break;
    }
    for (int d = 0; d < NV; d++) {
        double s = 0.0;
        for (int k = nnc; k < fb; k++) s = fma(R[k]->MiJ[d], R[k]->impPen, s);
        dvs[d] = s;
    }
    return 1;
}

/* ---- the same solve in Bullet's own form (tests only: bounds the row-space restatement's rounding) ----
 * btMultiBodyConstraintSolver::resolveSingleConstraintRowGeneric [ext] keeps the velocity delta deltaV of
 * every body and, per row, deltaImpulse = rhs - (J_A . deltaV_A + J_B . deltaV_B) * jacDiagABInv, then clamps
 * by assigning the bound: sum = applied + delta; sum < lo -> delta = lo - applied, applied = lo (hi likewise),
 * else applied = sum; deltaV += M^-1 J^T * delta.  Same row order, sweeps, friction bounds, residual and split
 * pass as pgs(); deltaV itself is the solver output.  Plain sums (no fma), as Bullet's C++ in double. */
static double solve_row_v(row* r, double* v, int pen) {
    double imp = pen ? r->impPen : r->imp;
    double dvn = 0.0;
    for (int d = 0; d < UG_NVP; d++) dvn += r->J[d] * v[d];
    double di = r->rhs - dvn * r->invD;
    if (pen) di = r->rhsPen - dvn * r->invD;
    double sum = imp + di;
    if (sum < r->lo) { di = r->lo - imp; imp = r->lo; }
    else if (sum > r->hi) { di = r->hi - imp; imp = r->hi; }
    else imp = sum;
    if (pen) r->impPen = imp; else r->imp = imp;
    for (int d = 0; d < UG_NVP; d++) v[d] += r->MiJ[d] * di;
    double rinv = r->invD == 0.0 ? 0.0 : 1.0 / r->invD;
    return di * rinv;
}
static int pgs_bullet(rowset* rs, double* dv, double* dvs) {
    row* R[MAXROWS];
    int n = 0, pos_of[MAXROWS];
    for (int j = 0; j < rs->nnc; j++) R[n++] = &rs->r[rs->idx_nc[j]];
    for (int j = 0; j < rs->nn; j++) R[n++] = &rs->r[rs->idx_n[j]];
    for (int j = 0; j < rs->nf; j++) R[n++] = &rs->r[rs->idx_f[j]];
    for (int j = 0; j < rs->nr; j++) R[n++] = &rs->r[rs->idx_r[j]];
    for (int p = 0; p < n; p++) pos_of[R[p] - rs->r] = p;
    const int nnc = rs->nnc, fb = rs->nnc + rs->nn;
    double v[UG_NVP];
    memset(v, 0, sizeof(v));
    for (int p = nnc; p < fb; p++) /* warm start: normals carry their scaled previous impulse */
        for (int d = 0; d < UG_NVP; d++) v[d] += R[p]->MiJ[d] * R[p]->imp;
    for (int it = 0; it < UG_PGS_ITERS; it++) {
        double res = 0.0;
        for (int j = 0; j < nnc; j++) {
            int p = (it & 1) ? j : nnc - 1 - j;
            double x = solve_row_v(R[p], v, 0);
            x = x * x;
            res = res > x ? res : x;
        }
        for (int p = nnc; p < fb; p++) {
            double x = solve_row_v(R[p], v, 0);
            x = x * x;
            res = res > x ? res : x;
        }
        for (int p = fb; p < n; p++) {
            row* f = R[p];
            double tot = R[pos_of[f->nrow]]->imp;
            if (tot > 0.0) {
                f->lo = -(f->fric * tot);
                f->hi = f->fric * tot;
                double x = solve_row_v(f, v, 0);
                x = x * x;
                res = res > x ? res : x;
            }
        }
        if (res <= UG_RESIDUAL_THR || it >= UG_PGS_ITERS - 1) break;
    }
    for (int d = 0; d < UG_NVP; d++) dv[d] = v[d];
    int any = 0;
    for (int p = nnc; p < fb; p++)
        if (R[p]->rhsPen != 0.0) any = 1;
    if (!any) return 0;
    memset(v, 0, sizeof(v));
    for (int it = 0; it < UG_PGS_ITERS; it++) {
        double res = 0.0;
        for (int p = nnc; p < fb; p++) {
            double x = solve_row_v(R[p], v, 1);
            x = x * x;
            res = res > x ? res : x;
        }
        if (res <= UG_RESIDUAL_THR || it >= UG_PGS_ITERS - 1) break;
    }
    for (int d = 0; d < UG_NVP; d++) dvs[d] = v[d];
    return 1;
}

/* ======================================================================== */
/* one p.stepSimulation()                                                    */
/* ======================================================================== */
/* a floating base's linear / angular velocity, per component (btMultiBody m_realBuf[0..5]) */
static v3 vclamp_coord(v3 v) {
    return V(ug_vclamp(v.x, UG_MAX_COORD_VEL), ug_vclamp(v.y, UG_MAX_COORD_VEL), ug_vclamp(v.z, UG_MAX_COORD_VEL));
}
static void substep(ugo_env* e) {
    const double dt = UG_DT;
    const scene* s = &e->sc;
    kin k;
    fk(e->q, &k);
    /* collision detection on current positions */
    const int ov0 = e->overflow;
    collide(e, &k);
    const int ov1 = e->overflow;
    if (ov1 != ov0) { e->stats[UG_STAT_MANCAP]++; e->flags |= UG_FLAG_DROPPED; }
    e->stats[UG_STAT_SUBSTEPS]++;
    /* external forces: robot (gravity, gyroscopic, damping) */
    double M[NB * NB], C[NB];
    robot_dynamics(e->qd, &k, s->gravity, M, C);
    ldlt(M, NB);
    double qdd[NB];
    for (int i = 0; i < NB; i++) qdd[i] = -C[i];
    ldlt_solve(M, NB, qdd);
    double v0[NV];
    memset(v0, 0, sizeof(v0));
    /* every dof velocity clamped to +-m_maxCoordinateVelocity (btMultiBody::applyDeltaVeeMultiDof [ext]) */
    for (int i = 0; i < NB; i++) { e->qd[i] = ug_vclamp(e->qd[i] + qdd[i] * dt, UG_MAX_COORD_VEL); v0[i] = e->qd[i]; }
    /* free objects: gravity + default damping + gyroscopic (btMultiBody floating base, 0 links) */
    for (int o = 0; o < s->nobj; o++) {
        if (!e->oactive[o]) continue;
        if (s->ojoint[o].kind != UGJ_FREE) {
            /* one-dof link on a fixed base (ug_joint.h): joint velocity in ov.x, joint position in ow.x */
            double Mj, Cj;
            ugj_dynamics(&s->ojoint[o], &e->oquat[o].x, e->ov[o].x, s->gravity, &Mj, &Cj);
            e->jM[o] = Mj;
            double qdd = -Cj / Mj;
            e->ov[o].x = ug_vclamp(e->ov[o].x + qdd * dt, UG_MAX_COORD_VEL);
            v0[NB + 6 * o] = e->ov[o].x;
            continue;
        }
        v3 v = e->ov[o];
        double vn = vlen(v);
        v3 a = vsub(V(0, 0, s->gravity), vscale(v, UG_LIN_DAMP + UG_LIN_DAMP * vn));
        e->ov[o] = vclamp_coord(vadd(v, vscale(a, dt)));
        m3 R = qmat(e->oquat[o]);
        v3 wl = mtv(&R, e->ow[o]);
        v3 I = s->oinertia[o];
        v3 Iw = V(I.x * wl.x, I.y * wl.y, I.z * wl.z);
        double wn = vlen(wl);
        v3 z = vadd(vscale(Iw, UG_ANG_DAMP + UG_ANG_DAMP * wn), vcross(wl, Iw));
        v3 al = V(-z.x / I.x, -z.y / I.y, -z.z / I.z);
        e->ow[o] = vclamp_coord(vadd(e->ow[o], vscale(mv(&R, al), dt)));
        int off = NB + 6 * o;
        v0[off] = e->ov[o].x; v0[off + 1] = e->ov[o].y; v0[off + 2] = e->ov[o].z;
        v0[off + 3] = e->ow[o].x; v0[off + 4] = e->ow[o].y; v0[off + 5] = e->ow[o].z;
    }
    /* constraint solve */
    static __thread rowset rs;
    build_rows(e, &k, M, v0, &rs);
    if (e->overflow != ov1) { e->stats[UG_STAT_ROWCAP]++; e->flags |= UG_FLAG_DROPPED; }
    double dv[UG_NVP], dvs[UG_NVP];
    memset(dv, 0, sizeof(dv));
    memset(dvs, 0, sizeof(dvs));
    int split = e->pgs_bullet ? pgs_bullet(&rs, dv, dvs) : pgs(&rs, dv, dvs);
    if (split) e->stats[UG_STAT_SPLIT]++;
    for (int i = 0; i < rs.nn; i++) {
        const row* r = &rs.r[rs.idx_n[i]];
        e->man[r->man].pt[r->pt].imp = r->imp;
    }
    for (int i = 0; i < rs.nf; i++) {
        const row* r = &rs.r[rs.idx_f[i]];
        if (r->kind == 2) e->man[r->man].pt[r->pt].imp1 = r->imp;
        else e->man[r->man].pt[r->pt].imp2 = r->imp;
    }
    /* the poses this substep's narrowphase saw, before they move (the contact query's world positions) */
    for (int i = 0; i < NB; i++) e->prevq[i] = e->q[i];
    for (int o = 0; o < MAXOBJ; o++) { e->prevpos[o] = e->opos[o]; e->prevquat[o] = e->oquat[o]; }
    /* velocities += solver delta; positions integrate (v + split velocity) */
    for (int i = 0; i < NB; i++) {
        e->qd[i] = ug_vclamp(e->qd[i] + dv[i], UG_MAX_COORD_VEL);
        double vi = split ? e->qd[i] + dvs[i] : e->qd[i];
        e->q[i] = e->q[i] + vi * dt;
    }
    for (int o = 0; o < s->nobj; o++) {
        if (!e->oactive[o]) continue;
        int off = NB + 6 * o;
        if (s->ojoint[o].kind != UGJ_FREE) {
            e->ov[o].x = ug_vclamp(e->ov[o].x + dv[off], UG_MAX_COORD_VEL);
            double vi = split ? e->ov[o].x + dvs[off] : e->ov[o].x;
            e->ow[o].x = e->ow[o].x + vi * dt;
            ugj_frame(&s->ojoint[o], e->ow[o].x, &e->oquat[o].x, &e->opos[o].x);
            continue;
        }
        e->ov[o] = vclamp_coord(vadd(e->ov[o], V(dv[off], dv[off + 1], dv[off + 2])));
        e->ow[o] = vclamp_coord(vadd(e->ow[o], V(dv[off + 3], dv[off + 4], dv[off + 5])));
        v3 vl = e->ov[o], wa = e->ow[o];
        if (split) {
            vl = vadd(vl, V(dvs[off], dvs[off + 1], dvs[off + 2]));
            wa = vadd(wa, V(dvs[off + 3], dvs[off + 4], dvs[off + 5]));
        }
        e->opos[o] = vadd(e->opos[o], vscale(vl, dt));
        /* btMultiBody::stepPositionsMultiDof base quaternion update [ext] */
        double ang = vlen(wa);
        if (ang * dt > UG_ANGULAR_MOTION_THR) ang = UG_ANGULAR_MOTION_THR / dt;
        v3 ax;
        if (ang < 0.001) ax = vscale(wa, 0.5 * dt - (dt * dt * dt) * 0.020833333333 * ang * ang);
        else ax = vscale(wa, ug_sin(0.5 * ang * dt) / ang);
        q4 dq = Q(ax.x, ax.y, ax.z, ug_cos(0.5 * ang * dt));
        e->oquat[o] = qnormalize(qmul(dq, e->oquat[o]));
    }
}

/* ======================================================================== */
/* robot control layer (urgym/base/robot.py)                                 */
/* ======================================================================== */
/* numpy pairwise sum of 12 |dq| (np.sum, env_ball_balance_v0.py:100) */
static double np_sum12(const double* a) {
    double r = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    for (int i = 8; i < 12; i++) r += a[i];
    return r;
}
static int state_finite(const ugo_env* e);
/* wait_until_stable (env_ball_balance_v0.py:94-103): returns substeps taken.  A state that went non-finite
 * ends the loop at once (the step's non-finite guard then terminates the episode) instead of spinning the
 * remaining substeps on NaNs. */
static void trace_substep(const ugo_env* e);
/* the non-finite guard voids a runaway state: q, qd and the active objects' state become NaN and the contacts are
 * dropped, so what a step returns once the guard fired does not depend on how the first NaN spread (the kernels
 * clamp with v_min / v_max, which drop a NaN operand that C's selects keep) */
static void poison(ugo_env* e) {
    for (int i = 0; i < NB; i++) e->q[i] = e->qd[i] = NAN;
    for (int o = 0; o < e->sc.nobj; o++) {
        if (!e->oactive[o]) continue;
        e->opos[o] = V(NAN, NAN, NAN);
        e->oquat[o] = Q(NAN, NAN, NAN, NAN);
        e->ov[o] = e->ow[o] = V(NAN, NAN, NAN);
    }
    e->nman = 0;
}
static int wait_until_stable(ugo_env* e) {
    double pos[NB];
    memcpy(pos, e->q, sizeof(pos));
    for (int i = 0; i < UG_STABLE_STEPS; i++) {
        trace_substep(e);
        substep(e);
        if (!state_finite(e)) { poison(e); return i + 1; }
        double a[NB];
        for (int j = 0; j < NB; j++) a[j] = ug_fabs(pos[j] - e->q[j]);
        if (np_sum12(a) < UG_STABLE_EPS) return i + 1;
        memcpy(pos, e->q, sizeof(pos));
    }
    /* "Warning: The robot configuration did not stabilize" (:102-103): surfaced as a flag and a counter */
    e->stats[UG_STAT_UNSTABLE]++;
    e->flags |= UG_FLAG_UNSTABLE;
    return UG_STABLE_STEPS;
}
/* UR5Robotiq85.move_gripper (robot.py:213-218) */
double ugo_gripper_angle(double L) { return 0.715 - ug_asin((L - 0.010) / 0.1143); }
static void open_gripper(ugo_env* e, double pct) {
    double L = UG_GRIP_MIN + (UG_GRIP_MAX - UG_GRIP_MIN) * (pct / 100.0);
    e->mtarget[6] = ugo_gripper_angle(L);
    e->mon[6] = 1;
}
static void close_gripper(ugo_env* e, double pct) {
    double L = UG_GRIP_MAX - (UG_GRIP_MAX - UG_GRIP_MIN) * (pct / 100.0);
    e->mtarget[6] = ugo_gripper_angle(L);
    e->mon[6] = 1;
}

/* p.calculateInverseKinematics(robot, 7, pos, orn, ..6-long arrays.., maxNumIterations=20)
 * [ext]: PhysicsServerCommandProcessor IK loop + IKTrajectoryHelper::computeIK with
 * IK2_VEL_DLS_WITH_ORIENTATION (null space skipped: arrays shorter than the dof count) */
static void ik_solve(const double* q0, v3 tp, q4 to, double* qout) {
    double q[NB];
    memcpy(q, q0, sizeof(q));
    double diff = 1e30;
    for (int it = 0; it < UG_IK_ITERS && diff > UG_IK_RESIDUAL; it++) {
        kin k;
        fk(q, &k);
        m3 Re;
        v3 pe;
        link_frame(&k, UG_EE_LINK, 1, &Re, &pe);
        q4 oe = mquat(&Re);
        diff = vlen(vsub(pe, tp));
        double ds[6];
        ds[0] = 1.0 * (tp.x - pe.x); ds[1] = 1.0 * (tp.y - pe.y); ds[2] = 1.0 * (tp.z - pe.z);
        q4 inv = Q(-oe.x, -oe.y, -oe.z, oe.w);
        q4 dq = qmul(to, inv);
        double w = dq.w;
        if (w < -1.0) w = -1.0;
        if (w > 1.0) w = 1.0;
        float angle = (float)(2.0 * ug_acos(w));
        if (angle > UG_PI) angle = (float)(angle - 2.0 * UG_PI);
        else if (angle < -UG_PI) angle = (float)(angle + 2.0 * UG_PI);
        v3 axis;
        double s2 = 1.0 - dq.w * dq.w;
        if (s2 < 10.0 * 2.220446049250313e-16) axis = V(1.0, 0.0, 0.0);
        else { double sq = 1.0 / ug_sqrt(s2); axis = V(dq.x * sq, dq.y * sq, dq.z * sq); }
        axis = vscale(axis, 1.0 / vlen(axis));
        ds[3] = 1.0 * ((double)angle * axis.x);
        ds[4] = 1.0 * ((double)angle * axis.y);
        ds[5] = 1.0 * ((double)angle * axis.z);
        /* Jacobian of the EE link origin wrt the 6 arm dofs (gripper columns are zero) */
        double J[6][6];
        for (int d = 0; d < 6; d++) {
            v3 jl = vcross(k.a[d], vsub(pe, k.p[d]));
            J[0][d] = jl.x; J[1][d] = jl.y; J[2][d] = jl.z;
            J[3][d] = k.a[d].x; J[4][d] = k.a[d].y; J[5][d] = k.a[d].z;
        }
        /* (J^T J + diag(0.5)) dtheta = J^T ds  (BussIK CalcDeltaThetasDLS2) */
        double U[36], rhs[6];
        for (int i = 0; i < 6; i++) {
            for (int j = 0; j < 6; j++) {
                double sum = 0.0;
                for (int r = 0; r < 6; r++) sum += J[r][i] * J[r][j];
                U[i * 6 + j] = sum;
            }
            U[i * 6 + i] += UG_IK_DAMPING;
            double sr = 0.0;
            for (int r = 0; r < 6; r++) sr += J[r][i] * ds[r];
            rhs[i] = sr;
        }
        ldlt(U, 6);
        ldlt_solve(U, 6, rhs);
        double mx = 0.0;
        for (int i = 0; i < 6; i++) mx = ug_fabs(rhs[i]) > mx ? ug_fabs(rhs[i]) : mx;
        if (mx > UG_IK_MAXANGLE)
            for (int i = 0; i < 6; i++) rhs[i] *= UG_IK_MAXANGLE / mx;
        for (int i = 0; i < 6; i++) q[i] = rhs[i] + q[i];
    }
    memcpy(qout, q, sizeof(q));
}
static void move_ee_end(ugo_env* e, v3 pos, q4 orn) {
    double qt[NB];
    ik_solve(e->q, pos, orn, qt);
    for (int i = 0; i < 6; i++) { e->mtarget[i] = qt[i]; e->mon[i] = 1; }
}
static void move_ee_joint(ugo_env* e, const double* q6) {
    for (int i = 0; i < 6; i++) { e->mtarget[i] = q6[i]; e->mon[i] = 1; }
}
/* getLinkState(robot, l)[0:2]: link COM world pose */
static void link_state(const ugo_env* e, int l, v3* p, q4* o) {
    kin k;
    fk(e->q, &k);
    m3 R;
    link_frame(&k, l, 1, &R, p);
    *o = mquat(&R);
}
/* get_gripper_geometrical_center (env_ball_balance_v0.py:249-275): union of getAABB(11), getAABB(16) */
static v3 gripper_center(const ugo_env* e) {
    kin k;
    fk(e->q, &k);
    double bl[2][3], bh[2][3];
    const int links[2] = {11, 16};
    for (int i = 0; i < 2; i++) {
        int l = links[i];
        m3 R;
        v3 p;
        link_frame(&k, l, 1, &R, &p);
        v3 c = vadd(mv(&R, V(UG_LINK_AABB_C[3 * l], UG_LINK_AABB_C[3 * l + 1], UG_LINK_AABB_C[3 * l + 2])), p);
        v3 h = V(UG_LINK_AABB_H[3 * l], UG_LINK_AABB_H[3 * l + 1], UG_LINK_AABB_H[3 * l + 2]);
        const double* r = R.m;
        v3 ext = V(ug_fabs(r[0]) * h.x + ug_fabs(r[1]) * h.y + ug_fabs(r[2]) * h.z,
                   ug_fabs(r[3]) * h.x + ug_fabs(r[4]) * h.y + ug_fabs(r[5]) * h.z,
                   ug_fabs(r[6]) * h.x + ug_fabs(r[7]) * h.y + ug_fabs(r[8]) * h.z);
        v3 mn = vsub(c, ext), mx = vadd(c, ext);
        bl[i][0] = mn.x; bl[i][1] = mn.y; bl[i][2] = mn.z;
        bh[i][0] = mx.x; bh[i][1] = mx.y; bh[i][2] = mx.z;
    }
    double ctr[3];
    ugg_union_center(bl[0], bh[0], bl[1], bh[1], ctr);
    return V(ctr[0], ctr[1], ctr[2]);
}
static void remove_object(ugo_env* e, int o) {
    e->oactive[o] = 0;
    int c0 = e->sc.ocol[o], c1 = c0 + e->sc.oncol[o];
    int k = 0;
    for (int m = 0; m < e->nman; m++) {
        const pairdef* P = &e->sc.pair[e->man[m].pair];
        if ((P->a >= c0 && P->a < c1) || (P->b >= c0 && P->b < c1)) continue;
        if (k != m) e->man[k] = e->man[m];
        k++;
    }
    e->nman = k;
}
static void place_object(ugo_env* e, int o, v3 pos, q4 orn) {
    e->oactive[o] = 1;
    e->opos[o] = pos;
    e->oquat[o] = orn;
    e->ov[o] = V(0, 0, 0);
    e->ow[o] = V(0, 0, 0);
}
/* RobotBase.reset -> reset_arm (robot.py:89-98) + reset_gripper/open_gripper (robot.py:100-106) */
static int robot_reset(ugo_env* e) {
    for (int i = 0; i < 6; i++) { e->q[i] = UG_ARM_REST[i]; e->qd[i] = 0.0; }
    int n = 0;
    while (n < 10) {
        substep(e);
        n++;
        if (!state_finite(e)) { poison(e); break; } /* as wait_until_stable: no substeps on NaNs */
    }
    open_gripper(e, 100.0);
    return n;
}

/* ======================================================================== */
/* tasks                                                                     */
/* ======================================================================== */
int ugo_obs_dim(int task) { return UG_OBS_DIM(task); }
int ugo_act_dim(int task) { return UG_ACT_DIM(task); }
int ugo_state_dim(void) { return STATE_DIM; }

static void bb_obs(const ugo_env* e, double* obs) {
    /* env_ball_balance_v0.py:137-143 */
    v3 eu = euler_from_quat(e->oquat[0]);
    obs[0] = eu.x; obs[1] = eu.y; obs[2] = eu.z;
    obs[3] = e->opos[0].x - e->opos[1].x;
    obs[4] = e->opos[0].y - e->opos[1].y;
    obs[5] = e->opos[0].z - e->opos[1].z;
}
/* create_ball (env_ball_balance_v0.py:186-205): 0.2 m + r above the paddle, x += U(-0.03,0.03), y += U(-0.08,0.02) */
static v3 bb_ball_position(ugo_env* e, const double* draws, v3 paddle) {
    v3 bp = V(paddle.x, paddle.y, paddle.z + 0.2 + UG_BB_BALL_R);
    bp.x += draws ? -0.03 + (0.03 - -0.03) * draws[0] : mt_uniform(&e->rng, -0.03, 0.03);
    bp.y += draws ? -0.08 + (0.02 - -0.08) * draws[1] : mt_uniform(&e->rng, -0.08, 0.02);
    return bp;
}
static int bb_reset(ugo_env* e, const double* draws, double* obs) {
    /* env_ball_balance_v0.py:145-170 */
    int n = robot_reset(e);
    remove_object(e, 0);
    remove_object(e, 1);
    move_ee_end(e, V(0.0, -0.60, 0.60), Q(0.50, -0.50, -0.50, 0.50));
    open_gripper(e, 20.0);
    n += wait_until_stable(e);
    v3 pe;
    q4 oe;
    link_state(e, UG_EE_LINK, &pe, &oe);
    v3 gc = gripper_center(e);
    v3 pose = V(pe.x, pe.y - 0.2, gc.z);
    place_object(e, 0, pose, Q(0, 0, 0, 1));
    place_object(e, 1, bb_ball_position(e, draws, pose), e->oquat[0]);
    close_gripper(e, 100.0);
    n += wait_until_stable(e);
    bb_obs(e, obs);
    return n;
}
/* ---- TwoBallsBalance (env_two_balls_balance_v0.py): the BallBalance scene with two balls ---- */
static void tb_obs(const ugo_env* e, double* obs) {
    /* :157-163: paddle euler, paddle - ball 1, paddle - ball 2 */
    v3 eu = euler_from_quat(e->oquat[0]);
    obs[0] = eu.x; obs[1] = eu.y; obs[2] = eu.z;
    for (int b = 0; b < 2; b++) {
        obs[3 + 3 * b] = e->opos[0].x - e->opos[1 + b].x;
        obs[4 + 3 * b] = e->opos[0].y - e->opos[1 + b].y;
        obs[5 + 3 * b] = e->opos[0].z - e->opos[1 + b].z;
    }
}
static int tb_reset(ugo_env* e, const double* draws, double* obs) {
    /* :165-190 (as BallBalance, create_balls(0.003) instead of create_ball) */
    int n = robot_reset(e);
    for (int o = 0; o < 3; o++) remove_object(e, o);
    move_ee_end(e, V(0.0, -0.60, 0.60), Q(0.50, -0.50, -0.50, 0.50));
    open_gripper(e, 20.0);
    n += wait_until_stable(e);
    v3 pe;
    q4 oe;
    link_state(e, UG_EE_LINK, &pe, &oe);
    v3 gc = gripper_center(e);
    v3 pose = V(pe.x, pe.y - 0.2, gc.z);
    place_object(e, 0, pose, Q(0, 0, 0, 1));
    double u[4], pd[3] = {pose.x, pose.y, pose.z}, b1[3], b2[3];
    for (int i = 0; i < 4; i++) u[i] = draws ? draws[i] : mt_random(&e->rng);
    ugg_tb_balls(pd, UG_TB_BALL_R, u, b1, b2);
    place_object(e, 1, V(b1[0], b1[1], b1[2]), e->oquat[0]);
    place_object(e, 2, V(b2[0], b2[1], b2[2]), e->oquat[0]);
    close_gripper(e, 100.0);
    n += wait_until_stable(e);
    tb_obs(e, obs);
    return n;
}
static int tb_step(ugo_env* e, const float* a, double* obs, double* rew, uint8_t* term, uint8_t* succ) {
    /* :106-146: the BallBalance action (euler + a), then the two-ball reward and termination */
    v3 pe;
    q4 oe;
    link_state(e, UG_EE_LINK, &pe, &oe);
    v3 eu = euler_from_quat(oe);
    eu.x += (double)a[0]; eu.y += (double)a[1]; eu.z += (double)a[2];
    move_ee_end(e, pe, quat_from_euler(eu));
    int n = wait_until_stable(e);
    double b1[3] = {e->opos[1].x, e->opos[1].y, e->opos[1].z}, b2[3] = {e->opos[2].x, e->opos[2].y, e->opos[2].z};
    *term = (uint8_t)ugg_tb_reward(a, b1, b2, e->opos[0].z, rew);
    *succ = 0;
    tb_obs(e, obs);
    return n;
}
static int bb_step(ugo_env* e, const float* a, double* obs, double* rew, uint8_t* term, uint8_t* succ) {
    /* env_ball_balance_v0.py:105-134 */
    v3 pe;
    q4 oe;
    link_state(e, UG_EE_LINK, &pe, &oe);
    v3 eu = euler_from_quat(oe);
    eu.x += (double)a[0]; eu.y += (double)a[1]; eu.z += (double)a[2];
    q4 qn = quat_from_euler(eu);
    move_ee_end(e, pe, qn);
    int n = wait_until_stable(e);
    *rew = 1.0;
    *term = e->opos[1].z < e->opos[0].z;
    *succ = 0;
    bb_obs(e, obs);
    return n;
}

/* ---- contact predicates over the manifold cache (p.getContactPoints existence) ---- */
/* any point between a robot link in [lmin, lmax] and the collider cb */
static int robot_contact(const ugo_env* e, int cb, int lmin, int lmax) {
    const scene* s = &e->sc;
    for (int m = 0; m < e->nman; m++) {
        const pairdef* P = &s->pair[e->man[m].pair];
        if (e->man[m].npts <= 0 || P->b != cb) continue;
        int l = s->col[P->a].link;
        if (l >= lmin && l <= lmax) return 1;
    }
    return 0;
}
static int static_collider(const scene* s, int ent) {
    for (int i = 0; i < s->ncol; i++)
        if (s->col[i].ent == ent) return i;
    return -1;
}

/* ---- CubesPush (env_cubes_push_v0.py) ---- */
static void cp_obs(const ugo_env* e, double* obs) {
    /* :198-205 ee position (link 7 COM) + both cube positions */
    v3 pe;
    q4 oe;
    link_state(e, UG_EE_LINK, &pe, &oe);
    obs[0] = pe.x; obs[1] = pe.y; obs[2] = pe.z;
    if (e->sc.variant == UG_TASK_CUBESPUSHDIFF) {
        /* env_cubes_push_diff_v0.py:202-212: cube positions relative to the ee (np.array(cube) - np.array(ee)) */
        for (int o = 0; o < 2; o++) {
            obs[3 + 3 * o] = e->opos[o].x - pe.x; obs[4 + 3 * o] = e->opos[o].y - pe.y; obs[5 + 3 * o] = e->opos[o].z - pe.z;
        }
        return;
    }
    for (int o = 0; o < 2; o++) { obs[3 + 3 * o] = e->opos[o].x; obs[4 + 3 * o] = e->opos[o].y; obs[5 + 3 * o] = e->opos[o].z; }
}
static int cp_reset(ugo_env* e, const double* draws, double* obs) {
    /* :207-227 */
    int n = robot_reset(e);
    remove_object(e, 0);
    remove_object(e, 1);
    place_object(e, 0, V(0.0, -0.5, 0.1), Q(0, 0, 0, 1));
    double x = ugg_cp_cube1_x(draws ? draws[0] : mt_random(&e->rng));
    place_object(e, 1, V(x, -0.7, 0.1), Q(0, 0, 0, 1));
    move_ee_end(e, V(x, -0.7, 0.1 + UG_CP_EE_DZ), Q(0.0, UG_VQ_S, 0.0, UG_VQ_C));
    close_gripper(e, 100.0);
    n += wait_until_stable(e);
    cp_obs(e, obs);
    return n;
}
static int cp_step(ugo_env* e, const float* a, double* obs, double* rew, uint8_t* term, uint8_t* succ) {
    /* :115-150 */
    v3 pe;
    q4 oe;
    link_state(e, UG_EE_LINK, &pe, &oe);
    move_ee_end(e, V(pe.x + (double)a[0], pe.y + (double)a[1], pe.z + (double)a[2]), Q(0.0, UG_VQ_S, 0.0, UG_VQ_C));
    int n = wait_until_stable(e);
    int table = robot_contact(e, static_collider(&e->sc, 10), 1, UG_NL - 1); /* :176-183 robot link != 0 */
    int touched = robot_contact(e, e->sc.ocol[1], 9, 18);                    /* :185-194 fingers 9..18 */
    double r;
    int success = ugg_cp_reward(table, touched, e->opos[0].x, e->opos[0].y, e->opos[0].z, e->opos[1].x,
                                e->opos[1].y, e->opos[1].z, e->sparse, &r);
    *rew = r;
    *term = (uint8_t)success;
    *succ = (uint8_t)success;
    cp_obs(e, obs);
    return n;
}

/* ---- CubesGrasp (env_cubes_grasp_v0.py) ---- */
/* get_gripper_opening_length (:349-376): link frames 11 and 16, distance - 0.052, clamp, normalise */
static double cg_opening(const ugo_env* e) {
    kin k;
    fk(e->q, &k);
    m3 R1, R2;
    v3 p1, p2;
    link_frame(&k, 11, 0, &R1, &p1);
    link_frame(&k, 16, 0, &R2, &p2);
    return ugg_cg_opening(ug_norm3(p2.x - p1.x, p2.y - p1.y, p2.z - p1.z));
}
static double cg_distance(const ugo_env* e) {
    /* distance_to_target (:199-204): gripper geometric centre to the cube position */
    v3 gc = gripper_center(e);
    return ug_norm3(gc.x - e->opos[0].x, gc.y - e->opos[0].y, gc.z - e->opos[0].z);
}
static int cg_grasped(const ugo_env* e) {
    /* object_grasped (:211-228): a point on a left link {11,12,13} and one on a right link {16,17,18} */
    return robot_contact(e, e->sc.ocol[0], 11, 13) && robot_contact(e, e->sc.ocol[0], 16, 18);
}
static void cg_obs(const ugo_env* e, double* obs) {
    /* :268-287 subgoal flags, ee pose (7), opening, cube pose (7) */
    v3 pe;
    q4 oe;
    link_state(e, UG_EE_LINK, &pe, &oe);
    obs[0] = e->goal_approached; obs[1] = e->goal_grasped;
    obs[2] = pe.x; obs[3] = pe.y; obs[4] = pe.z; obs[5] = oe.x; obs[6] = oe.y; obs[7] = oe.z; obs[8] = oe.w;
    obs[9] = cg_opening(e);
    obs[10] = e->opos[0].x; obs[11] = e->opos[0].y; obs[12] = e->opos[0].z;
    obs[13] = e->oquat[0].x; obs[14] = e->oquat[0].y; obs[15] = e->oquat[0].z; obs[16] = e->oquat[0].w;
}
static int cg_reset(ugo_env* e, const double* draws, double* obs) {
    /* :289-307 robot.reset, create_cubes (:310-330), move_ee(get_ee_pose) and settle */
    int n = robot_reset(e);
    remove_object(e, 0);
    double u0 = draws ? draws[0] : mt_random(&e->rng);
    double u1 = draws ? draws[1] : mt_random(&e->rng);
    double x, y;
    ugg_cg_cube_xy(u0, u1, &x, &y);
    place_object(e, 0, V(x, y, 0.1), Q(0, 0, 0, 1));
    v3 pe;
    q4 oe;
    link_state(e, UG_EE_LINK, &pe, &oe);
    move_ee_end(e, pe, oe);
    n += wait_until_stable(e);
    e->goal_approached = e->goal_grasped = 0;
    cg_obs(e, obs);
    return n;
}
static int cg_choose(ugo_env* e, float w0, float w1) { return ugg_cg_choose(w0, w1, mt_random(&e->rng)); }
static int cg_step(ugo_env* e, const float* a, double* obs, double* rew, uint8_t* term, uint8_t* succ) {
    /* :132-192 */
    int sel = cg_choose(e, a[0], a[1]);
    if (sel == 0) {
        double q6[6];
        for (int i = 0; i < 6; i++) q6[i] = (double)a[2 + i];
        move_ee_joint(e, q6);
    } else if (a[8] < 0.5f) {
        open_gripper(e, 100.0);
    } else {
        close_gripper(e, 100.0);
    }
    int n = wait_until_stable(e);
    int app = e->goal_approached, gr = e->goal_grasped;
    double d = cg_distance(e);
    double r;
    int success = ugg_cg_reward(&app, &gr, d, cg_opening(e), cg_grasped(e), e->opos[0].z, &r);
    e->goal_approached = app;
    e->goal_grasped = gr;
    *rew = r;
    *term = (uint8_t)success;
    *succ = (uint8_t)success;
    cg_obs(e, obs);
    return n;
}

/* ---- Golf (env_golf_v0.py) ---- */
/* any manifold point between a collider in [a0, a1) and one in [b0, b1) (either side of the pair) */
static int pair_contact(const ugo_env* e, int a0, int a1, int b0, int b1) {
    const scene* s = &e->sc;
    for (int m = 0; m < e->nman; m++) {
        const pairdef* P = &s->pair[e->man[m].pair];
        if (e->man[m].npts <= 0) continue;
        if ((P->a >= a0 && P->a < a1 && P->b >= b0 && P->b < b1) || (P->b >= a0 && P->b < a1 && P->a >= b0 && P->a < b1))
            return 1;
    }
    return 0;
}
static void drop_manifolds_of(ugo_env* e, int ci) {
    int k = 0;
    for (int m = 0; m < e->nman; m++) {
        const pairdef* P = &e->sc.pair[e->man[m].pair];
        if (P->a == ci || P->b == ci) continue;
        if (k != m) e->man[k] = e->man[m];
        k++;
    }
    e->nman = k;
}
/* club reference points: composite COM + R * offset (offsets along the base z axis) */
static v3 club_point(const ugo_env* e, double zoff) {
    m3 R = qmat(e->oquat[0]);
    return vadd(e->opos[0], mv(&R, V(0.0, 0.0, zoff - UG_GF_ZC)));
}
static void gf_obs(const ugo_env* e, double* obs) {
    if (e->sc.variant == UG_TASK_GOLFJOINTS) {
        /* env_golf_joints_v0.py:228-235: np.append(joints[0:6], [stick, ball - stick, hole - ball]) */
        for (int i = 0; i < 6; i++) obs[i] = e->q[i];
        obs += 6;
    }
    v3 st = club_point(e, UG_GF_FOOT_Z); /* getLinkState(stick, 0)[0] (:240-244) */
    double stick[3] = {st.x, st.y, st.z}, ball[3] = {e->opos[1].x, e->opos[1].y, e->opos[1].z};
    double hole[3] = {UG_GF_PITCH_X, UG_GF_PITCH_Y, UG_GF_PITCH_Z};
    ugg_gf_obs(stick, ball, hole, obs);
}
static int gf_reset(ugo_env* e, const double* draws, double* obs) {
    /* :238-267 */
    int n = robot_reset(e);
    remove_object(e, 0);
    remove_object(e, 1);
    drop_manifolds_of(e, static_collider(&e->sc, 12)); /* the pitch is removed and re-created (:246-248) */
    move_ee_end(e, V(0.0, -0.60, 0.40), Q(0.0, 0.0, -0.70, 0.70));
    open_gripper(e, 20.0);
    n += wait_until_stable(e);
    v3 gc = gripper_center(e);
    /* create_stick(pose): base at the gripper centre - 0.05 z, identity orientation -> COM above by zc */
    place_object(e, 0, V(gc.x, gc.y, gc.z - 0.05 + UG_GF_ZC), Q(0, 0, 0, 1));
    double u0 = draws ? draws[0] : mt_random(&e->rng);
    double u1 = draws ? draws[1] : mt_random(&e->rng);
    double bx, by;
    ugg_gf_ball_xy(u0, u1, &bx, &by);
    place_object(e, 1, V(bx, by, 0.1), Q(0, 0, 0, 1));
    close_gripper(e, 100.0);
    n += wait_until_stable(e);
    gf_obs(e, obs);
    return n;
}
static int gf_step(ugo_env* e, const float* a, double* obs, double* rew, uint8_t* term, uint8_t* succ) {
    /* :115-183 */
    if (e->sc.variant == UG_TASK_GOLFJOINTS) {
        /* env_golf_joints_v0.py:122-124: get_joint_states() + action (float64 + float32 -> float64), 'joint' */
        double q6[6];
        for (int i = 0; i < 6; i++) q6[i] = e->q[i] + (double)a[i];
        move_ee_joint(e, q6);
    } else {
        v3 pe;
        q4 oe;
        link_state(e, UG_EE_LINK, &pe, &oe);
        move_ee_end(e, V(pe.x + (double)a[0], pe.y + (double)a[1], pe.z + (double)a[2]), Q(0.0, 0.0, -0.70, 0.70));
    }
    int n = wait_until_stable(e);
    const scene* s = &e->sc;
    int c0 = s->ocol[0], c1 = c0 + s->oncol[0], cb = s->ocol[1], cp = static_collider(s, 12);
    int in_fingers = 0;
    for (int c = c0; c < c1; c++) in_fingers |= robot_contact(e, c, 9, 18);          /* :199-208 */
    int floor = robot_contact(e, cp, 0, UG_NL - 1) || pair_contact(e, c0, c1, cp, cp + 1); /* :185-197 */
    int touched = pair_contact(e, cb, cb + 1, c0, c1);                               /* :199-203 */
    v3 st = club_point(e, UG_GF_FOOT_Z);
    double stick[3] = {st.x, st.y, st.z}, ball[3] = {e->opos[1].x, e->opos[1].y, e->opos[1].z};
    double hole[3] = {UG_GF_PITCH_X, UG_GF_PITCH_Y, UG_GF_PITCH_Z};
    double r;
    int t;
    int success = ugg_gf_reward(ball, hole, stick, in_fingers, floor, touched, e->sparse, &r, &t);
    *rew = r;
    *term = (uint8_t)t;
    *succ = (uint8_t)success;
    gf_obs(e, obs);
    return n;
}

/* ---- Box (env_box_v0.py) ---- */
/* reset_box (:172-177): both joints to 0 at rest (resetJointState), the links' frames follow; the button's motor
 * (force 1, target 0) is always on in this scene and the door's has force 0 (build_rows) */
static void bx_place(ugo_env* e) {
    for (int o = 0; o < 2; o++) {
        e->oactive[o] = 1;
        e->ov[o] = V(0, 0, 0);
        e->ow[o] = V(0, 0, 0);
        ugj_frame(&e->sc.ojoint[o], 0.0, &e->oquat[o].x, &e->opos[o].x);
    }
}
/* get_ee_pose() in world coordinates (robot.py:142-145): the robot base stands at (0, UG_BX_ROBOT_Y, 0) with the
 * identity orientation, so the world pose is the base-frame pose shifted along y */
static void bx_ee_world(const ugo_env* e, double* w7) {
    v3 pe;
    q4 oe;
    link_state(e, UG_EE_LINK, &pe, &oe);
    w7[0] = pe.x; w7[1] = pe.y + UG_BX_ROBOT_Y; w7[2] = pe.z;
    w7[3] = oe.x; w7[4] = oe.y; w7[5] = oe.z; w7[6] = oe.w;
}
/* move_ee(world pose, 'end'): calculateInverseKinematics takes the target into the base frame
 * (PhysicsServerCommandProcessor: base transform inverse * btTransform(target) [ext]) -- the position shifted
 * back along y, the orientation through btMatrix3x3::setRotation / getRotation (unit norm) */
static void bx_move_ee(ugo_env* e, const double* w7) {
    q4 t = Q(w7[3], w7[4], w7[5], w7[6]);
    m3 R = qmat(t);
    move_ee_end(e, V(w7[0], w7[1] - UG_BX_ROBOT_Y, w7[2]), mquat(&R));
}
static void bx_obs(const ugo_env* e, double* obs) { bx_ee_world(e, obs); } /* :161-170 np.array(ee_pos) */
static int bx_reset(ugo_env* e, double* obs) {
    /* :179-186 robot.reset(), move_ee(get_ee_pose(), 'end'), reset_box() */
    int n = robot_reset(e);
    double w7[7];
    bx_ee_world(e, w7);
    bx_move_ee(e, w7);
    bx_place(e);
    e->goal_approached = e->goal_grasped = e->goal_closed = 0;
    bx_obs(e, obs);
    return n;
}
static int bx_step(ugo_env* e, const float* a, double* obs, double* rew, uint8_t* term, uint8_t* succ) {
    /* :118-139 */
    double w7[7], t7[7];
    bx_ee_world(e, w7);
    ugg_box_target(w7, a, t7);
    bx_move_ee(e, t7);
    e->mtarget[6] = ugo_gripper_angle((double)a[7]); /* move_gripper(action[-1]) (robot.py:213-218) */
    e->mon[6] = 1;
    int n = 0;
    while (n < UG_BX_STEPS) { /* :128-129 a fixed 120 substeps */
        substep(e);
        n++;
        if (!state_finite(e)) { poison(e); break; }
    }
    int bc = e->sc.ocol[1];
    int press = ugg_box_press(e->ow[1].x, e->button_mode, robot_contact(e, bc, 0, UG_NL - 1), robot_contact(e, bc, 9, 18));
    int op = e->goal_approached, pr = e->goal_grasped, cl = e->goal_closed;
    double r;
    int closed = ugg_box_reward(&op, &pr, &cl, e->ow[0].x, press, &r);
    e->goal_approached = op; e->goal_grasped = pr; e->goal_closed = cl;
    *rew = r;
    *term = (uint8_t)closed;
    *succ = (uint8_t)closed;
    bx_obs(e, obs);
    return n;
}

/* ======================================================================== */
/* public API                                                                */
/* ======================================================================== */
ugo_env* ugo_create(int task, uint32_t seed) { return ugo_create_ex(task, seed, 0); }
/* flags: UG_GEOM_LOD selects the collision LOD (urgym_create_ex's URGYM_FLAG_LOD_GEOMETRY); the default (0 or
 * UG_GEOM_FULL) is the full geometry */
ugo_env* ugo_create_ex(int task, uint32_t seed, int flags) {
    if (task < 0 || task >= UG_NTASK) return NULL;
    /* Box-v0 has cylinders on the robot's path (door handles, button): full geometry only */
    if (task == UG_TASK_BOX && !UG_GEOM_IS_FULL(flags)) return NULL;
    ugo_env* e = (ugo_env*)calloc(1, sizeof(ugo_env));
    build_scene(&e->sc, task, flags);
    mt_seed(&e->rng, seed);
    return e;
}
void ugo_destroy(ugo_env* e) { free(e); }
void ugo_substep(ugo_env* e) { substep(e); }
/* debug aid (tools/debug_gjk.py): the state before every substep of this thread's next calls (up to 600) */
#define TRACE_MAX 600
static __thread int g_trace_on, g_trace_n;
static __thread double* g_trace;
void ugo_trace(int on) {
    if (!g_trace) g_trace = (double*)malloc(sizeof(double) * STATE_DIM * TRACE_MAX);
    if (on) g_trace_n = 0;
    g_trace_on = on;
}
int ugo_traced(double* out, int max) {
    const int n = g_trace_n < max ? g_trace_n : max;
    if (n) memcpy(out, g_trace, sizeof(double) * STATE_DIM * (size_t)n);
    return g_trace_n;
}
static void trace_substep(const ugo_env* e) {
    if (g_trace_on && g_trace_n < TRACE_MAX) ugo_get_state(e, g_trace + (size_t)STATE_DIM * g_trace_n++);
}
/* non-finite state guard (failure detection): q, qd and the active objects' state */
static int state_finite(const ugo_env* e) {
    for (int i = 0; i < NB; i++)
        if (!isfinite(e->q[i]) || !isfinite(e->qd[i])) return 0;
    for (int o = 0; o < e->sc.nobj; o++) {
        if (!e->oactive[o]) continue;
        double v[13] = {e->opos[o].x, e->opos[o].y, e->opos[o].z, e->oquat[o].x, e->oquat[o].y, e->oquat[o].z,
                        e->oquat[o].w, e->ov[o].x, e->ov[o].y, e->ov[o].z, e->ow[o].x, e->ow[o].y, e->ow[o].z};
        for (int j = 0; j < 13; j++)
            if (!isfinite(v[j])) return 0;
    }
    return 1;
}
/* a reset of a non-finite state starts from a clean robot (all joints 0 at rest, motors off, no objects,
 * no contacts); a finite state is left to the task's own reset */
static void sanitize(ugo_env* e) {
    if (state_finite(e)) return;
    memset(e->q, 0, sizeof(e->q));
    memset(e->qd, 0, sizeof(e->qd));
    memset(e->mtarget, 0, sizeof(e->mtarget));
    memset(e->mon, 0, sizeof(e->mon));
    for (int o = 0; o < MAXOBJ; o++) {
        e->oactive[o] = 0;
        e->opos[o] = V(0, 0, 0); e->oquat[o] = Q(0, 0, 0, 0); e->ov[o] = V(0, 0, 0); e->ow[o] = V(0, 0, 0);
    }
    e->nman = 0;
}
static int reset_impl(ugo_env* e, const double* draws, double* obs) {
    sanitize(e);
    e->goal_approached = e->goal_grasped = e->goal_closed = 0;
    int n = -1;
    if (e->sc.variant == UG_TASK_TWOBALLS) n = tb_reset(e, draws, obs);
    else switch (e->sc.task) {
        case UG_TASK_BALLBALANCE: n = bb_reset(e, draws, obs); break;
        case UG_TASK_CUBESPUSH: n = cp_reset(e, draws, obs); break;
        case UG_TASK_CUBESGRASP: n = cg_reset(e, draws, obs); break;
        case UG_TASK_GOLF: n = gf_reset(e, draws, obs); break;
        case UG_TASK_BOX: n = bx_reset(e, obs); break;
    }
    /* a reset whose settling went non-finite is surfaced like a step's (flag + counter); its observation is
     * returned as computed */
    if (!state_finite(e)) {
        e->flags |= UG_FLAG_NONFINITE;
        e->stats[UG_STAT_NONFINITE]++;
    }
    return n;
}
int ugo_reset(ugo_env* e, double* obs) { return ugo_reset_draws(e, NULL, obs); }
int ugo_reset_draws(ugo_env* e, const double* draws, double* obs) {
    e->flags = 0;
    return reset_impl(e, draws, obs);
}
int ugo_step(ugo_env* e, const float* action, double* obs, double* reward, uint8_t* terminated, uint8_t* success) {
    e->flags = 0;
    int n = -1;
    if (e->sc.variant == UG_TASK_TWOBALLS) n = tb_step(e, action, obs, reward, terminated, success);
    else switch (e->sc.task) {
        case UG_TASK_BALLBALANCE: n = bb_step(e, action, obs, reward, terminated, success); break;
        case UG_TASK_CUBESPUSH: n = cp_step(e, action, obs, reward, terminated, success); break;
        case UG_TASK_CUBESGRASP: n = cg_step(e, action, obs, reward, terminated, success); break;
        case UG_TASK_GOLF: n = gf_step(e, action, obs, reward, terminated, success); break;
        case UG_TASK_BOX: n = bx_step(e, action, obs, reward, terminated, success); break;
    }
    if (!state_finite(e)) { /* terminate the episode, zero reward; the autoreset restarts from a clean state */
        *terminated = 1;
        *success = 0;
        *reward = 0.0;
        e->flags |= UG_FLAG_NONFINITE;
        e->stats[UG_STAT_NONFINITE]++;
    }
    return n;
}
/* p.getContactPoints(bodyA, bodyB, linkIndexA, linkIndexB) over the manifold cache of the last substep
 * (read by env_cubes_grasp_v0.py:209-226).  Bodies are entity codes: 0 robot, 1 + i object i,
 * 10 table, 11 plane, 12 pitch, -1 any; links: robot link index, object base -1 (Golf club: base -1, foot 0,
 * disc 1 as env_golf_v0.py:313-327 builds it), -2 any.  Each point is the pybullet tuple as 24 doubles:
 * flag 0, bodyA, bodyB, linkA, linkB, positionOnA[3], positionOnB[3], contactNormalOnB[3], distance,
 * normalForce, lateralFriction1, lateralFrictionDir1[3], lateralFriction2, lateralFrictionDir2[3]; forces are
 * the last solve's impulses / dt, the friction directions btPlaneSpace1 of the normal (the solver's rows),
 * world positions = the points' body-local anchors under the poses of the last substep's narrowphase (prevq /
 * prevpos / prevquat, taken before that substep's integration) -- Bullet's m_positionWorldOnA/B as its
 * refreshContactPoints left them.  Filters as pybullet applies them
 * (PhysicsServerCommandProcessor's contact query): the tuple is swapped (A/B fields exchanged, normal negated)
 * when bodyA names the pair's B side, then bodyB / linkA / linkB filter that orientation; a pair's A side is the
 * robot link for robot pairs, the object for object-static pairs, the sphere (else the lower object) for
 * object-object pairs.  Returns the number of matching points (at most max_pts written). */
static int link_of_collider(const scene* s, int ci) {
    const collider* c = &s->col[ci];
    if (c->ent == 0) return c->link;
    if (s->task == UG_TASK_BOX && (c->ent == 1 || c->ent == 2)) return c->ent == 1 ? 1 : 0; /* door = joint 1, button = 0 */
    if (c->ent >= 1 && c->ent <= MAXOBJ) return ci - s->ocol[c->ent - 1] - 1;
    return -1;
}
static int match(int want, int have) { return want == -1 || want == have; }
static int match_link(int want, int have) { return want == -2 || want == have; }
/* an owner frame as the last substep's narrowphase saw it (the poses in prevq / prevpos / prevquat) */
static xf prev_owner_xf(const ugo_env* e, const kin* k, int owner) {
    xf T;
    if (owner >= 0) { T.R = k->R[owner]; T.p = k->p[owner]; }
    else if (owner <= -2 && owner > -100) { int o = -2 - owner; T.R = qmat(e->prevquat[o]); T.p = e->prevpos[o]; }
    else { T.R = mident(); T.p = V(0, 0, 0); }
    return T;
}
int ugo_contact_points(const ugo_env* e, int bodyA, int bodyB, int linkA, int linkB, double* out, int max_pts) {
    const scene* s = &e->sc;
    kin k;
    fk(e->prevq, &k); /* the narrowphase's poses: Bullet reports m_positionWorldOnA/B from its last refresh */
    int cnt = 0;
    for (int m = 0; m < e->nman; m++) {
        const manifold* M = &e->man[m];
        const pairdef* P = &s->pair[M->pair];
        const int ea = s->col[P->a].ent, eb = s->col[P->b].ent;
        const int la = link_of_collider(s, P->a), lb = link_of_collider(s, P->b);
        /* pybullet's filter order: the orientation comes from bodyA alone (no swap without a bodyA filter, or
         * when it names the pair's A side), then bodyB and the link filters apply in that orientation */
        int swap = 0;
        if (bodyA != -1) {
            if (bodyA == ea) swap = 0;
            else if (bodyA == eb) swap = 1;
            else continue;
        }
        if (!match(bodyB, swap ? ea : eb) || !match_link(linkA, swap ? lb : la) || !match_link(linkB, swap ? la : lb))
            continue;
        xf OA = prev_owner_xf(e, &k, s->col[P->a].owner), OB = prev_owner_xf(e, &k, s->col[P->b].owner);
        for (int j = 0; j < M->npts; j++) {
            const cpoint* c = &M->pt[j];
            if (cnt < max_pts) {
                double* o = out + (size_t)cnt * 24;
                v3 pA = xf_apply(&OA, c->lpA), pB = xf_apply(&OB, c->lpB);
                v3 n = c->n, t1, t2;
                if (ug_fabs(n.z) > 0.7071067811865475244) { /* btPlaneSpace1 (the friction rows' directions) */
                    double a = n.y * n.y + n.z * n.z, kk = 1.0 / ug_sqrt(a);
                    t1 = V(0, -n.z * kk, n.y * kk);
                    t2 = V(a * kk, -n.x * t1.z, n.x * t1.y);
                } else {
                    double a = n.x * n.x + n.y * n.y, kk = 1.0 / ug_sqrt(a);
                    t1 = V(-n.y * kk, n.x * kk, 0);
                    t2 = V(-n.z * t1.y, n.z * t1.x, a * kk);
                }
                if (swap) { v3 t = pA; pA = pB; pB = t; n = vneg(n); }
                if (s->task == UG_TASK_BOX) { /* world coordinates (the restatement keeps the robot base at the origin) */
                    pA.y = pA.y + UG_BX_ROBOT_Y;
                    pB.y = pB.y + UG_BX_ROBOT_Y;
                }
                o[0] = 0.0;
                o[1] = swap ? eb : ea; o[2] = swap ? ea : eb;
                o[3] = swap ? lb : la; o[4] = swap ? la : lb;
                o[5] = pA.x; o[6] = pA.y; o[7] = pA.z;
                o[8] = pB.x; o[9] = pB.y; o[10] = pB.z;
                o[11] = n.x; o[12] = n.y; o[13] = n.z;
                o[14] = c->dist;
                o[15] = c->imp / UG_DT;
                o[16] = c->imp1 / UG_DT;
                o[17] = t1.x; o[18] = t1.y; o[19] = t1.z;
                o[20] = c->imp2 / UG_DT;
                o[21] = t2.x; o[22] = t2.y; o[23] = t2.z;
            }
            cnt++;
        }
    }
    return cnt;
}
/* Camera.shot() -> p.getCameraImage (utilities.py:84-89) restated as ray casting of the env's collision shapes
 * (ug_render.h, shared with the kernel): every pixel against every active collider, the last collider first (statics
 * and objects before the robot's hulls), nearest hit kept, ties to the lower collider index.  rgba H x W x 4,
 * depth H x W, seg H x W (each may be NULL).  Returns -1 for a singular P V. */
int ugo_camera(const ugo_env* e, const float* view16, const float* proj16, int W, int H, int flags, uint8_t* rgba,
               float* depth, int32_t* seg) {
    const scene* s = &e->sc;
    UgrCam cam;
    if (ugr_setup(view16, proj16, &cam) != 0) return -1;
    kin k;
    fk(e->q, &k);
    double R[MAXCOL][9], P[MAXCOL][3], rad[MAXCOL], box[MAXCOL][6];
    int on[MAXCOL];
    for (int ci = 0; ci < s->ncol; ci++) {
        const collider* c = &s->col[ci];
        const xf O = owner_xf(e, &k, c->owner);
        const xf T = shape_xf(&O, c);
        for (int m = 0; m < 9; m++) R[ci][m] = T.R.m[m];
        /* world coordinates: Box-v0's frame has the robot base at the origin (world y + UG_BX_ROBOT_Y) */
        P[ci][0] = T.p.x; P[ci][1] = s->task == UG_TASK_BOX ? T.p.y + UG_BX_ROBOT_Y : T.p.y; P[ci][2] = T.p.z;
        rad[ci] = ugr_radius(c->kind, c->half, UG_HULL_V + 3 * c->v0, c->nv);
        ugr_hull_box(UG_HULL_V + 3 * c->v0, c->kind == UG_SHAPE_HULL ? c->nv : 0, box[ci]);
        on[ci] = collider_active(e, c) != 0;
    }
    for (int pix = 0; pix < W * H; pix++) {
        double o[3], d[3], nb[3] = {0.0, 0.0, 0.0};
        ugr_ray(&cam, pix % W, pix / W, W, H, o, d);
        double best = UGR_MISS;
        int bc = -1;
        for (int ci = s->ncol - 1; ci >= 0; ci--) {
            if (!on[ci]) continue;
            const collider* c = &s->col[ci];
            double nw[3];
            const double t = ugr_shape(R[ci], P[ci], rad[ci], c->kind, c->half, UG_HULL_F + 4 * c->f0, c->nf, box[ci],
                                       best, o, d, nw);
            if (t < best || (t == best && t != UGR_MISS)) { best = t; bc = ci; nb[0] = nw[0]; nb[1] = nw[1]; nb[2] = nw[2]; }
        }
        const int ent = bc >= 0 ? s->col[bc].ent : -1, link = bc >= 0 ? link_of_collider(s, bc) : -1;
        unsigned char px[4];
        float dp;
        int sg;
        ugr_shade(&cam, s->variant, best, nb, ent, link, flags, o, d, px, &dp, &sg);
        if (rgba) { rgba[4 * pix] = px[0]; rgba[4 * pix + 1] = px[1]; rgba[4 * pix + 2] = px[2]; rgba[4 * pix + 3] = px[3]; }
        if (depth) depth[pix] = dp;
        if (seg) seg[pix] = sg;
    }
    return 0;
}
/* the robot's equations of motion at (q, qd) for the dynamics known-answer tests: mass matrix M (NB x NB,
 * CRBA), bias C (RNEA with qdd = 0: gravity g along z, Coriolis / gyroscopic, btMultiBody link damping) and
 * the body COMs (NB x 3, world) */
void ugo_dynamics(const double* q, const double* qd, double g, double* M, double* C, double* com) {
    kin k;
    fk(q, &k);
    robot_dynamics(qd, &k, g, M, C);
    for (int b = 0; b < NB; b++) { com[3 * b] = k.c[b].x; com[3 * b + 1] = k.c[b].y; com[3 * b + 2] = k.c[b].z; }
}
int ugo_flags(const ugo_env* e) { return e->flags; }
void ugo_get_stats(const ugo_env* e, int32_t* out) { memcpy(out, e->stats, sizeof(e->stats)); }
void ugo_set_reward_type(ugo_env* e, int sparse) { e->sparse = sparse != 0; }
void ugo_set_button_mode(ugo_env* e, int mode) { e->button_mode = mode; }
int ugo_g_box_reward(int* flags3, double door, int press, double* r) {
    return ugg_box_reward(&flags3[0], &flags3[1], &flags3[2], door, press, r);
}
void ugo_g_box_target(const double* ee7, const float* a, double* t7) { ugg_box_target(ee7, a, t7); }
/* the Box scene's jointed object o at joint state (q, qd): frame (quat 4, pos 3), M, C, then the link's mass, COM (3)
 * and principal inertia (3) -- for the known-answer tests (tests/test_box_kat.py) */
void ugo_box_joint(int o, double q, double qd, double* out) {
    UgJoint J[2];
    ugj_box_links(&J[0], &J[1]);
    const UgJoint* Jo = &J[o];
    ugj_frame(Jo, q, out, out + 4);
    ugj_dynamics(Jo, out, qd, -10.0, out + 7, out + 8);
    out[9] = Jo->mass;
    for (int i = 0; i < 3; i++) { out[10 + i] = Jo->com[i]; out[13 + i] = Jo->inertia[i]; }
}
int ugo_g_box_press(double button, int mode, int robot_touch, int finger_touch) {
    return ugg_box_press(button, mode, robot_touch, finger_touch);
}
void ugo_set_pgs_bullet(ugo_env* e, int on) { e->pgs_bullet = on != 0; }
/* checkpoint of the env's Python-random stream (624 words + index) */
void ugo_get_rng(const ugo_env* e, uint32_t* mt625) {
    memcpy(mt625, e->rng.mt, 624 * sizeof(uint32_t));
    mt625[624] = (uint32_t)e->rng.idx;
}
void ugo_set_rng(ugo_env* e, const uint32_t* mt625) {
    memcpy(e->rng.mt, mt625, 624 * sizeof(uint32_t));
    e->rng.idx = (int)mt625[624];
}
void ugo_get_state(const ugo_env* e, double* s) {
    memset(s, 0, sizeof(double) * STATE_DIM);
    int i = 0;
    for (int j = 0; j < NB; j++) s[i++] = e->q[j];
    for (int j = 0; j < NB; j++) s[i++] = e->qd[j];
    for (int j = 0; j < 7; j++) s[i++] = e->mtarget[j];
    for (int j = 0; j < 7; j++) s[i++] = e->mon[j];
    for (int o = 0; o < MAXOBJ; o++) s[i++] = e->oactive[o];
    for (int o = 0; o < MAXOBJ; o++) {
        s[i++] = e->opos[o].x; s[i++] = e->opos[o].y; s[i++] = e->opos[o].z;
        s[i++] = e->oquat[o].x; s[i++] = e->oquat[o].y; s[i++] = e->oquat[o].z; s[i++] = e->oquat[o].w;
        s[i++] = e->ov[o].x; s[i++] = e->ov[o].y; s[i++] = e->ov[o].z;
        s[i++] = e->ow[o].x; s[i++] = e->ow[o].y; s[i++] = e->ow[o].z;
    }
    s[i++] = e->nman;
    for (int m = 0; m < MAXMAN; m++) {
        const manifold* M = &e->man[m];
        s[i++] = m < e->nman ? M->pair : -1;
        s[i++] = m < e->nman ? M->npts : 0;
        for (int p = 0; p < 4; p++) {
            const cpoint* c = &M->pt[p];
            int live = m < e->nman && p < M->npts;
            double v[PT_DOUBLES] = {c->lpA.x, c->lpA.y, c->lpA.z, c->lpB.x, c->lpB.y, c->lpB.z,
                                    c->n.x, c->n.y, c->n.z, c->dist, c->imp, c->imp1, c->imp2};
            for (int t = 0; t < PT_DOUBLES; t++) s[i++] = live ? v[t] : 0.0;
        }
    }
    s[i++] = e->goal_approached;
    s[i++] = e->goal_grasped;
    s[i++] = e->overflow;
    s[i++] = e->goal_closed;
    for (int j = 0; j < NB; j++) s[i++] = e->prevq[j];
    for (int o = 0; o < MAXOBJ; o++) {
        s[i++] = e->prevpos[o].x; s[i++] = e->prevpos[o].y; s[i++] = e->prevpos[o].z;
        s[i++] = e->prevquat[o].x; s[i++] = e->prevquat[o].y; s[i++] = e->prevquat[o].z; s[i++] = e->prevquat[o].w;
    }
}
void ugo_set_state(ugo_env* e, const double* s) {
    int i = 0;
    for (int j = 0; j < NB; j++) e->q[j] = s[i++];
    for (int j = 0; j < NB; j++) e->qd[j] = s[i++];
    for (int j = 0; j < 7; j++) e->mtarget[j] = s[i++];
    for (int j = 0; j < 7; j++) e->mon[j] = (int)s[i++];
    for (int o = 0; o < MAXOBJ; o++) e->oactive[o] = (int)s[i++];
    for (int o = 0; o < MAXOBJ; o++) {
        e->opos[o].x = s[i++]; e->opos[o].y = s[i++]; e->opos[o].z = s[i++];
        e->oquat[o].x = s[i++]; e->oquat[o].y = s[i++]; e->oquat[o].z = s[i++]; e->oquat[o].w = s[i++];
        e->ov[o].x = s[i++]; e->ov[o].y = s[i++]; e->ov[o].z = s[i++];
        e->ow[o].x = s[i++]; e->ow[o].y = s[i++]; e->ow[o].z = s[i++];
    }
    e->nman = (int)s[i++];
    for (int m = 0; m < MAXMAN; m++) {
        manifold* M = &e->man[m];
        M->pair = (int)s[i++];
        M->npts = (int)s[i++];
        for (int p = 0; p < 4; p++) {
            cpoint* c = &M->pt[p];
            c->lpA = V(s[i], s[i + 1], s[i + 2]); c->lpB = V(s[i + 3], s[i + 4], s[i + 5]);
            c->n = V(s[i + 6], s[i + 7], s[i + 8]);
            c->dist = s[i + 9]; c->imp = s[i + 10]; c->imp1 = s[i + 11]; c->imp2 = s[i + 12];
            i += PT_DOUBLES;
        }
    }
    e->goal_approached = (int)s[i++];
    e->goal_grasped = (int)s[i++];
    e->overflow = (int)s[i++];
    e->goal_closed = (int)s[i++];
    for (int j = 0; j < NB; j++) e->prevq[j] = s[i++];
    for (int o = 0; o < MAXOBJ; o++) {
        e->prevpos[o].x = s[i++]; e->prevpos[o].y = s[i++]; e->prevpos[o].z = s[i++];
        e->prevquat[o].x = s[i++]; e->prevquat[o].y = s[i++]; e->prevquat[o].z = s[i++]; e->prevquat[o].w = s[i++];
    }
}
void ugo_rng_seed(ugo_env* e, uint32_t seed) { mt_seed(&e->rng, seed); }
double ugo_rng_random(ugo_env* e) { return mt_random(&e->rng); }
double ugo_gdr(double value, double ts, double tm) { return ugg_gdr(value, ts, tm); }
void ugo_euler_from_quat(const double* q, double* rpy) {
    v3 r = euler_from_quat(Q(q[0], q[1], q[2], q[3]));
    rpy[0] = r.x; rpy[1] = r.y; rpy[2] = r.z;
}
void ugo_quat_from_euler(const double* rpy, double* q) {
    q4 r = quat_from_euler(V(rpy[0], rpy[1], rpy[2]));
    q[0] = r.x; q[1] = r.y; q[2] = r.z; q[3] = r.w;
}
void ugo_link_state(const ugo_env* e, int link, double* pos7) {
    v3 p;
    q4 o;
    link_state(e, link, &p, &o);
    pos7[0] = p.x; pos7[1] = p.y; pos7[2] = p.z; pos7[3] = o.x; pos7[4] = o.y; pos7[5] = o.z; pos7[6] = o.w;
}
void ugo_ik(const ugo_env* e, const double* tp, const double* to, double* q_out) {
    ik_solve(e->q, V(tp[0], tp[1], tp[2]), Q(to[0], to[1], to[2], to[3]), q_out);
}
/* OpenMP threads of the next ugo_batch_step calls from this thread (bench.py's all-core and 16-thread samples) */
void ugo_set_threads(int n) {
#ifdef _OPENMP
    extern void omp_set_num_threads(int);
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}
long ugo_batch_step(ugo_env** envs, int n, const float* actions, double* obs, double* reward, uint8_t* terminated,
                    uint8_t* success, int32_t* substeps, int autoreset, int max_episode_steps, int32_t* elapsed) {
    long total = 0;
    if (n <= 0) return 0;
    int task = envs[0]->sc.variant;
    int A = ugo_act_dim(task), O = ugo_obs_dim(task);
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : total)
    for (int i = 0; i < n; i++) {
        int ns = ugo_step(envs[i], actions + (size_t)i * A, obs + (size_t)i * O, reward + i, terminated + i, success + i);
        if (elapsed) elapsed[i] += 1;
        int trunc = elapsed && max_episode_steps > 0 && elapsed[i] >= max_episode_steps;
        if (autoreset && (terminated[i] || trunc)) {
            ns += reset_impl(envs[i], NULL, obs + (size_t)i * O);
            if (elapsed) elapsed[i] = 0;
        }
        substeps[i] = ns;
        total += ns;
    }
    return total;
}

/* ---- hooks for known-answer / golden tests ---- */
void ugo_bb_ball_position(ugo_env* e, const double* paddle, double* out) {
    v3 b = bb_ball_position(e, NULL, V(paddle[0], paddle[1], paddle[2]));
    out[0] = b.x; out[1] = b.y; out[2] = b.z;
}
double ugo_stable_sum(const double* a12) { return np_sum12(a12); }
void ugo_observe(const ugo_env* e, double* obs) {
    if (e->sc.variant == UG_TASK_TWOBALLS) { tb_obs(e, obs); return; }
    switch (e->sc.task) {
        case UG_TASK_BALLBALANCE: bb_obs(e, obs); break;
        case UG_TASK_CUBESPUSH: cp_obs(e, obs); break;
        case UG_TASK_CUBESGRASP: cg_obs(e, obs); break;
        case UG_TASK_GOLF: gf_obs(e, obs); break;
    }
}
int ugo_terminated(const ugo_env* e) {
    if (e->sc.variant == UG_TASK_TWOBALLS) return e->opos[1].z < e->opos[0].z || e->opos[2].z < e->opos[0].z;
    if (e->sc.task == UG_TASK_BALLBALANCE) return e->opos[1].z < e->opos[0].z;
    return 0;
}
/* contact predicates and gripper geometry (A12/A13) for the golden and parity tests */
int ugo_robot_contact(const ugo_env* e, int obj_or_static, int lmin, int lmax) {
    int cb = obj_or_static >= 10 ? static_collider(&e->sc, obj_or_static) : e->sc.ocol[obj_or_static];
    return cb < 0 ? 0 : robot_contact(e, cb, lmin, lmax);
}
double ugo_gripper_opening(const ugo_env* e) { return cg_opening(e); }
void ugo_gripper_center(const ugo_env* e, double* out3) {
    v3 c = gripper_center(e);
    out3[0] = c.x; out3[1] = c.y; out3[2] = c.z;
}
int ugo_choose(ugo_env* e, float w0, float w1) { return cg_choose(e, w0, w1); }
double ugo_norm3(const double* v) { return ug_norm3(v[0], v[1], v[2]); }
/* the shared task glue (ug_glue.h), exported for the golden tests */
double ugo_g_cp_cube1_x(double u) { return ugg_cp_cube1_x(u); }
int ugo_g_cp_reward(int table, int touched, const double* c0, const double* c1, int sparse, double* r) {
    return ugg_cp_reward(table, touched, c0[0], c0[1], c0[2], c1[0], c1[1], c1[2], sparse, r);
}
void ugo_g_cg_cube_xy(double u0, double u1, double* xy) { ugg_cg_cube_xy(u0, u1, &xy[0], &xy[1]); }
int ugo_g_cg_choose(float w0, float w1, double u) { return ugg_cg_choose(w0, w1, u); }
double ugo_g_cg_opening(double d) { return ugg_cg_opening(d); }
int ugo_g_cg_reward(int* flags, double dist, double opening, int grasp, double cube_z, double* r) {
    return ugg_cg_reward(&flags[0], &flags[1], dist, opening, grasp, cube_z, r);
}
void ugo_g_union_center(const double* aabbs, double* c) { ugg_union_center(aabbs, aabbs + 3, aabbs + 6, aabbs + 9, c); }
void ugo_g_gf_ball_xy(double u0, double u1, double* xy) { ugg_gf_ball_xy(u0, u1, &xy[0], &xy[1]); }
int ugo_g_gf_reward(const double* ball, const double* hole, const double* stick, int in_fingers, int floor_contact,
                    int touched, int sparse, double* r, int* term) {
    return ugg_gf_reward(ball, hole, stick, in_fingers, floor_contact, touched, sparse, r, term);
}
void ugo_g_tb_balls(const double* paddle, const double* u4, double* b1, double* b2) {
    ugg_tb_balls(paddle, UG_TB_BALL_R, u4, b1, b2);
}
int ugo_g_tb_reward(const float* a, const double* b1, const double* b2, double paddle_z, double* r) {
    return ugg_tb_reward(a, b1, b2, paddle_z, r);
}
