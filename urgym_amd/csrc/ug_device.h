/* ug_device.h -- gfx950 device building blocks of the URGym hot path: vector /
 * quaternion algebra, MT19937, scene tables, forward kinematics, CRBA/RNEA
 * robot dynamics, LDL^T, per-pair narrowphases, persistent-manifold update,
 * damped-least-squares IK.  They are lane-serial functions; ug_team.h
 * composes them into the one-wavefront-per-env kernel.
 * Model constants (UR5/Robotiq tree, hulls) sit in __constant__ memory and
 * are wave-uniform (scalar loads).  Arithmetic follows the CPU restatement
 * (oracle/ug_oracle.c) operation for operation, compiled with
 * -ffp-contract=off, so the two produce bit-identical trajectories.
 */
#ifndef UG_DEVICE_H
#define UG_DEVICE_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#define UG_CONST static __constant__ const
#ifdef UG_ROBOT_R140 /* the UR5Robotiq140 build (liburgym_r140.so, robot.py:221-240) */
#include "model_data_r140.h"
#include "supcell_data_r140.h"
#else
#include "model_data.h"
#include "supcell_data.h"
#endif
#include "scene_data.h"
#include "ug_detmath.h"
#include "ug_joint.h"
#include "ug_layout.h"

#define NB UG_NB
#define MAXOBJ UG_MAXOBJ
#define NV (NB + 6 * MAXOBJ)
#define MAXMAN UG_MAXMAN
#define MAXROWS 128
#define MAXCOL 28
#define MAXPAIR 192
#define MAXCAND 4   /* per-pair narrowphases emit <= 4 points (box-box culls to 4) */

#define DF __device__ static
#define DFI __device__ static inline

namespace ugd {

/* ---------------- linear algebra (same evaluation order as the oracle) ---------------- */
struct v3 { double x, y, z; };
struct m3 { double m[9]; };
struct q4 { double x, y, z, w; };

DFI v3 V(double x, double y, double z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
DFI v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
/* a floating base's linear / angular velocity clamped per component to +-m_maxCoordinateVelocity (oracle vclamp_coord) */
DFI v3 vclamp_coord(v3 v) {
    return V(ug_vclamp(v.x, UG_MAX_COORD_VEL), ug_vclamp(v.y, UG_MAX_COORD_VEL), ug_vclamp(v.z, UG_MAX_COORD_VEL));
}
DFI v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
DFI v3 vscale(v3 a, double s) { return V(a.x * s, a.y * s, a.z * s); }
DFI v3 vneg(v3 a) { return V(-a.x, -a.y, -a.z); }
DFI double vdot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
DFI v3 vcross(v3 a, v3 b) { return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
DFI double vlen(v3 a) { return ug_sqrt(vdot(a, a)); }
DFI v3 mv(const m3& M, v3 v) {
    const double* m = M.m;
    return V(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[3] * v.x + m[4] * v.y + m[5] * v.z,
             m[6] * v.x + m[7] * v.y + m[8] * v.z);
}
DFI v3 mtv(const m3& M, v3 v) {
    const double* m = M.m;
    return V(m[0] * v.x + m[3] * v.y + m[6] * v.z, m[1] * v.x + m[4] * v.y + m[7] * v.z,
             m[2] * v.x + m[5] * v.y + m[8] * v.z);
}
DFI m3 mm(const m3& A, const m3& B) {
    m3 C;
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++)
            C.m[3 * i + j] = A.m[3 * i] * B.m[j] + A.m[3 * i + 1] * B.m[3 + j] + A.m[3 * i + 2] * B.m[6 + j];
    return C;
}
DFI m3 mtm(const m3& A, const m3& B) {
    m3 C;
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++)
            C.m[3 * i + j] = A.m[i] * B.m[j] + A.m[3 + i] * B.m[3 + j] + A.m[6 + i] * B.m[6 + j];
    return C;
}
DFI m3 mload(const double* p) {
    m3 r;
#pragma unroll
    for (int i = 0; i < 9; i++) r.m[i] = p[i];
    return r;
}
DFI m3 mident() {
    m3 r;
#pragma unroll
    for (int i = 0; i < 9; i++) r.m[i] = 0.0;
    r.m[0] = r.m[4] = r.m[8] = 1.0;
    return r;
}
DFI m3 inertia_world(const m3& R, const double* I6) {
    m3 I;
    I.m[0] = I6[0]; I.m[4] = I6[1]; I.m[8] = I6[2];
    I.m[1] = I.m[3] = I6[3]; I.m[2] = I.m[6] = I6[4]; I.m[5] = I.m[7] = I6[5];
    m3 T = mm(R, I);
    m3 C;
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++)
            C.m[3 * i + j] = T.m[3 * i] * R.m[3 * j] + T.m[3 * i + 1] * R.m[3 * j + 1] + T.m[3 * i + 2] * R.m[3 * j + 2];
    return C;
}
DFI m3 axis_angle(v3 a, double q) {
    double s, c;
    ug_sincos(q, &s, &c);
    double t = 1.0 - c;
    m3 R;
    R.m[0] = t * a.x * a.x + c;       R.m[1] = t * a.x * a.y - s * a.z; R.m[2] = t * a.x * a.z + s * a.y;
    R.m[3] = t * a.x * a.y + s * a.z; R.m[4] = t * a.y * a.y + c;       R.m[5] = t * a.y * a.z - s * a.x;
    R.m[6] = t * a.x * a.z - s * a.y; R.m[7] = t * a.y * a.z + s * a.x; R.m[8] = t * a.z * a.z + c;
    return R;
}
DFI q4 Q(double x, double y, double z, double w) { q4 r; r.x = x; r.y = y; r.z = z; r.w = w; return r; }
DFI q4 qmul(q4 a, q4 b) {
    return Q(a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z,
             a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z);
}
DFI q4 qnormalize(q4 a) {
    double l = ug_sqrt(a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w);
    return Q(a.x / l, a.y / l, a.z / l, a.w / l);
}
DFI m3 qmat(q4 q) {
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
DF q4 mquat(const m3& M) {
    const double* m = M.m;
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
DF v3 euler_from_quat(q4 q) {
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
DF q4 quat_from_euler(v3 rpy) {
    double phi = rpy.x / 2.0, the = rpy.y / 2.0, psi = rpy.z / 2.0;
    double sp = ug_sin(phi), cp = ug_cos(phi), st = ug_sin(the), ct = ug_cos(the), ss = ug_sin(psi), cs = ug_cos(psi);
    q4 q = Q(sp * ct * cs - cp * st * ss, cp * st * cs + sp * ct * ss, cp * ct * ss - sp * st * cs,
             cp * ct * cs + sp * st * ss);
    double len = ug_sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    return Q(q.x / len, q.y / len, q.z / len, q.w / len);
}

/* ---------------- MT19937 on SoA global state (word w of env i at mt[w * n + i]) ---------------- */
struct Rng {
    uint32_t* mt;
    int n, i;
    __device__ uint32_t& w(int k) const { return mt[(size_t)k * n + i]; }
};
DF uint32_t mt_next(const Rng& r) {
    uint32_t idx = r.w(624);
    if (idx >= 624) {
        for (int k = 0; k < 624; k++) {
            uint32_t y = (r.w(k) & 0x80000000u) | (r.w((k + 1) % 624) & 0x7fffffffu);
            r.w(k) = r.w((k + 397) % 624) ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        idx = 0;
    }
    uint32_t y = r.w(idx);
    r.w(624) = idx + 1;
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}
DF double mt_random(const Rng& r) {
    uint32_t a = mt_next(r) >> 5, b = mt_next(r) >> 6;
    return ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);
}
/* the random() the next mt_random(Rng{m, 1, 0}) would return, without advancing the stream (m: one env's 624 words +
 * index).  Past the end of a generation its first words are the next generation's, formed as mt_next's twist forms
 * words 0 and 1 (both read only words of the current generation: 0, 1, 2, 397, 398). */
DF uint32_t mt_temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}
DF uint32_t mt_twist_word(const uint32_t* m, int k) {
    const uint32_t y = (m[k] & 0x80000000u) | (m[k + 1] & 0x7fffffffu);
    return m[k + 397] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}
DF double mt_peek_random(const uint32_t* m) {
    const uint32_t idx = m[624];
    const uint32_t w0 = idx < 624 ? m[idx] : mt_twist_word(m, 0);
    const uint32_t w1 = idx + 1 < 624 ? m[idx + 1] : mt_twist_word(m, idx < 624 ? 0 : 1);
    const uint32_t a = mt_temper(w0) >> 5, b = mt_temper(w1) >> 6;
    return ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);
}

/* ---------------- scene (built on the host, read-only, wave-uniform) ---------------- */
struct Collider {
    int kind;
    double half[3];
    double margin;
    int v0, nv, f0, nf;
    int c0; /* full hulls: first chunk bounding sphere (UG_HULL_CS) */
    m3 R; v3 P;
    m3 aR; v3 aP;
    v3 ac, ah;
    double disc;
    double friction, restitution, rolling;
    int owner, ent, link;
    /* the convex-convex path (UG_CONTACT_GJK, ug_gjk.h): Bullet's shape as GJK sees it (oracle build_scene) */
    v3 gimp;        /* box / cylinder implicit dimensions (outer minus margin) */
    double gmargin; /* getMargin(): collision margin, a sphere's radius */
    int gjkbox;     /* a convex mesh kept as its box (the Golf pitch): every pair of it is convex-convex */
    double gradius; /* the largest distance of a core support point from the shape origin (certificate bound) */
    int compound;   /* btCompoundShape collision object: its child manifolds are refreshed before the narrowphase */
    int scb, sck;   /* a full hull's support-cell table (first cell, K; scb -1: none), set with the GJK parameters */
};
struct PairDef { int a, b; double thr, friction, restitution, rolling; };
struct Scene {
    int task;    /* base task: scene and physics */
    int variant; /* the env id's task (== task, or a variant's UG_TASK_*): step / obs glue */
    double gravity;
    int nobj;
    double omass[MAXOBJ];
    v3 oinertia[MAXOBJ];
    int ncol;
    Collider col[MAXCOL];
    int ocol[MAXOBJ];  /* first collider of each object */
    int oncol[MAXOBJ]; /* colliders of each object (consecutive) */
    UgJoint ojoint[MAXOBJ]; /* one-dof links on a fixed base (Box: door, button; ug_joint.h); kind UGJ_FREE otherwise */
    int njoint, jorder[MAXOBJ]; /* the jointed objects in the multibody's joint order (Box: button = joint 0, door = 1) */
    int npair;
    PairDef pair[MAXPAIR];
    int sparse; /* reward_type != 'dense' (urgym_set_reward_type) */
    int button_mode; /* Box-v0 button_touch_mode (UG_BX_TOUCH_*, urgym_set_button_mode) */
    int full;   /* full-geometry mode (UG_GEOM_FULL): robot hulls with every vertex and face */
    int gjk;    /* contact generation: 1 Bullet's convex-convex GJK / EPA (the default), 0 vertex-in-hull */
    /* the quiescent-collision bound (ug_team.h quiescent_ok): robot collider c's points move by at most
     * sum_j |q_j - q_ref_j| qsw[c][j] between two configurations (0 for dofs that do not move it, static colliders) */
    double qsw[MAXCOL][NB];
};

struct CPoint { v3 lpA, lpB, n; double dist, imp, imp1, imp2; };
struct Manifold { int pair, npts; CPoint pt[4]; };
/* the lane-per-pair working manifold lives in LDS (team_collide: g_sh.pm[lane]); LDS-qualified values are
 * moved field by field (plain aggregates have no address-space-qualified copy operations) */
typedef __attribute__((address_space(3))) Manifold LManifold;
typedef __attribute__((address_space(3))) CPoint LCPoint;
typedef __attribute__((address_space(3))) v3 Lv3;
__device__ static inline v3 ldv(const Lv3& a) { v3 r; r.x = a.x; r.y = a.y; r.z = a.z; return r; }
__device__ static inline void stv(Lv3& d, v3 a) { d.x = a.x; d.y = a.y; d.z = a.z; }
__device__ static inline void stpt(LCPoint& d, const CPoint& s) {
    stv(d.lpA, s.lpA); stv(d.lpB, s.lpB); stv(d.n, s.n);
    d.dist = s.dist; d.imp = s.imp; d.imp1 = s.imp1; d.imp2 = s.imp2;
}
__device__ static inline void cppt(LCPoint& d, const LCPoint& s) {
    stv(d.lpA, ldv(s.lpA)); stv(d.lpB, ldv(s.lpB)); stv(d.n, ldv(s.n));
    d.dist = s.dist; d.imp = s.imp; d.imp1 = s.imp1; d.imp2 = s.imp2;
}

/* ---------------- kinematics ---------------- */
struct Kin {
    m3 R[NB];
    v3 p[NB];
    v3 a[NB];
    v3 c[NB];
};
DF void fk(const double* q, Kin& k) {
    for (int b = 0; b < NB; b++) {
        int pb = UG_BODY_PARENT[b];
        m3 Rpb = mload(&UG_BODY_R[9 * b]);
        v3 Ppb = V(UG_BODY_P[3 * b], UG_BODY_P[3 * b + 1], UG_BODY_P[3 * b + 2]);
        v3 ax = V(UG_BODY_AXIS[3 * b], UG_BODY_AXIS[3 * b + 1], UG_BODY_AXIS[3 * b + 2]);
        m3 Rj = axis_angle(ax, q[b]);
        m3 Rp;
        v3 pp;
        if (pb < 0) { Rp = mident(); pp = V(0, 0, 0); }
        else { Rp = k.R[pb]; pp = k.p[pb]; }
        m3 Rtmp = mm(Rp, Rpb);
        k.R[b] = mm(Rtmp, Rj);
        k.p[b] = vadd(pp, mv(Rp, Ppb));
        k.a[b] = mv(Rtmp, ax);
        v3 com = V(UG_BODY_COM[3 * b], UG_BODY_COM[3 * b + 1], UG_BODY_COM[3 * b + 2]);
        k.c[b] = vadd(k.p[b], mv(k.R[b], com));
    }
}
DF void link_frame(const Kin& k, int l, int com, m3& R, v3& p) {
    int b = UG_LINK_BODY[l];
    m3 Rl = mload(com ? &UG_LINK_COMR[9 * l] : &UG_LINK_R[9 * l]);
    const double* P = com ? &UG_LINK_COMP[3 * l] : &UG_LINK_P[3 * l];
    v3 Pl = V(P[0], P[1], P[2]);
    if (b < 0) { R = Rl; p = Pl; return; }
    R = mm(k.R[b], Rl);
    p = vadd(k.p[b], mv(k.R[b], Pl));
}
DFI int moves(int d, int b) {
    while (b >= 0) {
        if (b == d) return 1;
        b = UG_BODY_PARENT[b];
    }
    return 0;
}

/* ---------------- robot dynamics (CRBA + RNEA, world-frame spatial algebra) ---------------- */
struct SV { v3 w, v; };
DFI SV spatial_inertia_mul(double m, v3 h, const m3& J, SV x) {
    SV r;
    r.w = vadd(mv(J, x.w), vcross(h, x.v));
    r.v = vsub(vscale(x.v, m), vcross(h, x.w));
    return r;
}
/* work arrays of robot_dynamics: the team kernels place them in LDS (a private array would live in
 * scratch, whose latency the serial recursions pay at every access) */
struct DynWork {
    double m[NB], cm[NB];
    v3 h[NB], ch[NB];
    m3 J[NB], cJ[NB];
    SV S[NB], Vb[NB], Ab[NB], f[NB];
    v3 fdl[UG_NL], tl[UG_NL]; /* link damping force / torque (team version) */
    double C[NB];             /* bias forces (team version) */
};
DF void robot_dynamics(const double* qd, const Kin& k, double g, double* M, double* C, DynWork& w) {
    double* m = w.m;
    v3* h = w.h;
    m3* J = w.J;
    double* cm = w.cm;
    v3* ch = w.ch;
    m3* cJ = w.cJ;
#pragma unroll
    for (int b = 0; b < NB; b++) {
        m[b] = UG_BODY_MASS[b];
        v3 c = k.c[b];
        h[b] = vscale(c, m[b]);
        m3 Iw = inertia_world(k.R[b], &UG_BODY_I[6 * b]);
        double cc = vdot(c, c);
        m3 Jb;
        Jb.m[0] = Iw.m[0] + m[b] * (cc - c.x * c.x); Jb.m[1] = Iw.m[1] - m[b] * (c.x * c.y); Jb.m[2] = Iw.m[2] - m[b] * (c.x * c.z);
        Jb.m[3] = Iw.m[3] - m[b] * (c.y * c.x); Jb.m[4] = Iw.m[4] + m[b] * (cc - c.y * c.y); Jb.m[5] = Iw.m[5] - m[b] * (c.y * c.z);
        Jb.m[6] = Iw.m[6] - m[b] * (c.z * c.x); Jb.m[7] = Iw.m[7] - m[b] * (c.z * c.y); Jb.m[8] = Iw.m[8] + m[b] * (cc - c.z * c.z);
        J[b] = Jb;
        cm[b] = m[b]; ch[b] = h[b]; cJ[b] = Jb;
    }
#pragma unroll
    for (int b = NB - 1; b >= 0; b--) {
        int p = UG_BODY_PARENT[b];
        if (p < 0) continue;
        cm[p] += cm[b];
        ch[p] = vadd(ch[p], ch[b]);
#pragma unroll
        for (int i = 0; i < 9; i++) cJ[p].m[i] += cJ[b].m[i];
    }
    SV* S = w.S;
#pragma unroll
    for (int b = 0; b < NB; b++) { S[b].w = k.a[b]; S[b].v = vcross(k.p[b], k.a[b]); }
#pragma unroll
    for (int i = 0; i < NB * NB; i++) M[i] = 0.0;
#pragma unroll
    for (int b = 0; b < NB; b++) {
        SV F = spatial_inertia_mul(cm[b], ch[b], cJ[b], S[b]);
        M[b * NB + b] = vdot(S[b].w, F.w) + vdot(S[b].v, F.v);
        int j = UG_BODY_PARENT[b];
#pragma unroll
        for (int depth = 0; depth < NB; depth++) { /* the ancestors of b (compile-time after unrolling) */
            if (j < 0) break;
            double x = vdot(S[j].w, F.w) + vdot(S[j].v, F.v);
            M[j * NB + b] = x;
            M[b * NB + j] = x;
            j = UG_BODY_PARENT[j];
        }
    }
    SV *Vb = w.Vb, *Ab = w.Ab, *f = w.f;
#pragma unroll
    for (int b = 0; b < NB; b++) {
        int p = UG_BODY_PARENT[b];
        SV Vp, Ap;
        if (p < 0) { Vp.w = V(0, 0, 0); Vp.v = V(0, 0, 0); Ap.w = V(0, 0, 0); Ap.v = V(0, 0, -g); }
        else { Vp = Vb[p]; Ap = Ab[p]; }
        SV vj; vj.w = vscale(S[b].w, qd[b]); vj.v = vscale(S[b].v, qd[b]);
        Vb[b].w = vadd(Vp.w, vj.w); Vb[b].v = vadd(Vp.v, vj.v);
        Ab[b].w = vadd(Ap.w, vcross(Vb[b].w, vj.w));
        Ab[b].v = vadd(Ap.v, vadd(vcross(Vb[b].w, vj.v), vcross(Vb[b].v, vj.w)));
        SV IA = spatial_inertia_mul(m[b], h[b], J[b], Ab[b]);
        SV IV = spatial_inertia_mul(m[b], h[b], J[b], Vb[b]);
        f[b].w = vadd(IA.w, vadd(vcross(Vb[b].w, IV.w), vcross(Vb[b].v, IV.v)));
        f[b].v = vadd(IA.v, vcross(Vb[b].w, IV.v));
        double wn = vlen(Vb[b].w);
        m3 D = inertia_world(k.R[b], &UG_BODY_DAMPI[6 * b]);
        v3 tau = vscale(mv(D, Vb[b].w), UG_ANG_DAMP + UG_ANG_DAMP * wn);
        f[b].w = vadd(f[b].w, tau);
    }
#pragma unroll
    for (int l = 1; l < UG_NL; l++) {
        int b = UG_LINK_BODY[l];
        if (b < 0) continue;
        v3 cl = vadd(k.p[b], mv(k.R[b], V(UG_LINK_COMP[3 * l], UG_LINK_COMP[3 * l + 1], UG_LINK_COMP[3 * l + 2])));
        v3 vl = vadd(Vb[b].v, vcross(Vb[b].w, cl));
        double vn = vlen(vl);
        v3 fd = vscale(vl, UG_LINK_MASS[l] * (UG_LIN_DAMP + UG_LIN_DAMP * vn));
        f[b].v = vadd(f[b].v, fd);
        f[b].w = vadd(f[b].w, vcross(cl, fd));
    }
#pragma unroll
    for (int b = NB - 1; b >= 0; b--) {
        C[b] = vdot(S[b].w, f[b].w) + vdot(S[b].v, f[b].v);
        int p = UG_BODY_PARENT[b];
        if (p >= 0) { f[p].w = vadd(f[p].w, f[b].w); f[p].v = vadd(f[p].v, f[b].v); }
    }
}
DF void ldlt(double* A, int n) {
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
DF void ldlt_solve(const double* A, int n, double* x) {
    for (int i = 0; i < n; i++)
        for (int k2 = 0; k2 < i; k2++) x[i] -= A[i * n + k2] * x[k2];
    for (int i = 0; i < n; i++) x[i] = x[i] / A[i * n + i];
    for (int i = n - 1; i >= 0; i--)
        for (int k2 = i + 1; k2 < n; k2++) x[i] -= A[k2 * n + i] * x[k2];
}

/* ---------------- collision ---------------- */
struct XF { m3 R; v3 p; };
DFI v3 xf_apply(const XF& T, v3 x) { return vadd(mv(T.R, x), T.p); }
DFI v3 xf_inv_apply(const XF& T, v3 x) { return mtv(T.R, vsub(x, T.p)); }
DFI XF shape_xf(const XF& O, const Collider& c) {
    XF T;
    T.R = mm(O.R, c.R);
    T.p = vadd(O.p, mv(O.R, c.P));
    return T;
}
DF void world_aabb(const XF& O, const Collider& c, v3& lo, v3& hi) {
    m3 Rw = mm(O.R, c.aR);
    v3 pw = vadd(O.p, mv(O.R, c.aP));
    v3 ctr = vadd(mv(Rw, c.ac), pw);
    const double* r = Rw.m;
    v3 ext = V(ug_fabs(r[0]) * c.ah.x + ug_fabs(r[1]) * c.ah.y + ug_fabs(r[2]) * c.ah.z,
               ug_fabs(r[3]) * c.ah.x + ug_fabs(r[4]) * c.ah.y + ug_fabs(r[5]) * c.ah.z,
               ug_fabs(r[6]) * c.ah.x + ug_fabs(r[7]) * c.ah.y + ug_fabs(r[8]) * c.ah.z);
    lo = vsub(ctr, ext);
    hi = vadd(ctr, ext);
}

struct Cand { v3 n, pB; double d; };
/* a pair's candidate slots: LDS (team_collide's u.cand.c[lane]), so the dynamically indexed list never goes
 * to scratch memory */
typedef __attribute__((address_space(3))) Cand LCand;
struct CandList { int n; LCand* c; };
DFI void cand_add(CandList& L, v3 n, v3 pB, double d) {
    if (L.n < MAXCAND) { stv(L.c[L.n].n, n); stv(L.c[L.n].pB, pB); L.c[L.n].d = d; L.n++; }
}

DF void nc_sphere_box(const XF& TA, const Collider& A, const XF& TB, const Collider& B, double thr, CandList& out) {
    double r = A.half[0];
    double bm = B.margin;
    v3 he = V(B.half[0] - bm, B.half[1] - bm, B.half[2] - bm);
    v3 rel = xf_inv_apply(TB, TA.p);
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
    cand_add(out, mv(TB.R, n), xf_apply(TB, pb), depth);
}
DF void nc_sphere_sphere(const XF& TA, const Collider& A, const XF& TB, const Collider& B, double thr, CandList& out) {
    v3 d = vsub(TA.p, TB.p);
    double len = vlen(d);
    double dist = len - (A.half[0] + B.half[0]);
    if (dist > thr) return;
    v3 n = len > 2.220446049250313e-16 ? vscale(d, 1.0 / len) : V(1, 0, 0);
    cand_add(out, n, vadd(TB.p, vscale(n, B.half[0])), dist);
}

/* box-box working arrays: one LDS slot per box-box lane (team_collide), so the dynamically indexed clip
 * buffers never go to scratch memory */
typedef __attribute__((address_space(3))) double ldouble;
typedef __attribute__((address_space(3))) int lint;
struct BoxScratch { double quad[8], ret[16], buffer[16], dep[8], ang[8], pt[24]; int avail[8], iret[8]; };
typedef __attribute__((address_space(3))) BoxScratch LBoxScratch;
DF int intersect_rect_quad(const double h[2], ldouble* p, ldouble* ret, ldouble* buffer) {
    int nq = 4, nr = 0;
    ldouble* q = p;
    ldouble* r = ret;
    for (int dir = 0; dir <= 1; dir++) {
        for (int sign = -1; sign <= 1; sign += 2) {
            ldouble* pq = q;
            ldouble* pr = r;
            nr = 0;
            for (int i = nq; i > 0; i--) {
                if (sign * pq[dir] < h[dir]) {
                    pr[0] = pq[0]; pr[1] = pq[1];
                    pr += 2; nr++;
                    if (nr & 8) { q = r; goto done; }
                }
                ldouble* nextq = (i > 1) ? pq + 2 : q;
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
    if (q != ret)
        for (int i = 0; i < nr * 2; i++) ret[i] = q[i];
    return nr;
}
DF void cull_points(int n, const ldouble* p, int m, int i0, lint* iret, ldouble* A, lint* avail) {
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
    for (int i = 0; i < n; i++) A[i] = ug_atan2(p[i * 2 + 1] - cy, p[i * 2] - cx);
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
DFI double col_dot(const m3& A, int i, const m3& B, int j) {
    return A.m[i] * B.m[j] + A.m[3 + i] * B.m[3 + j] + A.m[6 + i] * B.m[6 + j];
}
DFI double col_dotv(const m3& A, int i, v3 v) { return A.m[i] * v.x + A.m[3 + i] * v.y + A.m[6 + i] * v.z; }
DFI double vget(v3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
DFI void vsetc(v3& v, int i, double x) { if (i == 0) v.x = x; else if (i == 1) v.y = x; else v.z = x; }

DF void nc_box_box(const XF& TA, const Collider& A, const XF& TB, const Collider& B, double thr, CandList& out,
                   LBoxScratch& S) {
    (void)thr;
    const double fudge = 1.05;
    const m3& R1 = TA.R;
    const m3& R2 = TB.R;
    v3 p1 = TA.p, p2 = TB.p;
    v3 p = vsub(p2, p1);
    v3 pp = mtv(R1, p);
    double Ah[3] = {A.half[0], A.half[1], A.half[2]};
    double Bh[3] = {B.half[0], B.half[1], B.half[2]};
    double R11 = col_dot(R1, 0, R2, 0), R12 = col_dot(R1, 0, R2, 1), R13 = col_dot(R1, 0, R2, 2);
    double R21 = col_dot(R1, 1, R2, 0), R22 = col_dot(R1, 1, R2, 1), R23 = col_dot(R1, 1, R2, 2);
    double R31 = col_dot(R1, 2, R2, 0), R32 = col_dot(R1, 2, R2, 1), R33 = col_dot(R1, 2, R2, 2);
    double Q11 = ug_fabs(R11), Q12 = ug_fabs(R12), Q13 = ug_fabs(R13);
    double Q21 = ug_fabs(R21), Q22 = ug_fabs(R22), Q23 = ug_fabs(R23);
    double Q31 = ug_fabs(R31), Q32 = ug_fabs(R32), Q33 = ug_fabs(R33);
    double s = -1e300, s2, l, e1;
    int invert_normal = 0, code = 0;
    int nR = -1;
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
        const m3& Rn = nR < 3 ? R1 : R2;
        int c = nR % 3;
        normal = V(Rn.m[c], Rn.m[3 + c], Rn.m[6 + c]);
    } else {
        normal = mv(R1, normalC);
    }
    if (invert_normal) normal = vneg(normal);
    double depth = -s;
    if (code > 6) {
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
        int ia = (code - 7) / 3, ib = (code - 7) % 3;
        v3 ua = V(R1.m[ia], R1.m[3 + ia], R1.m[6 + ia]);
        v3 ub = V(R2.m[ib], R2.m[3 + ib], R2.m[6 + ib]);
        v3 pd = vsub(pb, pa);
        double uaub = vdot(ua, ub), q1 = vdot(ua, pd), q2 = -vdot(ub, pd);
        double d = 1.0 - uaub * uaub, beta;
        if (d <= 0.0001) { beta = 0; }
        else { d = 1.0 / d; beta = (uaub * q1 + q2) * d; }
        pb = vadd(pb, vscale(ub, beta));
        cand_add(out, vneg(normal), pb, -depth);
        return;
    }
    const m3* Ra;
    const m3* Rb;
    v3 pa, pb;
    const double* Sa;
    const double* Sb;
    if (code <= 3) { Ra = &R1; Rb = &R2; pa = p1; pb = p2; Sa = Ah; Sb = Bh; }
    else { Ra = &R2; Rb = &R1; pa = p2; pb = p1; Sa = Bh; Sb = Ah; }
    v3 normal2 = code <= 3 ? normal : vneg(normal);
    v3 nr = mtv(*Rb, normal2);
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
    ldouble* quad = S.quad;
    double c1 = col_dotv(*Ra, code1, center), c2 = col_dotv(*Ra, code2, center);
    double m11 = col_dot(*Ra, code1, *Rb, a1), m12 = col_dot(*Ra, code1, *Rb, a2);
    double m21 = col_dot(*Ra, code2, *Rb, a1), m22 = col_dot(*Ra, code2, *Rb, a2);
    {
        double k1 = m11 * Sb[a1], k2 = m21 * Sb[a1], k3 = m12 * Sb[a2], k4 = m22 * Sb[a2];
        quad[0] = c1 - k1 - k3; quad[1] = c2 - k2 - k4;
        quad[2] = c1 - k1 + k3; quad[3] = c2 - k2 + k4;
        quad[4] = c1 + k1 + k3; quad[5] = c2 + k2 + k4;
        quad[6] = c1 + k1 - k3; quad[7] = c2 + k2 - k4;
    }
    double rect[2] = {Sa[code1], Sa[code2]};
    ldouble* ret = S.ret;
    int n = intersect_rect_quad(rect, quad, ret, S.buffer);
    if (n < 1) return;
    ldouble* pt = S.pt;
    ldouble* dep = S.dep;
    double det1 = 1.0 / (m11 * m22 - m12 * m21);
    m11 *= det1; m12 *= det1; m21 *= det1; m22 *= det1;
    int cnum = 0;
    v3 rba1 = V(Rb->m[a1], Rb->m[3 + a1], Rb->m[6 + a1]);
    v3 rba2 = V(Rb->m[a2], Rb->m[3 + a2], Rb->m[6 + a2]);
    for (int j = 0; j < n; j++) {
        double k1 = m22 * (ret[j * 2] - c1) - m12 * (ret[j * 2 + 1] - c2);
        double k2 = -m21 * (ret[j * 2] - c1) + m11 * (ret[j * 2 + 1] - c2);
        const v3 pc = vadd(vadd(center, vscale(rba1, k1)), vscale(rba2, k2));
        pt[3 * cnum] = pc.x; pt[3 * cnum + 1] = pc.y; pt[3 * cnum + 2] = pc.z;
        dep[cnum] = Sa[codeN] - vdot(normal2, pc);
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
            v3 pw = vadd(V(pt[3 * j], pt[3 * j + 1], pt[3 * j + 2]), pa);
            if (code >= 4) pw = vsub(pw, vscale(normal, dep[j]));
            cand_add(out, vneg(normal), pw, -dep[j]);
        }
    } else {
        int i1 = 0;
        double maxdepth = dep[0];
        for (int i = 1; i < cnum; i++)
            if (dep[i] > maxdepth) { maxdepth = dep[i]; i1 = i; }
        lint* iret = S.iret;
        cull_points(cnum, ret, maxc, i1, iret, S.ang, S.avail);
        for (int j = 0; j < maxc; j++) {
            const int ij = iret[j];
            v3 pw = vadd(V(pt[3 * ij], pt[3 * ij + 1], pt[3 * ij + 2]), pa);
            if (code >= 4) pw = vsub(pw, vscale(normal, dep[ij]));
            cand_add(out, vneg(normal), pw, -dep[ij]);
        }
    }
}

/* max over the hull's face planes of the signed distance of y, first face attaining it (sequential scan
 * semantics).  Planes are fetched HP_BATCH at a time with every load issued before the first use: the
 * per-face loop would otherwise wait one memory latency per face. */
#define HP_BATCH 8
template <class C> /* a Collider, or any type with the hull range fields nf / f0 */
DFI void hull_plane_max(const C& A, v3 y, double& smax, int& fm) {
    const int nf = A.nf, f0 = A.f0;
    for (int b = 0; b < nf; b += HP_BATCH) {
        double F[HP_BATCH][4];
#pragma unroll
        for (int u = 0; u < HP_BATCH; u++) {
            const int f = b + u < nf ? b + u : nf - 1;
#pragma unroll
            for (int c = 0; c < 4; c++) F[u][c] = UG_HULL_F[4 * (f0 + f) + c];
        }
#pragma unroll
        for (int u = 0; u < HP_BATCH; u++)
#pragma unroll
            for (int c = 0; c < 4; c++) asm volatile("" : "+v"(F[u][c])); /* all loads complete here, together */
#pragma unroll
        for (int u = 0; u < HP_BATCH; u++) {
            double sd = F[u][0] * y.x + F[u][1] * y.y + F[u][2] * y.z - F[u][3];
            if (b + u < nf && sd > smax) { smax = sd; fm = b + u; }
        }
    }
}
/* ---- full geometry: the club disc as a true cylinder (UG_SHAPE_CYL), oracle cyl_point / cyl_support / nc_sphere_cyl
 * (the polytope pairs run on the whole wave: ug_team.h team_poly_cyl) ---- */
DFI double cyl_point(double r, double hh, v3 x, v3& nl, v3& pl) {
    const double rho = ug_sqrt(x.x * x.x + x.y * x.y);
    const double dr = rho - r, dz = ug_fabs(x.z) - hh;
    const double sz = x.z < 0 ? -1.0 : 1.0;
    if (dr <= 0 && dz <= 0) {
        if (dr > dz && rho > 0) {
            nl = V(x.x / rho, x.y / rho, 0.0);
            pl = V(nl.x * r, nl.y * r, x.z);
            return dr;
        }
        nl = V(0.0, 0.0, sz);
        pl = V(x.x, x.y, sz * hh);
        return dz;
    }
    const double k = rho > r ? r / rho : 1.0;
    const v3 q = V(x.x * k, x.y * k, ug_max(-hh, ug_min(hh, x.z)));
    const v3 d = vsub(x, q);
    const double len = vlen(d);
    nl = vscale(d, 1.0 / len);
    pl = q;
    return len;
}
/* support points along u (cylinder frame): returns their count (1, or the cap's 4 rim points when u is axial);
 * point j of 4 is (+-r, 0) / (0, +-r) in order */
DFI int cyl_support_n(v3 u) { return ug_sqrt(u.x * u.x + u.y * u.y) > 1e-9 ? 1 : 4; }
DFI v3 cyl_support_pt(double r, double hh, v3 u, int j) {
    const double sz = u.z < 0 ? -1.0 : 1.0;
    const double ur = ug_sqrt(u.x * u.x + u.y * u.y);
    if (ur > 1e-9) return V(r * (u.x / ur), r * (u.y / ur), sz * hh);
    return j == 0 ? V(r, 0.0, sz * hh) : j == 1 ? V(-r, 0.0, sz * hh) : j == 2 ? V(0.0, r, sz * hh) : V(0.0, -r, sz * hh);
}
DF void nc_sphere_cyl(const XF& TA, const Collider& A, const XF& TB, const Collider& B, double thr, CandList& out) {
    const v3 x = xf_inv_apply(TB, TA.p);
    v3 nl, pl;
    const double d = cyl_point(B.half[0], B.half[2], x, nl, pl);
    const double depth = d - A.half[0];
    if (depth < thr) cand_add(out, mv(TB.R, nl), xf_apply(TB, pl), depth);
}
/* hull (robot link) vs box: cooperative, one wavefront per pair -- ug_team.h team_hull_box */
DF void nc_hull_sphere(const XF& TA, const Collider& A, const XF& TB, const Collider& B, double thr, CandList& out) {
    v3 y = mtv(TA.R, vsub(TB.p, TA.p));
    double r = B.half[0];
    double smax = -1e300;
    int fm = -1;
    hull_plane_max(A, y, smax, fm);
    double depth = smax - r - A.margin;
    if (depth >= thr) return;
    const double* F = &UG_HULL_F[4 * (A.f0 + fm)];
    v3 nw = vneg(mv(TA.R, V(F[0], F[1], F[2])));
    cand_add(out, nw, vadd(TB.p, vscale(nw, r)), depth);
}

DF int sort_cached(const LManifold& M, const CPoint& pt) {
    int maxi = -1;
    double maxpen = pt.dist;
    for (int i = 0; i < 4; i++)
        if (M.pt[i].dist < maxpen) { maxi = i; maxpen = M.pt[i].dist; }
    double res[4] = {0, 0, 0, 0};
    if (maxi != 0) { v3 a = vsub(pt.lpA, ldv(M.pt[1].lpA)), b = vsub(ldv(M.pt[3].lpA), ldv(M.pt[2].lpA)); v3 c = vcross(a, b); res[0] = vdot(c, c); }
    if (maxi != 1) { v3 a = vsub(pt.lpA, ldv(M.pt[0].lpA)), b = vsub(ldv(M.pt[3].lpA), ldv(M.pt[2].lpA)); v3 c = vcross(a, b); res[1] = vdot(c, c); }
    if (maxi != 2) { v3 a = vsub(pt.lpA, ldv(M.pt[0].lpA)), b = vsub(ldv(M.pt[3].lpA), ldv(M.pt[1].lpA)); v3 c = vcross(a, b); res[2] = vdot(c, c); }
    if (maxi != 3) { v3 a = vsub(pt.lpA, ldv(M.pt[0].lpA)), b = vsub(ldv(M.pt[2].lpA), ldv(M.pt[1].lpA)); v3 c = vcross(a, b); res[3] = vdot(c, c); }
    int bi = -1;
    double bv = -1e300;
    for (int i = 0; i < 4; i++)
        if (ug_fabs(res[i]) > bv) { bv = ug_fabs(res[i]); bi = i; }
    return bi;
}
/* the pair's collider poses as LDS records (g_sh.O): read through an LDS-typed reference, so the reads are ds_*
 * instructions (a generic one would be a flat access that waits for every outstanding memory operation) */
typedef __attribute__((address_space(3))) const XF LXF;
DFI XF ldxf(const LXF& T) {
    XF r;
#pragma unroll
    for (int i = 0; i < 9; i++) r.R.m[i] = T.R.m[i];
    r.p = V(T.p.x, T.p.y, T.p.z);
    return r;
}
DFI const LXF& lxf(const XF& T) { return *(const LXF*)&T; }
DF void manifold_add(LManifold& M, const LXF& TA0, const LXF& TB0, const Cand c, double thr) {
    if (c.d > thr) return;
    const XF TA = ldxf(TA0), TB = ldxf(TB0);
    v3 pA = vadd(c.pB, vscale(c.n, c.d));
    CPoint np;
    np.lpA = xf_inv_apply(TA, pA);
    np.lpB = xf_inv_apply(TB, c.pB);
    np.n = c.n;
    np.dist = c.d;
    np.imp = np.imp1 = np.imp2 = 0.0;
    double shortest = thr * thr;
    int nearp = -1;
    for (int i = 0; i < M.npts; i++) {
        v3 d = vsub(ldv(M.pt[i].lpA), np.lpA);
        double x = vdot(d, d);
        if (x < shortest) { shortest = x; nearp = i; }
    }
    if (nearp >= 0) {
        np.imp = M.pt[nearp].imp; np.imp1 = M.pt[nearp].imp1; np.imp2 = M.pt[nearp].imp2;
        stpt(M.pt[nearp], np);
        return;
    }
    int ins = M.npts;
    if (ins == 4) ins = sort_cached(M, np);
    else M.npts++;
    if (ins < 0) ins = 0;
    stpt(M.pt[ins], np);
}
DF void manifold_refresh(LManifold& M, const LXF& TA0, const LXF& TB0, double thr) {
    const XF TA = ldxf(TA0), TB = ldxf(TB0);
    /* the world points of the first pass are kept (registers, compile-time slots) for the removal pass: the
     * removal pass visits slots in descending order and a removal only overwrites the slot just visited, so
     * every slot it reads still holds its original point */
    const int n0 = M.npts;
    v3 wA[4], wB[4];
#pragma unroll
    for (int i = 3; i >= 0; i--) {
        if (i < n0) {
            LCPoint& p = M.pt[i];
            wA[i] = xf_apply(TA, ldv(p.lpA));
            wB[i] = xf_apply(TB, ldv(p.lpB));
            p.dist = vdot(vsub(wA[i], wB[i]), ldv(p.n));
        }
    }
#pragma unroll
    for (int i = 3; i >= 0; i--) {
        if (i < n0) {
            LCPoint& p = M.pt[i];
            int rm = 0;
            if (p.dist > thr) rm = 1;
            else {
                v3 proj = vsub(wA[i], vscale(ldv(p.n), p.dist));
                v3 d = vsub(wB[i], proj);
                if (vdot(d, d) > thr * thr) rm = 1;
            }
            if (rm) {
                int last = M.npts - 1;
                if (i != last) cppt(M.pt[i], M.pt[last]);
                M.npts--;
            }
        }
    }
}
/* ---------------- robot control helpers (robot.py) ---------------- */
DFI double np_sum12(const double* a) {
    double r = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    for (int i = 8; i < 12; i++) r += a[i];
    return r;
}
DFI double gripper_angle(double L) { return 0.715 - ug_asin((L - 0.010) / 0.1143); }
/* ik_solve's kinematics: the 6 arm bodies only (their axes / points and the EE link frame are all the IK
 * reads), compile-time body indices so everything stays in registers; the same operations as fk() and
 * link_frame() for those bodies */
constexpr int kBodyParentIK[NB] = UG_BODY_PARENT_INIT;
#define UG_IK_NB 6 /* arm bodies 0..5; the EE link (UG_EE_LINK) is fixed to body 5 (UG_LINK_BODY) */
#define UG_IK_EE_BODY 5
struct ArmKin { m3 R[UG_IK_NB]; v3 p[UG_IK_NB]; v3 a[UG_IK_NB]; };
DFI void fk_arm(const double (&q)[NB], ArmKin& k) {
#pragma unroll
    for (int b = 0; b < UG_IK_NB; b++) {
        const int pb = kBodyParentIK[b];
        m3 Rpb = mload(&UG_BODY_R[9 * b]);
        v3 Ppb = V(UG_BODY_P[3 * b], UG_BODY_P[3 * b + 1], UG_BODY_P[3 * b + 2]);
        v3 ax = V(UG_BODY_AXIS[3 * b], UG_BODY_AXIS[3 * b + 1], UG_BODY_AXIS[3 * b + 2]);
        m3 Rj = axis_angle(ax, q[b]);
        m3 Rp;
        v3 pp;
        if (pb < 0) { Rp = mident(); pp = V(0, 0, 0); }
        else { Rp = k.R[pb < 0 ? 0 : pb]; pp = k.p[pb < 0 ? 0 : pb]; }
        m3 Rtmp = mm(Rp, Rpb);
        k.R[b] = mm(Rtmp, Rj);
        k.p[b] = vadd(pp, mv(Rp, Ppb));
        k.a[b] = mv(Rtmp, ax);
    }
}
/* ldlt() / ldlt_solve() of a fixed size with compile-time indices (same operations, same order) */
template <int N>
DFI void ldlt_n(double (&A)[N * N]) {
#pragma unroll
    for (int j = 0; j < N; j++) {
        double d = A[j * N + j];
#pragma unroll
        for (int k2 = 0; k2 < j; k2++) d -= A[j * N + k2] * A[j * N + k2] * A[k2 * N + k2];
        A[j * N + j] = d;
#pragma unroll
        for (int i = j + 1; i < N; i++) {
            double s = A[i * N + j];
#pragma unroll
            for (int k2 = 0; k2 < j; k2++) s -= A[i * N + k2] * A[j * N + k2] * A[k2 * N + k2];
            A[i * N + j] = s / d;
        }
    }
}
template <int N>
DFI void ldlt_solve_n(const double (&A)[N * N], double (&x)[N]) {
#pragma unroll
    for (int i = 0; i < N; i++)
#pragma unroll
        for (int k2 = 0; k2 < i; k2++) x[i] -= A[i * N + k2] * x[k2];
#pragma unroll
    for (int i = 0; i < N; i++) x[i] = x[i] / A[i * N + i];
#pragma unroll
    for (int i = N - 1; i >= 0; i--)
#pragma unroll
        for (int k2 = i + 1; k2 < N; k2++) x[i] -= A[k2 * N + i] * x[k2];
}
DF void ik_solve(const double* q0, v3 tp, q4 to, double* qout) {
    double q[NB];
#pragma unroll
    for (int i = 0; i < NB; i++) q[i] = q0[i];
    double diff = 1e30;
    const m3 Rl = mload(&UG_LINK_COMR[9 * UG_EE_LINK]);
    const v3 Pl = V(UG_LINK_COMP[3 * UG_EE_LINK], UG_LINK_COMP[3 * UG_EE_LINK + 1], UG_LINK_COMP[3 * UG_EE_LINK + 2]);
    for (int it = 0; it < UG_IK_ITERS && diff > UG_IK_RESIDUAL; it++) {
        ArmKin k;
        fk_arm(q, k);
        const m3 Re = mm(k.R[UG_IK_EE_BODY], Rl); /* link_frame(k, UG_EE_LINK, 1, ...) */
        const v3 pe = vadd(k.p[UG_IK_EE_BODY], mv(k.R[UG_IK_EE_BODY], Pl));
        q4 oe = mquat(Re);
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
        double J[6][6];
#pragma unroll
        for (int d = 0; d < 6; d++) {
            v3 jl = vcross(k.a[d], vsub(pe, k.p[d]));
            J[0][d] = jl.x; J[1][d] = jl.y; J[2][d] = jl.z;
            J[3][d] = k.a[d].x; J[4][d] = k.a[d].y; J[5][d] = k.a[d].z;
        }
        double U[36], rhs[6];
#pragma unroll
        for (int i = 0; i < 6; i++) {
#pragma unroll
            for (int j = 0; j < 6; j++) {
                double sum = 0.0;
#pragma unroll
                for (int r = 0; r < 6; r++) sum += J[r][i] * J[r][j];
                U[i * 6 + j] = sum;
            }
            U[i * 6 + i] += UG_IK_DAMPING;
            double sr = 0.0;
#pragma unroll
            for (int r = 0; r < 6; r++) sr += J[r][i] * ds[r];
            rhs[i] = sr;
        }
        ldlt_n<6>(U);
        ldlt_solve_n<6>(U, rhs);
        double mx = 0.0;
#pragma unroll
        for (int i = 0; i < 6; i++) mx = ug_fabs(rhs[i]) > mx ? ug_fabs(rhs[i]) : mx;
        if (mx > UG_IK_MAXANGLE)
#pragma unroll
            for (int i = 0; i < 6; i++) rhs[i] *= UG_IK_MAXANGLE / mx;
#pragma unroll
        for (int i = 0; i < 6; i++) q[i] = rhs[i] + q[i];
    }
#pragma unroll
    for (int i = 0; i < NB; i++) qout[i] = q[i];
}

}  // namespace ugd

#endif
