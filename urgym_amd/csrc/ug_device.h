/* ug_device.h -- gfx950 device code of the URGym hot path (one env per lane).
 *
 * Each lane owns one environment for a whole env-step: it loads the env's
 * state from the structure-of-arrays buffer (UG layout, coalesced across the
 * wavefront), runs move_ee -> wait_until_stable -> reward (and an autoreset
 * when the episode ends) entirely on-chip, and stores the state once.
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
#include "model_data.h"
#include "scene_data.h"
#include "ug_detmath.h"
#include "ug_layout.h"

#define NB UG_NB
#define MAXOBJ UG_MAXOBJ
#define NV (NB + 6 * MAXOBJ)
#define MAXMAN UG_MAXMAN
#define MAXROWS 128
#define MAXCOL 24
#define MAXPAIR 96
#define MAXCAND 64

#define DF __device__ static
#define DFI __device__ static inline

namespace ugd {

/* ---------------- linear algebra (same evaluation order as the oracle) ---------------- */
struct v3 { double x, y, z; };
struct m3 { double m[9]; };
struct q4 { double x, y, z, w; };

DFI v3 V(double x, double y, double z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
DFI v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
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
    double c = ug_cos(q), s = ug_sin(q), t = 1.0 - c;
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

/* ---------------- scene (built on the host, read-only, wave-uniform) ---------------- */
struct Collider {
    int kind;
    double half[3];
    double margin;
    int v0, nv, f0, nf;
    m3 R; v3 P;
    m3 aR; v3 aP;
    v3 ac, ah;
    double disc;
    double friction, restitution;
    int owner, ent, link;
};
struct PairDef { int a, b; double thr, friction, restitution; };
struct Scene {
    int task;
    double gravity;
    int nobj;
    double omass[MAXOBJ];
    v3 oinertia[MAXOBJ];
    int ncol;
    Collider col[MAXCOL];
    int ocol[MAXOBJ];
    int npair;
    PairDef pair[MAXPAIR];
};

struct CPoint { v3 lpA, lpB, n; double dist, imp, imp1, imp2; };
struct Manifold { int pair, npts; CPoint pt[4]; };

struct Env {
    const Scene* sc;
    double q[NB], qd[NB];
    double mtarget[7];
    int mon[7];
    int oactive[MAXOBJ];
    v3 opos[MAXOBJ];
    q4 oquat[MAXOBJ];
    v3 ov[MAXOBJ], ow[MAXOBJ];
    int nman;
    Manifold man[MAXMAN];
    int goal_approached, goal_grasped, overflow;
};

/* SoA <-> lane-private state */
DF void env_load(Env& e, const double* S, int n, int i) {
#define LD(f) S[(size_t)(f) * n + i]
    for (int j = 0; j < NB; j++) e.q[j] = LD(UG_F_Q + j);
    for (int j = 0; j < NB; j++) e.qd[j] = LD(UG_F_QD + j);
    for (int j = 0; j < 7; j++) e.mtarget[j] = LD(UG_F_MTARGET + j);
    for (int j = 0; j < 7; j++) e.mon[j] = (int)LD(UG_F_MON + j);
    for (int o = 0; o < MAXOBJ; o++) e.oactive[o] = (int)LD(UG_F_OACTIVE + o);
    for (int o = 0; o < MAXOBJ; o++) {
        int b = UG_F_OBJ + UG_OBJ_DOUBLES * o;
        e.opos[o] = V(LD(b), LD(b + 1), LD(b + 2));
        e.oquat[o] = Q(LD(b + 3), LD(b + 4), LD(b + 5), LD(b + 6));
        e.ov[o] = V(LD(b + 7), LD(b + 8), LD(b + 9));
        e.ow[o] = V(LD(b + 10), LD(b + 11), LD(b + 12));
    }
    e.nman = (int)LD(UG_F_NMAN);
    for (int m = 0; m < e.nman; m++) {
        int b = UG_F_MAN + m * UG_MAN_DOUBLES;
        Manifold& M = e.man[m];
        M.pair = (int)LD(b);
        M.npts = (int)LD(b + 1);
        for (int p = 0; p < M.npts; p++) {
            int c = b + 2 + p * UG_PT_DOUBLES;
            CPoint& P = M.pt[p];
            P.lpA = V(LD(c), LD(c + 1), LD(c + 2));
            P.lpB = V(LD(c + 3), LD(c + 4), LD(c + 5));
            P.n = V(LD(c + 6), LD(c + 7), LD(c + 8));
            P.dist = LD(c + 9); P.imp = LD(c + 10); P.imp1 = LD(c + 11); P.imp2 = LD(c + 12);
        }
    }
    e.goal_approached = (int)LD(UG_F_TASK);
    e.goal_grasped = (int)LD(UG_F_TASK + 1);
    e.overflow = (int)LD(UG_F_TASK + 2);
#undef LD
}
DF void env_store(const Env& e, double* S, int n, int i) {
#define ST(f, x) S[(size_t)(f) * n + i] = (x)
    for (int j = 0; j < NB; j++) ST(UG_F_Q + j, e.q[j]);
    for (int j = 0; j < NB; j++) ST(UG_F_QD + j, e.qd[j]);
    for (int j = 0; j < 7; j++) ST(UG_F_MTARGET + j, e.mtarget[j]);
    for (int j = 0; j < 7; j++) ST(UG_F_MON + j, (double)e.mon[j]);
    for (int o = 0; o < MAXOBJ; o++) ST(UG_F_OACTIVE + o, (double)e.oactive[o]);
    for (int o = 0; o < MAXOBJ; o++) {
        int b = UG_F_OBJ + UG_OBJ_DOUBLES * o;
        ST(b, e.opos[o].x); ST(b + 1, e.opos[o].y); ST(b + 2, e.opos[o].z);
        ST(b + 3, e.oquat[o].x); ST(b + 4, e.oquat[o].y); ST(b + 5, e.oquat[o].z); ST(b + 6, e.oquat[o].w);
        ST(b + 7, e.ov[o].x); ST(b + 8, e.ov[o].y); ST(b + 9, e.ov[o].z);
        ST(b + 10, e.ow[o].x); ST(b + 11, e.ow[o].y); ST(b + 12, e.ow[o].z);
    }
    ST(UG_F_NMAN, (double)e.nman);
    for (int m = 0; m < MAXMAN; m++) {
        int b = UG_F_MAN + m * UG_MAN_DOUBLES;
        const Manifold& M = e.man[m];
        int live = m < e.nman;
        ST(b, live ? (double)M.pair : -1.0);
        ST(b + 1, live ? (double)M.npts : 0.0);
        for (int p = 0; p < 4; p++) {
            int c = b + 2 + p * UG_PT_DOUBLES;
            int lp = live && p < M.npts;
            const CPoint& P = M.pt[p];
            ST(c, lp ? P.lpA.x : 0.0); ST(c + 1, lp ? P.lpA.y : 0.0); ST(c + 2, lp ? P.lpA.z : 0.0);
            ST(c + 3, lp ? P.lpB.x : 0.0); ST(c + 4, lp ? P.lpB.y : 0.0); ST(c + 5, lp ? P.lpB.z : 0.0);
            ST(c + 6, lp ? P.n.x : 0.0); ST(c + 7, lp ? P.n.y : 0.0); ST(c + 8, lp ? P.n.z : 0.0);
            ST(c + 9, lp ? P.dist : 0.0); ST(c + 10, lp ? P.imp : 0.0);
            ST(c + 11, lp ? P.imp1 : 0.0); ST(c + 12, lp ? P.imp2 : 0.0);
        }
    }
    ST(UG_F_TASK, (double)e.goal_approached);
    ST(UG_F_TASK + 1, (double)e.goal_grasped);
    ST(UG_F_TASK + 2, (double)e.overflow);
    ST(UG_F_TASK + 3, 0.0);
#undef ST
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
DF void robot_dynamics(const double* qd, const Kin& k, double g, double* M, double* C) {
    double m[NB];
    v3 h[NB];
    m3 J[NB];
    double cm[NB];
    v3 ch[NB];
    m3 cJ[NB];
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
    for (int b = NB - 1; b >= 0; b--) {
        int p = UG_BODY_PARENT[b];
        if (p < 0) continue;
        cm[p] += cm[b];
        ch[p] = vadd(ch[p], ch[b]);
        for (int i = 0; i < 9; i++) cJ[p].m[i] += cJ[b].m[i];
    }
    SV S[NB];
    for (int b = 0; b < NB; b++) { S[b].w = k.a[b]; S[b].v = vcross(k.p[b], k.a[b]); }
    for (int i = 0; i < NB * NB; i++) M[i] = 0.0;
    for (int b = 0; b < NB; b++) {
        SV F = spatial_inertia_mul(cm[b], ch[b], cJ[b], S[b]);
        M[b * NB + b] = vdot(S[b].w, F.w) + vdot(S[b].v, F.v);
        int j = UG_BODY_PARENT[b];
        while (j >= 0) {
            double x = vdot(S[j].w, F.w) + vdot(S[j].v, F.v);
            M[j * NB + b] = x;
            M[b * NB + j] = x;
            j = UG_BODY_PARENT[j];
        }
    }
    SV Vb[NB], Ab[NB], f[NB];
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
DF XF owner_xf(const Env& e, const Kin& k, int owner) {
    XF T;
    if (owner >= 0) { T.R = k.R[owner]; T.p = k.p[owner]; }
    else if (owner <= -2 && owner > -100) { int o = -2 - owner; T.R = qmat(e.oquat[o]); T.p = e.opos[o]; }
    else { T.R = mident(); T.p = V(0, 0, 0); }
    return T;
}
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
struct CandList { int n; Cand c[MAXCAND]; };
DFI void cand_add(CandList& L, v3 n, v3 pB, double d) {
    if (L.n < MAXCAND) { L.c[L.n].n = n; L.c[L.n].pB = pB; L.c[L.n].d = d; L.n++; }
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

DF int intersect_rect_quad(const double h[2], double p[8], double ret[16]) {
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
    if (q != ret)
        for (int i = 0; i < nr * 2; i++) ret[i] = q[i];
    return nr;
}
DF void cull_points(int n, const double p[], int m, int i0, int iret[]) {
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
DFI double col_dot(const m3& A, int i, const m3& B, int j) {
    return A.m[i] * B.m[j] + A.m[3 + i] * B.m[3 + j] + A.m[6 + i] * B.m[6 + j];
}
DFI double col_dotv(const m3& A, int i, v3 v) { return A.m[i] * v.x + A.m[3 + i] * v.y + A.m[6 + i] * v.z; }
DFI double vget(v3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
DFI void vsetc(v3& v, int i, double x) { if (i == 0) v.x = x; else if (i == 1) v.y = x; else v.z = x; }

DF void nc_box_box(const XF& TA, const Collider& A, const XF& TB, const Collider& B, double thr, CandList& out) {
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
    double quad[8];
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

DF void reduce4(CandList& L) {
    if (L.n <= 4) return;
    Cand sel[4];
    uint64_t used = 0;
    int best = 0;
    for (int i = 1; i < L.n; i++)
        if (L.c[i].d < L.c[best].d) best = i;
    sel[0] = L.c[best];
    used |= 1ull << best;
    for (int s = 1; s < 4; s++) {
        int bi = -1;
        double bd = -1.0;
        for (int i = 0; i < L.n; i++) {
            if (used & (1ull << i)) continue;
            double md = 1e300;
            for (int t = 0; t < s; t++) {
                v3 dd = vsub(L.c[i].pB, sel[t].pB);
                double x = vdot(dd, dd);
                if (x < md) md = x;
            }
            if (md > bd) { bd = md; bi = i; }
        }
        sel[s] = L.c[bi];
        used |= 1ull << bi;
    }
    for (int s = 0; s < 4; s++) L.c[s] = sel[s];
    L.n = 4;
}
DF void nc_hull_box(const XF& TA, const Collider& A, const XF& TB, const Collider& B, double thr, CandList& out) {
    m3 RAB = mtm(TB.R, TA.R);
    v3 pAB = mtv(TB.R, vsub(TA.p, TB.p));
    v3 h = V(B.half[0], B.half[1], B.half[2]);
    double mA = A.margin;
    CandList L;
    L.n = 0;
    for (int i = 0; i < A.nv; i++) {
        const double* vv = &UG_HULL_V[3 * (A.v0 + i)];
        v3 x = vadd(mv(RAB, V(vv[0], vv[1], vv[2])), pAB);
        v3 d = V(ug_fabs(x.x) - h.x, ug_fabs(x.y) - h.y, ug_fabs(x.z) - h.z);
        double dist;
        v3 nl, pl;
        if (d.x < 0 && d.y < 0 && d.z < 0) {
            int kk = 0;
            double dm = d.x;
            if (d.y > dm) { dm = d.y; kk = 1; }
            if (d.z > dm) { dm = d.z; kk = 2; }
            dist = dm;
            double sg = vget(x, kk) < 0 ? -1.0 : 1.0;
            nl = V(0, 0, 0); vsetc(nl, kk, sg);
            pl = x; vsetc(pl, kk, sg * vget(h, kk));
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
        if (depth < thr) cand_add(L, mv(TB.R, nl), xf_apply(TB, pl), depth);
    }
    m3 RBA = mtm(TA.R, TB.R);
    v3 pBA = mtv(TA.R, vsub(TB.p, TA.p));
    for (int c = 0; c < 8; c++) {
        v3 cl = V((c & 1) ? h.x : -h.x, (c & 2) ? h.y : -h.y, (c & 4) ? h.z : -h.z);
        v3 y = vadd(mv(RBA, cl), pBA);
        double smax = -1e300;
        int fm = -1;
        for (int f = 0; f < A.nf; f++) {
            const double* F = &UG_HULL_F[4 * (A.f0 + f)];
            double sd = F[0] * y.x + F[1] * y.y + F[2] * y.z - F[3];
            if (sd > smax) { smax = sd; fm = f; }
            if (sd - mA >= thr) break;
        }
        double depth = smax - mA;
        if (depth < thr) {
            const double* F = &UG_HULL_F[4 * (A.f0 + fm)];
            v3 nw = mv(TA.R, V(F[0], F[1], F[2]));
            cand_add(L, vneg(nw), xf_apply(TB, cl), depth);
        }
    }
    reduce4(L);
    for (int i = 0; i < L.n; i++) cand_add(out, L.c[i].n, L.c[i].pB, L.c[i].d);
}
DF void nc_hull_sphere(const XF& TA, const Collider& A, const XF& TB, const Collider& B, double thr, CandList& out) {
    v3 y = mtv(TA.R, vsub(TB.p, TA.p));
    double r = B.half[0];
    double smax = -1e300;
    int fm = -1;
    for (int f = 0; f < A.nf; f++) {
        const double* F = &UG_HULL_F[4 * (A.f0 + f)];
        double sd = F[0] * y.x + F[1] * y.y + F[2] * y.z - F[3];
        if (sd > smax) { smax = sd; fm = f; }
    }
    double depth = smax - r - A.margin;
    if (depth >= thr) return;
    const double* F = &UG_HULL_F[4 * (A.f0 + fm)];
    v3 nw = vneg(mv(TA.R, V(F[0], F[1], F[2])));
    cand_add(out, nw, vadd(TB.p, vscale(nw, r)), depth);
}

DF int sort_cached(const Manifold& M, const CPoint& pt) {
    int maxi = -1;
    double maxpen = pt.dist;
    for (int i = 0; i < 4; i++)
        if (M.pt[i].dist < maxpen) { maxi = i; maxpen = M.pt[i].dist; }
    double res[4] = {0, 0, 0, 0};
    if (maxi != 0) { v3 a = vsub(pt.lpA, M.pt[1].lpA), b = vsub(M.pt[3].lpA, M.pt[2].lpA); v3 c = vcross(a, b); res[0] = vdot(c, c); }
    if (maxi != 1) { v3 a = vsub(pt.lpA, M.pt[0].lpA), b = vsub(M.pt[3].lpA, M.pt[2].lpA); v3 c = vcross(a, b); res[1] = vdot(c, c); }
    if (maxi != 2) { v3 a = vsub(pt.lpA, M.pt[0].lpA), b = vsub(M.pt[3].lpA, M.pt[1].lpA); v3 c = vcross(a, b); res[2] = vdot(c, c); }
    if (maxi != 3) { v3 a = vsub(pt.lpA, M.pt[0].lpA), b = vsub(M.pt[2].lpA, M.pt[1].lpA); v3 c = vcross(a, b); res[3] = vdot(c, c); }
    int bi = -1;
    double bv = -1e300;
    for (int i = 0; i < 4; i++)
        if (ug_fabs(res[i]) > bv) { bv = ug_fabs(res[i]); bi = i; }
    return bi;
}
DF void manifold_add(Manifold& M, const XF& TA, const XF& TB, const Cand& c, double thr) {
    if (c.d > thr) return;
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
        v3 d = vsub(M.pt[i].lpA, np.lpA);
        double x = vdot(d, d);
        if (x < shortest) { shortest = x; nearp = i; }
    }
    if (nearp >= 0) {
        np.imp = M.pt[nearp].imp; np.imp1 = M.pt[nearp].imp1; np.imp2 = M.pt[nearp].imp2;
        M.pt[nearp] = np;
        return;
    }
    int ins = M.npts;
    if (ins == 4) ins = sort_cached(M, np);
    else M.npts++;
    if (ins < 0) ins = 0;
    M.pt[ins] = np;
}
DF void manifold_refresh(Manifold& M, const XF& TA, const XF& TB, double thr) {
    for (int i = M.npts - 1; i >= 0; i--) {
        CPoint& p = M.pt[i];
        v3 pA = xf_apply(TA, p.lpA), pB = xf_apply(TB, p.lpB);
        p.dist = vdot(vsub(pA, pB), p.n);
    }
    for (int i = M.npts - 1; i >= 0; i--) {
        CPoint& p = M.pt[i];
        int rm = 0;
        if (p.dist > thr) rm = 1;
        else {
            v3 pA = xf_apply(TA, p.lpA), pB = xf_apply(TB, p.lpB);
            v3 proj = vsub(pA, vscale(p.n, p.dist));
            v3 d = vsub(pB, proj);
            if (vdot(d, d) > thr * thr) rm = 1;
        }
        if (rm) {
            int last = M.npts - 1;
            if (i != last) M.pt[i] = M.pt[last];
            M.npts--;
        }
    }
}
DFI int collider_active(const Env& e, const Collider& c) {
    if (c.owner <= -2 && c.owner > -100) return e.oactive[-2 - c.owner];
    return 1;
}
DF void collide(Env& e, const Kin& k) {
    const Scene* s = e.sc;
    XF O[MAXCOL];
    v3 lo[MAXCOL], hi[MAXCOL];
    for (int i = 0; i < s->ncol; i++) {
        const Collider& c = s->col[i];
        O[i] = owner_xf(e, k, c.owner);
        world_aabb(O[i], c, lo[i], hi[i]);
        lo[i] = vsub(lo[i], V(UG_AABB_PAD, UG_AABB_PAD, UG_AABB_PAD));
        hi[i] = vadd(hi[i], V(UG_AABB_PAD, UG_AABB_PAD, UG_AABB_PAD));
    }
    for (int p = 0; p < s->npair; p++) {
        const PairDef& P = s->pair[p];
        int a = P.a, b = P.b;
        int slot = -1;
        for (int m = 0; m < e.nman; m++)
            if (e.man[m].pair == p) { slot = m; break; }
        int ov = collider_active(e, s->col[a]) && collider_active(e, s->col[b]) &&
                 !(lo[a].x > hi[b].x || hi[a].x < lo[b].x || lo[a].y > hi[b].y || hi[a].y < lo[b].y ||
                   lo[a].z > hi[b].z || hi[a].z < lo[b].z);
        if (!ov) {
            if (slot >= 0) {
                int last = e.nman - 1;
                if (slot != last) e.man[slot] = e.man[last];
                e.nman--;
            }
            continue;
        }
        const Collider& A = s->col[a];
        const Collider& B = s->col[b];
        XF TA = shape_xf(O[a], A), TB = shape_xf(O[b], B);
        CandList L;
        L.n = 0;
        if (A.kind == UG_SHAPE_SPHERE && B.kind == UG_SHAPE_BOX) nc_sphere_box(TA, A, TB, B, P.thr, L);
        else if (A.kind == UG_SHAPE_SPHERE && B.kind == UG_SHAPE_SPHERE) nc_sphere_sphere(TA, A, TB, B, P.thr, L);
        else if (A.kind == UG_SHAPE_BOX && B.kind == UG_SHAPE_BOX) nc_box_box(TA, A, TB, B, P.thr, L);
        else if (A.kind == UG_SHAPE_HULL && B.kind == UG_SHAPE_BOX) nc_hull_box(TA, A, TB, B, P.thr, L);
        else if (A.kind == UG_SHAPE_HULL && B.kind == UG_SHAPE_SPHERE) nc_hull_sphere(TA, A, TB, B, P.thr, L);
        else if (A.kind == UG_SHAPE_BOX && B.kind == UG_SHAPE_SPHERE) {
            CandList L2;
            L2.n = 0;
            nc_sphere_box(TB, B, TA, A, P.thr, L2);
            for (int i = 0; i < L2.n; i++)
                cand_add(L, vneg(L2.c[i].n), vadd(L2.c[i].pB, vscale(L2.c[i].n, L2.c[i].d)), L2.c[i].d);
        }
        if (slot < 0) {
            if (L.n == 0) continue;
            if (e.nman >= MAXMAN) { e.overflow++; continue; }
            slot = e.nman++;
            e.man[slot].pair = p;
            e.man[slot].npts = 0;
        }
        Manifold& M = e.man[slot];
        for (int i = 0; i < L.n; i++) manifold_add(M, O[a], O[b], L.c[i], P.thr);
        if (M.npts) manifold_refresh(M, O[a], O[b], P.thr);
        if (M.npts == 0) {
            int last = e.nman - 1;
            if (slot != last) e.man[slot] = e.man[last];
            e.nman--;
        }
    }
}

/* ---------------- constraint rows + PGS ---------------- */
struct Row {
    int entA, entB;
    double JA[NB], MiJA[NB];
    double JB[NB], MiJB[NB];
    double invD, rhs, rhsPen, lo, hi, imp, impPen, fric;
    int man, pt, kind, nrow;
};
struct RowSet {
    int n, nnc, nn, nf;
    Row r[MAXROWS];
    int idx_nc[MAXROWS], idx_n[MAXROWS], idx_f[MAXROWS];
};
DFI int ent_dofs(int ent) { return ent == 0 ? NB : 6; }
DFI int ent_off(int ent) { return ent == 0 ? 0 : NB + 6 * (ent - 1); }
DFI double ent_dot(int ent, const double* J, const double* v) {
    int n = ent_dofs(ent), o = ent_off(ent);
    double s = 0.0;
    for (int i = 0; i < n; i++) s += J[i] * v[o + i];
    return s;
}
DFI double ent_dot_local(int ent, const double* a, const double* b) {
    int n = ent_dofs(ent);
    double s = 0.0;
    for (int i = 0; i < n; i++) s += a[i] * b[i];
    return s;
}
DFI void ent_axpy(int ent, const double* MiJ, double a, double* v) {
    int n = ent_dofs(ent), o = ent_off(ent);
    for (int i = 0; i < n; i++) v[o + i] += MiJ[i] * a;
}
DFI void row_clear(Row& r) {
    for (int i = 0; i < NB; i++) { r.JA[i] = 0.0; r.MiJA[i] = 0.0; r.JB[i] = 0.0; r.MiJB[i] = 0.0; }
    r.entA = r.entB = -1;
    r.invD = r.rhs = r.rhsPen = r.lo = r.hi = r.imp = r.impPen = r.fric = 0.0;
    r.man = r.pt = r.kind = r.nrow = 0;
}
DF void point_jac(const Env& e, const Kin& k, int ent, int body, v3 p, v3 d, double* J, double* MiJ, const double* LDL) {
    if (ent == 0) {
        for (int i = 0; i < NB; i++) {
            J[i] = moves(i, body) ? vdot(d, vcross(k.a[i], vsub(p, k.p[i]))) : 0.0;
            MiJ[i] = J[i];
        }
        ldlt_solve(LDL, NB, MiJ);
    } else {
        int o = ent - 1;
        v3 r = vsub(p, e.opos[o]);
        v3 rn = vcross(r, d);
        J[0] = d.x; J[1] = d.y; J[2] = d.z; J[3] = rn.x; J[4] = rn.y; J[5] = rn.z;
        double im = 1.0 / e.sc->omass[o];
        m3 R = qmat(e.oquat[o]);
        v3 ir = mtv(R, rn);
        ir = V(ir.x / e.sc->oinertia[o].x, ir.y / e.sc->oinertia[o].y, ir.z / e.sc->oinertia[o].z);
        ir = mv(R, ir);
        MiJ[0] = d.x * im; MiJ[1] = d.y * im; MiJ[2] = d.z * im; MiJ[3] = ir.x; MiJ[4] = ir.y; MiJ[5] = ir.z;
    }
}
DFI int ent_of_collider(const Collider& c, int& body) {
    body = -1;
    if (c.owner >= 0) { body = c.owner; return 0; }
    if (c.owner == -1) return -1;
    if (c.owner > -100) return -1 - c.owner;
    return -1;
}
DF void contact_row(const Env& e, const Kin& k, const double* LDL, const double* v0, Row& r, int entA, int bodyA,
                    int entB, int bodyB, v3 pA, v3 pB, v3 d) {
    r.entA = entA; r.entB = entB;
    double dA = 0.0, dB = 0.0;
    double relv = 0.0;
    if (entA >= 0) {
        point_jac(e, k, entA, bodyA, pA, d, r.JA, r.MiJA, LDL);
        dA = ent_dot_local(entA, r.JA, r.MiJA);
        relv += ent_dot(entA, r.JA, v0);
    }
    if (entB >= 0) {
        point_jac(e, k, entB, bodyB, pB, vneg(d), r.JB, r.MiJB, LDL);
        dB = ent_dot_local(entB, r.JB, r.MiJB);
        relv += ent_dot(entB, r.JB, v0);
    }
    double den = dA + dB;
    r.invD = den > 2.220446049250313e-16 ? 1.0 / den : 0.0;
    r.rhs = relv;
}
DF void build_rows(Env& e, const Kin& k, const double* LDL, const double* v0, RowSet& rs) {
    rs.n = rs.nnc = rs.nn = rs.nf = 0;
    const double dt = UG_DT;
    for (int d = 0; d < NB; d++) {
        for (int side = 0; side < 2; side++) {
            double pen = side == 0 ? e.q[d] - UG_DOF_LOWER[d] : UG_DOF_UPPER[d] - e.q[d];
            if (pen > 0) continue;
            if (rs.n >= MAXROWS) { e.overflow++; continue; }
            Row& r = rs.r[rs.n];
            row_clear(r);
            r.entA = 0; r.entB = -1;
            r.JA[d] = side == 0 ? 1.0 : -1.0;
            for (int i = 0; i < NB; i++) r.MiJA[i] = r.JA[i];
            ldlt_solve(LDL, NB, r.MiJA);
            double den = ent_dot_local(0, r.JA, r.MiJA);
            r.invD = den > 2.220446049250313e-16 ? 1.0 / den : 0.0;
            double relv = ent_dot(0, r.JA, v0);
            double erp = (pen > UG_SPLIT_PEN_THR) ? UG_ERP : UG_ERP2;
            double perr = -pen * erp / dt, verr = -relv;
            double pimp = perr * r.invD, vimp = verr * r.invD;
            r.rhs = (pen > UG_SPLIT_PEN_THR) ? pimp + vimp : vimp;
            r.lo = 0.0; r.hi = UG_LIMIT_MAXIMP;
            r.kind = 0;
            rs.idx_nc[rs.nnc++] = rs.n++;
        }
    }
    for (int m = 0; m < 7; m++) {
        if (!e.mon[m]) continue;
        int d = m < 6 ? m : UG_FINGER_DOF;
        double maxImp = UG_DOF_MAXFORCE[d] * dt;
        if (rs.n >= MAXROWS) { e.overflow++; continue; }
        Row& r = rs.r[rs.n];
        row_clear(r);
        r.entA = 0; r.entB = -1;
        r.JA[d] = 1.0;
        for (int i = 0; i < NB; i++) r.MiJA[i] = r.JA[i];
        ldlt_solve(LDL, NB, r.MiJA);
        double den = ent_dot_local(0, r.JA, r.MiJA);
        r.invD = den > 2.220446049250313e-16 ? 1.0 / den : 0.0;
        double qd = v0[d];
        double pst = 1.0 * (e.mtarget[m] - e.q[d]) / dt;
        double verr = 0.0 - qd;
        double des = UG_MOTOR_KP * pst + qd + UG_MOTOR_KD * verr;
        double clamp = UG_DOF_MAXVEL[d];
        if (des > clamp) des = clamp;
        if (des < -clamp) des = -clamp;
        double relv = ent_dot(0, r.JA, v0);
        r.rhs = 0.0 * r.invD + (des - relv) * r.invD;
        r.lo = -maxImp; r.hi = maxImp;
        r.kind = 0;
        rs.idx_nc[rs.nnc++] = rs.n++;
    }
    for (int g = 0; g < 5; g++) {
        if (rs.n >= MAXROWS) { e.overflow++; continue; }
        int pa = UG_FINGER_DOF, cb = UG_GEAR_CHILD[g];
        double ratio = UG_GEAR_RATIO[g];
        Row& r = rs.r[rs.n];
        row_clear(r);
        r.entA = 0; r.entB = 0;
        r.JA[pa] = 1.0;
        r.JB[cb] = ratio;
        for (int i = 0; i < NB; i++) { r.MiJA[i] = r.JA[i]; r.MiJB[i] = r.JB[i]; }
        ldlt_solve(LDL, NB, r.MiJA);
        ldlt_solve(LDL, NB, r.MiJB);
        double den = ent_dot_local(0, r.JA, r.MiJA) + ent_dot_local(0, r.JB, r.MiJB);
        r.invD = den > 2.220446049250313e-16 ? 1.0 / den : 0.0;
        double relv = ent_dot(0, r.JA, v0) + ent_dot(0, r.JB, v0);
        double diff = e.q[cb] * ratio + e.q[pa];
        double pen = -UG_GEAR_ERP * (0.0 - diff);
        double perr = -pen * UG_ERP / dt, verr = 0.0 - relv;
        r.rhs = perr * r.invD + verr * r.invD;
        double maxImp = UG_GEAR_MAXF * dt;
        r.lo = -maxImp; r.hi = maxImp;
        r.kind = 0;
        rs.idx_nc[rs.nnc++] = rs.n++;
    }
    const Scene* s = e.sc;
    for (int m = 0; m < e.nman; m++) {
        const Manifold& M = e.man[m];
        const PairDef& P = s->pair[M.pair];
        int bodyA, bodyB;
        int entA = ent_of_collider(s->col[P.a], bodyA);
        int entB = ent_of_collider(s->col[P.b], bodyB);
        if (entA < 0 && entB < 0) continue;
        XF OA = owner_xf(e, k, s->col[P.a].owner), OB = owner_xf(e, k, s->col[P.b].owner);
        for (int j = 0; j < M.npts; j++) {
            if (rs.n + 3 > MAXROWS) { e.overflow++; continue; }
            const CPoint& cp = M.pt[j];
            v3 pA = xf_apply(OA, cp.lpA), pB = xf_apply(OB, cp.lpB);
            v3 n = cp.n;
            int ni = rs.n;
            Row& r = rs.r[ni];
            row_clear(r);
            contact_row(e, k, LDL, v0, r, entA, bodyA, entB, bodyB, pA, pB, n);
            if (r.invD == 0.0) continue;
            double relv = r.rhs;
            double pen = cp.dist + UG_LINEAR_SLOP;
            double rest = 0.0;
            if (!(ug_fabs(relv) < UG_REST_VEL_THR)) rest = P.restitution * -relv;
            if (rest <= 0.0) rest = 0.0;
            double verr = rest - relv, perr;
            double erp = (pen > UG_SPLIT_PEN_THR) ? UG_ERP : UG_ERP2;
            if (pen > 0) { perr = 0.0; verr -= pen / UG_DT; }
            else perr = -pen * erp / UG_DT;
            double pimp = perr * r.invD, vimp = verr * r.invD;
            if (pen > UG_SPLIT_PEN_THR) { r.rhs = pimp + vimp; r.rhsPen = 0.0; }
            else { r.rhs = vimp; r.rhsPen = pimp; }
            r.lo = 0.0; r.hi = 1e10;
            r.imp = cp.imp * UG_WARMSTART;
            r.kind = 1; r.man = m; r.pt = j;
            rs.idx_n[rs.nn++] = rs.n++;
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
                Row& f = rs.r[rs.n];
                row_clear(f);
                contact_row(e, k, LDL, v0, f, entA, bodyA, entB, bodyB, pA, pB, fdir == 0 ? t1 : t2);
                double frel = f.rhs;
                f.rhs = 0.0 * f.invD + (0.0 - frel) * f.invD;
                f.fric = P.friction;
                f.lo = 0.0; f.hi = 0.0;
                f.imp = 0.0;
                f.kind = 2 + fdir; f.man = m; f.pt = j; f.nrow = ni;
                rs.idx_f[rs.nf++] = rs.n++;
            }
        }
    }
}
DF double solve_row(Row& r, double* dv, int pen) {
    double imp = pen ? r.impPen : r.imp;
    double di = (pen ? r.rhsPen : r.rhs) - imp * 0.0;
    if (r.entA >= 0) di -= ent_dot(r.entA, r.JA, dv) * r.invD;
    if (r.entB >= 0) di -= ent_dot(r.entB, r.JB, dv) * r.invD;
    double sum = imp + di;
    if (sum < r.lo) { di = r.lo - imp; imp = r.lo; }
    else if (sum > r.hi) { di = r.hi - imp; imp = r.hi; }
    else imp = sum;
    if (pen) r.impPen = imp; else r.imp = imp;
    if (r.entA >= 0) ent_axpy(r.entA, r.MiJA, di, dv);
    if (r.entB >= 0) ent_axpy(r.entB, r.MiJB, di, dv);
    return di * (1.0 / r.invD);
}
DF void pgs(RowSet& rs, double* dv) {
    for (int i = 0; i < rs.nn; i++) {
        Row& r = rs.r[rs.idx_n[i]];
        if (r.imp != 0.0) {
            if (r.entA >= 0) ent_axpy(r.entA, r.MiJA, r.imp, dv);
            if (r.entB >= 0) ent_axpy(r.entB, r.MiJB, r.imp, dv);
        }
    }
    for (int it = 0; it < UG_PGS_ITERS; it++) {
        double res = 0.0;
        for (int j = 0; j < rs.nnc; j++) {
            int idx = (it & 1) ? j : rs.nnc - 1 - j;
            double x = solve_row(rs.r[rs.idx_nc[idx]], dv, 0);
            x = x * x;
            res = res > x ? res : x;
        }
        for (int j = 0; j < rs.nn; j++) {
            double x = solve_row(rs.r[rs.idx_n[j]], dv, 0);
            x = x * x;
            res = res > x ? res : x;
        }
        for (int j = 0; j < rs.nf; j++) {
            Row& f = rs.r[rs.idx_f[j]];
            double tot = rs.r[f.nrow].imp;
            if (tot > 0.0) {
                f.lo = -(f.fric * tot);
                f.hi = f.fric * tot;
                double x = solve_row(f, dv, 0);
                x = x * x;
                res = res > x ? res : x;
            }
        }
        if (res <= UG_RESIDUAL_THR || it >= UG_PGS_ITERS - 1) break;
    }
}
DF int pgs_split(RowSet& rs, double* dvs) {
    int any = 0;
    for (int j = 0; j < rs.nn; j++)
        if (rs.r[rs.idx_n[j]].rhsPen != 0.0) any = 1;
    if (!any) return 0;
    for (int it = 0; it < UG_PGS_ITERS; it++) {
        double res = 0.0;
        for (int j = 0; j < rs.nn; j++) {
            double x = solve_row(rs.r[rs.idx_n[j]], dvs, 1);
            x = x * x;
            res = res > x ? res : x;
        }
        if (res <= UG_RESIDUAL_THR || it >= UG_PGS_ITERS - 1) break;
    }
    return 1;
}

/* ---------------- one p.stepSimulation() ---------------- */
DF void substep(Env& e, RowSet& rs) {
    const double dt = UG_DT;
    const Scene* s = e.sc;
    Kin k;
    fk(e.q, k);
    collide(e, k);
    double M[NB * NB], C[NB];
    robot_dynamics(e.qd, k, s->gravity, M, C);
    ldlt(M, NB);
    double qdd[NB];
    for (int i = 0; i < NB; i++) qdd[i] = -C[i];
    ldlt_solve(M, NB, qdd);
    double v0[NV];
    for (int i = 0; i < NV; i++) v0[i] = 0.0;
    for (int i = 0; i < NB; i++) { e.qd[i] = e.qd[i] + qdd[i] * dt; v0[i] = e.qd[i]; }
    for (int o = 0; o < s->nobj; o++) {
        if (!e.oactive[o]) continue;
        v3 v = e.ov[o];
        double vn = vlen(v);
        v3 a = vsub(V(0, 0, s->gravity), vscale(v, UG_LIN_DAMP + UG_LIN_DAMP * vn));
        e.ov[o] = vadd(v, vscale(a, dt));
        m3 R = qmat(e.oquat[o]);
        v3 wl = mtv(R, e.ow[o]);
        v3 I = s->oinertia[o];
        v3 Iw = V(I.x * wl.x, I.y * wl.y, I.z * wl.z);
        double wn = vlen(wl);
        v3 z = vadd(vscale(Iw, UG_ANG_DAMP + UG_ANG_DAMP * wn), vcross(wl, Iw));
        v3 al = V(-z.x / I.x, -z.y / I.y, -z.z / I.z);
        e.ow[o] = vadd(e.ow[o], vscale(mv(R, al), dt));
        int off = NB + 6 * o;
        v0[off] = e.ov[o].x; v0[off + 1] = e.ov[o].y; v0[off + 2] = e.ov[o].z;
        v0[off + 3] = e.ow[o].x; v0[off + 4] = e.ow[o].y; v0[off + 5] = e.ow[o].z;
    }
    build_rows(e, k, M, v0, rs);
    double dv[NV], dvs[NV];
    for (int i = 0; i < NV; i++) { dv[i] = 0.0; dvs[i] = 0.0; }
    pgs(rs, dv);
    int split = pgs_split(rs, dvs);
    for (int i = 0; i < rs.nn; i++) {
        const Row& r = rs.r[rs.idx_n[i]];
        e.man[r.man].pt[r.pt].imp = r.imp;
    }
    for (int i = 0; i < rs.nf; i++) {
        const Row& r = rs.r[rs.idx_f[i]];
        if (r.kind == 2) e.man[r.man].pt[r.pt].imp1 = r.imp;
        else e.man[r.man].pt[r.pt].imp2 = r.imp;
    }
    for (int i = 0; i < NB; i++) {
        e.qd[i] = e.qd[i] + dv[i];
        double vi = split ? e.qd[i] + dvs[i] : e.qd[i];
        e.q[i] = e.q[i] + vi * dt;
    }
    for (int o = 0; o < s->nobj; o++) {
        if (!e.oactive[o]) continue;
        int off = NB + 6 * o;
        e.ov[o] = vadd(e.ov[o], V(dv[off], dv[off + 1], dv[off + 2]));
        e.ow[o] = vadd(e.ow[o], V(dv[off + 3], dv[off + 4], dv[off + 5]));
        v3 vl = e.ov[o], wa = e.ow[o];
        if (split) {
            vl = vadd(vl, V(dvs[off], dvs[off + 1], dvs[off + 2]));
            wa = vadd(wa, V(dvs[off + 3], dvs[off + 4], dvs[off + 5]));
        }
        e.opos[o] = vadd(e.opos[o], vscale(vl, dt));
        double ang = vlen(wa);
        if (ang * dt > UG_ANGULAR_MOTION_THR) ang = UG_ANGULAR_MOTION_THR / dt;
        v3 ax;
        if (ang < 0.001) ax = vscale(wa, 0.5 * dt - (dt * dt * dt) * 0.020833333333 * ang * ang);
        else ax = vscale(wa, ug_sin(0.5 * ang * dt) / ang);
        q4 dq = Q(ax.x, ax.y, ax.z, ug_cos(0.5 * ang * dt));
        e.oquat[o] = qnormalize(qmul(dq, e.oquat[o]));
    }
}

/* ---------------- robot control layer (robot.py) ---------------- */
DFI double np_sum12(const double* a) {
    double r = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    for (int i = 8; i < 12; i++) r += a[i];
    return r;
}
DF int wait_until_stable(Env& e, RowSet& rs) {
    double pos[NB];
    for (int j = 0; j < NB; j++) pos[j] = e.q[j];
    for (int i = 0; i < UG_STABLE_STEPS; i++) {
        substep(e, rs);
        double a[NB];
        for (int j = 0; j < NB; j++) a[j] = ug_fabs(pos[j] - e.q[j]);
        if (np_sum12(a) < UG_STABLE_EPS) return i + 1;
        for (int j = 0; j < NB; j++) pos[j] = e.q[j];
    }
    return UG_STABLE_STEPS;
}
DFI double gripper_angle(double L) { return 0.715 - ug_asin((L - 0.010) / 0.1143); }
DFI void open_gripper(Env& e, double pct) {
    double L = UG_GRIP_MIN + (UG_GRIP_MAX - UG_GRIP_MIN) * (pct / 100.0);
    e.mtarget[6] = gripper_angle(L);
    e.mon[6] = 1;
}
DFI void close_gripper(Env& e, double pct) {
    double L = UG_GRIP_MAX - (UG_GRIP_MAX - UG_GRIP_MIN) * (pct / 100.0);
    e.mtarget[6] = gripper_angle(L);
    e.mon[6] = 1;
}
DF void ik_solve(const double* q0, v3 tp, q4 to, double* qout) {
    double q[NB];
    for (int i = 0; i < NB; i++) q[i] = q0[i];
    double diff = 1e30;
    for (int it = 0; it < UG_IK_ITERS && diff > UG_IK_RESIDUAL; it++) {
        Kin k;
        fk(q, k);
        m3 Re;
        v3 pe;
        link_frame(k, UG_EE_LINK, 1, Re, pe);
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
        for (int d = 0; d < 6; d++) {
            v3 jl = vcross(k.a[d], vsub(pe, k.p[d]));
            J[0][d] = jl.x; J[1][d] = jl.y; J[2][d] = jl.z;
            J[3][d] = k.a[d].x; J[4][d] = k.a[d].y; J[5][d] = k.a[d].z;
        }
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
    for (int i = 0; i < NB; i++) qout[i] = q[i];
}
DF void move_ee_end(Env& e, v3 pos, q4 orn) {
    double qt[NB];
    ik_solve(e.q, pos, orn, qt);
    for (int i = 0; i < 6; i++) { e.mtarget[i] = qt[i]; e.mon[i] = 1; }
}
DF void link_state(const Env& e, int l, v3& p, q4& o) {
    Kin k;
    fk(e.q, k);
    m3 R;
    link_frame(k, l, 1, R, p);
    o = mquat(R);
}
DF v3 gripper_center(const Env& e) {
    Kin k;
    fk(e.q, k);
    v3 lo = V(1e300, 1e300, 1e300), hi = V(-1e300, -1e300, -1e300);
    for (int i = 0; i < 2; i++) {
        int l = i == 0 ? 11 : 16;
        m3 R;
        v3 p;
        link_frame(k, l, 1, R, p);
        v3 c = vadd(mv(R, V(UG_LINK_AABB_C[3 * l], UG_LINK_AABB_C[3 * l + 1], UG_LINK_AABB_C[3 * l + 2])), p);
        v3 h = V(UG_LINK_AABB_H[3 * l], UG_LINK_AABB_H[3 * l + 1], UG_LINK_AABB_H[3 * l + 2]);
        const double* r = R.m;
        v3 ext = V(ug_fabs(r[0]) * h.x + ug_fabs(r[1]) * h.y + ug_fabs(r[2]) * h.z,
                   ug_fabs(r[3]) * h.x + ug_fabs(r[4]) * h.y + ug_fabs(r[5]) * h.z,
                   ug_fabs(r[6]) * h.x + ug_fabs(r[7]) * h.y + ug_fabs(r[8]) * h.z);
        v3 mn = vsub(c, ext), mx = vadd(c, ext);
        lo = V(ug_min(lo.x, mn.x), ug_min(lo.y, mn.y), ug_min(lo.z, mn.z));
        hi = V(ug_max(hi.x, mx.x), ug_max(hi.y, mx.y), ug_max(hi.z, mx.z));
    }
    return V((hi.x + lo.x) / 2.0, (hi.y + lo.y) / 2.0, (hi.z + lo.z) / 2.0);
}
DF void remove_object(Env& e, int o) {
    e.oactive[o] = 0;
    int ci = e.sc->ocol[o];
    for (int m = e.nman - 1; m >= 0; m--) {
        const PairDef& P = e.sc->pair[e.man[m].pair];
        if (P.a == ci || P.b == ci) {
            int last = e.nman - 1;
            if (m != last) e.man[m] = e.man[last];
            e.nman--;
        }
    }
}
DFI void place_object(Env& e, int o, v3 pos, q4 orn) {
    e.oactive[o] = 1;
    e.opos[o] = pos;
    e.oquat[o] = orn;
    e.ov[o] = V(0, 0, 0);
    e.ow[o] = V(0, 0, 0);
}
DF int robot_reset(Env& e, RowSet& rs) {
    for (int i = 0; i < 6; i++) { e.q[i] = UG_ARM_REST[i]; e.qd[i] = 0.0; }
    for (int i = 0; i < 10; i++) substep(e, rs);
    open_gripper(e, 100.0);
    return 10;
}

/* ---------------- tasks ---------------- */
/* draws: source of random.random() values for resets: device MT19937 or caller-supplied */
struct Draws {
    const Rng* rng;
    const double* given;  /* n x ndraw or null */
    int k;
    __device__ double next() { return given ? given[k++] : mt_random(*rng); }
};
DFI double uniform(Draws& d, double a, double b) { return a + (b - a) * d.next(); }

DF void bb_obs(const Env& e, double* obs) {
    v3 eu = euler_from_quat(e.oquat[0]);
    obs[0] = eu.x; obs[1] = eu.y; obs[2] = eu.z;
    obs[3] = e.opos[0].x - e.opos[1].x;
    obs[4] = e.opos[0].y - e.opos[1].y;
    obs[5] = e.opos[0].z - e.opos[1].z;
}
/* create_ball (env_ball_balance_v0.py:186-205) */
DF v3 bb_ball_position(Draws& dr, v3 paddle) {
    v3 bp = V(paddle.x, paddle.y, paddle.z + 0.2 + UG_BB_BALL_R);
    bp.x += uniform(dr, -0.03, 0.03);
    bp.y += uniform(dr, -0.08, 0.02);
    return bp;
}
DF int bb_reset(Env& e, RowSet& rs, Draws& dr, double* obs) {
    int n = robot_reset(e, rs);
    remove_object(e, 0);
    remove_object(e, 1);
    move_ee_end(e, V(0.0, -0.60, 0.60), Q(0.50, -0.50, -0.50, 0.50));
    open_gripper(e, 20.0);
    n += wait_until_stable(e, rs);
    v3 pe;
    q4 oe;
    link_state(e, UG_EE_LINK, pe, oe);
    v3 gc = gripper_center(e);
    v3 pose = V(pe.x, pe.y - 0.2, gc.z);
    place_object(e, 0, pose, Q(0, 0, 0, 1));
    place_object(e, 1, bb_ball_position(dr, pose), e.oquat[0]);
    close_gripper(e, 100.0);
    n += wait_until_stable(e, rs);
    bb_obs(e, obs);
    return n;
}
DF int bb_step(Env& e, RowSet& rs, const float* a, double* obs, double* rew, int* term, int* succ) {
    v3 pe;
    q4 oe;
    link_state(e, UG_EE_LINK, pe, oe);
    v3 eu = euler_from_quat(oe);
    eu.x += (double)a[0]; eu.y += (double)a[1]; eu.z += (double)a[2];
    q4 qn = quat_from_euler(eu);
    move_ee_end(e, pe, qn);
    int n = wait_until_stable(e, rs);
    *rew = 1.0;
    *term = e.opos[1].z < e.opos[0].z;
    *succ = 0;
    bb_obs(e, obs);
    return n;
}
DF int task_reset(Env& e, RowSet& rs, Draws& dr, double* obs) {
    e.goal_approached = e.goal_grasped = 0;
    if (e.sc->task == UG_TASK_BALLBALANCE) return bb_reset(e, rs, dr, obs);
    return 0;
}
DF int task_step(Env& e, RowSet& rs, const float* a, double* obs, double* rew, int* term, int* succ) {
    if (e.sc->task == UG_TASK_BALLBALANCE) return bb_step(e, rs, a, obs, rew, term, succ);
    return 0;
}

}  // namespace ugd

#endif
