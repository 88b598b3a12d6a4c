// ug_capi.hip -- kernels + C-ABI (include/urgym.h) of the MI355X URGym hot path.
//
// One launch per batched env-step: k_step gives every environment one
// wavefront (block of 64 lanes) and runs the reference's whole step() -- IK,
// joint motors, wait_until_stable's <=480 physics substeps, reward /
// termination, and (gymnasium same-step autoreset) the reset of an env whose
// episode just ended -- without leaving the kernel (ug_team.h).  State is
// array-of-structs in HBM (ug_layout.h), loaded into LDS once and stored once
// per launch.  There is no CPU fallback: if this library is missing, nothing runs.
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/urgym.h"
#include "ug_team.h"
#include "ug_render.h"

using namespace ugd;

#define WAVE 64

// ---------------------------------------------------------------------------
// scene construction (device, one thread): statics, objects, collision pairs
// ---------------------------------------------------------------------------
__device__ static void box_collider(Collider* c, double hx, double hy, double hz, double margin, double friction) {
    c->kind = UG_SHAPE_BOX;
    c->half[0] = hx; c->half[1] = hy; c->half[2] = hz;
    c->margin = margin;
    c->v0 = c->nv = c->f0 = c->nf = c->c0 = 0;
    c->R = mident(); c->P = V(0, 0, 0);
    c->aR = mident(); c->aP = V(0, 0, 0);
    c->ac = V(0, 0, 0); c->ah = V(hx, hy, hz);
    c->disc = ug_sqrt(hx * hx + hy * hy + hz * hz);
    c->friction = friction;
    c->restitution = 0.0;
    c->rolling = 0.0;
    c->owner = -100; c->ent = 0;
    c->link = -1;
    c->gjkbox = 0;
    c->compound = 0;
}
__device__ static double safe_margin(double hx, double hy, double hz) {
    double m = hx < hy ? hx : hy;
    m = m < hz ? m : hz;
    m = 0.1 * m;
    return m < 0.04 ? m : 0.04;
}
/* the support-cell table of the hull with vertex range [v0, v0 + nv): a full hull's (tools/build_supcells.py), or none */
__device__ static void supcell_table(int v0, int nv, int* scb, int* sck) {
    *scb = -1;
    *sck = 0;
    for (int k = 0; k < UG_NSHAPE; k++)
        if (UG_SHAPE_KIND[k] == 1 && UG_SHAPE_FNV[k] > 0 && UG_SHAPE_FV0[k] == v0 && UG_SHAPE_FNV[k] == nv) {
            *scb = UG_SHAPE_SCB[k];
            *sck = UG_SHAPE_SCK[k];
        }
}
/* Bullet's shape parameters for GJK (oracle gjk_params) */
__device__ static void gjk_params(Collider* c) {
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
    /* a full hull's support-cell table (supcell_data.h), found by its vertex range */
    c->scb = -1;
    c->sck = 0;
    if (c->kind == UG_SHAPE_HULL) supcell_table(c->v0, c->nv, &c->scb, &c->sck);
    /* the certificate's rotation bound (team_collide): every core support point lies within gradius of the origin */
    double r2 = 0.0;
    if (c->kind == UG_SHAPE_HULL) {
        for (int i = 0; i < c->nv; i++) {
            const double* v = &UG_HULL_V[3 * (c->v0 + i)];
            const double x = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
            r2 = x > r2 ? x : r2;
        }
    } else if (c->kind == UG_SHAPE_BOX || c->kind == UG_SHAPE_CYL) {
        r2 = c->gimp.x * c->gimp.x + c->gimp.y * c->gimp.y + c->gimp.z * c->gimp.z;
    }
    c->gradius = ug_sqrt(r2) * (1.0 + 1e-12) + 1e-15;
}
__device__ static void add_pair(Scene* s, int a, int b) {
    PairDef* p = &s->pair[s->npair++];
    p->a = a; p->b = b;
    double d = s->col[a].disc < s->col[b].disc ? s->col[a].disc : s->col[b].disc;
    p->thr = d * UG_CONTACT_BREAK;
    double f = s->col[a].friction * s->col[b].friction;
    if (f < -UG_MAX_FRICTION) f = -UG_MAX_FRICTION;
    if (f > UG_MAX_FRICTION) f = UG_MAX_FRICTION;
    p->friction = f;
    p->restitution = s->col[a].restitution * s->col[b].restitution;
    double r = s->col[a].rolling * s->col[b].friction + s->col[a].friction * s->col[b].rolling;
    if (r < -UG_MAX_FRICTION) r = -UG_MAX_FRICTION;
    if (r > UG_MAX_FRICTION) r = UG_MAX_FRICTION;
    p->rolling = r;
}
__global__ void k_build_scene(Scene* s, int variant, int flags) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const int task = UG_BASE_TASK(variant);
    s->task = task;
    s->variant = variant;
    s->full = UG_GEOM_IS_FULL(flags);
    s->gjk = UG_CONTACT_IS_GJK(flags);
    s->gravity = task == UG_TASK_CUBESGRASP ? -10.0 : -9.8;
    s->nobj = 0;
    s->ncol = 0;
    s->npair = 0;
    s->sparse = 0;
    s->button_mode = UG_BX_TOUCH_ANY;
    s->njoint = 0;
    for (int o = 0; o < MAXOBJ; o++) { s->oncol[o] = 0; s->ojoint[o].kind = UGJ_FREE; }
    if (task == UG_TASK_BOX) s->gravity = -10.0; /* env_box_v0.py:60 */
    for (int l = 1; l < UG_NL; l++) {
        Collider* c = &s->col[s->ncol++];
        int si = -1;
        for (int k = 0; k < UG_NSHAPE; k++)
            if (UG_SHAPE_LINK[k] == l) si = k;
        c->kind = UG_SHAPE_KIND[si] == 0 ? UG_SHAPE_BOX : UG_SHAPE_HULL;
        c->half[0] = UG_SHAPE_HALF[3 * si]; c->half[1] = UG_SHAPE_HALF[3 * si + 1]; c->half[2] = UG_SHAPE_HALF[3 * si + 2];
        c->margin = UG_URDF_MARGIN;
        c->v0 = UG_SHAPE_V0[si]; c->nv = UG_SHAPE_NV[si]; c->f0 = UG_SHAPE_F0[si]; c->nf = UG_SHAPE_NF[si];
        c->c0 = 0;
        if (s->full) { /* PyBullet's hull of all mesh vertices instead of the collision LOD (oracle build_scene) */
            c->v0 = UG_SHAPE_FV0[si]; c->nv = UG_SHAPE_FNV[si]; c->f0 = UG_SHAPE_FF0[si]; c->nf = UG_SHAPE_FNF[si];
            c->c0 = UG_SHAPE_FC0[si];
        }
        c->R = mload(&UG_SHAPE_R[9 * si]);
        c->P = V(UG_SHAPE_P[3 * si], UG_SHAPE_P[3 * si + 1], UG_SHAPE_P[3 * si + 2]);
        c->aR = mload(&UG_LINK_COMR[9 * l]);
        c->aP = V(UG_LINK_COMP[3 * l], UG_LINK_COMP[3 * l + 1], UG_LINK_COMP[3 * l + 2]);
        c->ac = V(UG_LINK_AABB_C[3 * l], UG_LINK_AABB_C[3 * l + 1], UG_LINK_AABB_C[3 * l + 2]);
        c->ah = V(UG_LINK_AABB_H[3 * l], UG_LINK_AABB_H[3 * l + 1], UG_LINK_AABB_H[3 * l + 2]);
        c->disc = UG_LINK_DISC[l];
        c->friction = UG_DEFAULT_FRICTION;
        c->restitution = 0.0;
        c->rolling = 0.0;
        c->owner = UG_LINK_BODY[l];
        c->ent = 0;
        c->link = l;
        c->gjkbox = 0;
        /* a link whose collision frame is not its inertial frame collides through a btCompoundShape (oracle) */
        bool same = c->P.x == c->aP.x && c->P.y == c->aP.y && c->P.z == c->aP.z;
        for (int i = 0; i < 9; i++) same = same && c->R.m[i] == c->aR.m[i];
        c->compound = !same;
    }
    int nrobot = s->ncol;
    int statics[8], nstat = 0;
    if (task == UG_TASK_BALLBALANCE) {
        /* paddle, ball (env_ball_balance_v0.py:175-205); TwoBallsBalance: two balls of radius 0.003
         * (env_two_balls_balance_v0.py:187, 212-235) */
        const int two = variant == UG_TASK_TWOBALLS;
        s->nobj = two ? 3 : 2;
        double hx = UG_BB_PADDLE_HX, hy = UG_BB_PADDLE_HY, hz = UG_BB_PADDLE_HZ, m = UG_BB_PADDLE_MASS;
        s->omass[0] = m;
        s->oinertia[0] = V(m / 12.0 * (4.0 * hy * hy + 4.0 * hz * hz), m / 12.0 * (4.0 * hx * hx + 4.0 * hz * hz),
                           m / 12.0 * (4.0 * hx * hx + 4.0 * hy * hy));
        Collider* c = &s->col[s->ncol];
        box_collider(c, hx, hy, hz, safe_margin(hx, hy, hz), UG_DEFAULT_FRICTION);
        c->owner = -2; c->ent = 1;
        s->ocol[0] = s->ncol++;
        double r = two ? UG_TB_BALL_R : UG_BB_BALL_R, mb = UG_BB_BALL_MASS;
        for (int o = 1; o < s->nobj; o++) {
            s->omass[o] = mb;
            double ib = 0.4 * mb * r * r;
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
        s->nobj = task == UG_TASK_CUBESPUSH ? 2 : 1;
        for (int o = 0; o < s->nobj; o++) {
            double h = UG_CUBE_HALF, m = UG_CUBE_MASS;
            s->omass[o] = m;
            double ii = m / 12.0 * (4.0 * h * h + 4.0 * h * h);
            s->oinertia[o] = V(ii, ii, ii);
            Collider* c = &s->col[s->ncol];
            box_collider(c, h, h, h, UG_URDF_MARGIN, UG_CUBE_FRICTION);
            c->owner = -2 - o; c->ent = 1 + o;
            s->ocol[o] = s->ncol++;
        }
    }
    if (task == UG_TASK_CUBESGRASP) {
        Collider* c = &s->col[s->ncol];
        box_collider(c, UG_PLANE_HALF_XY, UG_PLANE_HALF_XY, UG_PLANE_HALF_Z, UG_URDF_MARGIN, UG_PLANE_FRICTION);
        c->P = V(0.0, 0.0, -UG_PLANE_HALF_Z); c->aP = c->P;
        c->disc = ug_sqrt(15.0 * 15.0 * 2.0 + 25.0) + 5.0;
        c->owner = -100; c->ent = 11;
        c->compound = 1;
        statics[nstat++] = s->ncol++;
    }
    if (task == UG_TASK_GOLF) {
        s->nobj = 2;
        double m = UG_GF_PART_MASS, zc = UG_GF_ZC;
        double bx = UG_GF_BASE_HX, bz = UG_GF_BASE_HZ, fx = UG_GF_FOOT_HX, fy = UG_GF_FOOT_HY;
        double r = UG_CYL_R, hh = UG_CYL_HH;
        v3 Ib = V(m / 12.0 * (4.0 * bx * bx + 4.0 * bz * bz), m / 12.0 * (4.0 * bx * bx + 4.0 * bz * bz),
                  m / 12.0 * (4.0 * bx * bx + 4.0 * bx * bx));
        v3 If = V(m / 12.0 * (4.0 * fy * fy + 4.0 * fy * fy), m / 12.0 * (4.0 * fx * fx + 4.0 * fy * fy),
                  m / 12.0 * (4.0 * fx * fx + 4.0 * fy * fy));
        double ic = m / 12.0 * (4.0 * hh * hh) + m / 4.0 * (r * r);
        v3 Ic = V(ic, ic, m / 2.0 * (r * r));
        double d0 = 0.0 - zc, d1 = UG_GF_FOOT_Z - zc, d2 = UG_GF_DISC_Z - zc;
        s->omass[0] = 3.0 * m;
        s->oinertia[0] = V(Ib.x + m * d0 * d0 + If.x + m * d1 * d1 + Ic.x + m * d2 * d2,
                           Ib.y + m * d0 * d0 + If.y + m * d1 * d1 + Ic.y + m * d2 * d2, Ib.z + If.z + Ic.z);
        s->ocol[0] = s->ncol;
        Collider* c = &s->col[s->ncol++];
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
        c->v0 = UG_CYL_V0; c->nv = UG_CYL_NV; c->f0 = UG_CYL_F0; c->nf = UG_CYL_NF;
        if (s->full) { /* GEOM_CYLINDER as a cylinder (oracle build_scene) */
            c->kind = UG_SHAPE_CYL;
            c->margin = 0.0;
        }
        c->P = V(0.0, 0.0, d2); c->aP = c->P;
        c->owner = -2; c->ent = 1;
        s->oncol[0] = 3;
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
        Collider* c = &s->col[s->ncol];
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
        Collider* c = &s->col[s->ncol];
        box_collider(c, UG_GF_PITCH_HX + UG_URDF_MARGIN, UG_GF_PITCH_HX + UG_URDF_MARGIN,
                     UG_GF_PITCH_HZ + UG_URDF_MARGIN, UG_URDF_MARGIN, UG_DEFAULT_FRICTION);
        c->P = V(UG_GF_PITCH_X, UG_GF_PITCH_Y, UG_GF_PITCH_Z); c->aP = c->P;
        c->owner = -100; c->ent = 12;
        c->gjkbox = 1;
        statics[nstat++] = s->ncol++;
    }
    if (task == UG_TASK_BOX) {
        /* skew-box-button.urdf (oracle build_scene): object 0 the door (box + three handle cylinders), object 1 the
         * button cylinder, the walls static (entity 13), plane.urdf at z = 0 (11); robot frame (box base at y -0.5) */
        const double by = -UG_BX_ROBOT_Y;
        s->nobj = 2;
        ugj_box_links(&s->ojoint[0], &s->ojoint[1]);
        s->njoint = 2;
        s->jorder[0] = 1;
        s->jorder[1] = 0;
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
        const double ddisc = ugj_disc(lo, hi);
        Collider* c = &s->col[s->ncol];
        box_collider(c, B[3], B[4], B[5], UG_URDF_MARGIN, UG_DEFAULT_FRICTION);
        c->P = V(B[0], B[1], B[2]); c->aP = c->P;
        c->disc = ddisc;
        c->owner = -2; c->ent = 1;
        c->compound = 1;
        s->ocol[0] = s->ncol++;
        for (int i = 0; i < 3; i++) {
            const double* H = &UG_BX_HANDLE[4 * i];
            c = &s->col[s->ncol++];
            box_collider(c, H[3], H[3], UG_BX_HANDLE_HH[i], 0.0, UG_DEFAULT_FRICTION);
            c->kind = UG_SHAPE_CYL;
            c->P = V(H[0], H[1], H[2]); c->aP = c->P;
            if (i == 2) { double qh[4]; ugj_box_h3_quat(qh); c->R = qmat(Q(qh[0], qh[1], qh[2], qh[3])); c->aR = c->R; }
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
        double wlo[3] = {1e30, 1e30, 1e30}, whi[3] = {-1e30, -1e30, -1e30};
        for (int w = 0; w < 4; w++)
            for (int k = 0; k < 3; k++) {
                double l = UG_BX_WALL_POS[3 * w + k] - UG_BX_WALL_HALF[3 * w + k], u = UG_BX_WALL_POS[3 * w + k] + UG_BX_WALL_HALF[3 * w + k];
                wlo[k] = l < wlo[k] ? l : wlo[k];
                whi[k] = u > whi[k] ? u : whi[k];
            }
        const double wdisc = ugj_disc(wlo, whi);
        for (int w = 0; w < 4; w++) {
            c = &s->col[s->ncol];
            box_collider(c, UG_BX_WALL_HALF[3 * w], UG_BX_WALL_HALF[3 * w + 1], UG_BX_WALL_HALF[3 * w + 2], UG_URDF_MARGIN,
                         UG_DEFAULT_FRICTION);
            c->P = V(UG_BX_WALL_POS[3 * w], UG_BX_WALL_POS[3 * w + 1] + by, UG_BX_WALL_POS[3 * w + 2]); c->aP = c->P;
            c->disc = wdisc;
            c->owner = -100; c->ent = 13;
            c->compound = 1;
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
    /* pairs in the oracle's order; Box: door box x button only among the objects, button x plane only among the
     * object-static pairs (oracle build_scene) */
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
                    if (s->col[b].kind == UG_SHAPE_SPHERE && s->col[a].kind != UG_SHAPE_SPHERE) { int t = a; a = b; b = t; }
                    add_pair(s, a, b);
                }
    for (int o = 0; o < s->nobj; o++)
        for (int c = s->ocol[o]; c < s->ocol[o] + s->oncol[o]; c++)
            for (int t = 0; t < nstat; t++) {
                if (task == UG_TASK_BOX && !(o == 1 && s->col[statics[t]].ent == 11)) continue;
                add_pair(s, c, statics[t]);
            }
    for (int i = 0; i < s->ncol; i++) gjk_params(&s->col[i]);
    /* the quiescent-collision bound: every point of robot collider i -- its core (within |P| + gradius of the body
     * origin) with its margin, and the corners of the box its AABB is formed from (|aP| + |ac| + |ah|) -- lies within
     * rho of its body's origin, which lies within l(j, b) (the summed joint offsets) of body j's origin, through which
     * joint j's axis passes: turning joint j by dq moves the point by at most |dq| (l + rho), whatever the other joints */
    for (int i = 0; i < s->ncol; i++) {
        const Collider& c = s->col[i];
        for (int j = 0; j < NB; j++) s->qsw[i][j] = 0.0;
        if (c.owner < 0) continue;
        const double rho = fmax(vlen(c.P) + c.gradius + c.gmargin, vlen(c.aP) + vlen(c.ac) + vlen(c.ah));
        for (int j = 0; j < NB; j++) {
            double l = 0.0;
            int b = c.owner;
            while (b >= 0 && b != j) {
                l += vlen(V(UG_BODY_P[3 * b], UG_BODY_P[3 * b + 1], UG_BODY_P[3 * b + 2]));
                b = UG_BODY_PARENT[b];
            }
            if (b == j) s->qsw[i][j] = (l + rho) * (1.0 + 1e-9) + 1e-12;
        }
    }
}

// development / test aid: convex-convex queries as the kernels run them, one per 16-lane group (GJK_NG per wave, each
// with its own EPA store), through the same support-cell tables (urgym_debug_gjk, tests/test_gpu_gjk.py).  Query i packs
// 39 doubles: per shape kind, v0, nv, imp[3], margin, R[9], p[3], then thr.
__global__ void __launch_bounds__(TEAM, 1) k_gjk_query(const double* q, int n, double* out, int* ok, ugk::EpaMem* E) {
    const int i = blockIdx.x * GJK_NG + gjk_grp();
    if (i >= n) return; /* a whole group: its lanes leave together */
    const double* Q = q + (size_t)i * 39;
    ugk::GShape S[2];
    ugk::gx T[2];
    for (int k = 0; k < 2; k++) {
        const double* P = Q + 19 * k;
        S[k].kind = (int)P[0]; S[k].v0 = (int)P[1]; S[k].nv = (int)P[2];
        S[k].imp = ugk::V3(P[3], P[4], P[5]);
        S[k].margin = P[6];
        S[k].scb = -1; S[k].sck = 0;
        if (S[k].kind == UG_SHAPE_HULL) supcell_table(S[k].v0, S[k].nv, &S[k].scb, &S[k].sck);
        for (int j = 0; j < 9; j++) T[k].R.m[j] = P[7 + j];
        T[k].p = ugk::V3(P[16], P[17], P[18]);
    }
    ugk::gv nn, pp;
    double d = 0.0;
    const bool r = ugk::gjk_pair((UGK_GMEM ugk::EpaMem*)(E + i), S[0], T[0], S[1], T[1], Q[38], nn, pp, d);
    if ((threadIdx.x & (GJK_G - 1)) == 0) {
        ok[i] = r ? 1 : 0;
        double* o = out + (size_t)i * 7;
        o[0] = nn.x; o[1] = nn.y; o[2] = nn.z; o[3] = pp.x; o[4] = pp.y; o[5] = pp.z; o[6] = d;
    }
}

// ---------------------------------------------------------------------------
// kernels: one wavefront (block of 64) per environment, state resident in LDS
// ---------------------------------------------------------------------------

static __device__ int task_obs_dim(int variant) { return UG_OBS_DIM(variant); }
static __device__ int task_act_dim(int variant) { return UG_ACT_DIM(variant); }
static __device__ int task_ndraw(int variant) { return UG_NDRAW(variant); }

static __device__ __forceinline__ void reset_env(const Scene* sc, double* S, uint32_t* mt, int* elapsed, double* ws,
                                                 const uint8_t* mask, const double* draws, double* obs,
                                                 int32_t* substeps, int* stats, uint8_t* flags, int i) {
    if (mask && !mask[i]) { /* nothing happened to a masked-out env in this call */
        if (threadIdx.x == 0) flags[i] = 0;
        return;
    }
    double* Si = S + (size_t)i * UG_STATE_DIM;
    team_load(Si, stats + (size_t)i * UG_NSTAT);
    RunIO io;
    io.act = nullptr;
    io.obs = obs + (size_t)i * task_obs_dim(sc->variant);
    io.final_obs = nullptr;
    io.dr = Draws{Rng{mt + (size_t)i * UG_MT_WORDS, 1, 0}, draws ? draws + (size_t)i * task_ndraw(sc->variant) : nullptr, 0};
    io.autoreset = 0;
    io.trunc = 0;
    PROF_T0(t_tot);
    int ns = team_run(sc, ws + (size_t)i * WS_STRIDE(sc->full, sc->gjk), G_RESET, io);
    PROF_ADD(PF_TOTAL, t_tot);
    team_store(Si, stats + (size_t)i * UG_NSTAT, flags + i);
    team_prof_flush();
    if (threadIdx.x == 0) {
        elapsed[i] = 0;
        if (substeps) substeps[i] = ns;
    }
}

/* The step and reset launches are work queues: one block per wave slot the device holds at once (urgym_handle::slots),
 * each taking the next env of the launch order from a global counter as soon as it is free, until the order is used
 * up.  With one block per env (the hardware dispatcher dealing the grid's blocks round-robin to the 8 XCDs in block
 * order) a wave slot sat idle 0.4-0.6 ms on average between the end of one block and the start of the next on it (p99
 * 3-4 ms; BallBalance x4096: 1.5 ms of idle per slot per 24.4 ms launch, tools/timeline.py's placement view,
 * profiles/round5_timeline_dispatch_hw.json).  The queue makes the launch the list schedule of the launch order.  An
 * env's result does not depend on which block ran it (its state, workspace and streams are its own); every block
 * leaves once the counter passes n.  The counter is zeroed (hipMemsetAsync on the launch's stream) before every
 * launch. */
__device__ __forceinline__ int queue_next(int* q) {
    int k = 0;
    if (threadIdx.x == 0) k = atomicAdd(q, 1);
    return __builtin_amdgcn_readfirstlane(k);
}

__global__ void __launch_bounds__(TEAM, 1) k_reset(const Scene* sc, double* S, uint32_t* mt, int* elapsed, double* ws,
                                                   int n, const uint8_t* mask, const double* draws, double* obs,
                                                   int32_t* substeps, int* stats, uint8_t* flags, int* queue) {
    for (;;) {
        const int i = queue_next(queue);
        if (i >= n) return;
        reset_env(sc, S, mt, elapsed, ws, mask, draws, obs, substeps, stats, flags, i);
    }
}

static __device__ __forceinline__ void step_env(const Scene* sc, double* S, uint32_t* mt, int* elapsed, double* ws,
                                                const float* act, double* obs, double* final_obs, double* rew,
                                                uint8_t* term, uint8_t* trunc, uint8_t* succ, int32_t* substeps,
                                                int autoreset, int max_steps, int i, int k, uint8_t* prio, int* stats,
                                                uint8_t* flags, double* pfeat) {
#ifdef UG_PROF
    const unsigned long long bt0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long lvl = prio[i]; /* the level this launch was ordered by */
#endif
    double* Si = S + (size_t)i * UG_STATE_DIM;
    team_load(Si, stats + (size_t)i * UG_NSTAT);
    const int O = task_obs_dim(sc->variant), A = task_act_dim(sc->variant);
    const int el = elapsed[i] + 1;
    RunIO io;
    io.act = act + (size_t)i * A;
    io.obs = obs + (size_t)i * O;
    io.final_obs = final_obs ? final_obs + (size_t)i * O : nullptr;
    io.dr = Draws{Rng{mt + (size_t)i * UG_MT_WORDS, 1, 0}, nullptr, 0};
    io.autoreset = autoreset;
    io.trunc = (max_steps > 0 && el >= max_steps) ? 1 : 0;
    io.reset_done = 0;
    PROF_T0(t_tot);
    int ns = team_run(sc, ws + (size_t)i * WS_STRIDE(sc->full, sc->gjk), G_STEP, io);
    PROF_ADD(PF_TOTAL, t_tot);
    team_store(Si, stats + (size_t)i * UG_NSTAT, flags + i);
    team_prof_flush();
    if (threadIdx.x == 0) {
        elapsed[i] = io.reset_done ? 0 : el;
        if (rew) rew[i] = io.rew;
        if (term) term[i] = (uint8_t)io.term;
        if (trunc) trunc[i] = (uint8_t)io.trunc;
        if (succ) succ[i] = (uint8_t)io.succ;
        if (substeps) substeps[i] = ns;
        prio[i] = (uint8_t)team_priority(sc, ns, elapsed[i] + 1, max_steps, autoreset,
                                         pfeat ? pfeat + (size_t)i * UG_PF_STRIDE : nullptr);
#ifdef UG_PROF
        if (k < UG_BT_MAX) { /* per launch-order position */
            unsigned long long* bt = &g_btime[4 * k];
            unsigned xcc, hwid; /* where the env ran: XCD, and SE / CU / SIMD (tools/timeline.py's placement view) */
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
            bt[0] = bt0;
            bt[1] = __builtin_amdgcn_s_memrealtime();
            bt[2] = (unsigned long long)i;
            bt[3] = (unsigned long long)ns | ((unsigned long long)io.reset_done << 16) |
                    ((unsigned long long)(xcc & 15u) << 20) | (lvl << 24) |
                    ((unsigned long long)hwid << 32);
        }
#endif
    }
}

__global__ void __launch_bounds__(TEAM, 1) k_step(const Scene* sc, double* S, uint32_t* mt, int* elapsed, double* ws,
                                                  int n, const float* act, double* obs, double* final_obs, double* rew,
                                                  uint8_t* term, uint8_t* trunc, uint8_t* succ, int32_t* substeps,
                                                  int autoreset, int max_steps, const int* order, uint8_t* prio,
                                                  int* stats, uint8_t* flags, int* queue, double* pfeat) {
    for (;;) {
        const int k = queue_next(queue);
        if (k >= n) return;
        step_env(sc, S, mt, elapsed, ws, act, obs, final_obs, rew, term, trunc, succ, substeps, autoreset, max_steps,
                 order[k], k, prio, stats, flags, pfeat);
    }
}

/* Launch levels from the step's own action (scheduling only; BallBalance, TwoBalls, CubesPush, CubesPushDiff, CubesGrasp,
 * Golf): per env, the state
 * inputs its last step left in pfeat (team_priority; the record's last double names the model) and the 3 action
 * components of this step -> the task's model -> the level; envs whose record is not flagged (a predicted truncation,
 * an inactive ball) keep their level.  One thread per env, before k_order. */
static_assert(UG_ACT_DIM(UG_TASK_TWOBALLS) == UG_PT_IN - UG_PT_STATE_IN, "TwoBalls' action: the model's last inputs");
static_assert(UG_ACT_DIM(UG_TASK_CUBESPUSH) == 3 && UG_ACT_DIM(UG_TASK_CUBESPUSHDIFF) == 3, "CubesPush's action: 3");
static_assert(UG_ACT_DIM(UG_TASK_BALLBALANCE) == 3, "BallBalance's action: 3");
static_assert(UG_ACT_DIM(UG_TASK_GOLF) == 3 && UG_ACT_DIM(UG_TASK_GOLFJOINTS) == 6, "Golf's action: 3, GolfJoints' 6");
/* CubesGrasp (model 4 / 5): the branch the step's random.choices will take, from the env's stream without consuming it */
__device__ static int cg_branch(const uint32_t* mt, const float* a, int i) {
    return ugg_cg_choose(a[0], a[1], mt_peek_random(mt + (size_t)i * UG_MT_WORDS));
}
/* a gradient-boosted tree ensemble's log-odds (tools/fit_priority.py tree_header: flat node arrays UG_PF_<P>_*, a leaf
 * has feature -1; x <= threshold goes left, so a NaN input goes right; the depth bound only guards a corrupt table) */
__device__ static double trees_logodds(const double* x, int ntrees, double base, const short* root, const signed char* feat,
                                       const double* thr, const short* left, const short* right, const double* val) {
    double lg = base;
    for (int t = 0; t < ntrees; t++) {
        int k = root[t];
        for (int d = 0; d < 64 && feat[k] >= 0; d++) k = x[feat[k]] <= thr[k] ? left[k] : right[k];
        lg += val[k];
    }
    return lg;
}
#define UG_TREES_LOGODDS(P, x)                                                                                          \
    trees_logodds(x, UG_PF_##P##_TREES, UG_PF_##P##_BASE, UG_PF_##P##_ROOT, UG_PF_##P##_FEAT, UG_PF_##P##_THR,         \
                  UG_PF_##P##_LEFT, UG_PF_##P##_RIGHT, UG_PF_##P##_VAL)
static_assert(UG_PF_TBT_IN == UG_PT_IN, "TwoBalls' trees take the MLP's inputs");
static_assert(UG_PF_CGT_IN == UG_PG_IN, "CubesGrasp's trees take the MLP's inputs");
__global__ void k_prio(const double* pfeat, const float* act, const uint32_t* mt, uint8_t* prio, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double* f = pfeat + (size_t)i * UG_PF_STRIDE;
    const double model = f[UG_PF_STRIDE - 1];
    if constexpr (NB == 12) {
        if (model == 4.0 || model == 5.0) { /* CubesGrasp: q, qd, targets - q, the branch, the truncation */
            const float* a = act + (size_t)i * UG_ACT_DIM(UG_TASK_CUBESGRASP);
            const int sel = cg_branch(mt, a, i);
            double x[UG_PG_IN];
            for (int k = 0; k < 2 * NB; k++) x[k] = f[k];
            for (int j = 0; j < 7; j++) {
                const double t = sel == 0 ? (j < 6 ? (double)a[2 + j] : f[2 * NB + 6])
                                          : (j < 6 ? f[2 * NB + j] : gripper_angle(a[8] < 0.5f ? UG_GRIP_MAX : UG_GRIP_MIN));
                x[2 * NB + j] = t - f[j];
            }
            x[2 * NB + 7] = (double)sel;
            x[2 * NB + 8] = model == 5.0 ? 1.0 : 0.0;
#ifdef UG_CG_MLP /* the round-6 MLP classifier (prio_model_cg.h); the trees replace it */
            prio[i] = (uint8_t)logit_level(mlp_logit<UG_PG_IN, UG_PG_HID>(x, UG_PG_MU, UG_PG_SD, UG_PG_W1, UG_PG_B1, UG_PG_W2,
                                                                           UG_PG_B2), UG_PG_L0, UG_PG_DL);
#else
            prio[i] = (uint8_t)logit_level(UG_TREES_LOGODDS(CGT, x), UG_PF_CGT_L0, UG_PF_CGT_DL);
#endif
            return;
        }
    }
    if (model == 1.0) { /* TwoBalls: 31 state inputs + the action -> the tree ensemble (round 6; the MLP of
                           * prio_model_tb.h under -DUG_TB_MLP) */
        double x[UG_PT_IN];
        for (int k = 0; k < UG_PT_STATE_IN; k++) x[k] = f[k];
        for (int a = 0; a < UG_PT_IN - UG_PT_STATE_IN; a++) x[UG_PT_STATE_IN + a] = (double)act[(size_t)i * 3 + a];
#ifdef UG_TB_MLP
        prio[i] = (uint8_t)logit_level(mlp_logit<UG_PT_IN, UG_PT_HID>(x, UG_PT_MU, UG_PT_SD, UG_PT_W1, UG_PT_B1, UG_PT_W2,
                                                                       UG_PT_B2), UG_PT_L0, UG_PT_DL);
#else
        prio[i] = (uint8_t)logit_level(UG_TREES_LOGODDS(TBT, x), UG_PF_TBT_L0, UG_PF_TBT_DL);
#endif
    } else if (model == 3.0) { /* BallBalance: the ball's 14 inputs + the action */
        double x[UG_PM_IN];
        for (int k = 0; k < UG_BALL_IN; k++) x[k] = f[k];
        for (int a = 0; a < 3; a++) x[UG_BALL_IN + a] = (double)act[(size_t)i * 3 + a];
        prio[i] = (uint8_t)logit_level(mlp_logit<UG_PM_IN, UG_PM_HID>(x, UG_PM_MU, UG_PM_SD, UG_PM_W1, UG_PM_B1, UG_PM_W2,
                                                                       UG_PM_B2), UG_PM_L0, UG_PM_DL);
    } else if (model == 6.0) { /* Golf: q, qd, the ball's position + the action -> the tree ensemble's log-odds */
        double x[UG_PF_GF_IN];
        for (int k = 0; k < UG_PF_GF_IN - 3; k++) x[k] = f[k];
        for (int a = 0; a < 3; a++) x[UG_PF_GF_IN - 3 + a] = (double)act[(size_t)i * 3 + a];
        prio[i] = (uint8_t)logit_level(UG_TREES_LOGODDS(GF, x), UG_PF_GF_L0, UG_PF_GF_DL);
    } else if (model == 7.0) { /* GolfJoints: the same state inputs + its 6 joint deltas -> its own trees */
        double x[UG_PF_GJ_IN];
        for (int k = 0; k < UG_PF_GJ_IN - 6; k++) x[k] = f[k];
        for (int a = 0; a < 6; a++) x[UG_PF_GJ_IN - 6 + a] = (double)act[(size_t)i * 6 + a];
        prio[i] = (uint8_t)logit_level(UG_TREES_LOGODDS(GJ, x), UG_PF_GJ_L0, UG_PF_GJ_DL);
    } else if (model == 2.0) { /* CubesPush(Diff): q, qd + the action */
        double x[UG_PC_IN];
        for (int k = 0; k < UG_PC_IN - 3; k++) x[k] = f[k];
        for (int a = 0; a < 3; a++) x[UG_PC_IN - 3 + a] = (double)act[(size_t)i * 3 + a];
        prio[i] = (uint8_t)logit_level(mlp_logit<UG_PC_IN, UG_PC_HID>(x, UG_PC_MU, UG_PC_SD, UG_PC_W1, UG_PC_B1, UG_PC_W2,
                                                                       UG_PC_B2), UG_PC_L0, UG_PC_DL);
    }
}

/* An explicit reset or set_state replaces the state the predictor record was taken from: clear the record's model flag
 * (k_prio then keeps the level k_iota or the last step left) for every env the call touched (mask NULL = all). */
__global__ void k_pfeat_clear(double* pfeat, const uint8_t* mask, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || (mask && !mask[i])) return;
    pfeat[(size_t)i * UG_PF_STRIDE + UG_PF_STRIDE - 1] = 0.0;
}

/* next launch order: envs by descending priority (0..255), ties by ascending env index (deterministic), one block.
 * Up to ORDER_LDS envs: a bitonic sort of (255 - priority) << 24 | env in LDS (78 stages for 4096 envs); more: a
 * two-pass stable counting sort by priority nibble (low, then high) through tmp. */
#define ORDER_THREADS 1024
#define ORDER_LDS 8192
__device__ static void order_pass(const uint8_t* prio, int shift, const int* src, int* dst, int n, int* wsum, int* base) {
    const int t = threadIdx.x, w = t / WAVE, l = t % WAVE;
    if (t == 0) *base = 0;
    __syncthreads();
    for (int b = 15; b >= 0; b--) {
        for (int c = 0; c < n; c += ORDER_THREADS) {
            const int i = c + t;
            const int e = i < n ? (src ? src[i] : i) : 0;
            const bool f = i < n && ((prio[e] >> shift) & 15) == b;
            const unsigned long long m = __ballot(f);
            if (l == 0) wsum[w] = __popcll(m);
            __syncthreads();
            int off = *base;
            for (int k = 0; k < w; k++) off += wsum[k];
            if (f) dst[off + __popcll(m & ((1ull << l) - 1ull))] = e;
            __syncthreads();
            if (t == 0)
                for (int k = 0; k < ORDER_THREADS / WAVE; k++) *base += wsum[k];
            __syncthreads();
        }
    }
}
__global__ void __launch_bounds__(ORDER_THREADS) k_order(const uint8_t* prio, int* order, int* tmp, int n) {
    __shared__ uint32_t sk[ORDER_LDS];
    __shared__ int wsum[ORDER_THREADS / WAVE];
    __shared__ int base;
    const int t = threadIdx.x;
    if (n > ORDER_LDS) {
        order_pass(prio, 0, nullptr, tmp, n, wsum, &base);
        __threadfence_block();
        __syncthreads();
        order_pass(prio, 4, tmp, order, n, wsum, &base);
        return;
    }
    int n2 = 1;
    while (n2 < n) n2 <<= 1;
    for (int i = t; i < n2; i += ORDER_THREADS) sk[i] = i < n ? ((255u - prio[i]) << 24) | (uint32_t)i : 0xFFFFFFFFu;
    __syncthreads();
    for (int k = 2; k <= n2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = t; i < n2; i += ORDER_THREADS) {
                const int x = i ^ j;
                if (x > i) {
                    const uint32_t a = sk[i], b = sk[x];
                    if ((a > b) == ((i & k) == 0)) { sk[i] = b; sk[x] = a; }
                }
            }
            __syncthreads();
        }
    }
    for (int i = t; i < n; i += ORDER_THREADS) order[i] = (int)(sk[i] & 0xFFFFFFu);
}
__global__ void k_iota(int* order, uint8_t* prio, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { order[i] = i; prio[i] = 0; }
}

__global__ void __launch_bounds__(TEAM, 1) k_substep(const Scene* sc, double* S, double* ws, int n, int* stats) {
    const int i = blockIdx.x;
    if (i >= n) return;
    double* Si = S + (size_t)i * UG_STATE_DIM;
    team_load(Si, stats + (size_t)i * UG_NSTAT);
    team_substep(sc, ws + (size_t)i * WS_STRIDE(sc->full, sc->gjk));
    team_store(Si, stats + (size_t)i * UG_NSTAT, nullptr);
}

// getLinkState / calculateInverseKinematics queries: one env per lane (not on the step path)
__global__ void __launch_bounds__(WAVE) k_link_state(const double* S, int n, int link, double* out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double q[NB];
    for (int j = 0; j < NB; j++) q[j] = S[(size_t)i * UG_STATE_DIM + UG_F_Q + j];
    v3 p;
    q4 o;
    link_state_of(q, link, p, o);
    double* r = out + (size_t)i * 7;
    r[0] = p.x; r[1] = p.y; r[2] = p.z; r[3] = o.x; r[4] = o.y; r[5] = o.z; r[6] = o.w;
}

__global__ void __launch_bounds__(WAVE) k_ik(const double* S, int n, const double* target, double* qout) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double q[NB], qo[NB];
    for (int j = 0; j < NB; j++) q[j] = S[(size_t)i * UG_STATE_DIM + UG_F_Q + j];
    const double* t = target + (size_t)i * 7;
    ik_solve(q, V(t[0], t[1], t[2]), Q(t[3], t[4], t[5], t[6]), qo);
    for (int j = 0; j < NB; j++) qout[(size_t)i * NB + j] = qo[j];
}

/* p.getContactPoints(bodyA, bodyB, linkIndexA, linkIndexB) over each env's manifold cache (lane per env; a
 * query, not on the step path).  Same definition as the oracle's ugo_contact_points: entity codes (0 robot,
 * 1 + i object i, 10 table, 11 plane, 12 pitch, -1 any), links (robot link index, object base -1 / club parts
 * 0, 1, -2 any), 24 doubles per point in pybullet's tuple order, forces = impulse / dt, friction directions
 * btPlaneSpace1 of the normal; the tuple is swapped when bodyA names the pair's B side, and bodyB / linkA /
 * linkB filter in that orientation (pybullet's order).  Positions are the points' local anchors under the poses of
 * the last substep's narrowphase (the state's UG_F_PREV record, taken before that substep's integration): Bullet's
 * m_positionWorldOnA/B as refreshContactPoints left them. */
__device__ static int link_of_collider(const Scene* s, int ci) {
    const Collider& c = s->col[ci];
    if (c.ent == 0) return c.link;
    if (s->task == UG_TASK_BOX && (c.ent == 1 || c.ent == 2)) return c.ent == 1 ? 1 : 0; /* door = joint 1, button = 0 */
    if (c.ent >= 1 && c.ent <= MAXOBJ) return ci - s->ocol[c.ent - 1] - 1;
    return -1;
}
__global__ void __launch_bounds__(WAVE) k_contacts(const Scene* sc, const double* S, int n, int bodyA, int bodyB,
                                                   int linkA, int linkB, int max_pts, double* out, int32_t* count) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const EnvState& e = *(const EnvState*)(S + (size_t)i * UG_STATE_DIM);
    Kin k;
    fk(e.prevq, k); /* the last narrowphase's poses */
    auto prev_xf = [&](int owner) {
        XF T;
        if (owner >= 0) { T.R = k.R[owner]; T.p = k.p[owner]; }
        else if (owner <= -2 && owner > -100) {
            const double* P = e.prevpose[-2 - owner];
            T.R = qmat(Q(P[3], P[4], P[5], P[6]));
            T.p = V(P[0], P[1], P[2]);
        } else { T.R = mident(); T.p = V(0, 0, 0); }
        return T;
    };
    int cnt = 0;
    const int nm = (int)e.nman;
    for (int m = 0; m < nm; m++) {
        const StMan& M = e.man[m];
        const PairDef& P = sc->pair[(int)M.pair];
        const int ea = sc->col[P.a].ent, eb = sc->col[P.b].ent;
        const int la = link_of_collider(sc, P.a), lb = link_of_collider(sc, P.b);
        auto mt = [](int want, int have) { return want == -1 || want == have; };
        auto ml = [](int want, int have) { return want == -2 || want == have; };
        int swap = 0; /* pybullet's order: orientation from bodyA alone, then the other filters */
        if (bodyA != -1) {
            if (bodyA == ea) swap = 0;
            else if (bodyA == eb) swap = 1;
            else continue;
        }
        if (!mt(bodyB, swap ? ea : eb) || !ml(linkA, swap ? lb : la) || !ml(linkB, swap ? la : lb)) continue;
        const XF OA = prev_xf(sc->col[P.a].owner), OB = prev_xf(sc->col[P.b].owner);
        const int np = (int)M.npts;
        for (int j = 0; j < np; j++) {
            const StPt& c = M.pt[j];
            if (cnt < max_pts) {
                double* o = out + ((size_t)i * max_pts + cnt) * 24;
                v3 pA = xf_apply(OA, c.lpA), pB = xf_apply(OB, c.lpB);
                v3 nn = c.n, t1, t2;
                if (ug_fabs(nn.z) > 0.7071067811865475244) {
                    double a = nn.y * nn.y + nn.z * nn.z, kk = 1.0 / ug_sqrt(a);
                    t1 = V(0, -nn.z * kk, nn.y * kk);
                    t2 = V(a * kk, -nn.x * t1.z, nn.x * t1.y);
                } else {
                    double a = nn.x * nn.x + nn.y * nn.y, kk = 1.0 / ug_sqrt(a);
                    t1 = V(-nn.y * kk, nn.x * kk, 0);
                    t2 = V(-nn.z * t1.y, nn.z * t1.x, a * kk);
                }
                if (swap) { v3 t = pA; pA = pB; pB = t; nn = vneg(nn); }
                if (sc->task == UG_TASK_BOX) { /* Box-v0 keeps the robot base at the origin: back to world y */
                    pA.y = pA.y + UG_BX_ROBOT_Y;
                    pB.y = pB.y + UG_BX_ROBOT_Y;
                }
                o[0] = 0.0;
                o[1] = swap ? eb : ea; o[2] = swap ? ea : eb;
                o[3] = swap ? lb : la; o[4] = swap ? la : lb;
                o[5] = pA.x; o[6] = pA.y; o[7] = pA.z;
                o[8] = pB.x; o[9] = pB.y; o[10] = pB.z;
                o[11] = nn.x; o[12] = nn.y; o[13] = nn.z;
                o[14] = c.dist;
                o[15] = c.imp / UG_DT;
                o[16] = c.imp1 / UG_DT;
                o[17] = t1.x; o[18] = t1.y; o[19] = t1.z;
                o[20] = c.imp2 / UG_DT;
                o[21] = t2.x; o[22] = t2.y; o[23] = t2.z;
            }
            cnt++;
        }
    }
    count[i] = cnt;
}

// Camera.shot() for a range of envs (ug_render.h), two launches.  k_camera_pose: block per env, lane per collider:
// its world pose (fk + owner / shape frame, the same functions the physics uses), culling bounds and active flag
// into a per-env record (CAM_REC doubles per collider).  k_camera: block = (8 x 8 pixel tile, env): the env's records
// into LDS, then every lane casts its pixel's ray against the active colliders, statics and objects first (their
// hits prune the robot's hulls behind them), keeping the nearest hit, ties to the lower collider index.
#define CAM_REC 20 /* R 9, p 3, bounding radius, vertex box 6, active */
__global__ void __launch_bounds__(WAVE) k_camera_pose(const Scene* sc, const double* S, int env0, double* rec) {
    __shared__ Kin k; /* the env's frames, once (lane 0), read by every collider's lane */
    const int lane = threadIdx.x;
    const EnvState& e = *(const EnvState*)(S + (size_t)(env0 + (int)blockIdx.x) * UG_STATE_DIM);
    if (lane == 0) fk(e.q, k);
    __syncthreads();
    if (lane >= sc->ncol) return;
    const Collider& c = sc->col[lane];
    const XF T = shape_xf(owner_xf(e, k, c.owner), c);
    double* r = rec + ((size_t)blockIdx.x * MAXCOL + lane) * CAM_REC;
    for (int m = 0; m < 9; m++) r[m] = T.R.m[m];
    /* the camera's view matrix is in world coordinates: Box-v0's poses are stored with the robot base at the origin
     * (scene_data.h), so they move back by the base's world offset */
    r[9] = T.p.x; r[10] = sc->task == UG_TASK_BOX ? T.p.y + UG_BX_ROBOT_Y : T.p.y; r[11] = T.p.z;
    r[12] = ugr_radius(c.kind, c.half, UG_HULL_V + 3 * c.v0, c.nv);
    ugr_hull_box(UG_HULL_V + 3 * c.v0, c.kind == UG_SHAPE_HULL ? c.nv : 0, r + 13);
    r[19] = collider_active(e, c) ? 1.0 : 0.0;
}
__global__ void __launch_bounds__(WAVE) k_camera(const Scene* sc, const double* rec, UgrCam cam, int W, int H,
                                                 int flags, uint8_t* rgba, float* depth, int32_t* seg) {
    __shared__ double sr[MAXCOL * CAM_REC];
    const int lane = threadIdx.x;
    const size_t img = blockIdx.y;
    const int nc = sc->ncol;
    const double* src = rec + img * MAXCOL * CAM_REC;
    for (int i = lane; i < nc * CAM_REC; i += WAVE) sr[i] = src[i];
    __syncthreads();
    const int tw = (W + 7) / 8;
    const int px = (blockIdx.x % tw) * 8 + (lane & 7), py = (blockIdx.x / tw) * 8 + (lane >> 3);
    if (px >= W || py >= H) return;
    double o[3], d[3], nb[3] = {0.0, 0.0, 0.0};
    ugr_ray(&cam, px, py, W, H, o, d);
    double best = UGR_MISS;
    int bc = -1;
    for (int ci = nc - 1; ci >= 0; ci--) {
        const double* r = sr + ci * CAM_REC;
        if (r[19] == 0.0) continue;
        const Collider& c = sc->col[ci];
        double nw[3];
        const double t = ugr_shape(r, r + 9, r[12], c.kind, c.half, UG_HULL_F + 4 * c.f0, c.nf, r + 13, best, o, d, nw);
        if (t < best || (t == best && t != UGR_MISS)) { best = t; bc = ci; nb[0] = nw[0]; nb[1] = nw[1]; nb[2] = nw[2]; }
    }
    const int ent = bc >= 0 ? sc->col[bc].ent : -1, link = bc >= 0 ? link_of_collider(sc, bc) : -1;
    unsigned char pxl[4];
    float dp;
    int sg;
    ugr_shade(&cam, sc->variant, best, nb, ent, link, flags, o, d, pxl, &dp, &sg);
    const size_t at = img * (size_t)(W * H) + (size_t)(py * W + px);
    if (rgba) { rgba[4 * at] = pxl[0]; rgba[4 * at + 1] = pxl[1]; rgba[4 * at + 2] = pxl[2]; rgba[4 * at + 3] = pxl[3]; }
    if (depth) depth[at] = dp;
    if (seg) seg[at] = sg;
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static std::string g_create_error;

struct urgym_handle {
    int task = 0, n = 0, dev = 0, flags = 0;
    hipStream_t stream = nullptr;
    Scene* d_scene = nullptr;
    double* d_state = nullptr;
    double* d_ws = nullptr;
    uint32_t* d_mt = nullptr;
    int* d_elapsed = nullptr;
    // staging for the host-pointer API
    float* d_act = nullptr;
    double *d_obs = nullptr, *d_final = nullptr, *d_rew = nullptr, *d_draws = nullptr, *d_aux = nullptr;
    uint8_t *d_term = nullptr, *d_trunc = nullptr, *d_succ = nullptr, *d_mask = nullptr;
    int32_t* d_sub = nullptr;
    int* d_order = nullptr;   // k_step launch order (queue position -> env), from the previous step's priorities
    int* d_order_tmp = nullptr; // k_order's first pass (more than ORDER_LDS envs)
    int* d_queue = nullptr;   // the step / reset work-queue counter
    int slots = 0;            // k_step / k_reset blocks: the wave slots the device holds at once (CUs x blocks per CU)
    uint8_t* d_prio = nullptr;
    double* d_pfeat = nullptr; // BallBalance, TwoBalls, CubesPush(Diff), CubesGrasp, Golf: per env the predictor's state inputs for k_prio (UG_PF_STRIDE doubles)
    int* d_stats = nullptr;   // UG_NSTAT event counters per env
    uint8_t* d_flags = nullptr; // UG_FLAG_* of the last step / reset per env
    int autoreset = 0, max_steps = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool timed = false;
    double* d_campose = nullptr; // k_camera_pose records (count x MAXCOL x CAM_REC), grown on demand
    size_t campose_envs = 0;
    std::string err;
};

static int fail(urgym_handle* h, const std::string& msg) {
    if (h) h->err = msg;
    else g_create_error = msg;
    return -1;
}
#define HIPCHK(h, call)                                                                       \
    do {                                                                                      \
        hipError_t _e = (call);                                                               \
        if (_e != hipSuccess) return fail((h), std::string(#call) + ": " + hipGetErrorString(_e)); \
    } while (0)

static int grid_of(int n) { return (n + WAVE - 1) / WAVE; }

// CPython random.seed(int) (init_by_array) -- host copy for per-env stream seeding
static void mt_seed_host(uint32_t* mt, uint32_t seed) {
    mt[0] = 19650218u;
    for (int i = 1; i < 624; i++) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    uint32_t key = seed;
    int i = 1, j = 0;
    for (int k = 624; k; k--) {
        mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key + (uint32_t)j;
        i++; j++;
        if (i >= 624) { mt[0] = mt[623]; i = 1; }
        if (j >= 1) j = 0;
    }
    for (int k = 623; k; k--) {
        mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
        i++;
        if (i >= 624) { mt[0] = mt[623]; i = 1; }
    }
    mt[0] = 0x80000000u;
    mt[624] = 624;
}

extern "C" {

int urgym_obs_dim(int task) { return UG_OBS_DIM(task); }
int urgym_act_dim(int task) { return UG_ACT_DIM(task); }
int urgym_state_dim(void) { return UG_STATE_DIM; }
int urgym_num_draws(int task) { return UG_NDRAW(task); }
int urgym_num_envs(const urgym_handle* h) { return h ? h->n : 0; }
const char* urgym_last_error(const urgym_handle* h) { return h ? h->err.c_str() : g_create_error.c_str(); }

static int create_impl(urgym_handle* h, int task, int n, int dev, uint32_t seed, int env_offset, int flags) {
    HIPCHK(h, hipSetDevice(dev));
    HIPCHK(h, hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
    HIPCHK(h, hipEventCreate(&h->ev0));
    HIPCHK(h, hipEventCreate(&h->ev1));
    // lane-serial helpers (dynamics, IK) keep their arrays in scratch
    HIPCHK(h, hipDeviceSetLimit(hipLimitStackSize, 16 * 1024));
    HIPCHK(h, hipMalloc(&h->d_scene, sizeof(Scene)));
    size_t N = (size_t)n;
    HIPCHK(h, hipMalloc(&h->d_state, sizeof(double) * UG_STATE_DIM * N));
    HIPCHK(h, hipMalloc(&h->d_mt, sizeof(uint32_t) * UG_MT_WORDS * N));
    HIPCHK(h, hipMalloc(&h->d_ws, sizeof(double) * WS_STRIDE(UG_GEOM_IS_FULL(flags), UG_CONTACT_IS_GJK(flags)) * N));
    HIPCHK(h, hipMalloc(&h->d_elapsed, sizeof(int) * N));
    HIPCHK(h, hipMalloc(&h->d_act, sizeof(float) * 9 * N));
    HIPCHK(h, hipMalloc(&h->d_obs, sizeof(double) * 17 * N));
    HIPCHK(h, hipMalloc(&h->d_final, sizeof(double) * 17 * N));
    HIPCHK(h, hipMalloc(&h->d_rew, sizeof(double) * N));
    HIPCHK(h, hipMalloc(&h->d_draws, sizeof(double) * 4 * N));
    HIPCHK(h, hipMalloc(&h->d_aux, sizeof(double) * UG_STATE_DIM * N));
    HIPCHK(h, hipMalloc(&h->d_term, N));
    HIPCHK(h, hipMalloc(&h->d_trunc, N));
    HIPCHK(h, hipMalloc(&h->d_succ, N));
    HIPCHK(h, hipMalloc(&h->d_mask, N));
    HIPCHK(h, hipMalloc(&h->d_sub, sizeof(int32_t) * N));
    HIPCHK(h, hipMalloc(&h->d_order, sizeof(int) * N));
    HIPCHK(h, hipMalloc(&h->d_order_tmp, sizeof(int) * N));
    HIPCHK(h, hipMalloc(&h->d_prio, N));
    /* URGYM_NO_PRIO_MODEL (a measurement aid, like URGYM_SLOTS): no predictor record, so every env is launched by the
     * fallback level (its last substep count, predicted truncation first) -- the A/B baseline of the k_prio models */
    const char* noprio = getenv("URGYM_NO_PRIO_MODEL");
    if ((!noprio || !*noprio || *noprio == '0') &&
        (task == URGYM_TASK_BALLBALANCE || task == URGYM_TASK_TWOBALLSBALANCE || task == URGYM_TASK_CUBESPUSH ||
         task == URGYM_TASK_CUBESPUSHDIFF || task == URGYM_TASK_CUBESGRASP || task == URGYM_TASK_GOLF ||
         task == URGYM_TASK_GOLFJOINTS)) {
        HIPCHK(h, hipMalloc(&h->d_pfeat, sizeof(double) * UG_PF_STRIDE * N));
        HIPCHK(h, hipMemsetAsync(h->d_pfeat, 0, sizeof(double) * UG_PF_STRIDE * N, h->stream));
    }
    HIPCHK(h, hipMalloc(&h->d_queue, sizeof(int)));
    {
        int cus = 0, per = 0;
        HIPCHK(h, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        HIPCHK(h, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_step, TEAM, 0));
        h->slots = (cus > 0 ? cus : 1) * (per > 0 ? per : 1);
        if (const char* e = getenv("URGYM_SLOTS")) h->slots = atoi(e) > 0 ? atoi(e) : h->slots; /* A/B measurement aid */
    }
    HIPCHK(h, hipMalloc(&h->d_stats, sizeof(int) * UG_NSTAT * N));
    HIPCHK(h, hipMalloc(&h->d_flags, N));
    HIPCHK(h, hipMemsetAsync(h->d_stats, 0, sizeof(int) * UG_NSTAT * N, h->stream));
    /* the workspace starts zeroed: its separation certificates (WS_PC) must read "none" until written */
    HIPCHK(h, hipMemsetAsync(h->d_ws, 0, sizeof(double) * WS_STRIDE(UG_GEOM_IS_FULL(flags), UG_CONTACT_IS_GJK(flags)) * N, h->stream));
    HIPCHK(h, hipMemsetAsync(h->d_flags, 0, N, h->stream));
    k_iota<<<grid_of(n), WAVE, 0, h->stream>>>(h->d_order, h->d_prio, n);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipMemsetAsync(h->d_state, 0, sizeof(double) * UG_STATE_DIM * N, h->stream));
    HIPCHK(h, hipMemsetAsync(h->d_elapsed, 0, sizeof(int) * N, h->stream));
    // per-env MT19937 streams seeded with seed + env_offset + i, UG_MT_WORDS words per env
    std::vector<uint32_t> host(UG_MT_WORDS * N);
    for (int i = 0; i < n; i++) mt_seed_host(host.data() + (size_t)i * UG_MT_WORDS, seed + (uint32_t)env_offset + (uint32_t)i);
    HIPCHK(h, hipMemcpyAsync(h->d_mt, host.data(), sizeof(uint32_t) * host.size(), hipMemcpyHostToDevice, h->stream));
    k_build_scene<<<1, 1, 0, h->stream>>>(h->d_scene, task, flags);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

urgym_handle* urgym_create(int task, int n, int dev, int precision, uint32_t seed, int env_offset) {
    return urgym_create_ex(task, n, dev, precision, seed, env_offset, 0);
}

urgym_handle* urgym_create_ex(int task, int n, int dev, int precision, uint32_t seed, int env_offset, int flags) {
    if ((flags & ~(URGYM_FLAG_FULL_GEOMETRY | URGYM_FLAG_LOD_GEOMETRY | URGYM_FLAG_CONTACT_GJK | URGYM_FLAG_CONTACT_VIH)) ||
        (flags & URGYM_FLAG_FULL_GEOMETRY && flags & URGYM_FLAG_LOD_GEOMETRY) ||
        (flags & URGYM_FLAG_CONTACT_GJK && flags & URGYM_FLAG_CONTACT_VIH)) {
        fail(nullptr, "urgym_create_ex: invalid flags " + std::to_string(flags));
        return nullptr;
    }
    if (task < URGYM_TASK_BALLBALANCE || task > URGYM_TASK_BOX) {
        fail(nullptr, "urgym_create: unknown task " + std::to_string(task));
        return nullptr;
    }
    if (task == URGYM_TASK_BOX && (flags & URGYM_FLAG_LOD_GEOMETRY)) {
        fail(nullptr, "urgym_create_ex: Box-v0 runs the full geometry only (its door handles and button are cylinders)");
        return nullptr;
    }
    if (n <= 0) { fail(nullptr, "urgym_create: n_envs must be > 0"); return nullptr; }
    if (precision != 64) { fail(nullptr, "urgym_create: only precision=64 (FP64) is supported"); return nullptr; }
    urgym_handle* h = new urgym_handle();
    h->task = task; h->n = n; h->dev = dev; h->flags = flags;
    if (create_impl(h, task, n, dev, seed, env_offset, flags) != 0) {
        g_create_error = h->err;
        urgym_destroy(h);
        return nullptr;
    }
    return h;
}

void urgym_destroy(urgym_handle* h) {
    if (!h) return;
    hipSetDevice(h->dev);
    if (h->stream) hipStreamSynchronize(h->stream);
    void* ptrs[] = {h->d_scene, h->d_state, h->d_ws, h->d_mt, h->d_elapsed, h->d_act, h->d_obs, h->d_final, h->d_rew,
                    h->d_draws, h->d_aux, h->d_term, h->d_trunc, h->d_succ, h->d_mask, h->d_sub, h->d_order, h->d_prio,
                    h->d_stats, h->d_flags, h->d_campose, h->d_queue, h->d_order_tmp, h->d_pfeat};
    for (void* p : ptrs)
        if (p) hipFree(p);
    if (h->ev0) hipEventDestroy(h->ev0);
    if (h->ev1) hipEventDestroy(h->ev1);
    if (h->stream) hipStreamDestroy(h->stream);
    delete h;
}

int urgym_set_autoreset(urgym_handle* h, int enable, int max_episode_steps) {
    if (!h) return -1;
    h->autoreset = enable;
    h->max_steps = max_episode_steps;
    return 0;
}

void* urgym_stream(urgym_handle* h) { return h ? (void*)h->stream : nullptr; }
int urgym_sync(urgym_handle* h) {
    if (!h) return -1;
    HIPCHK(h, hipSetDevice(h->dev));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}
double urgym_last_kernel_ms(const urgym_handle* h) {
    if (!h || !h->timed) return -1.0;
    float ms = 0.0f;
    if (hipEventElapsedTime(&ms, h->ev0, h->ev1) != hipSuccess) return -1.0;
    return (double)ms;
}

int urgym_reset_device(urgym_handle* h, const uint8_t* d_mask, const double* d_draws, double* d_obs) {
    if (!h) return -1;
    HIPCHK(h, hipSetDevice(h->dev));
    HIPCHK(h, hipMemsetAsync(h->d_queue, 0, sizeof(int), h->stream));
    HIPCHK(h, hipEventRecord(h->ev0, h->stream));
    k_reset<<<std::min(h->n, h->slots), TEAM, 0, h->stream>>>(h->d_scene, h->d_state, h->d_mt, h->d_elapsed, h->d_ws, h->n,
                                                               d_mask, d_draws, d_obs, nullptr, h->d_stats, h->d_flags,
                                                               h->d_queue);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipEventRecord(h->ev1, h->stream));
    if (h->d_pfeat) {
        k_pfeat_clear<<<grid_of(h->n), WAVE, 0, h->stream>>>(h->d_pfeat, d_mask, h->n);
        HIPCHK(h, hipGetLastError());
    }
    h->timed = true;
    return 0;
}

int urgym_reset(urgym_handle* h, const uint8_t* mask, const double* draws, double* obs) {
    if (!h) return -1;
    if (!obs) return fail(h, "urgym_reset: obs must not be NULL");
    size_t N = (size_t)h->n;
    int O = urgym_obs_dim(h->task);
    HIPCHK(h, hipSetDevice(h->dev));
    if (mask) HIPCHK(h, hipMemcpyAsync(h->d_mask, mask, N, hipMemcpyHostToDevice, h->stream));
    if (draws)
        HIPCHK(h, hipMemcpyAsync(h->d_draws, draws, sizeof(double) * urgym_num_draws(h->task) * N, hipMemcpyHostToDevice,
                                 h->stream));
    // unmasked rows must come back untouched
    HIPCHK(h, hipMemcpyAsync(h->d_obs, obs, sizeof(double) * O * N, hipMemcpyHostToDevice, h->stream));
    if (urgym_reset_device(h, mask ? h->d_mask : nullptr, draws ? h->d_draws : nullptr, h->d_obs) != 0) return -1;
    HIPCHK(h, hipMemcpyAsync(obs, h->d_obs, sizeof(double) * O * N, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int urgym_step_device(urgym_handle* h, const float* d_act, double* d_obs, double* d_final, double* d_rew,
                      uint8_t* d_term, uint8_t* d_trunc, uint8_t* d_succ, int32_t* d_sub) {
    if (!h) return -1;
    if (!d_act || !d_obs) return fail(h, "urgym_step_device: actions and obs must not be NULL");
    HIPCHK(h, hipSetDevice(h->dev));
    /* the launch order: the priorities the envs' last step left (TwoBalls: completed with this step's actions) */
    if (h->d_pfeat) {
        k_prio<<<grid_of(h->n), WAVE, 0, h->stream>>>(h->d_pfeat, d_act, h->d_mt, h->d_prio, h->n);
        HIPCHK(h, hipGetLastError());
    }
    k_order<<<1, ORDER_THREADS, 0, h->stream>>>(h->d_prio, h->d_order, h->d_order_tmp, h->n);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipMemsetAsync(h->d_queue, 0, sizeof(int), h->stream));
    HIPCHK(h, hipEventRecord(h->ev0, h->stream));
    k_step<<<std::min(h->n, h->slots), TEAM, 0, h->stream>>>(h->d_scene, h->d_state, h->d_mt, h->d_elapsed, h->d_ws, h->n,
                                                              d_act, d_obs, d_final, d_rew, d_term, d_trunc, d_succ, d_sub,
                                                              h->autoreset, h->max_steps, h->d_order, h->d_prio,
                                                              h->d_stats, h->d_flags, h->d_queue, h->d_pfeat);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipEventRecord(h->ev1, h->stream));
    h->timed = true;
    return 0;
}

int urgym_step(urgym_handle* h, const float* act, double* obs, double* final_obs, double* rew, uint8_t* term,
               uint8_t* trunc, uint8_t* succ, int32_t* sub) {
    if (!h) return -1;
    if (!act || !obs) return fail(h, "urgym_step: actions and obs must not be NULL");
    size_t N = (size_t)h->n;
    int O = urgym_obs_dim(h->task), A = urgym_act_dim(h->task);
    HIPCHK(h, hipSetDevice(h->dev));
    HIPCHK(h, hipMemcpyAsync(h->d_act, act, sizeof(float) * A * N, hipMemcpyHostToDevice, h->stream));
    if (final_obs)
        HIPCHK(h, hipMemcpyAsync(h->d_final, final_obs, sizeof(double) * O * N, hipMemcpyHostToDevice, h->stream));
    if (urgym_step_device(h, h->d_act, h->d_obs, final_obs ? h->d_final : nullptr, h->d_rew, h->d_term, h->d_trunc,
                          h->d_succ, h->d_sub) != 0)
        return -1;
    HIPCHK(h, hipMemcpyAsync(obs, h->d_obs, sizeof(double) * O * N, hipMemcpyDeviceToHost, h->stream));
    if (final_obs) HIPCHK(h, hipMemcpyAsync(final_obs, h->d_final, sizeof(double) * O * N, hipMemcpyDeviceToHost, h->stream));
    if (rew) HIPCHK(h, hipMemcpyAsync(rew, h->d_rew, sizeof(double) * N, hipMemcpyDeviceToHost, h->stream));
    if (term) HIPCHK(h, hipMemcpyAsync(term, h->d_term, N, hipMemcpyDeviceToHost, h->stream));
    if (trunc) HIPCHK(h, hipMemcpyAsync(trunc, h->d_trunc, N, hipMemcpyDeviceToHost, h->stream));
    if (succ) HIPCHK(h, hipMemcpyAsync(succ, h->d_succ, N, hipMemcpyDeviceToHost, h->stream));
    if (sub) HIPCHK(h, hipMemcpyAsync(sub, h->d_sub, sizeof(int32_t) * N, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int urgym_get_state(urgym_handle* h, double* state) {
    if (!h || !state) return -1;
    size_t tot = (size_t)h->n * UG_STATE_DIM;
    HIPCHK(h, hipSetDevice(h->dev));
    HIPCHK(h, hipMemcpyAsync(state, h->d_state, sizeof(double) * tot, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int urgym_set_state(urgym_handle* h, const double* state) {
    if (!h || !state) return -1;
    size_t tot = (size_t)h->n * UG_STATE_DIM;
    HIPCHK(h, hipSetDevice(h->dev));
    HIPCHK(h, hipMemcpyAsync(h->d_state, state, sizeof(double) * tot, hipMemcpyHostToDevice, h->stream));
    if (h->d_pfeat) {
        k_pfeat_clear<<<grid_of(h->n), WAVE, 0, h->stream>>>(h->d_pfeat, nullptr, h->n);
        HIPCHK(h, hipGetLastError());
    }
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int urgym_substep(urgym_handle* h) {
    if (!h) return -1;
    HIPCHK(h, hipSetDevice(h->dev));
    k_substep<<<h->n, TEAM, 0, h->stream>>>(h->d_scene, h->d_state, h->d_ws, h->n, h->d_stats);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int urgym_link_state(urgym_handle* h, int link, double* out) {
    if (!h || !out) return -1;
    if (link < 0 || link >= UG_NL) return fail(h, "urgym_link_state: link out of range");
    HIPCHK(h, hipSetDevice(h->dev));
    k_link_state<<<grid_of(h->n), WAVE, 0, h->stream>>>(h->d_state, h->n, link, h->d_aux);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipMemcpyAsync(out, h->d_aux, sizeof(double) * 7 * h->n, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int urgym_ik(urgym_handle* h, const double* target, double* q_out) {
    if (!h || !target || !q_out) return -1;
    size_t N = (size_t)h->n;
    HIPCHK(h, hipSetDevice(h->dev));
    double* d_t = h->d_aux;
    double* d_q = h->d_aux + 7 * N;
    HIPCHK(h, hipMemcpyAsync(d_t, target, sizeof(double) * 7 * N, hipMemcpyHostToDevice, h->stream));
    k_ik<<<grid_of(h->n), WAVE, 0, h->stream>>>(h->d_state, h->n, d_t, d_q);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipMemcpyAsync(q_out, d_q, sizeof(double) * NB * N, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int urgym_set_reward_type(urgym_handle* h, int sparse) {
    if (!h) return -1;
    const int v = sparse != 0;
    HIPCHK(h, hipSetDevice(h->dev));
    HIPCHK(h, hipMemcpyAsync((char*)h->d_scene + offsetof(Scene, sparse), &v, sizeof(int), hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int urgym_set_button_mode(urgym_handle* h, int mode) {
    if (!h) return -1;
    if (mode < UG_BX_TOUCH_ANY || mode > UG_BX_TOUCH_FINGERS) return fail(h, "urgym_set_button_mode: unknown mode " + std::to_string(mode));
    HIPCHK(h, hipSetDevice(h->dev));
    HIPCHK(h, hipMemcpyAsync((char*)h->d_scene + offsetof(Scene, button_mode), &mode, sizeof(int), hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int urgym_get_flags(urgym_handle* h, uint8_t* flags) {
    if (!h || !flags) return -1;
    HIPCHK(h, hipSetDevice(h->dev));
    HIPCHK(h, hipMemcpyAsync(flags, h->d_flags, (size_t)h->n, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}
const uint8_t* urgym_flags_device(urgym_handle* h) { return h ? h->d_flags : nullptr; }

int urgym_get_stats(urgym_handle* h, int32_t* stats) {
    if (!h || !stats) return -1;
    HIPCHK(h, hipSetDevice(h->dev));
    HIPCHK(h, hipMemcpyAsync(stats, h->d_stats, sizeof(int32_t) * UG_NSTAT * h->n, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int urgym_get_rng(urgym_handle* h, uint32_t* mt, int32_t* elapsed) {
    if (!h || !mt) return -1;
    HIPCHK(h, hipSetDevice(h->dev));
    HIPCHK(h, hipMemcpyAsync(mt, h->d_mt, sizeof(uint32_t) * UG_MT_WORDS * h->n, hipMemcpyDeviceToHost, h->stream));
    if (elapsed) HIPCHK(h, hipMemcpyAsync(elapsed, h->d_elapsed, sizeof(int) * h->n, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int urgym_set_rng(urgym_handle* h, const uint32_t* mt, const int32_t* elapsed) {
    if (!h || !mt) return -1;
    HIPCHK(h, hipSetDevice(h->dev));
    HIPCHK(h, hipMemcpyAsync(h->d_mt, mt, sizeof(uint32_t) * UG_MT_WORDS * h->n, hipMemcpyHostToDevice, h->stream));
    if (elapsed) HIPCHK(h, hipMemcpyAsync(h->d_elapsed, elapsed, sizeof(int) * h->n, hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int urgym_contact_points(urgym_handle* h, int body_a, int body_b, int link_a, int link_b, int max_pts, double* out,
                         int32_t* count) {
    if (!h || !out || !count || max_pts <= 0) return -1;
    size_t N = (size_t)h->n;
    HIPCHK(h, hipSetDevice(h->dev));
    double* d_out = nullptr;
    int32_t* d_cnt = nullptr;
    HIPCHK(h, hipMalloc(&d_out, sizeof(double) * 24 * (size_t)max_pts * N));
    HIPCHK(h, hipMalloc(&d_cnt, sizeof(int32_t) * N));
    HIPCHK(h, hipMemsetAsync(d_out, 0, sizeof(double) * 24 * (size_t)max_pts * N, h->stream));
    k_contacts<<<grid_of(h->n), WAVE, 0, h->stream>>>(h->d_scene, h->d_state, h->n, body_a, body_b, link_a, link_b,
                                                    max_pts, d_out, d_cnt);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(out, d_out, sizeof(double) * 24 * (size_t)max_pts * N, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(count, d_cnt, sizeof(int32_t) * N, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    hipFree(d_out);
    hipFree(d_cnt);
    if (e != hipSuccess) return fail(h, std::string("urgym_contact_points: ") + hipGetErrorString(e));
    return 0;
}

static int camera_args(urgym_handle* h, int env0, int count, const float* view16, const float* proj16, int width,
                       int height, UgrCam* cam) {
    if (!h) return -1;
    if (!view16 || !proj16) return fail(h, "urgym_camera_shot: view / projection matrix missing");
    if (env0 < 0 || count < 1 || count > 65535 || env0 + count > h->n)
        return fail(h, "urgym_camera_shot: env range [env0, env0 + count) outside the handle's envs (or count > 65535)");
    if (width < 1 || height < 1 || width > 4096 || height > 4096)
        return fail(h, "urgym_camera_shot: image size must be 1..4096 x 1..4096");
    if (ugr_setup(view16, proj16, cam) != 0) return fail(h, "urgym_camera_shot: projection * view is singular");
    return 0;
}

static hipError_t camera_launch(urgym_handle* h, int env0, int count, const UgrCam& cam, int width, int height, int flags,
                                uint8_t* d_rgba, float* d_depth, int32_t* d_seg) {
    if ((size_t)count > h->campose_envs) {
        if (h->d_campose) {
            hipError_t e = hipStreamSynchronize(h->stream);
            if (e == hipSuccess) e = hipFree(h->d_campose);
            h->d_campose = nullptr;
            h->campose_envs = 0;
            if (e != hipSuccess) return e;
        }
        hipError_t e = hipMalloc(&h->d_campose, sizeof(double) * (size_t)count * MAXCOL * CAM_REC);
        if (e != hipSuccess) return e;
        h->campose_envs = (size_t)count;
    }
    k_camera_pose<<<count, WAVE, 0, h->stream>>>(h->d_scene, h->d_state, env0, h->d_campose);
    dim3 grid((unsigned)(((width + 7) / 8) * ((height + 7) / 8)), (unsigned)count);
    k_camera<<<grid, WAVE, 0, h->stream>>>(h->d_scene, h->d_campose, cam, width, height, flags, d_rgba, d_depth, d_seg);
    return hipGetLastError();
}

int urgym_camera_shot_device(urgym_handle* h, int env0, int count, const float* view16, const float* proj16, int width,
                             int height, int flags, uint8_t* d_rgba, float* d_depth, int32_t* d_seg) {
    UgrCam cam;
    if (camera_args(h, env0, count, view16, proj16, width, height, &cam) != 0) return -1;
    HIPCHK(h, hipSetDevice(h->dev));
    HIPCHK(h, camera_launch(h, env0, count, cam, width, height, flags, d_rgba, d_depth, d_seg));
    return 0;
}

int urgym_camera_shot(urgym_handle* h, int env0, int count, const float* view16, const float* proj16, int width,
                      int height, int flags, uint8_t* rgba, float* depth, int32_t* seg) {
    UgrCam cam;
    if (camera_args(h, env0, count, view16, proj16, width, height, &cam) != 0) return -1;
    HIPCHK(h, hipSetDevice(h->dev));
    const size_t np = (size_t)width * (size_t)height * (size_t)count;
    uint8_t* d_rgba = nullptr;
    float* d_depth = nullptr;
    int32_t* d_seg = nullptr;
    hipError_t e = hipSuccess;
    if (rgba) e = hipMalloc(&d_rgba, 4 * np);
    if (e == hipSuccess && depth) e = hipMalloc(&d_depth, sizeof(float) * np);
    if (e == hipSuccess && seg) e = hipMalloc(&d_seg, sizeof(int32_t) * np);
    if (e == hipSuccess) e = camera_launch(h, env0, count, cam, width, height, flags, d_rgba, d_depth, d_seg);
    if (e == hipSuccess && rgba) e = hipMemcpyAsync(rgba, d_rgba, 4 * np, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess && depth) e = hipMemcpyAsync(depth, d_depth, sizeof(float) * np, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess && seg) e = hipMemcpyAsync(seg, d_seg, sizeof(int32_t) * np, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    hipFree(d_rgba);
    hipFree(d_depth);
    hipFree(d_seg);
    if (e != hipSuccess) return fail(h, std::string("urgym_camera_shot: ") + hipGetErrorString(e));
    return 0;
}

// Phase cycle counters of the team kernels (only a -DUG_PROF build records them):
// out16 receives the UG_NPROF (80) accumulators (ug_team.h PF_* / PC_*); reset != 0 zeroes them.
// reset == 2 instead copies the last k_step's block timeline (UG_BT_MAX x 4 words: start / end s_memrealtime,
// env, substeps | reset << 16), tools/timeline.py.
int urgym_debug_prof(urgym_handle* h, unsigned long long* out16, int reset) {
#ifdef UG_PROF
    if (!h || !out16) return -1;
    HIPCHK(h, hipSetDevice(h->dev));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (reset == 2) {
        HIPCHK(h, hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_btime), sizeof(unsigned long long) * 4 * UG_BT_MAX));
        return 0;
    }
    HIPCHK(h, hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_prof), sizeof(unsigned long long) * UG_NPROF));
    if (reset) {
        unsigned long long z[UG_NPROF] = {0};
        HIPCHK(h, hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof(z)));
    }
    return 0;
#else
    (void)h; (void)out16; (void)reset;
    return -1;
#endif
}

// Development aid: copy env's per-env workspace (count doubles from its start) to the host.
int urgym_debug_workspace(urgym_handle* h, int env, double* out, int count) {
    if (!h || !out || env < 0 || env >= h->n || count < 0 || count > (int)WS_STRIDE(UG_GEOM_IS_FULL(h->flags), UG_CONTACT_IS_GJK(h->flags))) return -1;
    HIPCHK(h, hipSetDevice(h->dev));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    HIPCHK(h, hipMemcpy(out, h->d_ws + (size_t)env * WS_STRIDE(UG_GEOM_IS_FULL(h->flags), UG_CONTACT_IS_GJK(h->flags)), sizeof(double) * count, hipMemcpyDeviceToHost));
    return 0;
}
int urgym_debug_ws_doubles(void) { return (int)WS_STRIDE(0, 0); } /* the LOD vertex-in-hull stride */

__global__ void k_cg_branch(const float* act, const uint32_t* mt, int* sel, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) sel[i] = cg_branch(mt, act + (size_t)i * UG_ACT_DIM(UG_TASK_CUBESGRASP), i);
}
int urgym_debug_cg_branch(urgym_handle* h, const float* act, int* sel) {
    if (!h || !act || !sel) return -1;
    if (h->task != URGYM_TASK_CUBESGRASP) return fail(h, "urgym_debug_cg_branch: not a CubesGrasp handle");
    const size_t N = (size_t)h->n;
    HIPCHK(h, hipSetDevice(h->dev));
    HIPCHK(h, hipMemcpyAsync(h->d_act, act, sizeof(float) * UG_ACT_DIM(UG_TASK_CUBESGRASP) * N, hipMemcpyHostToDevice,
                             h->stream));
    k_cg_branch<<<grid_of(h->n), WAVE, 0, h->stream>>>(h->d_act, h->d_mt, h->d_sub, h->n);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipMemcpyAsync(sel, h->d_sub, sizeof(int) * N, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

// Test aid: n convex-convex queries (39 doubles each, k_gjk_query) on device 0; out n x 7, ok n.
int urgym_debug_gjk(int n, const double* q, double* out, int* ok) {
    if (n <= 0 || !q || !out || !ok) return -1;
    double *dq = nullptr, *dout = nullptr;
    int* dok = nullptr;
    ugk::EpaMem* E = nullptr;
    int rc = 0;
    if (hipMalloc(&dq, sizeof(double) * 39 * n) != hipSuccess || hipMalloc(&dout, sizeof(double) * 7 * n) != hipSuccess ||
        hipMalloc(&dok, sizeof(int) * n) != hipSuccess || hipMalloc(&E, sizeof(ugk::EpaMem) * n) != hipSuccess)
        rc = -1;
    if (!rc && hipMemcpy(dq, q, sizeof(double) * 39 * n, hipMemcpyHostToDevice) != hipSuccess) rc = -1;
    if (!rc) {
        hipLaunchKernelGGL(k_gjk_query, dim3((n + GJK_NG - 1) / GJK_NG), dim3(TEAM), 0, 0, dq, n, dout, dok, E);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = -1;
    }
    if (!rc && hipMemcpy(out, dout, sizeof(double) * 7 * n, hipMemcpyDeviceToHost) != hipSuccess) rc = -1;
    if (!rc && hipMemcpy(ok, dok, sizeof(int) * n, hipMemcpyDeviceToHost) != hipSuccess) rc = -1;
    /* hipFree(nullptr) is a no-op: every path frees whatever was allocated */
    hipFree(dq); hipFree(dout); hipFree(dok); hipFree(E);
    return rc;
}

}  // extern "C"
