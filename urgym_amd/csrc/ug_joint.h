/* ug_joint.h -- one-dof links on a fixed base: the Box task's door (revolute) and button (prismatic) of
 * skew-box-button.urdf (env_box_v0.py:80-85).  Shared verbatim by the CPU restatement (oracle/ug_oracle.c) and the
 * HIP kernels (ug_team.h), so both evaluate the same operations in the same order (bit-identical FP64; both
 * sides build with -ffp-contract=off).
 *
 * Such a link is a separate btMultiBody (fixed base, URDF_MERGE_FIXED_LINKS merges the handles into the door),
 * so its equation of motion does not couple to the robot's: ABA (btMultiBody::computeAccelerationsArticulated-
 * BodyAlgorithmMultiDof [ext]) for a single link on a fixed base reduces to  M qdd = -C  with
 *   revolute  (axis a, COM offset r from the joint origin, r_perp^2 = |r|^2 - (a.r)^2):
 *     M = a^T I_w a + m r_perp^2
 *     C = -m g (a_x r_y - a_y r_x)                                (gravity (0, 0, g) at the COM)
 *         + qd a^T I_w a (k_a + k_a |qd|)                         (angular damping, the link's local inertia)
 *         + m qd r_perp^2 (k_l + k_l |qd| r_perp)                 (linear damping at the COM, |v| = |qd| r_perp)
 *   prismatic (axis a):  M = m,  C = -m g a_z + m qd (k_l + k_l |qd|)
 * (the Coriolis / gyroscopic terms of one link about a fixed axis project to zero and are not formed;
 * DAMPING_K1 = DAMPING_K2 = 0.04, btMultiBody's defaults [ext]).
 * Its link frame follows the joint: revolute btQuaternion(axis, q) about the joint origin (the rotation of
 * btMultiBody's m_cachedRotParentToThis, inverted), prismatic the joint origin + q axis.
 * The generalized velocity of such a link occupies the first of its object's six solver slots (the other five
 * stay zero): a row's Jacobian is J = d . (a x (p - o)) (revolute) or d . a (prismatic) for a point p along d,
 * u . a (revolute) or 0 (prismatic) for an angular row about u, and M^-1 J^T = J / M.
 */
#ifndef UG_JOINT_H
#define UG_JOINT_H

#include "ug_detmath.h"

#define UGJ_FREE 0
#define UGJ_REVOLUTE 1
#define UGJ_PRISMATIC 2

typedef struct {
    int kind;          /* UGJ_REVOLUTE / UGJ_PRISMATIC (UGJ_FREE: a free body, none of this applies) */
    double anchor[3];  /* joint origin, world (the fixed base does not move) */
    double axis[3];    /* unit joint axis, world */
    double mass;
    double com[3];     /* centre of mass in the link frame */
    double inertia[3]; /* principal inertia at the COM in the link frame's axes */
    double lower, upper;
} UgJoint;

/* btMatrix3x3::setRotation of (x, y, z, w), row-major (the same operations as the restatement's qmat) */
UG_HD void ugj_qmat(const double* q, double* R) {
    double d = q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
    double s = 2.0 / d;
    double xs = q[0] * s, ys = q[1] * s, zs = q[2] * s;
    double wx = q[3] * xs, wy = q[3] * ys, wz = q[3] * zs;
    double xx = q[0] * xs, xy = q[0] * ys, xz = q[0] * zs;
    double yy = q[1] * ys, yz = q[1] * zs, zz = q[2] * zs;
    R[0] = 1.0 - (yy + zz); R[1] = xy - wz; R[2] = xz + wy;
    R[3] = xy + wz; R[4] = 1.0 - (xx + zz); R[5] = yz - wx;
    R[6] = xz - wy; R[7] = yz + wx; R[8] = 1.0 - (xx + yy);
}

/* link frame at joint position q: quaternion (x, y, z, w) and origin (world) */
UG_HD void ugj_frame(const UgJoint* J, double q, double* quat, double* pos) {
    if (J->kind == UGJ_REVOLUTE) {
        double h = q * 0.5, s = ug_sin(h);
        quat[0] = J->axis[0] * s; quat[1] = J->axis[1] * s; quat[2] = J->axis[2] * s; quat[3] = ug_cos(h);
        pos[0] = J->anchor[0]; pos[1] = J->anchor[1]; pos[2] = J->anchor[2];
    } else {
        quat[0] = 0.0; quat[1] = 0.0; quat[2] = 0.0; quat[3] = 1.0;
        pos[0] = J->anchor[0] + J->axis[0] * q; pos[1] = J->anchor[1] + J->axis[1] * q; pos[2] = J->anchor[2] + J->axis[2] * q;
    }
}

/* equation of motion at (frame, qd): effective inertia *M and bias *C (header comment); g = gravity along z */
UG_HD void ugj_dynamics(const UgJoint* J, const double* quat, double qd, double g, double* M, double* C) {
    const double kl = 0.04, ka = 0.04; /* UG_LIN_DAMP, UG_ANG_DAMP */
    const double m = J->mass;
    const double aqd = ug_fabs(qd);
    if (J->kind == UGJ_REVOLUTE) {
        double R[9];
        ugj_qmat(quat, R);
        const double* a = J->axis;
        const double* c = J->com;
        double r0 = R[0] * c[0] + R[1] * c[1] + R[2] * c[2];
        double r1 = R[3] * c[0] + R[4] * c[1] + R[5] * c[2];
        double r2 = R[6] * c[0] + R[7] * c[1] + R[8] * c[2];
        /* a^T R diag(I) R^T a */
        double u0 = R[0] * a[0] + R[3] * a[1] + R[6] * a[2];
        double u1 = R[1] * a[0] + R[4] * a[1] + R[7] * a[2];
        double u2 = R[2] * a[0] + R[5] * a[1] + R[8] * a[2];
        double Ia = J->inertia[0] * (u0 * u0) + J->inertia[1] * (u1 * u1) + J->inertia[2] * (u2 * u2);
        double ar = a[0] * r0 + a[1] * r1 + a[2] * r2;
        double rr = r0 * r0 + r1 * r1 + r2 * r2;
        double rp2 = rr - ar * ar;
        rp2 = rp2 > 0.0 ? rp2 : 0.0;
        *M = Ia + m * rp2;
        double tg = m * g * (a[0] * r1 - a[1] * r0);
        double dang = qd * Ia * (ka + ka * aqd);
        double dlin = m * qd * rp2 * (kl + kl * (aqd * ug_sqrt(rp2)));
        *C = (-tg + dang) + dlin;
    } else {
        *M = m;
        *C = -(m * g * J->axis[2]) + m * qd * (kl + kl * aqd);
    }
}

/* Jacobian of a world point p along direction d (linear rows) */
UG_HD double ugj_point_jac(const UgJoint* J, const double* p, const double* d) {
    if (J->kind == UGJ_REVOLUTE) {
        const double* a = J->axis;
        double x0 = p[0] - J->anchor[0], x1 = p[1] - J->anchor[1], x2 = p[2] - J->anchor[2];
        double c0 = a[1] * x2 - a[2] * x1, c1 = a[2] * x0 - a[0] * x2, c2 = a[0] * x1 - a[1] * x0;
        return d[0] * c0 + d[1] * c1 + d[2] * c2;
    }
    return d[0] * J->axis[0] + d[1] * J->axis[1] + d[2] * J->axis[2];
}
/* Jacobian of the angular velocity along u (rolling-friction rows) */
UG_HD double ugj_ang_jac(const UgJoint* J, const double* u) {
    if (J->kind == UGJ_REVOLUTE) return u[0] * J->axis[0] + u[1] * J->axis[1] + u[2] * J->axis[2];
    return 0.0;
}

#ifdef UG_BX_ROBOT_Y /* scene_data.h: the Box task's two links */
/* h3's fixed joint rpy (1.57079632679, 0, 0) on h2 (URDF :218-223): UrdfParser's setEulerZYX(0, 0, roll) */
UG_HD void ugj_box_h3_quat(double* q) {
    double h = 1.57079632679 * 0.5;
    q[0] = ug_sin(h); q[1] = 0.0; q[2] = 0.0; q[3] = ug_cos(h);
}
/* the door (joint 1) and button (joint 0) links of skew-box-button.urdf in the restatement's frame (robot base at
 * the origin: the box base sits at (0, -UG_BX_ROBOT_Y, 0)).  URDF_MERGE_FIXED_LINKS [ext]: the door's mass is
 * the sum of door, h1, h2, h3 and its centre of mass their weighted mean (URDF order); the inertia is not read
 * from the URDF (no URDF_USE_INERTIA_FROM_FILE): btCompoundShape::calculateLocalInertia of the merged collision
 * compound, i.e. the box spanned by the compound's AABB in the inertial frame (COM origin, link axes). */
UG_HD void ugj_box_links(UgJoint* door, UgJoint* button) {
    const double by = -UG_BX_ROBOT_Y;
    door->kind = UGJ_REVOLUTE;
    door->anchor[0] = UG_BX_DOOR_X; door->anchor[1] = by; door->anchor[2] = UG_BX_DOOR_Z;
    door->axis[0] = 0.0; door->axis[1] = 1.0; door->axis[2] = 0.0;
    const double* mm = UG_BX_DOOR_MASSES;
    double m = ((mm[0] + mm[1]) + mm[2]) + mm[3];
    /* link COMs in the door frame: door at its origin, the handles at their centres */
    double cx[4] = {0.0, UG_BX_HANDLE[0], UG_BX_HANDLE[4], UG_BX_HANDLE[8]};
    double cy[4] = {0.0, UG_BX_HANDLE[1], UG_BX_HANDLE[5], UG_BX_HANDLE[9]};
    double cz[4] = {0.0, UG_BX_HANDLE[2], UG_BX_HANDLE[6], UG_BX_HANDLE[10]};
    double sx = 0.0, sy = 0.0, sz = 0.0;
    for (int i = 0; i < 4; i++) { sx = sx + mm[i] * cx[i]; sy = sy + mm[i] * cy[i]; sz = sz + mm[i] * cz[i]; }
    door->mass = m;
    door->com[0] = sx / m; door->com[1] = sy / m; door->com[2] = sz / m;
    /* compound AABB (door frame): the door box and the three handle cylinders (h3 lies along y) */
    const double* B = UG_BX_DOOR_BOX;
    double lo[3] = {B[0] - B[3], B[1] - B[4], B[2] - B[5]}, hi[3] = {B[0] + B[3], B[1] + B[4], B[2] + B[5]};
    for (int i = 0; i < 3; i++) {
        const double* H = &UG_BX_HANDLE[4 * i];
        double r = H[3], hh = UG_BX_HANDLE_HH[i];
        double e[3] = {r, i == 2 ? hh : r, i == 2 ? r : hh};
        for (int k = 0; k < 3; k++) {
            double l = H[k] - e[k], u = H[k] + e[k];
            lo[k] = l < lo[k] ? l : lo[k];
            hi[k] = u > hi[k] ? u : hi[k];
        }
    }
    double L[3];
    for (int k = 0; k < 3; k++) L[k] = 2.0 * ((hi[k] - lo[k]) * 0.5);
    door->inertia[0] = m / 12.0 * (L[1] * L[1] + L[2] * L[2]);
    door->inertia[1] = m / 12.0 * (L[0] * L[0] + L[2] * L[2]);
    door->inertia[2] = m / 12.0 * (L[0] * L[0] + L[1] * L[1]);
    door->lower = UG_BX_DOOR_LO; door->upper = UG_BX_DOOR_HI;

    button->kind = UGJ_PRISMATIC;
    button->anchor[0] = 0.0; button->anchor[1] = by; button->anchor[2] = UG_BX_BUTTON_Z;
    button->axis[0] = 0.0; button->axis[1] = 0.0; button->axis[2] = 1.0;
    button->mass = UG_BX_BUTTON_MASS;
    button->com[0] = button->com[1] = button->com[2] = 0.0;
    double bl[3] = {2.0 * UG_BX_BUTTON_R, 2.0 * UG_BX_BUTTON_R, 2.0 * UG_BX_BUTTON_HH};
    button->inertia[0] = UG_BX_BUTTON_MASS / 12.0 * (bl[1] * bl[1] + bl[2] * bl[2]);
    button->inertia[1] = UG_BX_BUTTON_MASS / 12.0 * (bl[0] * bl[0] + bl[2] * bl[2]);
    button->inertia[2] = UG_BX_BUTTON_MASS / 12.0 * (bl[0] * bl[0] + bl[1] * bl[1]);
    button->lower = UG_BX_BUTTON_LO; button->upper = UG_BX_BUTTON_HI;
}
/* angular motion disc of a compound (btCollisionShape::getAngularMotionDisc: |AABB centre| + half diagonal) from
 * its AABB in the collision-object frame */
UG_HD double ugj_disc(const double* lo, const double* hi) {
    double c0 = (lo[0] + hi[0]) * 0.5, c1 = (lo[1] + hi[1]) * 0.5, c2 = (lo[2] + hi[2]) * 0.5;
    double h0 = (hi[0] - lo[0]) * 0.5, h1 = (hi[1] - lo[1]) * 0.5, h2 = (hi[2] - lo[2]) * 0.5;
    return ug_sqrt(c0 * c0 + c1 * c1 + c2 * c2) + ug_sqrt(h0 * h0 + h1 * h1 + h2 * h2);
}
#endif

#endif
