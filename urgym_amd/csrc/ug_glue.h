/* ug_glue.h -- the tasks' pure scalar glue (rewards, subgoals, draws -> placements, action choice),
 * shared verbatim by the CPU restatement (oracle/ug_oracle.c) and the HIP kernels (ug_team.h), and
 * pinned against the reference's own Python glue by tests/golden (tools/gen_golden.py).
 * Inputs are the physics-derived quantities the reference queries through pybullet (contact
 * predicates, poses, gripper geometry); the arithmetic order follows the cited Python lines.
 */
#ifndef UG_GLUE_H
#define UG_GLUE_H

#include "ug_detmath.h"

/* geometric_distance_reward (utilities.py:192-207) */
UG_HD double ugg_gdr(double value, double ts, double tm) {
    value = value > 1e-10 ? value : 1e-10;
    double f1 = (value - ts) / value;
    double f2 = (tm - value) > 1e-10 ? (tm - value) : 1e-10;
    return -ug_tanh(f1 / f2);
}

/* get_gripper_geometrical_center (env_ball_balance_v0.py:249-275): centre of the union of two AABBs */
UG_HD void ugg_union_center(const double* lo1, const double* hi1, const double* lo2, const double* hi2, double* c) {
    for (int i = 0; i < 3; i++) {
        double lo = lo1[i] < lo2[i] ? lo1[i] : lo2[i];
        double hi = hi1[i] > hi2[i] ? hi1[i] : hi2[i];
        c[i] = (hi + lo) / 2.0;
    }
}

/* random.uniform(a, b) = a + (b - a) * random() */
UG_HD double ugg_uniform(double a, double b, double u) { return a + (b - a) * u; }

/* ---- TwoBallsBalance (env_two_balls_balance_v0.py) ---- */
/* create_balls (:212-223): ball 1 at the paddle + (U(-0.03, 0.03), U(-0.08, -0.045), 0.2 + r), ball 2 at the
 * paddle + (U(-0.03, 0.03), U(-0.015, 0.02), 0.2 - r); draws in that order (b1x, b1y, b2x, b2y) */
UG_HD void ugg_tb_balls(const double* paddle, double r, const double* u, double* b1, double* b2) {
    b1[0] = paddle[0] + ugg_uniform(-0.03, 0.03, u[0]);
    b1[1] = paddle[1] + ugg_uniform(-0.08, -0.045, u[1]);
    b1[2] = paddle[2] + 0.2 + r;
    b2[0] = paddle[0] + ugg_uniform(-0.03, 0.03, u[2]);
    b2[1] = paddle[1] + ugg_uniform(-0.015, 0.02, u[3]);
    b2[2] = paddle[2] + 0.2 - r;
}
/* reward_function (:148-151): 0 beyond 1, else 1 - x**2 */
UG_HD double ugg_tb_rf(double x) { return x > 1.0 ? 0.0 : 1.0 - x * x; }
/* step reward (:110-139): -|a_i| per action component, +1, then reward_function of |x|, |y| of each ball's
 * world position.  numpy 1.26 promotion (setup.py pins numpy 1.26.4): the float32 action components enter a
 * float64 sum (Python int 0 + numpy float32 scalar -> float64).  Returns terminated (a ball below the paddle). */
UG_HD int ugg_tb_reward(const float* a, const double* b1, const double* b2, double paddle_z, double* reward) {
    double r = 0.0;
    for (int i = 0; i < 3; i++) r = r + -ug_fabs((double)a[i]);
    r = r + 1.0;
    r = r + ugg_tb_rf(ug_fabs(b1[0]));
    r = r + ugg_tb_rf(ug_fabs(b1[1]));
    r = r + ugg_tb_rf(ug_fabs(b2[0]));
    r = r + ugg_tb_rf(ug_fabs(b2[1]));
    *reward = r;
    return b1[2] < paddle_z || b2[2] < paddle_z;
}

/* ---- CubesPush (env_cubes_push_v0.py) ---- */
/* create_cubes (:240-246): second cube x = uniform(-0.1, 0.1) */
UG_HD double ugg_cp_cube1_x(double u) { return ugg_uniform(-0.1, 0.1, u); }
/* step reward (:129-150 with update_reward :152-165); sparse (reward_type != 'dense', :159) drops the
 * distance shaping term; returns success */
UG_HD int ugg_cp_reward(int table_contact, int touched, double c0x, double c0y, double c0z, double c1x, double c1y,
                        double c1z, int sparse, double* reward) {
    double r = 0.0;
    int success = 0;
    if (table_contact) {
        r -= 0.01;
    } else if (touched) {
        double dist = ug_norm3(c0x - c1x, c0y - c1y, c0z - c1z);
        double ur = 0.0;
        if (!sparse) ur += ugg_gdr(dist, 0.1, 0.5) / 10.0;
        if (dist < 0.05) { ur += 10.0; success = 1; }
        r = ur + 0.1;
    }
    r -= 0.1;
    *reward = r;
    return success;
}

/* ---- CubesGrasp (env_cubes_grasp_v0.py) ---- */
/* create_cubes (:310-330): r = uniform(0.5, 0.8), theta = uniform(-pi, 0), (r cos theta, r sin theta, 0.1) */
UG_HD void ugg_cg_cube_xy(double u0, double u1, double* x, double* y) {
    double r = ugg_uniform(0.5, 0.8, u0);
    double th = ugg_uniform(-UG_PI, 0.0, u1);
    *x = r * ug_cos(th);
    *y = r * ug_sin(th);
}
/* random.choices([0, 1], weights=[w0, w1], k=1) (:141-147) with numpy 1.26 scalar promotion: float32
 * cumulative weights, total promoted to float64, x = random() * total, bisect_right */
UG_HD int ugg_cg_choose(float w0, float w1, double u) {
    float sum = w0 + w1;
    if (sum == 0.0f) return u * 1.0 < 0.5 ? 0 : 1;
    double x = u * ((double)sum + 0.0);
    return x < (double)w0 ? 0 : 1;
}
/* get_gripper_opening_length (:349-376) from the distance of link frames 11 and 16 */
UG_HD double ugg_cg_opening(double frame_dist) {
    double v = frame_dist - 0.052;
    double lo = 0.0, hi = 0.085;
    double t = v < hi ? v : hi;  /* min(max_opening, value) */
    v = t > lo ? t : lo;         /* max(min_opening, ...) */
    return (v - lo) / (hi - lo);
}
/* step reward and subgoal update (:156-192); flags in/out; returns success */
UG_HD int ugg_cg_reward(int* approached, int* grasped, double dist, double opening, int grasp_contact, double cube_z,
                        double* reward) {
    double r = 0.0;
    int success = 0;
    if (!*approached) {
        r += ugg_gdr(dist, 0.5, 2.0) / 4.0;
        if (dist < 0.05 && opening > 0.50) { *approached = 1; r += 5.0; }
    } else if (!*grasped) {
        if (grasp_contact) { *grasped = 1; r += 5.0; }
    } else if (grasp_contact && cube_z > 0.2) {
        r += 10.0;
        success = 1;
    }
    r -= 0.1;
    *reward = r;
    return success;
}

/* ---- Golf (env_golf_v0.py) ---- */
/* create_ball (:335-343): (0 + uniform(-0.2, 0.2), -0.7 + uniform(-0.1, 0.1), 0.1) */
UG_HD void ugg_gf_ball_xy(double u0, double u1, double* x, double* y) {
    *x = 0.0 + ugg_uniform(-0.2, 0.2, u0);
    *y = -0.7 + ugg_uniform(-0.1, 0.1, u1);
}
/* step reward, termination precedence (:129-183); hole = pitch base position; sparse (reward_type != 'dense',
 * :151, :163) drops both distance shaping terms; returns success */
UG_HD int ugg_gf_reward(const double* ball, const double* hole, const double* stick, int in_fingers, int floor_contact,
                        int touched, int sparse, double* reward, int* terminated) {
    double r = 0.0;
    int success = 0, term = 0;
    if (ug_norm3(hole[0] - ball[0], hole[1] - ball[1], hole[2] - ball[2]) < 0.05) { /* is_ball_in_hole :217-221 */
        r += 10.0;
        success = 1;
        term = 1;
    } else if (!in_fingers) { /* stick fell :136-140 */
        r -= 5.0;
        term = 1;
    } else if (ball[2] < 0.0) { /* ball off pitch :141-145, :224-228 */
        r -= 10.0;
        term = 1;
    } else {
        if (floor_contact) r -= 0.01;
        if (!sparse) {
            double d = ug_norm3(stick[0] - ball[0], stick[1] - ball[1], stick[2] - ball[2]);
            r += ugg_gdr(d, 0.1, 0.5) / 10.0;
        }
        if (touched) {
            r += 0.1;
            if (!sparse) {
                double dh = ug_norm3(hole[0] - ball[0], hole[1] - ball[1], hole[2] - ball[2]);
                r += ugg_gdr(dh, 0.1, 0.5) / 10.0;
            }
        }
    }
    r -= 0.1;
    *reward = r;
    *terminated = term;
    return success;
}
/* get_observation (:230-236): stick base (link 0 COM), stick - ball, hole - ball */
UG_HD void ugg_gf_obs(const double* stick, const double* ball, const double* hole, double* obs) {
    for (int i = 0; i < 3; i++) {
        obs[i] = stick[i];
        obs[3 + i] = stick[i] - ball[i];
        obs[6 + i] = hole[i] - ball[i];
    }
}

/* ---- Box (env_box_v0.py) ---- */
/* step head (:125): get_ee_pose() + action[:-1] -- the 7-tuple (world pose) plus the float32 action components, a
 * float64 array (numpy 1.26 promotion) */
UG_HD void ugg_box_target(const double* ee7, const float* a, double* t7) {
    for (int i = 0; i < 7; i++) t7[i] = ee7[i] + (double)a[i];
}
/* update_reward (:141-159) with the step penalty (:138): the state machine opened -> button pressed -> closed again;
 * flags in/out; returns box_closed (terminated and is_success, :132, :136) */
UG_HD int ugg_box_reward(int* opened, int* pressed, int* closed, double door, int button_press, double* reward) {
    double r = 0.0;
    if (!*opened) {
        if (door > 1.9) { *opened = 1; r = 1.0; }
    } else if (!*pressed) {
        if (button_press) { *pressed = 1; r = 1.0; }
    } else if (*opened && door < 0.1) {
        *closed = 1;
        r = 1.0;
    }
    r -= 0.1;
    *reward = r;
    return *closed;
}
/* valid_button_press (:191-216): the button joint below -0.02 and, unless the mode is 'any', a contact between the
 * button and the robot ('robot') or one of its finger links 9..18 ('fingers') */
UG_HD int ugg_box_press(double button, int mode, int robot_touch, int finger_touch) {
    if (!(button < -0.02)) return 0;
    if (mode == 0) return 1;
    return mode == 1 ? robot_touch : finger_touch;
}

#endif
