/* scene_data.h -- per-task scene constants (data, not code), restated from the
 * reference env files and PyBullet defaults.  Shared as *input data* by the CPU
 * restatement (oracle/) and the HIP kernels.  Every number cites its source;
 * [ext] marks a PyBullet/Bullet default that cannot be checked in this build
 * (SURVEY.md Appendix A).
 */
#ifndef URGYM_SCENE_DATA_H
#define URGYM_SCENE_DATA_H
#ifndef UG_CONST
#define UG_CONST static const
#endif

/* ---- world / solver (PyBullet defaults, none overridden by the reference) ---- */
#define UG_DT (1.0 / 240.0)            /* fixed 240 Hz step [ext], env_*:SIMULATION_STEP_DELAY */
#define UG_PGS_ITERS 50                /* m_numIterations [ext] */
#define UG_RESIDUAL_THR 1e-7           /* m_leastSquaresResidualThreshold [ext] */
#define UG_ERP 0.2                     /* m_erp (joints, shallow contacts) [ext] */
#define UG_ERP2 0.08                   /* m_erp2 (deep-penetration split impulse) [ext] */
#define UG_SPLIT_PEN_THR (-0.04)       /* m_splitImpulsePenetrationThreshold [ext] */
#define UG_WARMSTART 0.1               /* m_warmstartingFactor [ext] */
#define UG_LINEAR_SLOP 0.00001         /* m_linearSlop [ext] */
#define UG_REST_VEL_THR 0.2            /* m_restitutionVelocityThreshold [ext] */
#define UG_CONTACT_BREAK 0.02          /* gContactBreakingThreshold (relative to shape size) [ext] */
#define UG_AABB_PAD 0.02               /* broadphase AABB padding [ext] */
#define UG_LIN_DAMP 0.04               /* btMultiBody default linear damping [ext] */
#define UG_ANG_DAMP 0.04               /* btMultiBody default angular damping [ext] */
#define UG_MAX_FRICTION 10.0           /* MAX_FRICTION clamp of the combined friction [ext] */
#define UG_ANGULAR_MOTION_THR (0.5 * 1.5707963267948966)   /* ANGULAR_MOTION_THRESHOLD [ext] */
#define UG_MOTOR_KP 0.1                /* pybullet positionGain default [ext] */
#define UG_MOTOR_KD 1.0                /* pybullet velocityGain default [ext] */
#define UG_GEAR_MAXF 100.0             /* robot.py:211 maxForce=100 */
#define UG_GEAR_ERP 1.0                /* robot.py:211 erp=1 */
#define UG_LIMIT_MAXIMP 100.0          /* btMultiBodyJointLimitConstraint default max impulse [ext] */
#define UG_STABLE_STEPS 480            /* env_ball_balance_v0.py:94 sim_steps=480 */
#define UG_STABLE_EPS 5e-3             /* env_ball_balance_v0.py:100 */
#define UG_IK_ITERS 20                 /* robot.py:121 maxNumIterations=20 */
#define UG_IK_RESIDUAL 1e-4            /* pybullet IK residualThreshold default [ext] */
#define UG_IK_DAMPING 0.5              /* PhysicsServer IK joint damping default [ext] */
#define UG_IK_MAXANGLE (45.0 * 3.14159265358979311600e+00 / 180.0)  /* BussIK MaxAngleDLS [ext] */

/* ---- gripper (robot.py:188, 213-218; gear table robot.py:194-211) ---- */
#define UG_GRIP_MIN 0.0
#define UG_GRIP_MAX 0.085
#define UG_FINGER_DOF 6                /* finger_joint = link 9 = dof 6 */
/* constraints are created in joint-id order (robot.py:202 iterates self.joints): links 11,13,14,16,18
 * = dofs 7,8,9,10,11; gearRatio = -multiplier (robot.py:196-200, 211) */
UG_CONST int UG_GEAR_CHILD[5] = {7, 8, 9, 10, 11};
UG_CONST double UG_GEAR_RATIO[5] = {1.0, -1.0, -1.0, 1.0, -1.0};

/* ---- task ids (urgym/envs/__init__.py) ---- */
#define UG_TASK_BALLBALANCE 0
#define UG_TASK_CUBESPUSH 1
#define UG_TASK_CUBESGRASP 2
#define UG_TASK_GOLF 3
/* variants: same scene and physics as their base task, different step/obs glue */
#define UG_TASK_CUBESPUSHDIFF 4 /* env_cubes_push_diff_v0.py: obs = ee, cube - ee (x2) */
#define UG_TASK_GOLFJOINTS 5    /* env_golf_joints_v0.py: joint-space action[6], obs = joints + Golf obs */
#define UG_TASK_TWOBALLS 6      /* env_two_balls_balance_v0.py: BallBalance robot + paddle, two balls r 0.003 */
#define UG_NTASK 7
#define UG_BASE_TASK(t) ((t) == UG_TASK_CUBESPUSHDIFF ? UG_TASK_CUBESPUSH : \
                         ((t) == UG_TASK_GOLFJOINTS ? UG_TASK_GOLF : ((t) == UG_TASK_TWOBALLS ? UG_TASK_BALLBALANCE : (t))))
#define UG_OBS_DIM(t) ((t) == 0 ? 6 : ((t) == 2 ? 17 : ((t) == 5 ? 15 : 9)))
#define UG_ACT_DIM(t) ((t) == 2 ? 9 : ((t) == 5 ? 6 : 3))
#define UG_NDRAW(t) ((t) == 1 || (t) == 4 ? 1 : ((t) == 6 ? 4 : 2))

/* ---- shapes ---- */
#define UG_SHAPE_BOX 0
#define UG_SHAPE_HULL 1
#define UG_SHAPE_SPHERE 2
#define UG_SHAPE_CYL 3 /* full geometry: the Golf club's disc as a true cylinder (radius half[0], half height half[2],
                        * axis z of the shape frame; its outer surface, the safe margin included) */

/* statics: plane.urdf = 30x30x10 box, top at the load height, lateral friction 1 [ext];
 * table = box 1 x 2 x 0.5 centred at (0,0,-0.25) (env_ball_balance_v0.py:69-71, 216-247);
 * golf pitch = convex hull of golf_pitch.obj = 0.8 x 0.8 x 0.05 box at (0,-0.6,0.02) (env_golf_v0.py:87, 428-446) */
#define UG_PLANE_HALF_XY 15.0
#define UG_PLANE_HALF_Z 5.0
#define UG_PLANE_FRICTION 1.0
#define UG_DEFAULT_FRICTION 0.5        /* btCollisionObject / URDF default lateral friction [ext] */
#define UG_URDF_MARGIN 0.001           /* gUrdfDefaultCollisionMargin [ext] */

/* BallBalance (env_ball_balance_v0.py) */
#define UG_BB_PADDLE_HX 0.05           /* :177 halfExtents */
#define UG_BB_PADDLE_HY 0.1
#define UG_BB_PADDLE_HZ 0.005
#define UG_BB_PADDLE_MASS 0.1          /* :183 */
#define UG_BB_BALL_R 0.02              /* :186 */
#define UG_BB_BALL_MASS 0.01           /* :202 */
/* TwoBallsBalance (env_two_balls_balance_v0.py): same paddle; create_balls(0.003) (:187) -> two spheres of
 * radius 0.003, 0.01 kg (:213-233), ball 1 at +0.2 + r, ball 2 at +0.2 - r above the paddle */
#define UG_TB_BALL_R 0.003

/* CubesPush / CubesGrasp: cube.urdf x 0.04 (mass 1, lateral friction 1) [ext] */
#define UG_CUBE_HALF 0.02
#define UG_CUBE_MASS 1.0
#define UG_CUBE_FRICTION 1.0

/* "vertical" EE orientation = quaternion_multiply((0,0,0,1), getQuaternionFromAxisAngle([0,1,0], pi/2))
 * (env_cubes_push_v0.py:222-223, utilities.py:134-174): (0, sin(pi/4), 0, cos(pi/4)) with the libm
 * values Bullet's btQuaternion::setRotation produces */
#define UG_VQ_S 0.7071067811865475
#define UG_VQ_C 0.7071067811865476

/* CubesPush (env_cubes_push_v0.py) */
#define UG_CP_RADIUS 0.1               /* :90 positive_reward_radius */
#define UG_CP_DMAX 0.5                 /* :156 geometric_distance_reward(d, 0.1, 0.5) / 10 */
#define UG_CP_CLOSE 0.05               /* :159 are_cubes_close(..., 0.05) */
#define UG_CP_EE_DZ 0.2                /* :220 */

/* CubesGrasp (env_cubes_grasp_v0.py) */
#define UG_CG_RAISE 0.2                /* :20 OBJECT_RAISE_HEIGHT */
#define UG_CG_APPROACH 0.05            /* :209 */
#define UG_CG_OPEN_MIN 0.50            /* :209 */
#define UG_CG_OPEN_OFF 0.052           /* :359 */
#define UG_CG_RMIN 0.5                 /* :313 */
#define UG_CG_RMAX 0.8                 /* :314 */

/* Golf (env_golf_v0.py).  Club = multibody: base box 0.03x0.03x0.15 (1 kg), fixed links: box 0.1x0.03x0.03
 * (1 kg) at z -0.09 and cylinder r 0.04 h 0.01 (1 kg) at z +0.08 (:289-332); base friction 10, restitution
 * 0.1 (:330).  Restated as one rigid body at the composite COM with the composite (diagonal) inertia. */
#define UG_GF_BASE_HX 0.015
#define UG_GF_BASE_HZ 0.075
#define UG_GF_FOOT_HX 0.05
#define UG_GF_FOOT_HY 0.015
#define UG_GF_FOOT_Z (-(0.075 + 0.015)) /* :309 -(vertical/2 + transversal/2) */
#define UG_GF_DISC_Z (0.075 + 0.005)    /* :310 vertical/2 + disc/2 */
#define UG_GF_PART_MASS 1.0
#define UG_GF_ZC ((0.0 + UG_GF_FOOT_Z + UG_GF_DISC_Z) / 3.0) /* composite COM height in the base frame */
#define UG_GF_BASE_FRICTION 10.0
#define UG_GF_BASE_RESTITUTION 0.1
/* ball (:335-358): r 0.015, 0.01 kg, rolling friction 10, restitution 0.1, default lateral friction */
#define UG_GF_BALL_R 0.015
#define UG_GF_BALL_MASS 0.01
#define UG_GF_BALL_ROLLING 10.0
#define UG_GF_BALL_RESTITUTION 0.1
/* pitch (:87, 428-446): convex hull of golf_pitch.obj = 0.8 x 0.8 x 0.05 slab at (0, -0.6, 0.02), static;
 * mesh hull margin outside -> box half extents + margin */
#define UG_GF_PITCH_X 0.0
#define UG_GF_PITCH_Y (-0.6)
#define UG_GF_PITCH_Z 0.02
#define UG_GF_PITCH_HX 0.4
#define UG_GF_PITCH_HZ 0.025

#endif
