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
/* Box (env_box_v0.py, skew-box-button.urdf loaded with URDF_MERGE_FIXED_LINKS | URDF_USE_SELF_COLLISION, fixed base
 * at the origin, :80-85).  The robot stands at (0, 0.5, 0) (:55); the restatement keeps the robot base at its own
 * origin, so every world position of this task is stored shifted by -UG_BX_ROBOT_Y (observations and IK targets
 * convert, as PyBullet's base transform does).  Gravity -10 (:60), plane.urdf at z = 0 (:65), no table. */
#define UG_BX_ROBOT_Y 0.5
#define UG_BX_STEPS 120                /* :128 for _ in range(120): step_simulation() */
#define UG_BX_OPENED 1.9               /* :144 door joint > 1.9 */
#define UG_BX_CLOSED 0.1               /* :155 door joint < 0.1 */
#define UG_BX_PRESSED (-0.02)          /* :193 button joint < -0.02 */
#define UG_BX_BUTTON_FORCE 1.0         /* :175 setJointMotorControl2(box, 0, POSITION_CONTROL, force=1), target 0 */
/* merged base_link: walls box1..box4 (URDF :14-118), box half extents / centres in the box base frame */
UG_CONST double UG_BX_WALL_HALF[12] = {0.005, 0.1, 0.045, 0.005, 0.1, 0.045, 0.075, 0.005, 0.045, 0.075, 0.005, 0.045};
UG_CONST double UG_BX_WALL_POS[12] = {0.075, 0.0, 0.045, -0.075, 0.0, 0.045, 0.0, 0.1, 0.045, 0.0, -0.1, 0.045};
/* door link (revolute about y at (0.075, 0, 0.1), limits [0, 2], URDF :120-147) merged with its fixed handles
 * h1, h2 (cylinders r 0.005, length 0.05) and h3 (r 0.01, length 0.1, rpy (pi/2, 0, 0) on h2) (:149-223) */
#define UG_BX_DOOR_X 0.075
#define UG_BX_DOOR_Z 0.1
#define UG_BX_DOOR_LO 0.0
#define UG_BX_DOOR_HI 2.0
UG_CONST double UG_BX_DOOR_BOX[6] = {-0.076, 0.0, 0.0, 0.08, 0.1, 0.005}; /* centre, half extents */
/* handles: centre (door frame), radius, half length, axis (0 = z, 1 = the h3 rotation: z -> -y) */
UG_CONST double UG_BX_HANDLE[12] = {-0.13, 0.05, 0.025, 0.005, -0.13, -0.05, 0.025, 0.005, -0.13, 0.0, 0.05, 0.01};
UG_CONST double UG_BX_HANDLE_HH[3] = {0.025, 0.025, 0.05};
/* link masses (URDF :122, :151, :176, :202): door 0.1, h1 0.05, h2 0.05, h3 0.1 */
UG_CONST double UG_BX_DOOR_MASSES[4] = {0.1, 0.05, 0.05, 0.1};
/* button link (prismatic along z at (0, 0, 0.07), limits [-0.05, 0], mass 0.01; collision cylinder r 0.02,
 * length 0.05, URDF :225-252) */
#define UG_BX_BUTTON_Z 0.07
#define UG_BX_BUTTON_LO (-0.05)
#define UG_BX_BUTTON_HI 0.0
#define UG_BX_BUTTON_MASS 0.01
#define UG_BX_BUTTON_R 0.02
#define UG_BX_BUTTON_HH 0.025
/* button_touch_mode (ctor kwarg, :20, :191-216; registered default 'any', envs/__init__.py:3-8) */
#define UG_BX_TOUCH_ANY 0
#define UG_BX_TOUCH_ROBOT 1
#define UG_BX_TOUCH_FINGERS 2

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
#ifndef UG_MAX_COORD_VEL /* (a -D override: the fidelity tools compare against the unclamped dynamics) */
#define UG_MAX_COORD_VEL 100.0         /* btMultiBody m_maxCoordinateVelocity default (100.f) [ext]: every dof velocity is
                                          clamped to +-this in applyDeltaVeeMultiDof, after the force step and after the
                                          constraint solve's delta (processDeltaVeeMultiDof2) */
#endif
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
#ifdef UG_ROBOT_R140 /* UR5Robotiq140.__post_load__ (robot.py:231-240): every multiplier's sign flipped */
UG_CONST double UG_GEAR_RATIO[5] = {-1.0, 1.0, 1.0, -1.0, 1.0};
#else
UG_CONST double UG_GEAR_RATIO[5] = {1.0, -1.0, -1.0, 1.0, -1.0};
#endif

/* ---- task ids (urgym/envs/__init__.py) ---- */
#define UG_TASK_BALLBALANCE 0
#define UG_TASK_CUBESPUSH 1
#define UG_TASK_CUBESGRASP 2
#define UG_TASK_GOLF 3
/* variants: same scene and physics as their base task, different step/obs glue */
#define UG_TASK_CUBESPUSHDIFF 4 /* env_cubes_push_diff_v0.py: obs = ee, cube - ee (x2) */
#define UG_TASK_GOLFJOINTS 5    /* env_golf_joints_v0.py: joint-space action[6], obs = joints + Golf obs */
#define UG_TASK_TWOBALLS 6      /* env_two_balls_balance_v0.py: BallBalance robot + paddle, two balls r 0.003 */
#define UG_TASK_BOX 7           /* env_box_v0.py: the skew box with a door and a button */
#define UG_NTASK 8
#define UG_BASE_TASK(t) ((t) == UG_TASK_CUBESPUSHDIFF ? UG_TASK_CUBESPUSH : \
                         ((t) == UG_TASK_GOLFJOINTS ? UG_TASK_GOLF : ((t) == UG_TASK_TWOBALLS ? UG_TASK_BALLBALANCE : (t))))
#define UG_OBS_DIM(t) ((t) == 0 ? 6 : ((t) == 2 ? 17 : ((t) == 5 ? 15 : ((t) == 7 ? 7 : 9))))
#define UG_ACT_DIM(t) ((t) == 2 ? 9 : ((t) == 5 ? 6 : ((t) == 7 ? 8 : 3)))
#define UG_NDRAW(t) ((t) == 1 || (t) == 4 ? 1 : ((t) == 6 ? 4 : ((t) == 7 ? 0 : 2)))

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

/* Box (env_box_v0.py, skew-box-button.urdf loaded with URDF_MERGE_FIXED_LINKS | URDF_USE_SELF_COLLISION, fixed base
 * at the origin, :80-85).  The robot stands at (0, 0.5, 0) (:55); the restatement keeps the robot base at its own
 * origin, so every world position of this task is stored shifted by -UG_BX_ROBOT_Y (observations and IK targets
 * convert, as PyBullet's base transform does).  Gravity -10 (:60), plane.urdf at z = 0 (:65), no table. */
#define UG_BX_ROBOT_Y 0.5
#define UG_BX_STEPS 120                /* :128 for _ in range(120): step_simulation() */
#define UG_BX_OPENED 1.9               /* :144 door joint > 1.9 */
#define UG_BX_CLOSED 0.1               /* :155 door joint < 0.1 */
#define UG_BX_PRESSED (-0.02)          /* :193 button joint < -0.02 */
#define UG_BX_BUTTON_FORCE 1.0         /* :175 setJointMotorControl2(box, 0, POSITION_CONTROL, force=1), target 0 */
/* merged base_link: walls box1..box4 (URDF :14-118), box half extents / centres in the box base frame */
UG_CONST double UG_BX_WALL_HALF[12] = {0.005, 0.1, 0.045, 0.005, 0.1, 0.045, 0.075, 0.005, 0.045, 0.075, 0.005, 0.045};
UG_CONST double UG_BX_WALL_POS[12] = {0.075, 0.0, 0.045, -0.075, 0.0, 0.045, 0.0, 0.1, 0.045, 0.0, -0.1, 0.045};
/* door link (revolute about y at (0.075, 0, 0.1), limits [0, 2], URDF :120-147) merged with its fixed handles
 * h1, h2 (cylinders r 0.005, length 0.05) and h3 (r 0.01, length 0.1, rpy (pi/2, 0, 0) on h2) (:149-223) */
#define UG_BX_DOOR_X 0.075
#define UG_BX_DOOR_Z 0.1
#define UG_BX_DOOR_LO 0.0
#define UG_BX_DOOR_HI 2.0
UG_CONST double UG_BX_DOOR_BOX[6] = {-0.076, 0.0, 0.0, 0.08, 0.1, 0.005}; /* centre, half extents */
/* handles: centre (door frame), radius, half length, axis (0 = z, 1 = the h3 rotation: z -> -y) */
UG_CONST double UG_BX_HANDLE[12] = {-0.13, 0.05, 0.025, 0.005, -0.13, -0.05, 0.025, 0.005, -0.13, 0.0, 0.05, 0.01};
UG_CONST double UG_BX_HANDLE_HH[3] = {0.025, 0.025, 0.05};
/* link masses (URDF :122, :151, :176, :202): door 0.1, h1 0.05, h2 0.05, h3 0.1 */
UG_CONST double UG_BX_DOOR_MASSES[4] = {0.1, 0.05, 0.05, 0.1};
/* button link (prismatic along z at (0, 0, 0.07), limits [-0.05, 0], mass 0.01; collision cylinder r 0.02,
 * length 0.05, URDF :225-252) */
#define UG_BX_BUTTON_Z 0.07
#define UG_BX_BUTTON_LO (-0.05)
#define UG_BX_BUTTON_HI 0.0
#define UG_BX_BUTTON_MASS 0.01
#define UG_BX_BUTTON_R 0.02
#define UG_BX_BUTTON_HH 0.025
/* button_touch_mode (ctor kwarg, :20, :191-216; registered default 'any', envs/__init__.py:3-8) */
#define UG_BX_TOUCH_ANY 0
#define UG_BX_TOUCH_ROBOT 1
#define UG_BX_TOUCH_FINGERS 2

#endif
