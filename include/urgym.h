/* urgym.h -- C-ABI of the MI355X-native URGym hot path (liburgym.so).
 *
 * The reference reaches its physics through the `pybullet` module's free
 * functions, one env per process.  This boundary replaces
 * that per-substep Python<->C traffic with one batched call per env-step:
 * the whole move_ee -> wait_until_stable -> reward pipeline runs on the GPU.
 * Each entry point names the reference interface it replaces.
 *
 * Conventions: plain pointers and sizes, no torch types.  Host-pointer entry
 * points are synchronous; *_device variants take device pointers, enqueue on
 * the handle's HIP stream and return immediately (urgym_sync waits).
 * Return 0 on success, <0 on error (message via urgym_last_error).  A handle
 * owns its device memory and stream; it is not thread-safe, distinct handles
 * are.  One handle per GPU (device_ordinal); env batches shard across GPUs
 * by creating one handle per rank.
 *
 * Three builds of the same sources export this ABI (__graft_entry__.build):
 *   liburgym.so      UR5Robotiq85, 16-lane GJK groups -- every task;
 *   liburgym_g8.so   UR5Robotiq85, 8-lane GJK groups (-DUG_GJK_G=8) -- the same results bit for bit, faster for
 *                    Golf-v0 / GolfJoints-v0 (6.3 convex queries per substep: one round of eight pairs instead of
 *                    two of four); the Python binding loads it for those two tasks (urgym_amd/_native.py G8_TASKS),
 *                    a C caller picks it the same way or keeps liburgym.so (Golf ~3 % slower);
 *   liburgym_r140.so the UR5Robotiq140 arm (robot.py:221-240).
 * bench.py's JSON line names the library it ran (config.library).
 */
#ifndef URGYM_H
#define URGYM_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct urgym_handle urgym_handle;

#define URGYM_TASK_BALLBALANCE 0 /* urgym/envs/__init__.py:28-32  URGym/BallBalance-v0 */
#define URGYM_TASK_CUBESPUSH 1   /* urgym/envs/__init__.py:10-14  URGym/CubesPush-v0   */
#define URGYM_TASK_CUBESGRASP 2  /* urgym/envs/__init__.py:22-26  URGym/CubesGrasp-v0  */
#define URGYM_TASK_GOLF 3        /* urgym/envs/__init__.py:40-44  URGym/Golf-v0        */
#define URGYM_TASK_CUBESPUSHDIFF 4 /* urgym/envs/__init__.py:16-20  URGym/CubesPushDiff-v0 (env_cubes_push_diff_v0.py) */
#define URGYM_TASK_GOLFJOINTS 5    /* urgym/envs/__init__.py:46-50  URGym/GolfJoints-v0 (env_golf_joints_v0.py)      */
#define URGYM_TASK_TWOBALLSBALANCE 6 /* urgym/envs/__init__.py:34-38 URGym/TwoBallsBalance-v0 (env_two_balls_balance_v0.py) */
#define URGYM_TASK_BOX 7             /* urgym/envs/__init__.py:3-8   URGym/Box-v0 (env_box_v0.py; full geometry only) */

/* Replaces: gym.make(id) -> Env.__init__ (p.connect(DIRECT), loadURDF plane/table/robot,
 *   UR5Robotiq85.load(), env_ball_balance_v0.py:34-80; robot.py:178-211).
 * n_envs independent environments on GPU `device_ordinal`; precision must be 64
 * (FP64, PyBullet's double build [ext]); env i seeds its Python-`random`-compatible
 * MT19937 stream with seed + env_offset + i (env_*: random.uniform draws).
 * Returns NULL on error (urgym_last_error(NULL) explains). */
urgym_handle* urgym_create(int task_id, int n_envs, int device_ordinal, int precision, uint32_t seed,
                           int env_offset);

/* urgym_create with creation flags (0 = urgym_create).  The default geometry (0 or URGYM_FLAG_FULL_GEOMETRY) is the
 * reference's: the robot's mesh colliders are PyBullet's convex hulls of all mesh vertices (URDF2Bullet:
 * btConvexHullShape + optimizeConvexHull, up to 865 vertices / 1306 faces per link) and the Golf club's disc
 * (GEOM_CYLINDER, env_golf_v0.py:305) a true cylinder.  URGYM_FLAG_LOD_GEOMETRY selects the collision LOD instead
 * (<= 48-vertex hulls, a 16-gon disc prism; same contact algorithm): faster, knowingly off the reference's geometry.
 * Both are bit-identical to the CPU restatement's same mode; both flags together are an error. */
#define URGYM_FLAG_FULL_GEOMETRY 1 /* == UG_GEOM_FULL (urgym_amd/csrc/ug_layout.h) */
#define URGYM_FLAG_LOD_GEOMETRY 2  /* == UG_GEOM_LOD */
/* Contact generation.  The default (0 or URGYM_FLAG_CONTACT_GJK) is the path PyBullet takes for the robot's mesh hulls
 * (no URDF_INITIALIZE_SAT_FEATURES, robot.py:186-187): btConvexConvexAlgorithm's GJK + EPA pair detector, one new point
 * per pair and substep merged into the persistent manifold, for every pair without a dedicated Bullet algorithm
 * (sphere-sphere, sphere-box and box-box keep theirs).  URGYM_FLAG_CONTACT_VIH selects rounds 1-3's vertex-in-hull
 * generator (up to 4 points per pair and substep).  Both flags together are an error. */
#define URGYM_FLAG_CONTACT_GJK 4   /* == UG_CONTACT_GJK */
#define URGYM_FLAG_CONTACT_VIH 8   /* == UG_CONTACT_VIH */
urgym_handle* urgym_create_ex(int task_id, int n_envs, int device_ordinal, int precision, uint32_t seed,
                              int env_offset, int flags);

/* Replaces: Env.close() -> p.disconnect (env_ball_balance_v0.py:172-173). */
void urgym_destroy(urgym_handle* h);

/* Last error message for h (or the last creation error when h == NULL). */
const char* urgym_last_error(const urgym_handle* h);

/* Static shapes: observation_space / action_space (env_ball_balance_v0.py:52-54 etc.). */
int urgym_obs_dim(int task_id);
int urgym_act_dim(int task_id);
int urgym_state_dim(void);
int urgym_num_envs(const urgym_handle* h);

/* gymnasium TimeLimit (envs/__init__.py max_episode_steps) and VectorEnv same-step autoreset:
 * when enabled, an env that terminates or truncates inside urgym_step is reset in the same call
 * (obs then holds the reset observation, final_obs the terminal one). max_episode_steps <= 0
 * disables truncation. */
int urgym_set_autoreset(urgym_handle* h, int enable, int max_episode_steps);

/* Replaces: Env.reset() (env_ball_balance_v0.py:145-170 and per-env reset()).
 * mask: n_envs bytes (nonzero = reset that env) or NULL for all.
 * reset_draws: n_envs x urgym_num_draws(task) uniforms in [0,1) replacing random.random()
 * for each env's reset, or NULL to use the per-env device MT19937 streams.
 * obs: n_envs x obs_dim (FP64), rows of unmasked envs untouched. */
int urgym_reset(urgym_handle* h, const uint8_t* mask, const double* reset_draws, double* obs);
int urgym_num_draws(int task_id);

/* Replaces: Env.step(action) (env_ball_balance_v0.py:105-134; robot.py:113-128 move_ee ->
 * p.calculateInverseKinematics + p.setJointMotorControl2; wait_until_stable :94-103 ->
 * <=480 x p.stepSimulation + getJointState/getLinkState; reward/termination).
 * actions: n_envs x act_dim float32.  Outputs (any may be NULL except obs):
 * obs n x obs_dim, final_obs n x obs_dim (only rows of reset envs written), reward n,
 * terminated n, truncated n, success n (info['is_success']), substeps n (int32: physics
 * substeps spent in this call, reset included). */
int urgym_step(urgym_handle* h, const float* actions, double* obs, double* final_obs, double* reward,
               uint8_t* terminated, uint8_t* truncated, uint8_t* success, int32_t* substeps);

/* Same as urgym_step with device pointers; asynchronous on the handle's stream. */
int urgym_step_device(urgym_handle* h, const float* d_actions, double* d_obs, double* d_final_obs,
                      double* d_reward, uint8_t* d_terminated, uint8_t* d_truncated, uint8_t* d_success,
                      int32_t* d_substeps);
int urgym_reset_device(urgym_handle* h, const uint8_t* d_mask, const double* d_reset_draws, double* d_obs);
int urgym_sync(urgym_handle* h);
/* hipStream_t of the handle (as void*), for callers that order their own work after ours. */
void* urgym_stream(urgym_handle* h);

/* Checkpoint / parity: full per-env simulator state, n_envs x urgym_state_dim() doubles
 * (layout: urgym_amd/csrc/ug_layout.h).  No reference counterpart (the reference never
 * saves env state). */
int urgym_get_state(urgym_handle* h, double* state);
int urgym_set_state(urgym_handle* h, const double* state);

/* Replaces: the ctor kwarg reward_type ('dense' / 'sparse', env_cubes_push_v0.py:42,159; env_golf_v0.py:151,163).
 * sparse != 0 drops the distance-shaping terms of CubesPush(Diff) / Golf(Joints); BallBalance, TwoBallsBalance and
 * CubesGrasp store but never read it in the reference, so it changes nothing there. */
int urgym_set_reward_type(urgym_handle* h, int sparse);

/* Replaces: the Box-v0 ctor kwarg button_touch_mode (env_box_v0.py:20, valid_button_press :191-216; registered as
 * 'any', urgym/envs/__init__.py:3-8): 0 'any' (the button joint below -0.02 suffices), 1 'robot' (and a contact
 * between the button and any robot link), 2 'fingers' (and a contact with a finger link 9..18).  Other tasks ignore
 * it; an unknown mode is an error. */
int urgym_set_button_mode(urgym_handle* h, int mode);

/* Failure surfacing (no reference counterpart beyond the "did not stabilize" print, env_ball_balance_v0.py:102-103,
 * SURVEY.md 5).  flags: n_envs bytes, UG_FLAG_* bits (urgym_amd/csrc/ug_layout.h) of the last step / reset call:
 * 1 a wait_until_stable loop hit 480 substeps unsettled, 2 the state went non-finite (the env was terminated with
 * reward 0 and, with autoreset, reset from a clean state), 4 contacts were dropped at a capacity limit.
 * A reset (urgym_reset, or a step's autoreset) whose settling ends non-finite also sets bit 2 and counts; envs
 * masked out of urgym_reset get flags 0 (nothing happened to them in that call).
 * stats: n_envs x 8 int32 cumulative counters (UG_STAT_*: unstable waits, split-impulse substeps, row-capacity
 * substeps, manifold-capacity substeps, non-finite terminations or resets, substeps). */
int urgym_get_flags(urgym_handle* h, uint8_t* flags);
const uint8_t* urgym_flags_device(urgym_handle* h);
int urgym_get_stats(urgym_handle* h, int32_t* stats);

/* Checkpoint companion of urgym_get_state/urgym_set_state: each env's Python-random MT19937 stream
 * (n_envs x 625 uint32: 624 words + index) and its elapsed episode steps (n_envs int32, may be NULL). */
int urgym_get_rng(urgym_handle* h, uint32_t* mt, int32_t* elapsed);
int urgym_set_rng(urgym_handle* h, const uint32_t* mt, const int32_t* elapsed);

/* Replaces: p.getContactPoints(bodyA, bodyB, linkIndexA, linkIndexB) (env_cubes_grasp_v0.py:209-226) for every
 * env.  Bodies are entity codes (0 robot, 1 + i task object i, 10 table, 11 plane, 12 golf pitch, 13 the Box's walls,
 * -1 any), links the robot link index / -1 object base (Golf club parts 0, 1; Box: the door 1, the button 0 -- their
 * pybullet joint indices) / -2 any.  out: n_envs x max_pts x 24 doubles,
 * pybullet's tuple (flag, bodyA, bodyB, linkA, linkB, positionOnA[3], positionOnB[3], contactNormalOnB[3],
 * distance, normalForce, lateralFriction1, lateralFrictionDir1[3], lateralFriction2, lateralFrictionDir2[3]);
 * count: n_envs matching points (may exceed max_pts; only max_pts are written).
 * Filters apply in pybullet's order: body_a alone decides the orientation (no swap when it is -1 or names the
 * pair's A side; A/B fields exchanged and the normal negated when it names the B side), then body_b, link_a and
 * link_b filter in that orientation.  A pair's A side: the robot link (robot pairs), the object (object-static
 * pairs), the sphere or else the lower-numbered object (object-object pairs).
 * Positions: the points' world positions at the last substep's narrowphase (their local anchors under the poses it
 * saw, kept in the state record before that substep's integration), as Bullet's refreshContactPoints leaves
 * m_positionWorldOnA/B. */
int urgym_contact_points(urgym_handle* h, int body_a, int body_b, int link_a, int link_b, int max_pts, double* out,
                         int32_t* count);

/* Replaces: Camera.shot() -> p.getCameraImage(width, height, viewMatrix, projectionMatrix) (utilities.py:84-89;
 * env_box_v0.py:163-164) for envs [env0, env0 + count) of the handle, one image each, rendered on the GPU.
 * view16 / proj16: the 16 floats p.computeViewMatrix / p.computeProjectionMatrixFOV return (column-major;
 * urgym_amd/camera.py restates them).  Outputs (each may be NULL): rgba count x height x width x 4 (u8), depth
 * count x height x width (f32, OpenGL depth-buffer value, 1 = nothing hit), seg count x height x width (i32: body
 * code as in urgym_contact_points, plus ((link + 1) << 24) when flags & 1 -- pybullet's
 * ER_SEGMENTATION_MASK_OBJECT_AND_LINKINDEX -- and -1 = nothing hit).  Pixel (i, j) casts the ray of the
 * reference's rgbd_2_world inverse, NDC ((2i - W) / W, -(2j - H) / H) (urgym_amd/csrc/ug_render.h).
 * Deviations (unpinned: pybullet is absent): the collision shapes are drawn, not the visual meshes (the same for the
 * tasks' primitives; the robot's hulls cover its concave visual meshes); a flat colour per shape with a headlight
 * replaces TinyRenderer's lighting and textures; body codes, not pybullet's body unique ids.
 * urgym_camera_shot_device: device output pointers, asynchronous on urgym_stream(h). */
int urgym_camera_shot(urgym_handle* h, int env0, int count, const float* view16, const float* proj16, int width,
                      int height, int flags, uint8_t* rgba, float* depth, int32_t* seg);
int urgym_camera_shot_device(urgym_handle* h, int env0, int count, const float* view16, const float* proj16, int width,
                             int height, int flags, uint8_t* d_rgba, float* d_depth, int32_t* d_seg);

/* Replaces: one p.stepSimulation() for every env (fine-grained parity tests). */
int urgym_substep(urgym_handle* h);
/* Replaces: p.getLinkState(robot, link)[0:2] -> n_envs x 7 (pos, quat xyzw). */
int urgym_link_state(urgym_handle* h, int link, double* out);
/* Replaces: p.calculateInverseKinematics(robot, 7, pos, orn, ...) (robot.py:119-121):
 * target n_envs x 7 (pos, quat) -> q_out n_envs x 12, from each env's current joints. */
int urgym_ik(urgym_handle* h, const double* target, double* q_out);

/* Device time (ms) of the most recent step/reset kernel, measured with HIP events on the
 * handle's stream (bench.py roofline). */
double urgym_last_kernel_ms(const urgym_handle* h);
/* Development aid, no reference counterpart: phase cycle counters of the step/reset kernels
 * (collision, dynamics, row build, PGS, split, integration, glue, total, then event counts and sub-phase
 * timers; out16 must hold 48 values).  Returns -1 unless the library was built with -DUG_PROF. */
int urgym_debug_prof(urgym_handle* h, unsigned long long* out16, int reset);
/* Development aid: copy the first count doubles of env's device workspace to out; the workspace size
 * (doubles per env) is urgym_debug_ws_doubles().  A -DUG_DEBUG_DUMP build stores the last PGS call's
 * Delassus rows, w and impulses there. */
int urgym_debug_workspace(urgym_handle* h, int env, double* out, int count);
int urgym_debug_ws_doubles(void);
/* Test aid, no reference counterpart: n convex-convex queries (Bullet's btGjkPairDetector as the kernels run it,
 * one wave per query) on the current device.  Query i = 39 doubles: for shape A then B kind (UG_SHAPE_*), hull vertex
 * start, vertex count, implicit dimensions[3], margin, R[9] (row-major), p[3]; then the contact breaking threshold.
 * out: n x 7 (normal on B, point on B, distance), ok: n (1 = a point).  Returns 0 on success. */
int urgym_debug_gjk(int n, const double* q, double* out, int* ok);
/* Test aid, no reference counterpart: for a CubesGrasp handle, the branch each env's next urgym_step would take for the
 * given actions (n x 9 floats, host) -- random.choices([0, 1], weights=[a0, a1]) on the env's next random()
 * (env_cubes_grasp_v0.py:127-130), peeked from its MT19937 stream as k_prio does for the launch order, nothing
 * consumed.  sel: n ints, 0 = the joint move, 1 = the gripper command.  Returns 0 on success. */
int urgym_debug_cg_branch(urgym_handle* h, const float* act, int* sel);

#ifdef __cplusplus
}
#endif
#endif
