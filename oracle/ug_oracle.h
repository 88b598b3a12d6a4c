/* ug_oracle.h -- CPU restatement of URGym's per-step hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle for the HIP product
 * path (urgym_amd/csrc).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it (oracle/_build/libugoracle.so).  The product
 * never links or calls it.
 *
 * What it restates (file:line in /root/reference):
 *   env.step()              urgym/envs/env_ball_balance_v0.py:105-134 (and the other envs)
 *   robot.move_ee / IK      urgym/base/robot.py:113-128  -> p.calculateInverseKinematics [ext]
 *   wait_until_stable       urgym/envs/env_ball_balance_v0.py:94-103
 *   p.stepSimulation        PyBullet/Bullet3 btMultiBodyDynamicsWorld [ext, parity unpinned]
 *   obs/reward/termination  per env file (see oracle/ug_oracle.c)
 * Parity vs PyBullet itself is UNPINNED (pybullet absent);
 * the glue (rewards, euler/quaternion conventions, gripper map, RNG) is
 * pinned by tests/golden fixtures generated from the reference's own code.
 */
#ifndef UG_ORACLE_H
#define UG_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ugo_env ugo_env;

/* task: 0 BallBalance, 1 CubesPush, 2 CubesGrasp, 3 Golf, 4 CubesPushDiff, 5 GolfJoints, 6 TwoBallsBalance */
ugo_env* ugo_create(int task, uint32_t seed);
/* flags: UG_GEOM_LOD (ug_layout.h) -- the collision LOD instead of the default full geometry */
ugo_env* ugo_create_ex(int task, uint32_t seed, int flags);
void ugo_destroy(ugo_env* e);
int ugo_obs_dim(int task);
int ugo_act_dim(int task);
int ugo_state_dim(void);
/* reset(): fills obs; returns substeps spent */
int ugo_reset(ugo_env* e, double* obs);
/* reset with caller-supplied uniforms in [0,1) replacing the env's random() draws (NULL: use the stream) */
int ugo_reset_draws(ugo_env* e, const double* draws, double* obs);
/* step(): action float32[act_dim]; returns substeps spent in wait_until_stable */
int ugo_step(ugo_env* e, const float* action, double* obs, double* reward, uint8_t* terminated,
             uint8_t* success);
void ugo_get_state(const ugo_env* e, double* s);
/* UG_FLAG_* of the last ugo_step / ugo_reset call; UG_STAT_* counters (UG_NSTAT int32) */
int ugo_flags(const ugo_env* e);
void ugo_get_stats(const ugo_env* e, int32_t* out);
/* reward_type: 0 'dense', 1 'sparse' (ctor kwarg of every reference env) */
void ugo_set_reward_type(ugo_env* e, int sparse);
/* Box-v0 button_touch_mode: 0 'any', 1 'robot', 2 'fingers' (env_box_v0.py:20, :191-216) */
void ugo_set_button_mode(ugo_env* e, int mode);
/* tests only: 1 = solve with Bullet's velocity-space PGS form (clamp-and-assign) instead of the row-space
 * restatement the kernels reproduce; bounds the restatement's rounding against Bullet's arithmetic */
void ugo_set_pgs_bullet(ugo_env* e, int on);
/* Python-random stream checkpoint: 624 MT words + index */
void ugo_get_rng(const ugo_env* e, uint32_t* mt625);
void ugo_set_rng(ugo_env* e, const uint32_t* mt625);
/* robot equations of motion at (q, qd): M (12 x 12), C (12), body COMs (12 x 3) -- dynamics KATs */
void ugo_dynamics(const double* q, const double* qd, double g, double* M, double* C, double* com);
/* p.getContactPoints over the manifold cache: 24 doubles per point (see ug_oracle.c); returns the count */
int ugo_contact_points(const ugo_env* e, int bodyA, int bodyB, int linkA, int linkB, double* out, int max_pts);
int ugo_camera(const ugo_env* e, const float* view16, const float* proj16, int W, int H, int flags, uint8_t* rgba,
               float* depth, int32_t* seg);
void ugo_set_state(ugo_env* e, const double* s);
/* one physics substep (p.stepSimulation) -- for fine-grained parity tests */
void ugo_substep(ugo_env* e);
/* last substep's PGS shape (this thread): n, nnc, nn, nf, nr, sweeps, split sweeps, 0 */
void ugo_debug_rows(int* out);
/* last PGS call: A [128][128] row-major, then w4 = w after warm start | w after sweeps | impulses (128 each) */
void ugo_debug_pgs(double* A, double* w4);
/* helpers exposed for known-answer tests */
void ugo_rng_seed(ugo_env* e, uint32_t seed);
double ugo_rng_random(ugo_env* e);
double ugo_gdr(double value, double thr_sign, double thr_max);
void ugo_euler_from_quat(const double* q, double* rpy);
void ugo_quat_from_euler(const double* rpy, double* q);
double ugo_gripper_angle(double open_length);
void ugo_link_state(const ugo_env* e, int link, double* pos7);
void ugo_ik(const ugo_env* e, const double* target_pos, const double* target_orn, double* q_out);
void ugo_bb_ball_position(ugo_env* e, const double* paddle, double* out);
double ugo_stable_sum(const double* a12);
void ugo_observe(const ugo_env* e, double* obs);
int ugo_terminated(const ugo_env* e);
/* contact predicate: a manifold point between a robot link in [lmin, lmax] and object i (0..) or the
 * static with id obj_or_static (10 table, 11 plane) -- p.getContactPoints existence */
int ugo_robot_contact(const ugo_env* e, int obj_or_static, int lmin, int lmax);
double ugo_gripper_opening(const ugo_env* e);
void ugo_gripper_center(const ugo_env* e, double* out3);
int ugo_choose(ugo_env* e, float w0, float w1);
double ugo_norm3(const double* v);
/* shared task glue (urgym_amd/csrc/ug_glue.h) for the golden tests */
double ugo_g_cp_cube1_x(double u);
int ugo_g_cp_reward(int table, int touched, const double* c0, const double* c1, int sparse, double* r);
void ugo_g_cg_cube_xy(double u0, double u1, double* xy);
int ugo_g_cg_choose(float w0, float w1, double u);
double ugo_g_cg_opening(double d);
int ugo_g_cg_reward(int* flags, double dist, double opening, int grasp, double cube_z, double* r);
void ugo_g_union_center(const double* aabbs, double* c);
void ugo_g_gf_ball_xy(double u0, double u1, double* xy);
int ugo_g_gf_reward(const double* ball, const double* hole, const double* stick, int in_fingers, int floor_contact,
                    int touched, int sparse, double* r, int* term);
void ugo_g_tb_balls(const double* paddle, const double* u4, double* b1, double* b2);
int ugo_g_tb_reward(const float* a, const double* b1, const double* b2, double paddle_z, double* r);
/* one convex-convex (GJK / EPA) query, Bullet's btGjkPairDetector (oracle/ug_gjk_ref.h): shapes kind (UG_SHAPE_*),
 * hull vertex range, implicit dimensions, margin; poses R (row-major) + p; out = normal on B, point on B, distance.
 * Returns 1 when a point is reported. */
int ugo_gjk_pair(int kA, int v0A, int nvA, const double* impA, double mA, const double* RA, const double* pA, int kB, int v0B,
                 int nvB, const double* impB, double mB, const double* RB, const double* pB, double thr, double* out);
/* debug aid: record this thread's convex-convex queries (urgym_debug_gjk's 39-double packing + ok + normal, point,
 * distance = 47 doubles each, up to 512); ugo_gjk_records returns how many were recorded */
void ugo_gjk_record(int on);
/* debug aid: record the state (UG_STATE_DIM doubles) before every wait_until_stable substep, up to 600 */
void ugo_trace(int on);
int ugo_traced(double* out, int max);
int ugo_gjk_records(double* out, int max);
/* OpenMP threads of this thread's next ugo_batch_step calls */
void ugo_set_threads(int n);
/* batched CPU baseline: n envs, OpenMP over envs; returns total substeps */
long ugo_batch_step(ugo_env** envs, int n, const float* actions, double* obs, double* reward,
                    uint8_t* terminated, uint8_t* success, int32_t* substeps, int autoreset,
                    int max_episode_steps, int32_t* elapsed);

#ifdef __cplusplus
}
#endif
#endif
