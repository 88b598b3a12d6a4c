"""ctypes binding of the CPU restatement (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  It builds nothing at import time; run `make -C oracle` (done by
__graft_entry__.build()).
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# URGYM_ORACLE_LIB: another build of the restatement (make -C oracle asan -> tools/oracle_asan.sh)
LIB_PATH = os.environ.get("URGYM_ORACLE_LIB") or os.path.join(_HERE, "_build", "libugoracle.so")
LIB_PATH_R140 = os.path.join(_HERE, "_build", "libugoracle_r140.so")  # the UR5Robotiq140 restatement

_libs = {}


def lib(path=None):
    """the restatement's library (default: oracle/_build/libugoracle.so; tools/collision_fidelity.py passes the
    paths of its fidelity builds)"""
    path = path or LIB_PATH
    if path not in _libs:
        if not os.path.exists(path):
            raise RuntimeError(f"oracle library {path} not built: run `make -C oracle`")
        L = ctypes.CDLL(path)
        P, D, I, U32 = ctypes.c_void_p, ctypes.c_double, ctypes.c_int, ctypes.c_uint32
        L.ugo_create.restype = P
        L.ugo_create.argtypes = [I, U32]
        L.ugo_create_ex.restype = P
        L.ugo_create_ex.argtypes = [I, U32, I]
        L.ugo_destroy.argtypes = [P]
        L.ugo_obs_dim.argtypes = [I]
        L.ugo_act_dim.argtypes = [I]
        L.ugo_state_dim.argtypes = []
        L.ugo_reset.argtypes = [P, P]
        L.ugo_reset_draws.argtypes = [P, P, P]
        L.ugo_robot_contact.argtypes = [P, I, I, I]
        L.ugo_gripper_opening.argtypes = [P]
        L.ugo_gripper_opening.restype = D
        L.ugo_gripper_center.argtypes = [P, P]
        L.ugo_choose.argtypes = [P, ctypes.c_float, ctypes.c_float]
        L.ugo_norm3.argtypes = [P]
        L.ugo_norm3.restype = D
        L.ugo_g_cp_cube1_x.argtypes = [D]
        L.ugo_g_cp_cube1_x.restype = D
        L.ugo_g_cp_reward.argtypes = [I, I, P, P, I, P]
        L.ugo_g_cg_cube_xy.argtypes = [D, D, P]
        L.ugo_g_cg_choose.argtypes = [ctypes.c_float, ctypes.c_float, D]
        L.ugo_g_cg_opening.argtypes = [D]
        L.ugo_g_cg_opening.restype = D
        L.ugo_g_cg_reward.argtypes = [P, D, D, I, D, P]
        L.ugo_g_box_reward.argtypes = [P, D, I, P]
        L.ugo_g_box_press.argtypes = [D, I, I, I]
        L.ugo_g_box_target.argtypes = [P, P, P]
        L.ugo_box_joint.argtypes = [I, D, D, P]
        L.ugo_g_union_center.argtypes = [P, P]
        L.ugo_g_gf_ball_xy.argtypes = [D, D, P]
        L.ugo_g_gf_reward.argtypes = [P, P, P, I, I, I, I, P, P]
        L.ugo_g_tb_balls.argtypes = [P, P, P, P]
        L.ugo_g_tb_reward.argtypes = [P, P, P, D, P]
        L.ugo_flags.argtypes = [P]
        L.ugo_get_stats.argtypes = [P, P]
        L.ugo_set_reward_type.argtypes = [P, I]
        L.ugo_set_button_mode.argtypes = [P, I]
        L.ugo_get_rng.argtypes = [P, P]
        L.ugo_set_rng.argtypes = [P, P]
        L.ugo_contact_points.argtypes = [P, I, I, I, I, P, I]
        L.ugo_camera.argtypes = [P, P, P, I, I, I, P, P, P]
        L.ugo_dynamics.argtypes = [P, P, D, P, P, P]
        L.ugo_set_pgs_bullet.argtypes = [P, I]
        L.ugo_step.argtypes = [P, P, P, P, P, P]
        L.ugo_get_state.argtypes = [P, P]
        L.ugo_set_state.argtypes = [P, P]
        L.ugo_substep.argtypes = [P]
        L.ugo_rng_seed.argtypes = [P, U32]
        L.ugo_rng_random.argtypes = [P]
        L.ugo_rng_random.restype = D
        L.ugo_gdr.argtypes = [D, D, D]
        L.ugo_gdr.restype = D
        L.ugo_euler_from_quat.argtypes = [P, P]
        L.ugo_quat_from_euler.argtypes = [P, P]
        L.ugo_gripper_angle.argtypes = [D]
        L.ugo_gripper_angle.restype = D
        L.ugo_link_state.argtypes = [P, I, P]
        L.ugo_ik.argtypes = [P, P, P, P]
        L.ugo_bb_ball_position.argtypes = [P, P, P]
        L.ugo_stable_sum.argtypes = [P]
        L.ugo_stable_sum.restype = D
        L.ugo_observe.argtypes = [P, P]
        L.ugo_terminated.argtypes = [P]
        L.ugo_batch_step.restype = ctypes.c_long
        L.ugo_batch_step.argtypes = [P, I, P, P, P, P, P, P, I, I, P]
        _libs[path] = L
    return _libs[path]


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class OracleEnv:
    """One environment of the CPU restatement."""

    def __init__(self, task, seed, lib_path=None, flags=0):
        """flags: 0 / 1 = full geometry (the default), 2 = the collision LOD (UG_GEOM_LOD)"""
        self.L = lib(lib_path)
        self.task = task
        self.h = self.L.ugo_create_ex(task, seed, flags)
        if not self.h:
            raise ValueError(f"ugo_create_ex refused task {task} with flags {flags}")
        self.obs_dim = self.L.ugo_obs_dim(task)
        self.act_dim = self.L.ugo_act_dim(task)
        self.state_dim = self.L.ugo_state_dim()

    def __del__(self):
        try:
            self.L.ugo_destroy(self.h)
        except Exception:
            pass

    def reset(self, draws=None):
        obs = np.zeros(self.obs_dim)
        if draws is None:
            n = self.L.ugo_reset(self.h, _p(obs))
        else:
            d = np.ascontiguousarray(draws, dtype=np.float64)
            n = self.L.ugo_reset_draws(self.h, _p(d), _p(obs))
        return obs, n

    def robot_contact(self, obj_or_static, lmin, lmax):
        return bool(self.L.ugo_robot_contact(self.h, obj_or_static, lmin, lmax))

    def gripper_opening(self):
        return self.L.ugo_gripper_opening(self.h)

    def gripper_center(self):
        out = np.zeros(3)
        self.L.ugo_gripper_center(self.h, _p(out))
        return out

    def choose(self, w0, w1):
        return self.L.ugo_choose(self.h, w0, w1)

    def step(self, action):
        a = np.ascontiguousarray(action, dtype=np.float32)
        obs = np.zeros(self.obs_dim)
        rew = np.zeros(1)
        term = np.zeros(1, np.uint8)
        succ = np.zeros(1, np.uint8)
        n = self.L.ugo_step(self.h, _p(a), _p(obs), _p(rew), _p(term), _p(succ))
        return obs, float(rew[0]), bool(term[0]), bool(succ[0]), n

    def substep(self):
        self.L.ugo_substep(self.h)

    def flags(self):
        """UG_FLAG_* bits of the last step / reset call"""
        return self.L.ugo_flags(self.h)

    def stats(self):
        out = np.zeros(8, np.int32)
        self.L.ugo_get_stats(self.h, _p(out))
        return out

    def set_reward_type(self, reward_type):
        self.L.ugo_set_reward_type(self.h, int(reward_type == "sparse"))

    def set_button_mode(self, mode):
        """Box-v0 button_touch_mode: 'any', 'robot' or 'fingers' (env_box_v0.py:20)"""
        self.L.ugo_set_button_mode(self.h, {"any": 0, "robot": 1, "fingers": 2}[mode])

    def set_pgs_bullet(self, on):
        """solve with Bullet's velocity-space PGS form (tests only)"""
        self.L.ugo_set_pgs_bullet(self.h, int(on))

    def get_rng(self):
        out = np.zeros(625, np.uint32)
        self.L.ugo_get_rng(self.h, _p(out))
        return out

    def set_rng(self, mt):
        self.L.ugo_set_rng(self.h, _p(np.ascontiguousarray(mt, np.uint32)))

    def contact_points(self, body_a=-1, body_b=-1, link_a=-2, link_b=-2, max_pts=64):
        out = np.zeros((max_pts, 24))
        n = self.L.ugo_contact_points(self.h, body_a, body_b, link_a, link_b, _p(out), max_pts)
        return out[:min(n, max_pts)]

    def camera(self, view16, proj16, width, height, link_index=False):
        """ugo_camera: the restated Camera.shot() of this env -> rgb (H, W, 4) u8, depth (H, W) f32, seg (H, W) i32"""
        v = np.ascontiguousarray(view16, dtype=np.float32)
        p = np.ascontiguousarray(proj16, dtype=np.float32)
        rgb = np.zeros((height, width, 4), np.uint8)
        depth = np.zeros((height, width), np.float32)
        seg = np.zeros((height, width), np.int32)
        rc = self.L.ugo_camera(self.h, _p(v), _p(p), width, height, 1 if link_index else 0, _p(rgb), _p(depth), _p(seg))
        assert rc == 0, "singular projection * view"
        return rgb, depth, seg

    def get_state(self):
        s = np.zeros(self.state_dim)
        self.L.ugo_get_state(self.h, _p(s))
        return s

    def set_state(self, s):
        s = np.ascontiguousarray(s, dtype=np.float64)
        self.L.ugo_set_state(self.h, _p(s))

    def observe(self):
        obs = np.zeros(self.obs_dim)
        self.L.ugo_observe(self.h, _p(obs))
        return obs

    def terminated(self):
        return bool(self.L.ugo_terminated(self.h))

    def rng_seed(self, seed):
        self.L.ugo_rng_seed(self.h, seed)

    def rng_random(self):
        return self.L.ugo_rng_random(self.h)

    def bb_ball_position(self, paddle):
        out = np.zeros(3)
        self.L.ugo_bb_ball_position(self.h, _p(np.asarray(paddle, np.float64)), _p(out))
        return out

    def link_state(self, link):
        out = np.zeros(7)
        self.L.ugo_link_state(self.h, link, _p(out))
        return out

    def ik(self, pos, orn):
        q = np.zeros(12)
        self.L.ugo_ik(self.h, _p(np.asarray(pos, np.float64)), _p(np.asarray(orn, np.float64)), _p(q))
        return q


def dynamics(q, qd, g=-9.8):
    """(M 12x12, C 12, body COMs 12x3) of the restatement's CRBA / RNEA at (q, qd)"""
    M = np.zeros((12, 12))
    C = np.zeros(12)
    com = np.zeros((12, 3))
    lib().ugo_dynamics(_p(np.ascontiguousarray(q, np.float64)), _p(np.ascontiguousarray(qd, np.float64)), g, _p(M),
                       _p(C), _p(com))
    return M, C, com


def norm3(v):
    return lib().ugo_norm3(_p(np.ascontiguousarray(v, dtype=np.float64)))


def gdr(v, s, m):
    return lib().ugo_gdr(v, s, m)


def euler_from_quat(q):
    out = np.zeros(3)
    lib().ugo_euler_from_quat(_p(np.asarray(q, np.float64)), _p(out))
    return out


def quat_from_euler(e):
    out = np.zeros(4)
    lib().ugo_quat_from_euler(_p(np.asarray(e, np.float64)), _p(out))
    return out


def gripper_angle(L):
    return lib().ugo_gripper_angle(L)


def stable_sum(a12):
    return lib().ugo_stable_sum(_p(np.ascontiguousarray(a12, np.float64)))
