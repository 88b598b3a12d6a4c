"""ctypes binding of liburgym.so (the HIP product path, include/urgym.h).

There is deliberately no CPU fallback: if the in-tree library is missing, or
no GPU is visible, constructing an environment raises.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("URGYM_LIB") or os.path.join(_HERE, "_lib", "liburgym.so")

# C-ABI symbols declared in include/urgym.h (tests/test_capi.py checks that the library exports each one)
SYMBOLS = [
    "urgym_create", "urgym_create_ex", "urgym_destroy", "urgym_last_error", "urgym_obs_dim", "urgym_act_dim", "urgym_state_dim",
    "urgym_num_envs", "urgym_set_autoreset", "urgym_reset", "urgym_num_draws", "urgym_step", "urgym_step_device",
    "urgym_reset_device", "urgym_sync", "urgym_stream", "urgym_get_state", "urgym_set_state", "urgym_substep",
    "urgym_link_state", "urgym_ik", "urgym_last_kernel_ms", "urgym_debug_prof", "urgym_debug_workspace",
    "urgym_debug_ws_doubles", "urgym_set_reward_type", "urgym_get_flags", "urgym_flags_device", "urgym_get_stats",
    "urgym_get_rng", "urgym_set_rng", "urgym_contact_points", "urgym_set_button_mode",
    "urgym_camera_shot", "urgym_camera_shot_device", "urgym_debug_gjk", "urgym_debug_cg_branch",
]

# UG_FLAG_* / UG_STAT_* (urgym_amd/csrc/ug_layout.h)
FLAG_UNSTABLE, FLAG_NONFINITE, FLAG_DROPPED = 1, 2, 4
GEOM_FULL, GEOM_LOD = 1, 2  # urgym_create_ex flags: the full geometry (the default) / the collision LOD
CONTACT_GJK, CONTACT_VIH = 4, 8  # contact generation: Bullet's GJK / EPA (the default) / rounds 1-3's vertex-in-hull
STAT_NAMES = ["unstable_waits", "split_substeps", "row_capacity_substeps", "manifold_capacity_substeps",
              "nonfinite_terminations", "substeps", "reserved6", "reserved7"]
CONTACT_FIELDS = 24  # pybullet getContactPoints tuple, flattened

# robot.py's arm + gripper classes -> their build of the library (same sources, the robot's model header):
# UR5Robotiq85 (every registered env) and UR5Robotiq140 (robot.py:221-240, liburgym_r140.so)
ROBOT_LIBS = {"ur5_robotiq_85": LIB_PATH, "ur5_robotiq_140": os.path.join(_HERE, "_lib", "liburgym_r140.so")}
# Golf-v0 / GolfJoints-v0 run the build with 8-lane GJK groups (UG_GJK_G 8: eight convex pairs per round; Golf's
# 6.3 GJK queries per substep fit one round instead of two -- Golf +3 %, GolfJoints +7 %; BallBalance, 3.4 queries,
# loses 1.4 % with it, so every other task keeps the 16-lane build).  Same sources, same results bit for bit.
G8_LIB = os.path.join(_HERE, "_lib", "liburgym_g8.so")
G8_TASKS = (3, 5)
_libs = {}


def lib(robot="ur5_robotiq_85", task=None):
    if robot not in ROBOT_LIBS:
        raise ValueError(f"robot must be one of {sorted(ROBOT_LIBS)}, not {robot!r}")
    path = ROBOT_LIBS[robot]
    if robot == "ur5_robotiq_85" and task in G8_TASKS and not os.environ.get("URGYM_LIB"):
        path = G8_LIB
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise RuntimeError(f"{os.path.basename(path)} not built ({path}); run __graft_entry__.build() -- "
                           "no CPU fallback exists")
    # torch, when installed, is loaded first: it bundles its own HIP runtime, and importing it after this library
    # has initialised the /opt/rocm runtime leaves torch.cuda unavailable in the process (measured on MI355X,
    # tools/gpu.sh history: round 3's load-order diagnosis); the other order works, and the device tensors / streams of vec.py need torch's side
    try:
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is part of this image
        pass
    L = ctypes.CDLL(path)
    P, I, D, U32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_uint32
    L.urgym_create.restype = P
    L.urgym_create.argtypes = [I, I, I, I, U32, I]
    L.urgym_create_ex.restype = P
    L.urgym_create_ex.argtypes = [I, I, I, I, U32, I, I]
    L.urgym_destroy.argtypes = [P]
    L.urgym_last_error.restype = ctypes.c_char_p
    L.urgym_last_error.argtypes = [P]
    for name in ("urgym_obs_dim", "urgym_act_dim", "urgym_num_draws"):
        getattr(L, name).argtypes = [I]
    L.urgym_state_dim.argtypes = []
    L.urgym_num_envs.argtypes = [P]
    L.urgym_set_autoreset.argtypes = [P, I, I]
    L.urgym_reset.argtypes = [P, P, P, P]
    L.urgym_reset_device.argtypes = [P, P, P, P]
    L.urgym_step.argtypes = [P, P, P, P, P, P, P, P, P]
    L.urgym_step_device.argtypes = [P, P, P, P, P, P, P, P, P]
    L.urgym_sync.argtypes = [P]
    L.urgym_stream.restype = P
    L.urgym_stream.argtypes = [P]
    L.urgym_get_state.argtypes = [P, P]
    L.urgym_set_state.argtypes = [P, P]
    L.urgym_substep.argtypes = [P]
    L.urgym_link_state.argtypes = [P, I, P]
    L.urgym_ik.argtypes = [P, P, P]
    L.urgym_last_kernel_ms.restype = D
    L.urgym_last_kernel_ms.argtypes = [P]
    L.urgym_debug_prof.argtypes = [P, P, I]
    L.urgym_debug_workspace.argtypes = [P, I, P, I]
    L.urgym_debug_ws_doubles.argtypes = []
    L.urgym_debug_gjk.argtypes = [I, P, P, P]
    L.urgym_debug_cg_branch.argtypes = [P, P, P]
    L.urgym_set_reward_type.argtypes = [P, I]
    L.urgym_set_button_mode.argtypes = [P, I]
    L.urgym_get_flags.argtypes = [P, P]
    L.urgym_flags_device.restype = P
    L.urgym_flags_device.argtypes = [P]
    L.urgym_get_stats.argtypes = [P, P]
    L.urgym_get_rng.argtypes = [P, P, P]
    L.urgym_set_rng.argtypes = [P, P, P]
    L.urgym_contact_points.argtypes = [P, I, I, I, I, I, P, P]
    L.urgym_camera_shot.argtypes = [P, I, I, P, P, I, I, I, P, P, P]
    L.urgym_camera_shot_device.argtypes = [P, I, I, P, P, I, I, I, P, P, P]
    _libs[path] = L
    return L


def ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class Sim:
    """One handle = n_envs environments of one task on one GPU."""

    def __init__(self, task, n_envs, device=0, seed=0, env_offset=0, flags=0, robot="ur5_robotiq_85"):
        """flags: 0 or GEOM_FULL = the full geometry (default), GEOM_LOD = the collision LOD; robot: the arm +
        gripper (robot.py's UR5Robotiq85, every registered env's, or UR5Robotiq140)"""
        self.L = lib(robot, task)
        self.robot = robot
        self.task = task
        self.n = n_envs
        self.create_flags = flags
        self.h = self.L.urgym_create_ex(task, n_envs, device, 64, seed & 0xFFFFFFFF, env_offset, flags)
        if not self.h:
            raise RuntimeError("urgym_create failed: " + self.L.urgym_last_error(None).decode())
        self.obs_dim = self.L.urgym_obs_dim(task)
        self.act_dim = self.L.urgym_act_dim(task)
        self.state_dim = self.L.urgym_state_dim()
        self.ndraw = self.L.urgym_num_draws(task)
        # callables run before any call that changes the simulated state (the vector env's deferred camera batch
        # renders there, so its images stay those of the state its last step / reset returned)
        self.before_mutate = []

    def _mutating(self):
        for f in self.before_mutate:
            f()

    def _chk(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what} failed: " + self.L.urgym_last_error(self.h).decode())

    def close(self):
        if getattr(self, "h", None):
            self.L.urgym_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_autoreset(self, enable, max_episode_steps):
        self._chk(self.L.urgym_set_autoreset(self.h, int(enable), int(max_episode_steps)), "urgym_set_autoreset")

    def reset(self, mask=None, draws=None, obs=None):
        self._mutating()
        if obs is None:
            obs = np.zeros((self.n, self.obs_dim))
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        d = None if draws is None else np.ascontiguousarray(draws, dtype=np.float64)
        self._chk(self.L.urgym_reset(self.h, ptr(m), ptr(d), ptr(obs)), "urgym_reset")
        return obs

    def step(self, actions):
        self._mutating()
        a = np.ascontiguousarray(actions, dtype=np.float32).reshape(self.n, self.act_dim)
        n = self.n
        out = dict(obs=np.zeros((n, self.obs_dim)), final_obs=np.zeros((n, self.obs_dim)), reward=np.zeros(n),
                   terminated=np.zeros(n, np.uint8), truncated=np.zeros(n, np.uint8), success=np.zeros(n, np.uint8),
                   substeps=np.zeros(n, np.int32))
        self._chk(self.L.urgym_step(self.h, ptr(a), ptr(out["obs"]), ptr(out["final_obs"]), ptr(out["reward"]),
                                    ptr(out["terminated"]), ptr(out["truncated"]), ptr(out["success"]),
                                    ptr(out["substeps"])), "urgym_step")
        return out

    def step_device(self, d_act, d_obs, d_final=0, d_rew=0, d_term=0, d_trunc=0, d_succ=0, d_sub=0):
        """Device-pointer variant (ints = device addresses, e.g. torch.Tensor.data_ptr())."""
        self._mutating()
        v = ctypes.c_void_p
        self._chk(self.L.urgym_step_device(self.h, v(d_act), v(d_obs), v(d_final or None), v(d_rew or None),
                                           v(d_term or None), v(d_trunc or None), v(d_succ or None),
                                           v(d_sub or None)), "urgym_step_device")

    def sync(self):
        self._chk(self.L.urgym_sync(self.h), "urgym_sync")

    def last_kernel_ms(self):
        return self.L.urgym_last_kernel_ms(self.h)

    def get_state(self):
        s = np.zeros((self.n, self.state_dim))
        self._chk(self.L.urgym_get_state(self.h, ptr(s)), "urgym_get_state")
        return s

    def set_state(self, s):
        self._mutating()
        s = np.ascontiguousarray(s, dtype=np.float64).reshape(self.n, self.state_dim)
        self._chk(self.L.urgym_set_state(self.h, ptr(s)), "urgym_set_state")

    def substep(self):
        self._mutating()
        self._chk(self.L.urgym_substep(self.h), "urgym_substep")

    def link_state(self, link):
        out = np.zeros((self.n, 7))
        self._chk(self.L.urgym_link_state(self.h, int(link), ptr(out)), "urgym_link_state")
        return out

    def set_reward_type(self, reward_type):
        if reward_type not in ("dense", "sparse"):
            raise ValueError(f"reward_type must be 'dense' or 'sparse', not {reward_type!r}")
        self._chk(self.L.urgym_set_reward_type(self.h, int(reward_type == "sparse")), "urgym_set_reward_type")

    def set_button_mode(self, mode):
        """Box-v0 button_touch_mode: 'any', 'robot' or 'fingers' (env_box_v0.py:20)"""
        modes = {"any": 0, "robot": 1, "fingers": 2}
        if mode not in modes:
            raise ValueError(f"button_touch_mode must be one of {sorted(modes)}, not {mode!r}")
        self._chk(self.L.urgym_set_button_mode(self.h, modes[mode]), "urgym_set_button_mode")

    def flags(self):
        """UG_FLAG_* bits per env of the last step / reset call"""
        f = np.zeros(self.n, np.uint8)
        self._chk(self.L.urgym_get_flags(self.h, ptr(f)), "urgym_get_flags")
        return f

    def stats(self):
        out = np.zeros((self.n, 8), np.int32)
        self._chk(self.L.urgym_get_stats(self.h, ptr(out)), "urgym_get_stats")
        return out

    def get_rng(self):
        """(MT19937 streams n x 625 uint32, elapsed episode steps n int32): checkpoint companion of get_state"""
        mt = np.zeros((self.n, 625), np.uint32)
        el = np.zeros(self.n, np.int32)
        self._chk(self.L.urgym_get_rng(self.h, ptr(mt), ptr(el)), "urgym_get_rng")
        return mt, el

    def set_rng(self, mt, elapsed=None):
        m = np.ascontiguousarray(mt, np.uint32).reshape(self.n, 625)
        e = None if elapsed is None else np.ascontiguousarray(elapsed, np.int32).reshape(self.n)
        self._chk(self.L.urgym_set_rng(self.h, ptr(m), ptr(e)), "urgym_set_rng")

    def contact_points(self, body_a=-1, body_b=-1, link_a=-2, link_b=-2, max_pts=64):
        """p.getContactPoints for every env: (n x max_pts x 24 tuples, n counts)"""
        out = np.zeros((self.n, max_pts, CONTACT_FIELDS))
        cnt = np.zeros(self.n, np.int32)
        self._chk(self.L.urgym_contact_points(self.h, body_a, body_b, link_a, link_b, max_pts, ptr(out), ptr(cnt)),
                  "urgym_contact_points")
        return out, cnt

    def ik(self, target):
        t = np.ascontiguousarray(target, dtype=np.float64).reshape(self.n, 7)
        q = np.zeros((self.n, 12))
        self._chk(self.L.urgym_ik(self.h, ptr(t), ptr(q)), "urgym_ik")
        return q
