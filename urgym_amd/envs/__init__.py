"""URGym environments on MI355X: same IDs, spaces, ctor kwargs and 5-tuple as the reference.

Registry restated from /root/reference/urgym/envs/__init__.py:3-50 (IDs and
max_episode_steps).  Tasks not yet implemented on the GPU raise on
construction (no silent fallback).
"""
import math

import numpy as np

try:  # real gymnasium when available, else the local stand-ins
    from gymnasium import Env as _EnvBase  # noqa: F401
    from gymnasium.spaces import Box
except Exception:  # pragma: no cover - gymnasium absent in this image
    _EnvBase = object
    from ..spaces import Box

from .core import URGymEnv, URGymVectorEnv

TASKS = {
    # id: (task index, max_episode_steps)   envs/__init__.py lines
    "URGym/BallBalance-v0": (0, 500),   # :28-32
    "URGym/CubesPush-v0": (1, 50),      # :10-14
    "URGym/CubesGrasp-v0": (2, 20),     # :22-26
    "URGym/Golf-v0": (3, 100),          # :40-44
    "URGym/CubesPushDiff-v0": (4, 50),  # :16-20  (variant of CubesPush: relative obs)
    "URGym/GolfJoints-v0": (5, 100),    # :46-50  (variant of Golf: joint-space action, joints in obs)
    "URGym/TwoBallsBalance-v0": (6, 500),  # :34-38  (BallBalance scene with two balls)
    "URGym/Box-v0": (7, 200),           # :3-8    (skew box with door and button; kwargs button_touch_mode='any')
}
UNSUPPORTED = {}  # every id the reference registers is built


def spaces_for(task):
    """observation_space / action_space exactly as the reference declares them."""
    if task == 0:  # env_ball_balance_v0.py:52-54
        obs = Box(low=np.array([-math.pi] * 3 + [-1.0] * 3), high=np.array([math.pi] * 3 + [1.0] * 3), dtype=np.float64)
        act = Box(low=np.array([-0.1] * 3), high=np.array([+0.1] * 3), dtype=np.float32)
    elif task == 6:  # env_two_balls_balance_v0.py:52-54
        obs = Box(low=np.array([-math.pi] * 3 + [-1.0] * 6), high=np.array([math.pi] * 3 + [1.0] * 6), dtype=np.float64)
        act = Box(low=np.array([-0.1] * 3), high=np.array([+0.1] * 3), dtype=np.float32)
    elif task in (1, 3, 4):  # env_cubes_push_v0.py:58-60, env_golf_v0.py:58-60, env_cubes_push_diff_v0.py:58-62
        obs = Box(low=np.array([-1.0] * 9), high=np.array([1.0] * 9), dtype=np.float64)
        act = Box(low=np.array([-0.1] * 3), high=np.array([+0.1] * 3), dtype=np.float32)
    elif task == 7:  # env_box_v0.py:41-43
        obs = Box(low=np.array([-1.0, -1.0, -1.0, -math.pi, -math.pi, -math.pi, -math.pi]),
                  high=np.array([1.0, 1.0, 1.0, math.pi, math.pi, math.pi, math.pi]), dtype=np.float64)
        act = Box(low=np.array([-0.05] * 3 + [-math.pi / 10] * 4 + [0.0]),
                  high=np.array([+0.05] * 3 + [+math.pi / 10] * 4 + [0.085]), dtype=np.float32)
    elif task == 5:  # env_golf_joints_v0.py:59-63
        obs = Box(low=np.array([-2 * math.pi] * 6 + [-1.0] * 3 + [-1.0] * 3 + [-1.0] * 3),
                  high=np.array([2 * math.pi] * 6 + [1.0] * 3 + [1.0] * 3 + [1.0] * 3), dtype=np.float64)
        act = Box(low=np.array([-0.1] * 6), high=np.array([+0.1] * 6), dtype=np.float32)
    else:  # env_cubes_grasp_v0.py:72-74
        obs = Box(low=np.array([0] * 2 + [-1.0] * 3 + [-1] * 4 + [0] + [-1.0] * 3 + [-1.0] * 4),
                  high=np.array([1] * 2 + [1.0] * 3 + [1.0] * 4 + [1] + [1.0] * 3 + [1.0] * 4), dtype=np.float64)
        act = Box(low=np.array([0] * 2 + [-math.pi] * 6 + [0]), high=np.array([1] * 2 + [+math.pi] * 6 + [1]),
                  dtype=np.float32)
    return obs, act


def make(env_id, num_envs=None, device=0, seed=0, env_offset=0, **kwargs):
    """gym.make(id) equivalent.  num_envs=None -> single Env (TimeLimit applied);
    num_envs=N -> URGymVectorEnv with same-step autoreset."""
    if env_id in UNSUPPORTED:
        raise NotImplementedError(f"{env_id} is outside this build's hot-path scope (SURVEY.md 8(f))")
    if env_id not in TASKS:
        raise KeyError(env_id)
    task, max_steps = TASKS[env_id]
    if task == 7:
        kwargs.setdefault("button_touch_mode", "any")  # the registry's kwargs (envs/__init__.py:7)
    if num_envs is None:
        return URGymEnv(task, max_episode_steps=max_steps, device=device, seed=seed, **kwargs)
    return URGymVectorEnv(task, num_envs, max_episode_steps=max_steps, device=device, seed=seed,
                          env_offset=env_offset, **kwargs)


def BallBalance(camera=None, reward_type="dense", render_mode="human", **kw):
    """env_ball_balance_v0.BallBalance(camera, reward_type, render_mode) signature."""
    return URGymEnv(0, max_episode_steps=None, camera=camera, reward_type=reward_type, render_mode=render_mode, **kw)


def CubesPush(camera=None, reward_type="dense", render_mode="human", **kw):
    """env_cubes_push_v0.CubesPush(camera, reward_type, render_mode) signature."""
    return URGymEnv(1, max_episode_steps=None, camera=camera, reward_type=reward_type, render_mode=render_mode, **kw)


def CubesGrasp(camera=None, reward_type="dense", render_mode="human", **kw):
    """env_cubes_grasp_v0.CubesGrasp(camera, reward_type, render_mode) signature."""
    return URGymEnv(2, max_episode_steps=None, camera=camera, reward_type=reward_type, render_mode=render_mode, **kw)


def Golf(camera=None, reward_type="dense", render_mode="human", **kw):
    """env_golf_v0.Golf(camera, reward_type, render_mode) signature."""
    return URGymEnv(3, max_episode_steps=None, camera=camera, reward_type=reward_type, render_mode=render_mode, **kw)


def CubesPushDiff(camera=None, reward_type="dense", render_mode="human", **kw):
    """env_cubes_push_diff_v0.CubesPushDiff(camera, reward_type, render_mode) signature."""
    return URGymEnv(4, max_episode_steps=None, camera=camera, reward_type=reward_type, render_mode=render_mode, **kw)


def GolfJoints(camera=None, reward_type="dense", render_mode="human", **kw):
    """env_golf_joints_v0.GolfJoints(camera, reward_type, render_mode) signature."""
    return URGymEnv(5, max_episode_steps=None, camera=camera, reward_type=reward_type, render_mode=render_mode, **kw)


def TwoBallsBalance(camera=None, reward_type="dense", render_mode="human", **kw):
    """env_two_balls_balance_v0.TwoBallsBalance(camera, reward_type, render_mode) signature."""
    return URGymEnv(6, max_episode_steps=None, camera=camera, reward_type=reward_type, render_mode=render_mode, **kw)


def BoxManipulation(button_touch_mode="any", camera=None, render_mode="human", **kw):
    """env_box_v0.BoxManipulation(button_touch_mode, camera, render_mode) signature."""
    return URGymEnv(7, max_episode_steps=None, camera=camera, render_mode=render_mode,
                    button_touch_mode=button_touch_mode, **kw)


__all__ = ["make", "TASKS", "URGymEnv", "URGymVectorEnv", "BallBalance", "CubesPush", "CubesGrasp", "Golf",
           "CubesPushDiff", "GolfJoints", "TwoBallsBalance", "BoxManipulation", "spaces_for"]
