"""The C-ABI library: builds, loads, exports every symbol include/urgym.h declares, and refuses to
run without a GPU (no CPU fallback)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "urgym.h")).read()
    return sorted(set(re.findall(r"\b(urgym_[a-z_]+)\s*\(", txt)))


def test_header_and_binding_agree(built):
    from urgym_amd._native import SYMBOLS
    assert sorted(SYMBOLS) == header_symbols()


@pytest.mark.parametrize("robot", ["ur5_robotiq_85", "ur5_robotiq_140", "g8"])
def test_library_exports_every_declared_symbol(built, robot):
    from urgym_amd._native import G8_LIB, ROBOT_LIBS
    L = ctypes.CDLL(G8_LIB if robot == "g8" else ROBOT_LIBS[robot])  # every build carries the whole C-ABI
    for s in header_symbols():
        assert hasattr(L, s), s


def test_robot_builds_differ_only_in_the_robot():
    """UR5Robotiq140's restatement (robot.py:221-240): the same tree, its own limits / finger axis / mimic signs;
    the same task shapes and state layout as the Robotiq-85 build"""
    from oracle.pyoracle import LIB_PATH_R140, lib as olib
    a, b = olib(), olib(LIB_PATH_R140)
    assert a.ugo_state_dim() == b.ugo_state_dim()
    assert [a.ugo_obs_dim(t) for t in range(8)] == [b.ugo_obs_dim(t) for t in range(8)]
    from urgym_amd._native import lib
    with pytest.raises(ValueError):
        lib("panda")  # robot.py:150-175, not built


def test_static_shapes(built):
    from urgym_amd._native import lib
    L = lib()
    assert [L.urgym_obs_dim(t) for t in range(7)] == [6, 9, 17, 9, 9, 15, 9]
    assert [L.urgym_act_dim(t) for t in range(7)] == [3, 3, 9, 3, 3, 6, 3]
    assert [L.urgym_num_draws(t) for t in range(7)] == [2, 1, 2, 2, 1, 2, 4]
    from oracle.pyoracle import lib as olib
    assert L.urgym_state_dim() == olib().ugo_state_dim()


def test_spaces_match_reference(built):
    import numpy as np
    from urgym_amd.envs import spaces_for
    obs, act = spaces_for(0)
    assert obs.shape == (6,) and act.shape == (3,) and act.dtype == np.float32 and obs.dtype == np.float64
    assert np.allclose(act.low, -0.1) and np.allclose(obs.high[:3], np.pi)
    obs, act = spaces_for(5)  # GolfJoints: 6 joint deltas, joints + Golf obs
    assert obs.shape == (15,) and act.shape == (6,) and np.allclose(obs.high[:6], 2 * np.pi)
    from urgym_amd.envs import TASKS
    assert TASKS["URGym/CubesPushDiff-v0"] == (4, 50) and TASKS["URGym/GolfJoints-v0"] == (5, 100)
    assert TASKS["URGym/TwoBallsBalance-v0"] == (6, 500)
    obs, act = spaces_for(6)  # TwoBallsBalance: euler + two relative ball positions
    assert obs.shape == (9,) and act.shape == (3,) and np.allclose(obs.low[3:], -1.0)


def test_wrappers_refuse_what_they_do_not_implement(built):
    import numpy as np
    from urgym_amd.envs import make, TASKS, spaces_for
    assert TASKS["URGym/Box-v0"] == (7, 200)  # envs/__init__.py:3-8
    obs, act = spaces_for(7)  # env_box_v0.py:41-43: ee pose; pose deltas + gripper opening
    assert obs.shape == (7,) and act.shape == (8,) and act.high[7] == np.float32(0.085)
    from urgym_amd.envs.core import _check_button
    with pytest.raises(ValueError):
        _check_button(7, "elbow")
    with pytest.raises(TypeError):
        _check_button(0, "any")  # button_touch_mode is Box-v0's kwarg only
    with pytest.raises(KeyError):
        make("URGym/NoSuchEnv-v0")
    from urgym_amd.envs.core import _check_kwargs
    with pytest.raises(ValueError):
        _check_kwargs(None, "shaped")
    with pytest.raises(TypeError):
        _check_kwargs(object(), "dense")  # a camera must be urgym_amd.camera.Camera (utilities.py:62)
    from urgym_amd.camera import Camera
    _check_kwargs(Camera((1, 1, 1), (0, 0, 0), (0, 0, 1), 0.1, 5, (32, 32), 40), "dense")
    _check_kwargs(None, "sparse")


@pytest.mark.skipif(os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK), reason="GPU present")
def test_no_cpu_fallback_without_gpu(built):
    from urgym_amd._native import Sim
    with pytest.raises(RuntimeError):
        Sim(0, 4)
