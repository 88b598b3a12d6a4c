"""Box-v0 glue (env_box_v0.py:118-216) pinned against fixtures recorded from the reference's
own BoxManipulation with scripted physics (tools/gen_golden.py box -> box_glue.json): the step head (world ee pose
+ float32 action -> the IK target, the last component -> the gripper command, its asin within 1 ulp), the fixed 120 substeps, the
opened -> pressed -> closed reward state machine with the step penalty, termination / is_success, the observation,
valid_button_press in the three button_touch_modes, and reset's structure.  Bit-exact.
"""
import ctypes
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")
MODES = {"any": 0, "robot": 1, "fingers": 2}
ROBOT, BOX = 1, 2


@pytest.fixture(scope="module")
def L(built):
    from oracle import pyoracle
    return pyoracle.lib()


def P(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def load():
    with open(os.path.join(GOLD, "box_glue.json")) as f:
        return json.load(f)


def touches(contacts):
    """the two predicates valid_button_press reads from getContactPoints() (:199-213): a point between the button
    (box link 0) and the robot, in either orientation; and the same restricted to the finger links 9..18"""
    robot = finger = False
    for c in contacts:
        _, a, b, la, lb = c[:5]
        if a == BOX and la == 0 and b == ROBOT:
            robot = True
            finger |= 9 <= lb <= 18
        if a == ROBOT and b == BOX and lb == 0:
            robot = True
            finger |= 9 <= la <= 18
    return int(robot), int(finger)


def test_box_step_glue(L):
    flags = {}
    for c in load()["box_step"]:
        a = np.array(c["action"], np.float32)
        ee = np.array(c["ee_pose"], np.float64)
        t7 = np.zeros(7)
        L.ugo_g_box_target(P(ee), P(a), P(t7))
        assert t7.tolist() == c["move_target"] and c["control"] == "end"
        # the gripper map 0.715 - asin(..): fdlibm's asin (ug_detmath.h) within 1 ulp of glibc's, an absolute
        # 4e-16 after the subtraction (the bar of tests/test_golden.py's gripper map)
        g = L.ugo_gripper_angle(float(a[7]))
        assert abs(g - c["gripper_target"]) <= 4e-16
        assert c["substeps"] == 120
        f = flags.setdefault(c["mode"], np.zeros(3, np.int32))
        rt, ft = touches(c["contacts"])
        press = L.ugo_g_box_press(c["button"], MODES[c["mode"]], rt, ft)
        r = np.zeros(1)
        closed = L.ugo_g_box_reward(P(f), c["door"], press, P(r))
        assert r[0] == c["reward"], c
        assert bool(closed) == c["terminated"] == c["is_success"]
        assert [bool(x) for x in f] == c["flags"]
        assert c["obs"] == c["ee_pose"]  # np.array(robot.get_joint_obs()['ee_pos'])


def test_box_button_press_modes(L):
    for c in load()["box_press"]:
        rt, ft = touches(c["contacts"])
        assert bool(L.ugo_g_box_press(c["button"], MODES[c["mode"]], rt, ft)) == c["valid"], c


def test_box_reset_structure(built):
    """reset (:179-186): robot.reset (10 substeps), move_ee(current pose, 'end'), both box joints to 0 at rest, the
    flags cleared, obs = the ee world pose"""
    from oracle.pyoracle import OracleEnv
    g = load()["box_reset"]
    names = [c[0] for c in g["calls"]]
    assert names == ["robot.reset", "move_ee", "resetJointState", "resetJointState", "setJointMotorControl2",
                     "setJointMotorControl2"]
    assert g["calls"][1][1] == g["obs"] and g["calls"][1][2] == "end"
    assert g["calls"][4][2] == {"force": 1} and g["calls"][5][2] == {"force": 0}
    assert g["flags"] == [False, False, False]
    e = OracleEnv(7, 3)
    obs, n = e.reset()
    assert n == 10
    st = e.get_state()
    from urgym_amd.layout import F_OBJ, OBJ_DOUBLES, F_TASK
    for o in range(2):
        rec = st[F_OBJ + o * OBJ_DOUBLES: F_OBJ + (o + 1) * OBJ_DOUBLES]
        assert rec[7] == 0.0 and rec[10] == 0.0  # joint velocity, joint position
    assert st[F_TASK] == 0 and st[F_TASK + 1] == 0 and st[F_TASK + 3] == 0
    # obs: the ee world pose (robot base at (0, 0.5, 0))
    assert obs.shape == (7,)
