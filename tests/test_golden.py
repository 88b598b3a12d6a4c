"""Oracle (CPU restatement) pinned against fixtures generated from the reference's own code.

tests/golden/*.json were produced by tools/gen_golden.py, which imports
/root/reference/urgym with stub pybullet/gymnasium/cv2 modules (the physics is
scripted, the glue is the reference's).  Bar: bit-exact for the glue.
"""
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def ora(built):
    from oracle import pyoracle
    return pyoracle


def test_geometric_distance_reward(ora):
    # utilities.py:192-207; oracle uses fdlibm-style tanh -> within 1 ulp of numpy's
    for v, s, m, want in load("utilities.json")["geometric_distance_reward"]:
        got = ora.gdr(v, s, m)
        assert got == pytest.approx(want, rel=4e-16, abs=1e-300), (v, s, m)


def test_gripper_angle_map(ora):
    # robot.py:103-111 + UR5Robotiq85.move_gripper robot.py:213-218 (asin within 1 ulp)
    for kind, pct, target, force, maxvel in load("gripper.json")["gripper"]:
        L = 0 + (0.085 - 0) * (pct / 100) if kind == "open" else 0.085 - (0.085 - 0) * (pct / 100)
        assert ora.gripper_angle(L) == pytest.approx(target, rel=0, abs=4e-16)
        assert force == 1000.0 and maxvel == 2.0  # URDF finger_joint effort / velocity


def test_python_random_stream_bit_exact(ora):
    # CPython random.seed(int) + random.random(): MT19937 restated in C
    e = ora.OracleEnv(0, 0)
    for seed, vals in load("random.json")["random"]:
        e.rng_seed(seed)
        assert [e.rng_random() for _ in vals] == vals


def test_ballbalance_create_ball_bit_exact(ora):
    # env_ball_balance_v0.py:186-205: draw order x then y, ball 0.2 + r above the paddle
    e = ora.OracleEnv(0, 0)
    for seed, paddle, want in load("random.json")["ballbalance_create_ball"]:
        e.rng_seed(seed)
        assert e.bb_ball_position(paddle).tolist() == want


def test_ballbalance_step_glue(ora):
    """euler + float32 action (numpy float64 promotion), obs = paddle euler ++ (paddle - ball),
    terminated = ball_z < paddle_z, reward 1, info {} (env_ball_balance_v0.py:105-143)."""
    for c in load("ballbalance_glue.json")["ballbalance_step"]:
        a = np.array(c["action"], dtype=np.float32)
        got = (np.array(c["ee_euler"]) + a.astype(np.float64)).tolist()
        assert got == c["euler_plus_action"]
        assert c["ik_target"][:3] == c["ee_pose"][:3] and c["ik_method"] == "end"
        # obs via the oracle's observe() on a state holding the scripted paddle/ball poses
        e = ora.OracleEnv(0, 0)
        s = e.get_state()
        from urgym_amd import layout as LY
        s[LY.F_OACTIVE:LY.F_OACTIVE + 2] = 1  # objects active
        s[LY.obj(0):LY.obj(0) + 7] = c["paddle"]
        s[LY.obj(1):LY.obj(1) + 3] = c["ball"]
        e.set_state(s)
        obs = e.observe()
        assert obs[3:].tolist() == c["obs"][3:]
        # the paddle euler part is pybullet's getEulerFromQuaternion (scripted in the fixture)
        assert obs[:3].tolist() == ora.euler_from_quat(c["paddle"][3:]).tolist()
        assert e.terminated() == c["terminated"]
        assert c["reward"] == 1 and c["truncated"] is False and c["info"] == {}


def test_wait_until_stable_sum(ora):
    # np.sum pairwise order over 12 |dq| (env_ball_balance_v0.py:100) reproduced bit-exactly
    g = load("wait_until_stable.json")
    qs = np.array(g["positions"])
    for k, want in enumerate(g["abs_sums"]):
        assert ora.stable_sum(np.abs(qs[k] - qs[k + 1])) == want
    assert g["stable"] is False
