"""Variant-env glue (CubesPushDiff-v0, GolfJoints-v0) pinned against fixtures
recorded from the reference's own classes with scripted physics (tools/gen_golden.py variants ->
variants_glue.json): PushDiff's relative observation, GolfJoints' joint-space target (float64 joints +
float32 action), its 15-long observation and its reward (the shared Golf glue, ug_glue.h).  Bit-exact.
"""
import ctypes
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def L(built):
    from oracle import pyoracle
    return pyoracle.lib()


def P(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def load():
    with open(os.path.join(GOLD, "variants_glue.json")) as f:
        return json.load(f)


def test_push_diff_observation():
    # cp_obs (oracle) / cpd_obs (kernel): obs[3+3o] = cube_o - ee, the same IEEE subtraction
    for c in load()["push_diff_obs"]:
        ee, c0, c1 = (np.array(c[k]) for k in ("ee", "cube0", "cube1"))
        assert c["obs"] == list(ee) + list(c0 - ee) + list(c1 - ee)


def test_golf_joints_step(L):
    for c in load()["golf_joints_step"]:
        a = np.array(c["action"], np.float32)
        q6 = np.array(c["q6"])
        assert c["control"] == "joint"
        # gf_step (oracle) / glue G_STEP (kernel): q6[i] = q[i] + (double)a[i]
        assert c["move_target"] == [c["q6"][i] + float(a[i]) for i in range(6)]
        stick, ball, hole = np.array(c["stick"]), np.array(c["ball"]), np.array(c["hole"])
        assert c["obs"] == list(q6) + list(stick) + list(stick - ball) + list(hole - ball)
        r = np.zeros(1)
        t = np.zeros(1, np.int32)
        L.ugo_g_gf_reward(P(ball), P(hole), P(stick), 1, 0, 0, 0, P(r), P(t))  # stick in fingers, no floor/touch
        assert r[0] == pytest.approx(c["reward"], rel=0, abs=4e-16) and bool(t[0]) == c["terminated"]
