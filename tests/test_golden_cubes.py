"""CubesPush / CubesGrasp glue (urgym_amd/csrc/ug_glue.h, shared by oracle and HIP kernels) pinned
against fixtures generated from the reference's own Python (tools/gen_golden.py -> cubes_glue.json).

The physics queries (contacts, AABBs, link states, poses) are scripted in the fixture; what is compared
is the reference's arithmetic on them: draws -> placements, IK targets, random.choices, subgoal and
reward logic, gripper opening and centre.  Bar: bit-exact, except where a transcendental (tanh in the
distance reward, sin/cos of the placement angle) is involved: within 2 ulp of glibc.
"""
import ctypes
import json
import os
import random

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load():
    with open(os.path.join(GOLD, "cubes_glue.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def L(built):
    from oracle import pyoracle
    return pyoracle.lib()


def P(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def test_cubespush_reset_placement_and_target(L):
    for case in load()["cubespush_reset"]:
        random.seed(case["seed"])
        x = L.ugo_g_cp_cube1_x(random.random())
        assert case["cubes"][0] == [0.0, -0.5, 0.1]
        assert case["cubes"][1] == [x, -0.7, 0.1]                       # env_cubes_push_v0.py:240-246
        (name, pose, method), close = case["calls"]
        assert name == "move_ee" and method == "end" and close == ["close", 100]
        assert pose[:3] == [x, -0.7, 0.1 + 0.2]                          # :219-220
        assert pose[3:] == [0.0, 0.7071067811865475, 0.0, 0.7071067811865476] == case["vertical_quaternion"]


def test_cubespush_step_reward_and_target(L):
    for c in load()["cubespush_step"]:
        a = np.array(c["action"], np.float32)
        want_target = [c["ee_pose"][i] + float(a[i]) for i in range(3)] + [0.0, 0.7071067811865475, 0.0, 0.7071067811865476]
        assert c["ik_target"] == want_target                             # :121-125
        table = any(l != 0 for l in c["table_links"])                    # :176-183
        touched = any(9 <= l <= 18 for l in c["cube1_links"])            # :185-194
        r = np.zeros(1)
        sparse = int(c["reward_type"] == "sparse")                      # :159 reward_type
        succ = L.ugo_g_cp_reward(int(table), int(touched), P(np.array(c["cube0"])), P(np.array(c["cube1"])), sparse,
                                 P(r))
        assert r[0] == pytest.approx(c["reward"], rel=0, abs=4e-16), c
        assert bool(succ) == c["is_success"] == c["terminated"]
        assert c["obs"] == c["ee_pose"][:3] + c["cube0"] + c["cube1"]   # :196-205


def test_cubesgrasp_create_cube(L):
    for c in load()["cubesgrasp_create"]:
        random.seed(c["seed"])
        u0, u1 = random.random(), random.random()
        assert random.random() == c["next_random"]                       # exactly two draws
        xy = np.zeros(2)
        L.ugo_g_cg_cube_xy(u0, u1, P(xy))
        assert xy[0] == pytest.approx(c["cube"][0], rel=5e-16)
        assert xy[1] == pytest.approx(c["cube"][1], rel=5e-16)
        assert c["cube"][2] == 0.1


def test_cubesgrasp_random_choices(L):
    cases = load()["cubesgrasp_choose"]
    assert len(cases) >= 30
    for c in cases:
        random.seed(c["seed"])
        u = random.random()
        assert u == c["u"]
        assert L.ugo_g_cg_choose(c["w"][0], c["w"][1], u) == c["selected"], c


def test_cubesgrasp_step_glue(L):
    norm3 = lambda v: L.ugo_norm3(P(np.ascontiguousarray(v, dtype=np.float64)))
    for c in load()["cubesgrasp_step"]:
        aabbs = np.array(c["aabb11"][0] + c["aabb11"][1] + c["aabb16"][0] + c["aabb16"][1], np.float64)
        ctr = np.zeros(3)
        L.ugo_g_union_center(P(aabbs), P(ctr))
        dist = norm3(ctr - np.array(c["cube"]))
        assert dist == c["distance"]                                     # :199-204 (numpy norm: fused dot)
        opening = L.ugo_g_cg_opening(norm3(np.array(c["frame16"]) - np.array(c["frame11"])))
        assert opening == c["opening"]                                   # :349-376
        left = any(l in (11, 12, 13) for l in c["robot_links"])
        right = any(l in (16, 17, 18) for l in c["robot_links"])
        flags = np.array([c["flags_in"]["approached"], c["flags_in"]["grasped"]], np.int32)
        r = np.zeros(1)
        succ = L.ugo_g_cg_reward(P(flags), dist, opening, int(left and right), c["cube"][2], P(r))
        assert r[0] == pytest.approx(c["reward"], rel=0, abs=4e-16), c
        assert [bool(flags[0]), bool(flags[1])] == [c["flags_out"]["approached"], c["flags_out"]["grasped"]]
        assert bool(succ) == c["is_success"] == c["terminated"]
        # action 0.9/0.1 under random.seed(3) picks the move branch: move_ee(joint) with action[2:8]
        random.seed(3)
        sel = L.ugo_g_cg_choose(np.float32(c["action"][0]), np.float32(c["action"][1]), random.random())
        assert sel == 0 and c["calls"] == [["move_ee", c["action"][2:8], "joint"]]
        obs = c["obs"]
        assert obs[:2] == [float(c["flags_out"]["approached"]), float(c["flags_out"]["grasped"])]
        assert obs[9] == opening and obs[10:13] == c["cube"]


def test_numpy_norm3_matches_image_numpy(L):
    rng = np.random.default_rng(3)
    for _ in range(2000):
        v = rng.uniform(-1, 1, 3)
        assert L.ugo_norm3(P(np.ascontiguousarray(v))) == np.linalg.norm(v)
