"""UR5Robotiq140 (robot.py:221-240): liburgym_r140.so -- the same kernels over the Robotiq-140
model header (tools/build_model.py on ur5_robotiq_140.urdf: its meshes' full hulls, masses, limits, the finger
joint's -x axis) and the flipped mimic multipliers -- bit-exact against the restatement built the same way
(oracle libugoracle_r140.so) through autoreset steps on the tasks whose glue drives the gripper hardest (BallBalance
grasps the paddle at reset, CubesGrasp opens / closes on cubes, Box-v0 presses with the fingers), and different from
the Robotiq-85 build on the same seeds (the robot is really swapped)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 777
R140 = "ur5_robotiq_140"


@pytest.fixture(scope="module")
def mods(built):
    from urgym_amd._native import Sim
    from oracle.pyoracle import LIB_PATH_R140, OracleEnv
    return Sim, OracleEnv, LIB_PATH_R140


def actions(task, rng, n):
    if task == 2:
        lo = np.array([0, 0] + [-np.pi] * 6 + [0], np.float64)
        hi = np.array([1, 1] + [np.pi] * 6 + [1], np.float64)
        return rng.uniform(lo, hi, size=(n, 9)).astype(np.float32)
    if task == 7:
        lo = np.array([-0.05] * 3 + [-np.pi / 10] * 4 + [0.0])
        hi = np.array([0.05] * 3 + [np.pi / 10] * 4 + [0.085])
        return rng.uniform(lo, hi, size=(n, 8)).astype(np.float32)
    return rng.uniform(-0.1, 0.1, size=(n, 3)).astype(np.float32)


@pytest.mark.parametrize("task,steps,max_steps", [(0, 6, 4), (2, 8, 5), (7, 3, 2)])
def test_r140_bit_exact(mods, task, steps, max_steps):
    Sim, OracleEnv, lib140 = mods
    n = 6
    sim = Sim(task, n, seed=SEED, robot=R140)
    sim.set_autoreset(True, max_steps)
    obs = sim.reset()
    ref = [OracleEnv(task, SEED + i, lib_path=lib140) for i in range(n)]
    for i, r in enumerate(ref):
        assert np.array_equal(obs[i], r.reset()[0]), i
    rng = np.random.default_rng(task)
    el = np.zeros(n, int)
    for t in range(steps):
        act = actions(task, rng, n)
        out = sim.step(act)
        for i, r in enumerate(ref):
            o, rew, term, succ, ns = r.step(act[i])
            el[i] += 1
            trunc = el[i] >= max_steps
            assert out["reward"][i] == rew and bool(out["terminated"][i]) == term, (t, i)
            assert bool(out["truncated"][i]) == trunc and bool(out["success"][i]) == succ, (t, i)
            if term or trunc:
                assert np.array_equal(out["final_obs"][i], o), (t, i)
                o, ns2 = r.reset()
                ns += ns2
                el[i] = 0
            assert np.array_equal(out["obs"][i], o), (t, i)
            assert out["substeps"][i] == ns, (t, i)
    st = sim.get_state()
    for i, r in enumerate(ref):
        assert np.array_equal(st[i], r.get_state()), i
    sim.close()


def test_r140_is_a_different_robot(mods):
    """same seeds, same actions: the Robotiq-140 build's reset (the paddle grasp) ends elsewhere than the 85's, and
    its gripper joints sit within the 140's limits (finger_joint in [0, 0.7], the mimic children's signs flipped)"""
    Sim, _, _ = mods
    a, b = Sim(0, 4, seed=SEED), Sim(0, 4, seed=SEED, robot=R140)
    oa, ob = a.reset(), b.reset()
    assert not np.array_equal(oa, ob)
    qa, qb = a.get_state()[:, 6:12], b.get_state()[:, 6:12]
    assert np.all(qb[:, 0] >= -1e-3) and np.all(qb[:, 0] <= 0.7 + 1e-3)
    assert np.all(np.sign(qb[:, 1:]) == -np.sign(qa[:, 1:]))  # the mimic children turn the other way
    a.close()
    b.close()
