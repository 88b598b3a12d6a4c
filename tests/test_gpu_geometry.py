"""The two collision geometries.  The default, full geometry is the reference's: the robot's mesh
colliders are PyBullet's convex hulls of all mesh vertices (up to 865 vertices / 1306 faces per link, SURVEY App. A.3;
URDF2Bullet btConvexHullShape + optimizeConvexHull) and the Golf club's disc a true cylinder (GEOM_CYLINDER,
env_golf_v0.py:305) -- every other GPU test runs it (urgym_create's default).  URGYM_FLAG_LOD_GEOMETRY selects the
collision LOD (<= 48-vertex hulls, a 16-gon disc prism), round 2's default.  Here: the LOD mode bit-exact against the
restatement's LOD mode on every task through autoresets and at config B's size; the explicit full flag equal to the
default; the two modes differing; the disc cylinder's contacts (getContactPoints on the club's disc link) exercised
and bit-exact."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20241220
FULL, LOD = 1, 2
MAX_STEPS = {0: 500, 1: 50, 2: 20, 3: 100, 4: 50, 5: 100, 6: 500}


@pytest.fixture(scope="module")
def mods(built):
    from urgym_amd._native import Sim
    from oracle.pyoracle import OracleEnv
    return Sim, OracleEnv


def actions(task, rng, n):
    if task == 2:
        lo = np.array([0, 0] + [-np.pi] * 6 + [0], np.float64)
        hi = np.array([1, 1] + [np.pi] * 6 + [1], np.float64)
        return rng.uniform(lo, hi, size=(n, 9)).astype(np.float32)
    if task == 5:
        return rng.uniform(-0.1, 0.1, size=(n, 6)).astype(np.float32)
    return rng.uniform(-0.1, 0.1, size=(n, 3)).astype(np.float32)


def run(Sim, OracleEnv, task, n, T, max_steps, seed=SEED, flags=LOD):
    sim = Sim(task, n, seed=seed, flags=flags)
    sim.set_autoreset(True, max_steps)
    obs = sim.reset()
    ref = [OracleEnv(task, seed + i, flags=flags) for i in range(n)]
    for i, r in enumerate(ref):
        assert np.array_equal(obs[i], r.reset()[0]), (task, i)
    rng = np.random.default_rng(seed + 31 * task)
    el = np.zeros(n, int)
    ended = 0
    for t in range(T):
        act = actions(task, rng, n)
        out = sim.step(act)
        fl = sim.flags()
        for i, r in enumerate(ref):
            o, rew, term, succ, ns = r.step(act[i])
            f = r.flags()
            el[i] += 1
            trunc = el[i] >= max_steps
            assert out["reward"][i] == rew and bool(out["terminated"][i]) == term, (task, t, i)
            assert bool(out["success"][i]) == succ and bool(out["truncated"][i]) == trunc, (task, t, i)
            if term or trunc:
                assert np.array_equal(out["final_obs"][i], o), (task, t, i)
                o, ns2 = r.reset()
                ns += ns2
                f |= r.flags()
                el[i] = 0
                ended += 1
            assert np.array_equal(out["obs"][i], o), (task, t, i)
            assert out["substeps"][i] == ns, (task, t, i)
            assert fl[i] == f, (task, t, i)
    st = sim.get_state()
    for i, r in enumerate(ref):
        assert np.array_equal(st[i], r.get_state()), (task, i)
        assert np.array_equal(sim.stats()[i], r.stats()), (task, i)
    sim.close()
    return ended


@pytest.mark.parametrize("task", [0, 1, 2, 3, 4, 5, 6])
def test_lod_geometry_bit_exact_every_task(mods, task):
    """every task in the LOD mode, 6 envs x 6 autoreset steps (truncation at 4 steps, so each env resets and keeps
    going), against the restatement's LOD mode"""
    Sim, OracleEnv = mods
    ended = run(Sim, OracleEnv, task, 6, 6, 4)
    assert ended >= 6


def test_full_geometry_grasp_episode(mods):
    """CubesGrasp through its 20-step limit with the default full finger hulls (the grasp-by-friction task where the
    geometry matters most, profiles/collision_fidelity.md)"""
    Sim, OracleEnv = mods
    run(Sim, OracleEnv, 2, 4, 21, MAX_STEPS[2], flags=0)


def test_full_flag_is_the_default_and_lod_differs(mods):
    """urgym_create == urgym_create_ex(..., URGYM_FLAG_FULL_GEOMETRY); the LOD mode is a different trajectory"""
    Sim, _ = mods
    a, b, c = Sim(0, 8, seed=SEED), Sim(0, 8, seed=SEED, flags=FULL), Sim(0, 8, seed=SEED, flags=LOD)
    oa, ob, oc = a.reset(), b.reset(), c.reset()
    assert np.array_equal(oa, ob) and not np.array_equal(oa, oc)
    act = np.random.default_rng(0).uniform(-0.1, 0.1, size=(8, 3)).astype(np.float32)
    ra, rb = a.step(act), b.step(act)
    for key in ra:
        assert np.array_equal(ra[key], rb[key]), key
    for s in (a, b, c):
        s.close()


def test_cylinder_disc_contacts_bit_exact(mods):
    """Golf, full geometry: the club's disc (object 1, link 1) is a true cylinder; its contacts with the robot, the
    ball and the statics come through getContactPoints bit-exact against the restatement, and some exist"""
    Sim, OracleEnv = mods
    n = 8
    sim = Sim(3, n, seed=SEED)
    sim.reset()
    ref = [OracleEnv(3, SEED + i) for i in range(n)]
    for r in ref:
        r.reset()
    rng = np.random.default_rng(9)
    total = 0
    for _ in range(4):
        act = rng.uniform(-0.1, 0.1, size=(n, 3)).astype(np.float32)
        sim.step(act)
        for i, r in enumerate(ref):
            r.step(act[i])
        out, cnt = sim.contact_points(1, -1, 1, -2, max_pts=64)
        for i, r in enumerate(ref):
            want = r.contact_points(1, -1, 1, -2, max_pts=64)
            assert cnt[i] == len(want) and np.array_equal(out[i, :cnt[i]], want), i
            total += cnt[i]
    assert total > 0
    sim.close()


def test_lod_geometry_config_b_size(mods):
    """BallBalance x 4096 in the LOD mode: finite, bounded substeps, sampled envs bit-exact over 3 steps"""
    Sim, OracleEnv = mods
    n = 4096
    sim = Sim(0, n, seed=SEED, flags=LOD)
    sim.set_autoreset(True, 500)
    obs = sim.reset()
    rng = np.random.default_rng(SEED)
    acts = [actions(0, rng, n) for _ in range(3)]
    outs = [sim.step(a) for a in acts]
    for out in outs:
        assert np.all(np.isfinite(out["obs"])) and np.all((out["substeps"] >= 1) & (out["substeps"] <= 3 * 480 + 10))
    st = sim.get_state()
    for i in [0, 777, n // 2, n - 1]:
        r = OracleEnv(0, SEED + i, flags=LOD)
        assert np.array_equal(obs[i], r.reset()[0])
        for t, a in enumerate(acts):
            o, rew, term, succ, ns = r.step(a[i])
            assert outs[t]["reward"][i] == rew and bool(outs[t]["terminated"][i]) == term, (i, t)
            if term:
                r.reset()
        assert np.array_equal(st[i], r.get_state()), i
    sim.close()
