"""GPU parity: the HIP product path (liburgym.so) against the CPU restatement (oracle/).

Both implement the same algorithm with the same operation order and no FMA
contraction, so the bar is bit-identical FP64 state, observations, rewards,
terminations and substep counts (tolerance 0).  At the full 4096-env config
we check size-independent properties (finiteness, ball on paddle after reset,
determinism across runs) plus bit-exact parity on a sample of envs.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20241220


@pytest.fixture(scope="module")
def mods(built):
    from urgym_amd._native import Sim
    from oracle.pyoracle import OracleEnv
    return Sim, OracleEnv


def _oracles(OracleEnv, n, seed, idx=None):
    idx = range(n) if idx is None else idx
    return {i: OracleEnv(0, seed + i) for i in idx}


def test_reset_bit_exact(mods):
    Sim, OracleEnv = mods
    n = 64
    sim = Sim(0, n, seed=SEED)
    obs = sim.reset()
    st = sim.get_state()
    ref = _oracles(OracleEnv, n, SEED)
    for i, r in ref.items():
        o, _ = r.reset()
        assert np.array_equal(obs[i], o), i
        assert np.array_equal(st[i], r.get_state()), i


def test_substep_bit_exact_from_shared_state(mods):
    """Same input state -> one p.stepSimulation() -> identical state (contacts active)."""
    Sim, OracleEnv = mods
    n = 32
    sim = Sim(0, n, seed=SEED)
    sim.reset()
    st = sim.get_state()
    ref = _oracles(OracleEnv, n, SEED)
    for k in range(5):
        sim.substep()
        for i, r in ref.items():
            if k == 0:
                r.set_state(st[i])
            r.substep()
    st2 = sim.get_state()
    for i, r in ref.items():
        assert np.array_equal(st2[i], r.get_state()), i


def test_steps_bit_exact_with_autoreset(mods):
    Sim, OracleEnv = mods
    n, T = 64, 12
    sim = Sim(0, n, seed=SEED)
    sim.set_autoreset(True, 500)
    obs = sim.reset()
    ref = _oracles(OracleEnv, n, SEED)
    for r in ref.values():
        r.reset()
    rng = np.random.default_rng(SEED)
    for t in range(T):
        act = rng.uniform(-0.1, 0.1, size=(n, 3)).astype(np.float32)
        out = sim.step(act)
        for i, r in ref.items():
            o, rew, term, succ, ns = r.step(act[i])
            assert bool(out["terminated"][i]) == term, (t, i)
            assert out["reward"][i] == rew
            if term:
                assert np.array_equal(out["final_obs"][i], o), (t, i)
                o2, ns2 = r.reset()
                ns += ns2
                o = o2
            assert np.array_equal(out["obs"][i], o), (t, i)
            assert out["substeps"][i] == ns, (t, i)
    st = sim.get_state()
    for i, r in ref.items():
        assert np.array_equal(st[i], r.get_state()), i


def test_ik_and_link_state_bit_exact(mods):
    Sim, OracleEnv = mods
    n = 16
    sim = Sim(0, n, seed=SEED)
    sim.reset()
    st = sim.get_state()
    ref = _oracles(OracleEnv, n, SEED)
    ls = sim.link_state(7)
    rng = np.random.default_rng(1)
    tgt = np.concatenate([ls[:, :3] + rng.uniform(-0.05, 0.05, (n, 3)), ls[:, 3:]], axis=1)
    q = sim.ik(tgt)
    for i, r in ref.items():
        r.set_state(st[i])
        assert np.array_equal(ls[i], r.link_state(7))
        assert np.array_equal(q[i], r.ik(tgt[i, :3], tgt[i, 3:]))


def test_full_config_properties(mods):
    """BallBalance x 4096 (config B): finite, ball resting on the paddle after reset, determinism,
    and bit-exact parity on a sample of envs."""
    Sim, OracleEnv = mods
    n = 4096
    a = Sim(0, n, seed=SEED)
    a.set_autoreset(True, 500)
    obs = a.reset()
    assert np.all(np.isfinite(obs))
    # obs[:,5] = paddle_z - ball_z: the ball starts above the paddle
    assert np.all(obs[:, 5] < 0)
    rng = np.random.default_rng(SEED)
    act = rng.uniform(-0.1, 0.1, size=(n, 3)).astype(np.float32)
    out = a.step(act)
    assert np.all(np.isfinite(out["obs"]))
    assert np.all(out["reward"] == 1.0)
    assert np.all((out["substeps"] >= 1) & (out["substeps"] <= 480 * 3 + 10))
    st = a.get_state()
    sample = [0, 1, 63, 64, 1000, 2047, 4095]
    for i in sample:
        r = OracleEnv(0, SEED + i)
        r.reset()
        o, rew, term, succ, ns = r.step(act[i])
        if term:
            r.reset()
        assert np.array_equal(st[i], r.get_state()), i
    # run-to-run determinism on the GPU (no atomics, no data races)
    b = Sim(0, n, seed=SEED)
    b.set_autoreset(True, 500)
    b.reset()
    out_b = b.step(act)
    assert np.array_equal(out["obs"], out_b["obs"])
    assert np.array_equal(b.get_state(), st)


def _task_actions(task, rng, n):
    """uniform in the reference's action_space (SURVEY.md 8(d) synthetic inputs)"""
    if task == 2:
        lo = np.array([0, 0] + [-np.pi] * 6 + [0], np.float64)
        hi = np.array([1, 1] + [np.pi] * 6 + [1], np.float64)
        return rng.uniform(lo, hi, size=(n, 9)).astype(np.float32)
    if task == 5:  # GolfJoints: 6 joint deltas (TwoBallsBalance (6) has BallBalance's 3 euler deltas)
        return rng.uniform(-0.1, 0.1, size=(n, 6)).astype(np.float32)
    return rng.uniform(-0.1, 0.1, size=(n, 3)).astype(np.float32)


@pytest.mark.parametrize("task,max_steps", [(1, 50), (2, 20), (3, 100), (4, 50), (5, 100), (6, 500)])
def test_cube_tasks_bit_exact_with_autoreset(mods, task, max_steps):
    """CubesPush / CubesGrasp / Golf and the variants CubesPushDiff / GolfJoints
    (8(f) rank 1): reset, steps with contact-predicate rewards, subgoal flags, random.choices draws, the
    compound club, rolling friction, joint-space control and same-step autoreset, bit-identical to the
    oracle."""
    Sim, OracleEnv = mods
    n, T = 32, 6
    sim = Sim(task, n, seed=SEED)
    sim.set_autoreset(True, max_steps)
    obs = sim.reset()
    ref = {i: OracleEnv(task, SEED + i) for i in range(n)}
    for i, r in ref.items():
        o, _ = r.reset()
        assert np.array_equal(obs[i], o), (task, i)
    rng = np.random.default_rng(SEED + task)
    elapsed = np.zeros(n, int)
    for t in range(T):
        act = _task_actions(task, rng, n)
        out = sim.step(act)
        for i, r in ref.items():
            o, rew, term, succ, ns = r.step(act[i])
            elapsed[i] += 1
            assert out["reward"][i] == rew, (task, t, i)
            assert bool(out["terminated"][i]) == term and bool(out["success"][i]) == succ, (task, t, i)
            if term or elapsed[i] >= max_steps:
                assert np.array_equal(out["final_obs"][i], o), (task, t, i)
                o, ns2 = r.reset()
                ns += ns2
                elapsed[i] = 0
            assert np.array_equal(out["obs"][i], o), (task, t, i)
            assert out["substeps"][i] == ns, (task, t, i)
    st = sim.get_state()
    for i, r in ref.items():
        assert np.array_equal(st[i], r.get_state()), (task, i)


@pytest.mark.parametrize("task", [1, 2, 3, 4, 5])
def test_cube_tasks_reset_draws(mods, task):
    """urgym_reset with caller-supplied draws == oracle reset with the same draws"""
    Sim, OracleEnv = mods
    n = 8
    sim = Sim(task, n, seed=SEED)
    draws = np.random.default_rng(7).uniform(0, 1, size=(n, sim.ndraw))
    obs = sim.reset(draws=draws)
    for i in range(n):
        o, _ = OracleEnv(task, SEED + i).reset(draws=draws[i])
        assert np.array_equal(obs[i], o), (task, i)
