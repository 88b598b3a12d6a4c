"""GPU parity of the round-2 surface: TwoBallsBalance-v0, reward_type='sparse', failure surfacing (flags, event
counters, the non-finite guard), the RNG/elapsed checkpoint, the getContactPoints query, env sharding, the
full-size configs C-E, the gymnasium-style wrappers and long horizons through truncation.  Bar: bit-identical
to the CPU restatement (tolerance 0) wherever a value is compared."""
import numpy as np
import pytest

from urgym_amd import layout as LY

pytestmark = pytest.mark.gpu

SEED = 20241220
MAX_STEPS = {0: 500, 1: 50, 2: 20, 3: 100, 4: 50, 5: 100, 6: 500}


@pytest.fixture(scope="module")
def mods(built):
    from urgym_amd._native import Sim
    from oracle.pyoracle import OracleEnv
    return Sim, OracleEnv


def actions(task, rng, n):
    """uniform in the reference's action_space (SURVEY.md 8(d) synthetic inputs)"""
    if task == 2:
        lo = np.array([0, 0] + [-np.pi] * 6 + [0], np.float64)
        hi = np.array([1, 1] + [np.pi] * 6 + [1], np.float64)
        return rng.uniform(lo, hi, size=(n, 9)).astype(np.float32)
    if task == 5:
        return rng.uniform(-0.1, 0.1, size=(n, 6)).astype(np.float32)
    return rng.uniform(-0.1, 0.1, size=(n, 3)).astype(np.float32)


def run_parity(Sim, OracleEnv, task, n, T, max_steps, reward_type="dense", seed=SEED, inject=None):
    """n envs x T autoreset steps on the GPU and in the oracle: obs, final obs, reward, terminated, truncated,
    success, substeps, flags compared every step; state and event counters at the end.  inject(t, sim, ref)
    may edit both sides before step t.  Returns (sim, ref, per-step GPU outputs)."""
    sim = Sim(task, n, seed=seed)
    sim.set_reward_type(reward_type)
    sim.set_autoreset(True, max_steps)
    obs = sim.reset()
    ref = [OracleEnv(task, seed + i) for i in range(n)]
    for i, r in enumerate(ref):
        r.set_reward_type(reward_type)
        o, _ = r.reset()
        assert np.array_equal(obs[i], o), (task, i)
    rng = np.random.default_rng(seed + 17 * task)
    elapsed = np.zeros(n, int)
    outs = []
    for t in range(T):
        if inject is not None:
            inject(t, sim, ref)
        act = actions(task, rng, n)
        out = sim.step(act)
        fl = sim.flags()
        outs.append(out)
        for i, r in enumerate(ref):
            o, rew, term, succ, ns = r.step(act[i])
            f = r.flags()
            elapsed[i] += 1
            assert out["reward"][i] == rew, (task, t, i)
            assert bool(out["terminated"][i]) == term and bool(out["success"][i]) == succ, (task, t, i)
            trunc = elapsed[i] >= max_steps
            assert bool(out["truncated"][i]) == trunc, (task, t, i)
            if term or trunc:
                if f & 2:  # non-finite guard: the terminal obs of a NaN state is not compared -- NaN propagation
                    # is not specified bit-for-bit (v_max_f64 / v_min_f64 return the non-NaN operand of the PGS clamp,
                    # the C ternaries the NaN); the flag, reward 0, termination and the clean reset are
                    assert fl[i] & 2, (task, t, i)
                else:
                    assert np.array_equal(out["final_obs"][i], o), (task, t, i)
                o, ns2 = r.reset()
                f |= r.flags()
                ns += ns2
                elapsed[i] = 0
            assert np.array_equal(out["obs"][i], o), (task, t, i)
            assert out["substeps"][i] == ns, (task, t, i)
            assert fl[i] == f, (task, t, i, fl[i], f)
    st = sim.get_state()
    stats = sim.stats()
    for i, r in enumerate(ref):
        assert np.array_equal(st[i], r.get_state()), (task, i)
        assert np.array_equal(stats[i], r.stats()), (task, i, stats[i], r.stats())
    return sim, ref, outs


def test_twoballs_bit_exact_with_autoreset(mods):
    """TwoBallsBalance-v0: third free body, two r = 0.003 balls, per-axis shaping reward,
    action penalty, two-ball termination; reset draws in the reference's order."""
    Sim, OracleEnv = mods
    sim, ref, outs = run_parity(Sim, OracleEnv, 6, 32, 8, MAX_STEPS[6])
    assert any(o["terminated"].any() for o in outs)       # an episode ended (and was auto-reset) in the run
    draws = np.random.default_rng(7).uniform(0, 1, size=(8, 4))
    s2 = Sim(6, 8, seed=SEED)
    obs = s2.reset(draws=draws)
    for i in range(8):
        o, _ = OracleEnv(6, SEED + i).reset(draws=draws[i])
        assert np.array_equal(obs[i], o), i


@pytest.mark.parametrize("task", [1, 3, 4, 5])
def test_sparse_reward_bit_exact(mods, task):
    """reward_type='sparse' (env_cubes_push_v0.py:159, env_golf_v0.py:151,163): shaping terms dropped"""
    Sim, OracleEnv = mods
    run_parity(Sim, OracleEnv, task, 16, 4, MAX_STEPS[task], reward_type="sparse")


def test_nonfinite_guard_terminates_and_resets(mods):
    """a non-finite state (injected NaN / inf velocity) ends the episode with reward 0 and the flag set; the
    same-step autoreset starts from a clean robot; identical to the oracle."""
    Sim, OracleEnv = mods
    bad = {2: np.nan, 5: np.inf}

    def inject(t, sim, ref):
        if t != 1:
            return
        st = sim.get_state()
        for i, v in bad.items():
            st[i, LY.F_QD + 3] = v
            s = ref[i].get_state()
            s[LY.F_QD + 3] = v
            ref[i].set_state(s)
        sim.set_state(st)

    sim, ref, outs = run_parity(Sim, OracleEnv, 0, 8, 3, 500, inject=inject)
    from urgym_amd._native import FLAG_NONFINITE
    for i in range(8):
        hit = i in bad
        assert bool(outs[1]["terminated"][i]) == hit or not hit
        if hit:
            assert outs[1]["reward"][i] == 0.0 and outs[1]["terminated"][i] == 1
            assert np.all(np.isfinite(outs[1]["obs"][i]))       # the reset observation
    assert [int(x) for x in sim.stats()[:, 4]] == [1 if i in bad else 0 for i in range(8)]
    assert np.all(np.isfinite(sim.get_state()))
    assert FLAG_NONFINITE == 2


def test_checkpoint_with_rng_and_elapsed_round_trips(mods):
    """get_state + get_rng, run across an autoreset (truncation at 3 steps draws new reset randoms), restore,
    run again: identical outputs (the checkpoint must carry the MT streams and elapsed counters)."""
    Sim, _ = mods
    n = 16
    sim = Sim(0, n, seed=SEED)
    sim.set_autoreset(True, 3)
    sim.reset()
    rng = np.random.default_rng(5)
    acts = [rng.uniform(-0.1, 0.1, size=(n, 3)).astype(np.float32) for _ in range(6)]
    sim.step(acts[0])
    st, (mt, el) = sim.get_state(), sim.get_rng()
    first = [sim.step(a) for a in acts[1:]]
    sim.set_state(st)
    sim.set_rng(mt, el)
    again = [sim.step(a) for a in acts[1:]]
    assert any(o["truncated"].any() for o in first)
    for a, b in zip(first, again):
        for k in a:
            assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("task", [2, 3])
def test_contact_points_bit_exact(mods, task):
    """getContactPoints-shaped query: normalForce / lateral frictions / directions / positions
    against the oracle, and consistent with the contact predicates the rewards use."""
    Sim, OracleEnv = mods
    n = 8
    sim = Sim(task, n, seed=SEED)
    sim.reset()
    rng = np.random.default_rng(3)
    ref = [OracleEnv(task, SEED + i) for i in range(n)]
    for r in ref:
        r.reset()
    for _ in range(2):
        act = actions(task, rng, n)
        sim.step(act)
        for i, r in enumerate(ref):
            r.step(act[i])
    st = sim.get_state()
    queries = [(-1, -1, -2, -2), (0, 1, -2, -2), (1, 0, -2, -2), (0, -1, 11, -2), (0, 1, 16, -2)]
    if task == 3:
        queries += [(1, 0, 0, -2), (2, 1, -2, -2), (0, 12, -2, -2)]
    total = 0
    for q in queries:
        out, cnt = sim.contact_points(*q, max_pts=64)
        for i, r in enumerate(ref):
            r.set_state(st[i])
            want = r.contact_points(*q, max_pts=64)
            assert cnt[i] == len(want), (q, i)
            assert np.array_equal(out[i, :cnt[i]], want), (q, i)
            total += cnt[i]
            if q == (0, 1, -2, -2):  # normal forces are non-negative (lo = 0 on normal rows)
                assert np.all(out[i, :cnt[i], 15] >= 0.0)
    assert total > 0
    if task == 2:  # object_grasped predicate == the query restricted to the finger links (env_cubes_grasp_v0.py:206-226)
        out, cnt = sim.contact_points(0, 1, -2, -2)
        for i, r in enumerate(ref):
            links = set(out[i, :cnt[i], 3].astype(int).tolist())
            assert r.robot_contact(0, 11, 13) == bool(links & {11, 12, 13})
            assert r.robot_contact(0, 16, 18) == bool(links & {16, 17, 18})


@pytest.mark.parametrize("task", [0, 3])
def test_sharded_equals_unsharded(mods, task):
    """two handles holding env ids [0, n/2) and [n/2, n) (env_offset) == one handle of n, bit for
    bit, over autoreset steps -- results do not depend on the sharding (the multi-GPU weak-scaling contract)."""
    Sim, _ = mods
    n, T = 64, 10
    full = Sim(task, n, seed=SEED)
    parts = [Sim(task, n // 2, seed=SEED, env_offset=0), Sim(task, n // 2, seed=SEED, env_offset=n // 2)]
    for s in [full] + parts:
        s.set_autoreset(True, 6)
    o_full = full.reset()
    o_parts = np.concatenate([p.reset() for p in parts])
    assert np.array_equal(o_full, o_parts)
    rng = np.random.default_rng(11)
    for t in range(T):
        act = actions(task, rng, n)
        a = full.step(act)
        b = [parts[0].step(act[:n // 2]), parts[1].step(act[n // 2:])]
        for k in a:
            assert np.array_equal(a[k], np.concatenate([b[0][k], b[1][k]])), (t, k)
    assert np.array_equal(full.get_state(), np.concatenate([p.get_state() for p in parts]))


@pytest.mark.parametrize("task,n", [(1, 4096), (2, 8192), (3, 8192)])
def test_full_size_configs(mods, task, n):
    """configs C (CubesPush x 4096), D (CubesGrasp x 8192), E per GPU (Golf x 8192): finite, bounded substeps,
    run-to-run determinism, and bit-exact parity on sampled envs."""
    Sim, OracleEnv = mods
    a = Sim(task, n, seed=SEED)
    a.set_autoreset(True, MAX_STEPS[task])
    obs = a.reset()
    assert np.all(np.isfinite(obs))
    rng = np.random.default_rng(SEED)
    acts = [actions(task, rng, n) for _ in range(2)]
    outs = [a.step(x) for x in acts]
    for out in outs:
        assert np.all(np.isfinite(out["obs"])) and np.all(np.isfinite(out["reward"]))
        assert np.all((out["substeps"] >= 1) & (out["substeps"] <= 480 * 3 + 10))
    st = a.get_state()
    for i in [0, 1, n // 2 + 3, n - 1]:
        r = OracleEnv(task, SEED + i)
        r.reset()
        for t, x in enumerate(acts):
            o, rew, term, succ, ns = r.step(x[i])
            assert outs[t]["reward"][i] == rew, (task, i, t)
            if term:
                r.reset()
        assert np.array_equal(st[i], r.get_state()), (task, i)
    b = Sim(task, n, seed=SEED)
    b.set_autoreset(True, MAX_STEPS[task])
    b.reset()
    out_b = b.step(acts[0])
    assert np.array_equal(outs[0]["obs"], out_b["obs"])


def test_gym_wrappers_truncation_and_final_observation(mods):
    """make() -> URGymVectorEnv (same-step autoreset, final_observation, TimeLimit truncation) and URGymEnv
    (single env, info keys) against the oracle; CubesGrasp's 20-step limit is crossed."""
    _, OracleEnv = mods
    from urgym_amd.envs import make
    n, T = 8, 22
    venv = make("URGym/CubesGrasp-v0", num_envs=n, seed=SEED)
    obs, info = venv.reset()
    ref = [OracleEnv(2, SEED + i) for i in range(n)]
    for i, r in enumerate(ref):
        assert np.array_equal(obs[i], r.reset()[0])
    rng = np.random.default_rng(2)
    elapsed = np.zeros(n, int)
    saw_trunc = False
    for t in range(T):
        act = actions(2, rng, n)
        obs, rew, term, trunc, infos = venv.step(act)
        for i, r in enumerate(ref):
            o, rw, tm, sc, ns = r.step(act[i])
            elapsed[i] += 1
            assert rew[i] == rw and term[i] == tm and infos["is_success"][i] == sc
            assert trunc[i] == (elapsed[i] >= 20)
            if tm or elapsed[i] >= 20:
                saw_trunc |= bool(trunc[i])
                assert infos["_final_observation"][i]
                assert np.array_equal(infos["final_observation"][i], o)
                o, _ = r.reset()
                elapsed[i] = 0
            assert np.array_equal(obs[i], o)
    assert saw_trunc
    venv.close()
    env = make("URGym/BallBalance-v0", seed=SEED)
    o, info = env.reset()
    r = OracleEnv(0, SEED)
    assert np.array_equal(o, r.reset()[0]) and info == {}
    a = np.array([0.05, -0.02, 0.01], np.float32)
    o, rw, tm, tr, info = env.step(a)
    o2, rw2, tm2, _, _ = r.step(a)
    assert np.array_equal(o, o2) and rw == rw2 and tm == tm2 and tr is False
    assert set(info) <= {"unstable", "nonfinite", "contacts_dropped"}
    env.close()
    env = make("URGym/CubesPush-v0", seed=SEED, reward_type="sparse")
    env.reset()
    _, _, _, _, info = env.step(np.zeros(3, np.float32))
    assert "is_success" in info
    env.close()


@pytest.mark.parametrize("task,max_steps,n,T", [(0, 8, 4, 20), (1, 50, 6, 52), (3, 100, 3, 102), (6, 6, 4, 14)])
def test_long_horizon_through_truncation(mods, task, max_steps, n, T):
    """each task through at least one full episode ending in truncation at max_episode_steps (BallBalance /
    TwoBalls with a shortened limit), every value bit-exact, event counters equal the oracle's."""
    Sim, OracleEnv = mods
    sim, ref, outs = run_parity(Sim, OracleEnv, task, n, T, max_steps)
    assert any(o["truncated"].any() for o in outs)
    print("stats", task, sim.stats().sum(0).tolist())


def _quat_axis_angle(ax, ang):
    ax = np.asarray(ax, np.float64) / np.linalg.norm(ax)
    s = np.sin(ang / 2.0)
    return np.array([ax[0] * s, ax[1] * s, ax[2] * s, np.cos(ang / 2.0)])


def _quat_mul(a, b):
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by, aw * by - ax * bz + ay * bw + az * bx,
                     aw * bz + ax * by - ay * bx + az * bw, aw * bw - ax * bx - ay * by - az * bz])


def test_box_box_clip_cull_and_edge_paths(mods):
    """The box-box narrowphase's rare branches (ug_team.h team_box_box vs the oracle's serial dBoxBox2): a cube
    stacked on a cube rotated about z (octagonal clip polygon -> 8 points -> cullPoints), at 0 degrees (4
    points), tilted so an edge or a corner leads (edge-edge / single-point contacts), and offset to the edge of
    the lower cube (partial clips).  Three substeps from each crafted state, bit-identical to the oracle."""
    Sim, OracleEnv = mods
    n = 25
    sim = Sim(1, n, seed=SEED)
    sim.reset()
    st = sim.get_state().copy()
    rng = np.random.default_rng(7)
    h = 0.02
    for i in range(n):
        o0, o1 = LY.obj(0), LY.obj(1)
        c0 = np.array([0.10, -0.60, h - 1e-5])  # resting on the table, away from the gripper
        st[i, o0:o0 + 3] = c0
        st[i, o0 + 3:o0 + 7] = [0.0, 0.0, 0.0, 1.0]
        st[i, o0 + 7:o0 + 13] = 0.0
        kind = i % 5
        if kind == 0:    # rotated about z: octagon, cull to 4
            q = _quat_axis_angle([0, 0, 1], np.pi / 4 + 0.05 * rng.standard_normal())
            c1 = c0 + np.array([0.0, 0.0, 2 * h - 0.0008])
        elif kind == 1:  # aligned: 4 corner points, no clipping
            q = _quat_axis_angle([0, 0, 1], 0.02 * rng.standard_normal())
            c1 = c0 + np.array([0.003 * rng.standard_normal(), 0.003 * rng.standard_normal(), 2 * h - 0.0006])
        elif kind == 2:  # tilted 45 degrees about x and rotated about z: an edge leads, crossing the top face edge
            q = _quat_mul(_quat_axis_angle([0, 0, 1], 0.6 + 0.1 * rng.standard_normal()), _quat_axis_angle([1, 0, 0], np.pi / 4))
            c1 = c0 + np.array([h * 0.9, 0.0, h + h * np.sqrt(2.0) - 0.0007])
        elif kind == 3:  # offset over the edge of the lower cube: a partial clip
            q = _quat_axis_angle([0, 0, 1], 0.3 + 0.1 * rng.standard_normal())
            c1 = c0 + np.array([1.3 * h, 0.7 * h, 2 * h - 0.0005])
        else:            # both on an edge, the edges crossed: an edge-edge contact
            r2 = np.sqrt(2.0)
            c0 = np.array([0.10, -0.60, h * r2 - 1e-5])
            st[i, o0:o0 + 3] = c0
            st[i, o0 + 3:o0 + 7] = _quat_axis_angle([0, 1, 0], np.pi / 4)
            q = _quat_mul(_quat_axis_angle([0, 0, 1], 0.1 * rng.standard_normal()), _quat_axis_angle([1, 0, 0], np.pi / 4))
            c1 = c0 + np.array([0.002 * rng.standard_normal(), 0.002 * rng.standard_normal(), 2 * h * r2 - 0.0007])
        st[i, o1:o1 + 3] = c1
        st[i, o1 + 3:o1 + 7] = q / np.linalg.norm(q)
        st[i, o1 + 7:o1 + 13] = 0.0
    sim.set_state(st)
    ref = {i: OracleEnv(1, SEED + i) for i in range(n)}
    for i, r in ref.items():
        r.set_state(st[i])
    npts = 0
    for k in range(3):
        sim.substep()
        got = sim.get_state()
        for i, r in ref.items():
            r.substep()
            assert np.array_equal(got[i], r.get_state()), (k, i)
        npts += int(got[:, LY.F_NMAN].sum())
    assert npts > 0
