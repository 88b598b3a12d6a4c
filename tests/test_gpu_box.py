"""Box-v0 on the GPU (env_box_v0.py) against the CPU restatement: the door (revolute) and
button (prismatic) links of the fixed-base box (ug_joint.h), its compound colliders (a box and three handle
cylinders on the door, the button cylinder, the walls), the door-button self-collision, the button motor and both
joint limits, the 120-substep step, the opened -> pressed -> closed reward state machine in the three
button_touch_modes and the reset through the 200-step truncation.  Bar: bit-identical FP64 (tolerance 0) for
states, observations, rewards, terminations, truncations, substep counts and contact tuples.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 4242
TASK = 7


@pytest.fixture(scope="module")
def mods(built):
    from urgym_amd._native import Sim
    from oracle.pyoracle import OracleEnv
    return Sim, OracleEnv


def _actions(rng, n):
    lo = np.array([-0.05] * 3 + [-np.pi / 10] * 4 + [0.0])
    hi = np.array([0.05] * 3 + [np.pi / 10] * 4 + [0.085])
    return rng.uniform(lo, hi, size=(n, 8)).astype(np.float32)


def _run(Sim, OracleEnv, n, T, seed, mode="any", max_steps=200, idx=None, state_fn=None):
    sim = Sim(TASK, n, seed=seed)
    sim.set_button_mode(mode)
    sim.set_autoreset(True, max_steps)
    obs = sim.reset()
    idx = range(n) if idx is None else idx
    ref = {i: OracleEnv(TASK, seed + i) for i in idx}
    for i, r in ref.items():
        r.set_button_mode(mode)
        o, ns = r.reset()
        assert np.array_equal(obs[i], o), i
    st = sim.get_state()
    for i, r in ref.items():
        assert np.array_equal(st[i], r.get_state()), i
    if state_fn is not None:  # crafted states, installed on both sides
        st = state_fn(st)
        sim.set_state(st)
        for i, r in ref.items():
            r.set_state(st[i])
    rng = np.random.default_rng(seed)
    el = {i: 0 for i in ref}
    seen = {"reward": set(), "term": 0, "trunc": 0}
    for t in range(T):
        act = _actions(rng, n)
        out = sim.step(act)
        for i, r in ref.items():
            o, rew, term, succ, ns = r.step(act[i])
            el[i] += 1
            trunc = (not term) and el[i] >= max_steps
            assert bool(out["terminated"][i]) == term, (t, i)
            assert bool(out["truncated"][i]) == trunc, (t, i)
            assert out["reward"][i] == rew, (t, i)
            assert bool(out["success"][i]) == succ
            seen["reward"].add(rew)
            seen["term"] += term
            seen["trunc"] += trunc
            if term or trunc:
                assert np.array_equal(out["final_obs"][i], o), (t, i)
                o, ns2 = r.reset()
                ns += ns2
                el[i] = 0
            assert np.array_equal(out["obs"][i], o), (t, i)
            assert out["substeps"][i] == ns, (t, i)
    st = sim.get_state()
    for i, r in ref.items():
        assert np.array_equal(st[i], r.get_state()), i
        assert sim.stats()[i].tolist() == r.stats().tolist()
    return sim, ref, seen


def test_box_reset_and_steps_bit_exact(mods):
    Sim, OracleEnv = mods
    sim, ref, seen = _run(Sim, OracleEnv, 16, 10, SEED)
    out, cnt = sim.contact_points(-1, -1, -2, -2, 64)
    for i, r in ref.items():  # the door resting on the button: the door-button manifold, pybullet tuples
        pts = r.contact_points(-1, -1, -2, -2, 64)
        assert cnt[i] == len(pts) > 0
        assert np.array_equal(out[i][: len(pts)], pts), i


def test_box_through_truncation(mods):
    """a 200-step episode (24,000 substeps) into the TimeLimit truncation and the autoreset after it"""
    Sim, OracleEnv = mods
    sim, ref, seen = _run(Sim, OracleEnv, 4, 202, SEED + 1)
    assert seen["trunc"] == 4


def _door_at(st, q, flags=None):
    """the door at joint position q, its frame quaternion following (ug_joint.h); optionally the task words
    (box_opened, button_pressed, -, box_closed)"""
    from urgym_amd.layout import F_TASK, obj
    st = st.copy()
    h = 0.5 * q
    for i in range(len(st)):
        st[i, obj(0) + 10] = q                                           # joint position (w.x)
        st[i, obj(0) + 3: obj(0) + 7] = [0.0, np.sin(h), 0.0, np.cos(h)]  # frame quaternion (set on both sides)
        if flags is not None:
            st[i, F_TASK], st[i, F_TASK + 1] = flags
    return st


def _door_open(st):
    return _door_at(st, 1.95)  # past the opened threshold 1.9


@pytest.mark.parametrize("mode", ["any", "robot", "fingers"])
def test_box_reward_state_machine(mods, mode):
    """from an opened door: the opened reward fires on the first step, then the button predicate of each
    button_touch_mode runs on the GPU's manifolds exactly as on the restatement's"""
    Sim, OracleEnv = mods
    sim, ref, seen = _run(Sim, OracleEnv, 8, 6, SEED + 2, mode=mode, state_fn=_door_open)
    assert any(abs(r - 0.9) < 1e-12 for r in seen["reward"])  # box_opened: 1 - 0.1


def test_box_closing_terminates_and_resets(mods):
    """opened and pressed already, the door down at 0.05 rad: box_closed fires (reward 0.9), the episode terminates
    with is_success and the same-step autoreset restarts it"""
    Sim, OracleEnv = mods
    sim, ref, seen = _run(Sim, OracleEnv, 8, 3, SEED + 4, state_fn=lambda st: _door_at(st, 0.05, (1.0, 1.0)))
    assert seen["term"] == 8 and any(abs(r - 0.9) < 1e-12 for r in seen["reward"])


def test_box_at_size(mods):
    """1024 envs, 3 steps: finite everywhere, sampled envs bit-exact"""
    Sim, OracleEnv = mods
    sim, ref, seen = _run(Sim, OracleEnv, 1024, 3, SEED + 3, idx=[0, 511, 1023])
    assert np.all(np.isfinite(sim.get_state()))


def test_box_refuses_lod(mods):
    Sim, _ = mods
    from urgym_amd._native import GEOM_LOD
    with pytest.raises(RuntimeError):
        Sim(TASK, 2, flags=GEOM_LOD)


# arm offsets from the reset pose (shoulder pan .. wrist 3) that press the gripper's hulls 0.6-3.7 cm into the door
# compound (its box and handle cylinders) -- found with the restatement (the hull-cylinder pass's
# candidate list under a deep press, team_poly_cyl's FC_MAX cap)
DOOR_PRESS = [[0.0, 0.502, 0.248, -0.339, -0.245, -1.029], [-0.213, 0.156, 0.637, -1.129, 0.122, 0.396],
              [-0.17, 0.619, 0.338, 0.981, -1.024, -0.772], [-0.549, 0.362, 0.42, 0.227, 0.907, 0.257],
              [-0.23, 0.718, 0.007, 0.699, -0.419, 0.375], [-0.033, 0.623, 0.059, 0.415, -0.855, 0.259]]


@pytest.mark.parametrize("contact", ["gjk", "vih"])
def test_box_gripper_pressed_into_the_door(mods, contact):
    """the gripper's full hulls pushed into the door's box and handle cylinders: after one substep the restatement
    reports contacts deeper than 5 mm, and two env-steps from those states are bit-exact on the GPU (state,
    observation, reward, substeps, contact tuples) in both contact modes"""
    Sim, OracleEnv = mods
    from urgym_amd import layout as LY
    from urgym_amd._native import CONTACT_VIH
    fl = CONTACT_VIH if contact == "vih" else 0
    n = len(DOOR_PRESS)
    sim = Sim(TASK, n, seed=SEED, flags=fl)
    sim.set_autoreset(False, 0)
    sim.reset()
    st = sim.get_state()
    ref = [OracleEnv(TASK, SEED + i, flags=fl) for i in range(n)]
    deepest = []
    for i, r in enumerate(ref):
        r.reset()
        assert np.array_equal(st[i], r.get_state()), i
        st[i, LY.F_Q:LY.F_Q + 6] += DOOR_PRESS[i]
        st[i, LY.F_QD:LY.F_QD + 12] = 0.0
        probe = OracleEnv(TASK, SEED + i, flags=fl)
        probe.reset()
        probe.set_state(st[i])
        probe.substep()
        cp = probe.contact_points()
        m = cp[(cp[:, 3] >= 8) & (cp[:, 2] == 1)]
        deepest.append(m[:, 14].min() if len(m) else 0.0)
        r.set_state(st[i])
    assert min(deepest) < -0.02 and sum(d < -0.005 for d in deepest) >= 5, deepest
    sim.set_state(st)
    rng = np.random.default_rng(7)
    for t in range(2):
        act = _actions(rng, n)
        out = sim.step(act)
        got = sim.get_state()
        cps, cnt = sim.contact_points()
        for i, r in enumerate(ref):
            o, rew, term, succ, ns = r.step(act[i])
            assert np.array_equal(out["obs"][i], o) and out["reward"][i] == rew, (t, i)
            assert out["substeps"][i] == ns and np.array_equal(got[i], r.get_state()), (t, i)
            rc = r.contact_points()
            assert cnt[i] == len(rc) and np.array_equal(cps[i, :cnt[i]], rc), (t, i)
    sim.close()
