"""The launch as a work queue (ug_capi.hip k_step / k_reset: one block per wave slot, each taking the next env of the
launch order from a global counter) and the launch order's two sorts (k_order: a bitonic sort in LDS up to 8192
envs, a two-pass counting sort past it).  Every env must be stepped exactly once per launch whatever the order and
the block that takes it, so an env's results do not depend on the handle's size: the first envs of an 8200-env
handle (the counting-sort path, more envs than wave slots) equal a 16-env handle's (the bitonic path) bit for bit,
and every env's episode counter advances by one per step."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20241220


def test_every_env_stepped_once_per_launch(built):
    from urgym_amd._native import Sim
    from urgym_amd.envs import spaces_for
    task, big, small, steps = 1, 8200, 16, 3  # CubesPush: a short reset and step
    act = spaces_for(task)[1]
    lo, hi = np.asarray(act.low, np.float64), np.asarray(act.high, np.float64)
    acts = [np.random.default_rng(t).uniform(lo, hi, size=(big, len(lo))).astype(np.float32) for t in range(steps)]
    sims = {n: Sim(task, n, seed=SEED) for n in (big, small)}
    outs = {}
    for n, sim in sims.items():
        sim.set_autoreset(False, 0)
        sim.reset()
        for t in range(steps):
            out = sim.step(acts[t][:n])
            assert (out["substeps"] > 0).all(), f"n={n}: an env ran no substep in step {t}"
        outs[n] = (out, sim.get_state(), sim.get_rng()[1])
    (ob, sb, eb), (os_, ss, es) = outs[big], outs[small]
    assert (eb == steps).all() and (es == steps).all()
    for k in ("obs", "reward", "substeps", "terminated"):
        assert np.array_equal(ob[k][:small], os_[k]), k
    assert np.array_equal(sb[:small], ss)


@pytest.mark.parametrize("task", [2, 0, 1, 6, 3, 5])
def test_launch_order_models_change_no_result(built, task, monkeypatch):
    """The k_prio models only order the launch (CubesGrasp's peeks each env's MT19937 stream for the branch its
    random.choices will take; Golf, GolfJoints, TwoBalls and CubesGrasp walk tree ensembles): a handle with the models and one without them (URGYM_NO_PRIO_MODEL: the last-substep
    order) give the same results, states and streams bit for bit, across an autoreset (CubesGrasp truncates at 20)."""
    from urgym_amd._native import Sim
    from urgym_amd.envs import spaces_for
    n, steps = 256, 22
    act = spaces_for(task)[1]
    lo, hi = np.asarray(act.low, np.float64), np.asarray(act.high, np.float64)
    acts = [np.random.default_rng(100 + t).uniform(lo, hi, size=(n, len(lo))).astype(np.float32) for t in range(steps)]
    res = []
    for off in ("0", "1"):
        monkeypatch.setenv("URGYM_NO_PRIO_MODEL", off)
        sim = Sim(task, n, seed=SEED)
        sim.set_autoreset(True, {0: 500, 1: 50, 2: 20, 6: 500, 3: 100, 5: 100}[task])
        sim.reset()
        outs = [sim.step(a) for a in acts]
        res.append((outs, sim.get_state(), sim.get_rng()))
        sim.close()
    (oa, sa, ra), (ob, sb, rb) = res
    for t in range(steps):
        for k in ("obs", "reward", "substeps", "terminated", "truncated"):
            assert np.array_equal(oa[t][k], ob[t][k]), (t, k)
    assert np.array_equal(sa, sb)
    assert np.array_equal(ra[0], rb[0]) and np.array_equal(ra[1], rb[1])


def test_cubesgrasp_branch_peek_is_exact(built):
    """k_prio's branch (urgym_debug_cg_branch: the env's next random() peeked, ugg_cg_choose) is the branch the step then
    takes -- read back from the motor targets the step set (the move: the 6 arm targets = the action; the gripper
    command: the finger target) -- and the peek consumes nothing (the streams equal a twin handle's that never peeked)."""
    from urgym_amd import layout as LY
    from urgym_amd._native import Sim, ptr
    from urgym_amd.envs import spaces_for
    n, steps = 512, 24
    act = spaces_for(2)[1]
    lo, hi = np.asarray(act.low, np.float64), np.asarray(act.high, np.float64)
    sim, twin = Sim(2, n, seed=SEED), Sim(2, n, seed=SEED)
    for s in (sim, twin):
        s.set_autoreset(True, 20)
        s.reset()
    seen = [0, 0]
    for t in range(steps):
        a = np.random.default_rng(7 + t).uniform(lo, hi, size=(n, 9)).astype(np.float32)
        a[: n // 8, 0] = 0.0  # weights (0, w): always the gripper; (0, 0): the random() < 0.5 rule
        a[: n // 16, 1] = 0.0
        sel = np.zeros(n, np.int32)
        for _ in range(2):  # peeking twice changes nothing
            assert sim.L.urgym_debug_cg_branch(sim.h, ptr(a), ptr(sel)) == 0
        out = sim.step(a)
        twin.step(a)
        mt = sim.get_state()[:, LY.F_MTARGET:LY.F_MTARGET + 7]
        moved = (mt[:, :6] == a[:, 2:8].astype(np.float64)).all(1)
        live = ~(out["terminated"] | out["truncated"]).astype(bool)  # an autoreset rewrites the targets
        assert np.array_equal(moved[live], sel[live] == 0), t
        seen[0] += int((sel[live] == 0).sum())
        seen[1] += int((sel[live] == 1).sum())
        assert np.array_equal(sim.get_rng()[0], twin.get_rng()[0]), t
    assert min(seen) > 1000, seen
