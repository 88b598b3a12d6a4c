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
