"""Config E at its stated size and the multi-rank path with the real simulator:

* Golf x 65536 as eight env_offset shards of 8192 (what the 8 ranks of config E hold) == one 65536-env handle, bit
  for bit, over 10 autoreset steps (a synchronized truncation reset of every env included), with envs sampled
  from every shard checked against the CPU restatement step by step;
* two gloo ranks (torch.distributed.run children, both on this GPU) stepping their shards of a batch and
  all-gathering the returns each step == one handle stepping the whole batch; the same through RCCL (nccl backend,
  device tensors) with one rank;
* full episodes at the configs' sizes: CubesPush x 4096 through its 50-step truncation, CubesGrasp x 8192 through
  its 20-step truncation, sampled envs bit-exact against the restatement at every step.
Reference: BASELINE.json configs[2..4]; /root/reference/urgym/envs/env_golf_v0.py:115-446,
env_cubes_push_v0.py:115-251, env_cubes_grasp_v0.py:112-405."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20241220
KEYS = ("obs", "final_obs", "reward", "terminated", "truncated", "success", "substeps")


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
    return rng.uniform(-0.1, 0.1, size=(n, 3)).astype(np.float32)


class Sampled:
    """the restatement replaying a few envs of a GPU batch, compared at every step"""

    def __init__(self, OracleEnv, task, ids, seed, max_steps, obs0):
        self.ids, self.max_steps = list(ids), max_steps
        self.ref = {i: OracleEnv(task, seed + i) for i in self.ids}
        self.el = {i: 0 for i in self.ids}
        for i, r in self.ref.items():
            assert np.array_equal(obs0[i], r.reset()[0]), i

    def step(self, act, out, tag):
        for i, r in self.ref.items():
            o, rew, term, succ, ns = r.step(act[i])
            self.el[i] += 1
            trunc = self.el[i] >= self.max_steps
            assert out["reward"][i] == rew and bool(out["terminated"][i]) == term, (tag, i)
            assert bool(out["truncated"][i]) == trunc and bool(out["success"][i]) == succ, (tag, i)
            if term or trunc:
                assert np.array_equal(out["final_obs"][i], o), (tag, i)
                o, ns2 = r.reset()
                ns += ns2
                self.el[i] = 0
            assert np.array_equal(out["obs"][i], o), (tag, i)
            assert out["substeps"][i] == ns, (tag, i)

    def check_state(self, st, tag):
        for i, r in self.ref.items():
            assert np.array_equal(st[i], r.get_state()), (tag, i)


def test_config_e_eight_shards_equal_one_65536_handle(mods):
    """config E (Golf x 65536 = 8 x 8192): eight handles at env offsets r * 8192 == one handle of 65536, every
    output of every step and the final states bit-identical; two envs of every shard replayed by the oracle.
    Truncation at 7 steps puts a synchronized reset of all 65536 envs inside the 10 steps."""
    Sim, OracleEnv = mods
    task, world, per, T, max_steps = 3, 8, 8192, 10, 7
    n = world * per
    full = Sim(task, n, seed=SEED)
    shards = [Sim(task, per, seed=SEED, env_offset=r * per) for r in range(world)]
    for s in [full] + shards:
        s.set_autoreset(True, max_steps)
    o_full = full.reset()
    assert np.array_equal(o_full, np.concatenate([s.reset() for s in shards]))
    sample = Sampled(OracleEnv, task, [r * per + k for r in range(world) for k in (r % 3, per - 1 - r)], SEED,
                     max_steps, o_full)
    rng = np.random.default_rng(SEED)
    resets = 0
    for t in range(T):
        act = actions(task, rng, n)
        a = full.step(act)
        b = [s.step(act[r * per:(r + 1) * per]) for r, s in enumerate(shards)]
        for k in KEYS:
            assert np.array_equal(a[k], np.concatenate([x[k] for x in b])), (t, k)
        assert np.all(np.isfinite(a["obs"])) and np.all(np.isfinite(a["reward"]))
        sample.step(act, a, t)
        resets += int((a["terminated"] | a["truncated"]).sum())
    assert resets >= n  # the step-7 truncation reset every env
    st = full.get_state()
    for r, s in enumerate(shards):
        assert np.array_equal(st[r * per:(r + 1) * per], s.get_state()), r
    sample.check_state(st, "end")
    for s in [full] + shards:
        s.close()


@pytest.mark.parametrize("backend,world", [("gloo", 2), ("nccl", 1)])
def test_ranks_gather_real_sim_outputs(mods, tmp_path, backend, world):
    """ranks (torch.distributed.run children on this GPU) step their shards of a BallBalance batch and all-gather
    every return (obs, final_obs, reward, terminated, truncated, success, substeps) each step through one
    ReturnGather; the gathered batches equal one handle stepping the whole batch with the same action stream
    (autoreset through truncation at 4 steps).  gloo: two ranks sharing the GPU, returns through host memory.
    nccl: RCCL, the production branch (device tensors gathered from HBM, parallel.py ReturnGather) -- one rank,
    since RCCL refuses two ranks on one GPU and this box has one; the 8-rank node run is the driver's."""
    Sim, _ = mods
    from urgym_amd.parallel import spawn_ranks
    task, total, steps, max_steps, seed = 0, 256, 6, 4, 4242
    out = tmp_path / "gathered.npz"
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_sim_rank_worker.py")
    rc = spawn_ranks(world, worker, [str(out), str(task), str(total), str(steps), str(max_steps), str(seed), backend])
    assert rc == 0
    g = np.load(out)
    assert int(g["world"]) == world and str(g["backend"]) == backend
    sim = Sim(task, total, seed=seed)
    sim.set_autoreset(True, max_steps)
    sim.reset()
    rng = np.random.default_rng(seed)
    for t in range(steps):
        r = sim.step(rng.uniform(-0.1, 0.1, size=(total, 3)).astype(np.float32))
        assert np.array_equal(g["obs"][t], r["obs"]), t
        assert np.array_equal(g["reward"][t], r["reward"]), t
        assert np.array_equal(g["terminated"][t], r["terminated"].astype(bool)), t
        assert np.array_equal(g["truncated"][t], r["truncated"].astype(bool)), t
        assert np.array_equal(g["success"][t], r["success"].astype(bool)), t
        assert np.array_equal(g["substeps"][t], r["substeps"]), t
        done = r["terminated"].astype(bool) | r["truncated"].astype(bool)
        assert np.array_equal(g["final_obs"][t][done], r["final_obs"][done]), t  # the autoreset envs' terminal obs
    assert g["truncated"].any()
    sim.close()


@pytest.mark.parametrize("task,n,max_steps", [(1, 4096, 50), (2, 8192, 20)])
def test_full_episode_at_config_size(mods, task, n, max_steps):
    """configs C and D through a whole episode: max_steps + 2 autoreset steps at full size, every step finite with
    bounded substeps, the truncation step resetting every env that had not terminated, and four sampled envs
    (first, last, two inside) bit-exact against the restatement at every step."""
    Sim, OracleEnv = mods
    sim = Sim(task, n, seed=SEED)
    sim.set_autoreset(True, max_steps)
    obs = sim.reset()
    sample = Sampled(OracleEnv, task, [0, 1 + n // 3, n // 2 + 5, n - 1], SEED, max_steps, obs)
    rng = np.random.default_rng(SEED + task)
    ended = 0
    for t in range(max_steps + 2):
        act = actions(task, rng, n)
        out = sim.step(act)
        assert np.all(np.isfinite(out["obs"])) and np.all(np.isfinite(out["reward"])), t
        assert np.all((out["substeps"] >= 1) & (out["substeps"] <= 3 * 480 + 10)), t
        sample.step(act, out, t)
        ended += int((out["terminated"] | out["truncated"]).sum())
    assert ended >= n  # every env ended at least one episode (truncation at max_steps)
    sample.check_state(sim.get_state(), "end")
    sim.close()
