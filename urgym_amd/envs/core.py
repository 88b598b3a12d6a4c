"""gymnasium-compatible Env / VectorEnv over the batched C-ABI (urgym_amd._native.Sim)."""
import numpy as np

from .._native import Sim


class URGymVectorEnv:
    """N envs of one task on one GPU, gymnasium 0.29 VectorEnv semantics:
    step() returns (obs, rewards, terminated, truncated, infos) with same-step
    autoreset -- a finished env is reset inside the same call and its terminal
    observation is in infos['final_observation'] (masked by '_final_observation').
    """

    def __init__(self, task, num_envs, max_episode_steps=None, device=0, seed=0, env_offset=0,
                 camera=None, reward_type="dense", render_mode="rgb_array"):
        from . import spaces_for
        if camera is not None:
            raise NotImplementedError("camera rendering is outside the hot-path scope")
        if reward_type != "dense":
            raise NotImplementedError("only reward_type='dense' is implemented")
        self.task = task
        self.num_envs = num_envs
        self.single_observation_space, self.single_action_space = spaces_for(task)
        self.sim = Sim(task, num_envs, device=device, seed=seed, env_offset=env_offset)
        self.max_episode_steps = max_episode_steps or 0
        self.sim.set_autoreset(True, self.max_episode_steps)
        self.render_mode = render_mode  # 'human' GUI is not supported (documented deviation)

    def reset(self, *, seed=None, options=None):
        obs = self.sim.reset()
        return obs, {}

    def step(self, actions):
        out = self.sim.step(actions)
        term = out["terminated"].astype(bool)
        trunc = out["truncated"].astype(bool)
        done = term | trunc
        infos = {"is_success": out["success"].astype(bool), "substeps": out["substeps"]}
        if done.any():
            fo = np.empty(self.num_envs, dtype=object)
            for i in np.nonzero(done)[0]:
                fo[i] = out["final_obs"][i].copy()
            infos["final_observation"] = fo
            infos["_final_observation"] = done
        return out["obs"], out["reward"], term, trunc, infos

    def close(self):
        self.sim.close()


class URGymEnv:
    """Single env with the reference's surface: reset(*, seed, options) -> (obs, info),
    step(a) -> (obs, float reward, bool terminated, bool truncated, info)."""

    def __init__(self, task, max_episode_steps=None, device=0, seed=0, camera=None, reward_type="dense",
                 render_mode="human"):
        from . import spaces_for
        if camera is not None:
            raise NotImplementedError("camera rendering is outside the hot-path scope")
        self.task = task
        self.observation_space, self.action_space = spaces_for(task)
        self.sim = Sim(task, 1, device=device, seed=seed)
        self.max_episode_steps = max_episode_steps or 0
        self.sim.set_autoreset(False, 0)
        self._elapsed = 0
        self.render_mode = render_mode

    def reset(self, *, seed=None, options=None):
        self._elapsed = 0
        return self.sim.reset()[0].copy(), {}

    def step(self, action):
        out = self.sim.step(np.asarray(action, dtype=np.float32).reshape(1, -1))
        self._elapsed += 1
        trunc = bool(self.max_episode_steps and self._elapsed >= self.max_episode_steps)
        info = {} if self.task == 0 else {"is_success": bool(out["success"][0])}
        return out["obs"][0].copy(), float(out["reward"][0]), bool(out["terminated"][0]), trunc, info

    def close(self):
        self.sim.close()
