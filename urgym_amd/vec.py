"""Stable-Baselines3-shaped vectorized environments over the batched C-ABI.

The reference's consumers are SB3 algorithms driving one env per process (training.py:25-41,
optuna_training.py:35-67).  Here one handle steps thousands of envs per call:

* `URGymSB3VecEnv` -- the SB3 `VecEnv` protocol (reset() -> obs, step_async / step_wait -> (obs, rewards, dones,
  infos) with SB3's auto-reset: infos[i]['terminal_observation'], infos[i]['TimeLimit.truncated'], plus
  'is_success' where the reference reports it), so `PPO("MlpPolicy", URGymSB3VecEnv(...))` runs on it.  When
  stable_baselines3 is importable the class subclasses its VecEnv; in this image it is absent and the class
  stands alone with the same methods.
* `URGymTorchVecEnv` -- device-resident rollouts: actions in, observations / rewards / flags out as torch tensors
  in HBM, every kernel ordered on the handle's HIP stream (policy forward passes included, `stream_context()`),
  no host round trip per step.  `rollout(policy, steps)` runs a policy on the device for a batch of steps.
"""
import numpy as np

from ._native import Sim

try:  # pragma: no cover - SB3 is absent in this image
    from stable_baselines3.common.vec_env import VecEnv as _SB3VecEnv
except Exception:  # pragma: no cover
    _SB3VecEnv = object


class URGymSB3VecEnv(_SB3VecEnv):
    """n envs of one URGym task on one GPU behind SB3's VecEnv protocol."""

    def __init__(self, env_id, num_envs, device=0, seed=0, env_offset=0, reward_type="dense"):
        from .envs import TASKS, UNSUPPORTED, spaces_for
        if env_id in UNSUPPORTED:
            raise NotImplementedError(f"{env_id} is outside this build's hot-path scope (SURVEY.md 8(f))")
        self.task, self.max_episode_steps = TASKS[env_id]
        self.render_mode = None
        obs_space, act_space = spaces_for(self.task)
        if _SB3VecEnv is not object:  # pragma: no cover - SB3 is absent in this image
            # SB3's constructor sets num_envs / spaces / reset_infos / _seeds / _options / render_mode
            _SB3VecEnv.__init__(self, num_envs, obs_space, act_space)
        self.num_envs = num_envs
        self.observation_space, self.action_space = obs_space, act_space
        self.sim = Sim(self.task, num_envs, device=device, seed=seed, env_offset=env_offset)
        self.sim.set_reward_type(reward_type)
        self.sim.set_autoreset(True, self.max_episode_steps)
        self._actions = None
        self.reset_infos = [{} for _ in range(num_envs)]

    # -- SB3 VecEnv protocol --
    def reset(self):
        return self.sim.reset()

    def step_async(self, actions):
        self._actions = np.asarray(actions, dtype=np.float32).reshape(self.num_envs, -1)

    def step_wait(self):
        out = self.sim.step(self._actions)
        term = out["terminated"].astype(bool)
        trunc = out["truncated"].astype(bool)
        dones = term | trunc
        infos = []
        report_success = self.task not in (0, 6)  # BallBalance / TwoBalls return info {} (env_ball_balance_v0.py:134)
        for i in range(self.num_envs):
            info = {"is_success": bool(out["success"][i])} if report_success else {}
            if dones[i]:
                info["terminal_observation"] = out["final_obs"][i].copy()
                info["TimeLimit.truncated"] = bool(trunc[i] and not term[i])
            infos.append(info)
        return out["obs"], out["reward"].astype(np.float32), dones, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def close(self):
        self.sim.close()

    def seed(self, seed=None):
        return [None] * self.num_envs  # per-env streams are seeded at construction (seed + env id)

    def get_attr(self, attr_name, indices=None):
        return [getattr(self, attr_name)] * len(self._indices(indices))

    def set_attr(self, attr_name, value, indices=None):
        setattr(self, attr_name, value)

    def env_method(self, method_name, *args, indices=None, **kwargs):
        raise NotImplementedError("per-env methods do not exist: the envs live in one GPU batch")

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False] * len(self._indices(indices))

    def get_images(self):
        return [None] * self.num_envs

    def render(self, mode=None):
        return None

    def _indices(self, indices):
        if indices is None:
            return range(self.num_envs)
        return [indices] if isinstance(indices, int) else indices


class URGymTorchVecEnv:
    """Device-resident batch: torch tensors in, torch tensors out, one HIP stream for env and policy."""

    def __init__(self, env_id, num_envs, device=0, seed=0, env_offset=0, reward_type="dense"):
        import torch
        from .envs import TASKS, spaces_for
        self.torch = torch
        self.task, self.max_episode_steps = TASKS[env_id]
        self.num_envs = num_envs
        self.observation_space, self.action_space = spaces_for(self.task)
        self.sim = Sim(self.task, num_envs, device=device, seed=seed, env_offset=env_offset)
        self.sim.set_reward_type(reward_type)
        self.sim.set_autoreset(True, self.max_episode_steps)
        self.device = torch.device("cuda", device)
        self.stream = torch.cuda.ExternalStream(self.sim.L.urgym_stream(self.sim.h), device=self.device)
        n, O = num_envs, self.sim.obs_dim
        f64, u8 = torch.float64, torch.uint8
        self.obs = torch.zeros(n, O, dtype=f64, device=self.device)
        self.final_obs = torch.zeros(n, O, dtype=f64, device=self.device)
        self.reward = torch.zeros(n, dtype=f64, device=self.device)
        self.terminated = torch.zeros(n, dtype=u8, device=self.device)
        self.truncated = torch.zeros(n, dtype=u8, device=self.device)
        self.success = torch.zeros(n, dtype=u8, device=self.device)
        self.substeps = torch.zeros(n, dtype=torch.int32, device=self.device)
        self.low = torch.as_tensor(np.asarray(self.action_space.low), dtype=torch.float32, device=self.device)
        self.high = torch.as_tensor(np.asarray(self.action_space.high), dtype=torch.float32, device=self.device)
        # the buffers were zero-filled on the caller's stream; the handle's stream is non-blocking
        self.stream.wait_stream(torch.cuda.current_stream(self.device))

    def stream_context(self):
        """with env.stream_context(): torch work (the policy) is ordered with the env kernels"""
        return self.torch.cuda.stream(self.stream)

    def _enter(self):
        """order the env stream after the caller's current stream (actions produced there); returns it"""
        cur = self.torch.cuda.current_stream(self.device)
        if cur != self.stream:
            self.stream.wait_stream(cur)
        return cur

    def _leave(self, cur):
        """order the caller's current stream after the env kernels, so it may read the outputs directly"""
        if cur != self.stream:
            cur.wait_stream(self.stream)

    def reset(self):
        import ctypes
        v = ctypes.c_void_p
        cur = self._enter()
        self.sim._chk(self.sim.L.urgym_reset_device(self.sim.h, None, None, v(self.obs.data_ptr())), "urgym_reset_device")
        self._leave(cur)
        return self.obs

    def step(self, actions):
        """actions: (n, act_dim) CUDA tensor from any stream of the env's device (the env stream waits for the
        caller's current stream).  Returns the device buffers (obs, reward, terminated, truncated, final_obs),
        ordered before later work on the caller's current stream and overwritten by the next step."""
        cur = self._enter()
        with self.stream_context():  # the float32 copy (if any) is made on the env stream
            a = actions.to(dtype=self.torch.float32).contiguous()
        if a.data_ptr() == actions.data_ptr():
            a.record_stream(self.stream)  # the caller's tensor: not reused before the kernel has read it
        self.sim.step_device(a.data_ptr(), self.obs.data_ptr(), self.final_obs.data_ptr(), self.reward.data_ptr(),
                             self.terminated.data_ptr(), self.truncated.data_ptr(), self.success.data_ptr(),
                             self.substeps.data_ptr())
        self._leave(cur)
        return self.obs, self.reward, self.terminated, self.truncated, self.final_obs

    def rollout(self, policy, steps):
        """Run `policy(obs) -> actions` (a torch module / function on the device) for `steps` batched env steps
        on the env stream; returns per-step reward sums and done counts (tensors on the device)."""
        torch = self.torch
        cur = self._enter()
        with self.stream_context():
            rew = torch.zeros(steps, dtype=torch.float64, device=self.device)
            done = torch.zeros(steps, dtype=torch.int64, device=self.device)
            obs = self.obs
            for t in range(steps):
                with torch.no_grad():
                    act = policy(obs.to(torch.float32))
                act = torch.maximum(torch.minimum(act, self.high), self.low)
                obs, r, term, trunc, _ = self.step(act)
                rew[t] = r.sum()
                done[t] = (term | trunc).sum()
        self._leave(cur)
        return rew, done

    def sync(self):
        self.sim.sync()

    def close(self):
        self.sim.close()
