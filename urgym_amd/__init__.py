"""urgym_amd -- MI355X-native hot path of URGym (UR5 + Robotiq-85 manipulation).

`import urgym_amd` mirrors `import urgym`: it exposes make() for the same
URGym/* ids (and registers them with gymnasium when gymnasium is installed).
The physics runs only in liburgym.so (HIP, gfx950); there is no CPU fallback.
"""
from .envs import TASKS, URGymEnv, URGymVectorEnv, make  # noqa: F401

try:  # pragma: no cover - gymnasium is not installed in this image
    from gymnasium.envs.registration import register

    for _id, (_task, _max) in TASKS.items():
        register(id=_id, entry_point="urgym_amd.envs.core:URGymEnv", max_episode_steps=_max, kwargs={"task": _task})
except Exception:
    pass

__all__ = ["make", "TASKS", "URGymEnv", "URGymVectorEnv"]
