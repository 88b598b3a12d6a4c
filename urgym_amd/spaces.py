"""Minimal gymnasium.spaces.Box stand-in (gymnasium is not installed in this image).

If gymnasium is importable, urgym_amd.envs uses the real Box instead.
"""
import numpy as np


class Box:
    def __init__(self, low, high, dtype=np.float32, shape=None):
        self.dtype = np.dtype(dtype)
        low = np.asarray(low, dtype=self.dtype)
        high = np.asarray(high, dtype=self.dtype)
        if shape is not None:
            low = np.broadcast_to(low, shape).copy()
            high = np.broadcast_to(high, shape).copy()
        self.low, self.high = low, high
        self.shape = low.shape
        self._rng = np.random.default_rng()

    def seed(self, seed=None):
        self._rng = np.random.default_rng(seed)

    def sample(self):
        return self._rng.uniform(self.low, self.high).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self):
        return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"
