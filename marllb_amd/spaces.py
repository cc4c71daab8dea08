"""Action/observation spaces with the gym==0.17.2 surface the reference uses (env.py:163-182).

gym is not a dependency: these two classes carry exactly the attributes and methods the reference
environment, its tests (test_env.py:37-61) and the problem-04 trainer (trainer.py:106) touch —
shape, dtype, low/high, nvec, sample(), seed(), contains().
"""
from __future__ import annotations

import numpy as np


class Box:
    """gym.spaces.Box: a (possibly unbounded) box in R^shape."""

    def __init__(self, low, high, shape=None, dtype=np.float32):
        self.dtype = np.dtype(dtype)
        if shape is None:
            shape = np.broadcast(np.asarray(low), np.asarray(high)).shape
        self.shape = tuple(int(x) for x in shape)
        self.low = np.full(self.shape, low, dtype=self.dtype)
        self.high = np.full(self.shape, high, dtype=self.dtype)
        self.np_random = np.random.RandomState()

    def seed(self, seed=None):
        self.np_random = np.random.RandomState(seed)
        return [seed]

    def sample(self):
        """Uniform on bounded dims, exponential/normal on unbounded ones (gym 0.17 Box.sample)."""
        lo_b = np.isfinite(self.low)
        hi_b = np.isfinite(self.high)
        out = np.empty(self.shape, dtype=np.float64)
        both = lo_b & hi_b
        out[both] = self.np_random.uniform(self.low[both], self.high[both])
        lo_only = lo_b & ~hi_b
        out[lo_only] = self.low[lo_only] + self.np_random.exponential(size=int(lo_only.sum()))
        hi_only = ~lo_b & hi_b
        out[hi_only] = self.high[hi_only] - self.np_random.exponential(size=int(hi_only.sum()))
        neither = ~lo_b & ~hi_b
        out[neither] = self.np_random.normal(size=int(neither.sum()))
        return out.astype(self.dtype)

    def contains(self, x) -> bool:
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self):
        return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"


class MultiDiscrete:
    """gym.spaces.MultiDiscrete: one categorical of size nvec[i] per server."""

    def __init__(self, nvec):
        self.nvec = np.asarray(nvec, dtype=np.int64)
        self.shape = self.nvec.shape
        self.dtype = np.dtype(np.int64)
        self.np_random = np.random.RandomState()

    def seed(self, seed=None):
        self.np_random = np.random.RandomState(seed)
        return [seed]

    def sample(self):
        return (self.np_random.random_sample(self.nvec.shape) * self.nvec).astype(self.dtype)

    def contains(self, x) -> bool:
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= 0) and np.all(x < self.nvec))

    def __repr__(self):
        return f"MultiDiscrete({self.nvec})"
