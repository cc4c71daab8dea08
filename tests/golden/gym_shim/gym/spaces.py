"""gym.spaces.Box / MultiDiscrete subset (shape/low/high/nvec/sample) for gen_golden.py."""
import numpy as np


class Box:
    def __init__(self, low, high, shape=None, dtype=np.float32):
        self.dtype = np.dtype(dtype)
        self.shape = tuple(shape) if shape is not None else np.shape(low)
        self.low = np.full(self.shape, low, dtype=self.dtype)
        self.high = np.full(self.shape, high, dtype=self.dtype)
        self.np_random = np.random.RandomState()

    def sample(self):
        hi = np.where(np.isinf(self.high), 1.0, self.high)
        return self.np_random.uniform(self.low, hi).astype(self.dtype)


class MultiDiscrete:
    def __init__(self, nvec):
        self.nvec = np.asarray(nvec, dtype=np.int64)
        self.shape = self.nvec.shape
        self.np_random = np.random.RandomState()

    def sample(self):
        return (self.np_random.random_sample(self.nvec.shape) * self.nvec).astype(np.int64)
