"""Stand-in spaces (fixture generation only)."""
import numpy as np


class Space:
    def __init__(self, shape=None, dtype=None):
        self.shape = shape
        self.dtype = dtype


class Discrete(Space):
    def __init__(self, n, start=0):
        super().__init__((), np.int64)
        self.n = int(n)
        self.start = start


class MultiDiscrete(Space):
    def __init__(self, nvec, dtype=np.int64):
        self.nvec = np.asarray(nvec)
        super().__init__(self.nvec.shape, dtype)


class Box(Space):
    def __init__(self, low, high, shape=None, dtype=np.float32):
        if shape is None:
            shape = np.shape(low) if np.ndim(low) else np.shape(high)
        self.low = np.broadcast_to(np.asarray(low, dtype=dtype), shape)
        self.high = np.broadcast_to(np.asarray(high, dtype=dtype), shape)
        super().__init__(tuple(shape), dtype)
