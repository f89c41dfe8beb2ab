"""Observation/action spaces. Uses gymnasium's when importable (the reference's dependency);
otherwise minimal equivalents with the same attributes (n, shape, dtype, low/high, sample())."""
import numpy as np

try:  # pragma: no cover - gymnasium is not installed in the build image
    from gymnasium.spaces import Box, Discrete, MultiDiscrete  # noqa: F401
    from gymnasium.vector.utils import batch_space  # noqa: F401
    HAVE_GYMNASIUM = True
except Exception:  # noqa: BLE001
    HAVE_GYMNASIUM = False

    class Space:
        def __init__(self, shape=None, dtype=None, seed=None):
            self.shape = shape
            self.dtype = np.dtype(dtype) if dtype is not None else None
            self._rng = np.random.default_rng(seed)

        def seed(self, seed=None):
            self._rng = np.random.default_rng(seed)

    class Discrete(Space):
        def __init__(self, n, start=0, seed=None):
            assert int(n) > 0, "Discrete needs n > 0"
            super().__init__((), np.int64, seed)
            self.n = int(n)
            self.start = int(start)

        def sample(self):
            return int(self.start + self._rng.integers(self.n))

        def contains(self, x):
            return self.start <= int(x) < self.start + self.n

        def __repr__(self):
            return f"Discrete({self.n})"

    class MultiDiscrete(Space):
        def __init__(self, nvec, dtype=np.int64, seed=None):
            self.nvec = np.asarray(nvec, dtype=np.int64)
            super().__init__(self.nvec.shape, dtype, seed)

        def sample(self):
            return (self._rng.random(self.nvec.shape) * self.nvec).astype(self.dtype)

        def __repr__(self):
            return f"MultiDiscrete({self.nvec.tolist()})"

    class Box(Space):
        def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
            if shape is None:
                shape = np.broadcast(np.asarray(low), np.asarray(high)).shape
            shape = tuple(shape)
            self.low = np.broadcast_to(np.asarray(low, dtype=dtype), shape).copy()
            self.high = np.broadcast_to(np.asarray(high, dtype=dtype), shape).copy()
            super().__init__(shape, dtype, seed)

        def sample(self):
            if np.issubdtype(self.dtype, np.integer):
                return self._rng.integers(self.low, self.high + 1, self.shape).astype(self.dtype)
            return self._rng.uniform(self.low, self.high, self.shape).astype(self.dtype)

        def __repr__(self):
            return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"

    def batch_space(space, n=1):
        if isinstance(space, Discrete):
            return MultiDiscrete(np.full((n,), space.n))
        if isinstance(space, Box):
            return Box(np.stack([space.low] * n), np.stack([space.high] * n), (n,) + space.shape, space.dtype)
        raise NotImplementedError(type(space))
