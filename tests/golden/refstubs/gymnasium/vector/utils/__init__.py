import numpy as np
from ...spaces import Discrete, MultiDiscrete, Box


def batch_space(space, n=1):
    if isinstance(space, Discrete):
        return MultiDiscrete(np.full((n,), space.n))
    if isinstance(space, Box):
        return Box(np.stack([space.low] * n), np.stack([space.high] * n), (n,) + space.shape, space.dtype)
    return space
