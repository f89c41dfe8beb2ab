"""ORACLE / TEST INFRASTRUCTURE — draw providers for the pure oracle step functions.

The reference consumes one numpy Generator per env object (SURVEY.md §8(a) RNG contract). The
oracle steps take a *draw provider* so the same restated step can be driven either
  * seed-identically by a numpy Generator (`NumpyDraws`), or
  * by pre-decided per-env values (`ReplayDraws`), which is how the GPU's replay mode is
    checked for envs whose numpy stream cannot be reproduced in parallel (Taxi multinomial,
    C-ROOMS ziggurat normals).
"""
import numpy as np


class NumpyDraws:
    """Exactly the reference's calls on `np.random.Generator`."""

    def __init__(self, gen):
        self.gen = gen

    # Generator.random(B) (action_utils.py:84)
    def uniform(self, n):
        return self.gen.random(n)

    # Generator.choice(values, b) over the masked (ascending) envs (msrooms.py:350-364)
    def choice(self, values, mask, site):
        return self.gen.choice(values, int(mask.sum()))

    # Generator.normal(scale=s, size=(n, 2)) (crooms.py:178, :324)
    def normal(self, scale, n, site):
        return self.gen.normal(scale=scale, size=(n, 2))

    # Generator.multinomial(ns, p, b).argmax(-1) (extended_taxi.py:348-350)
    def multinomial_argmax(self, ns, p, mask, site):
        return self.gen.multinomial(ns, p, int(mask.sum())).argmax(-1)

    # Generator.integers(k, size=b) (extended_taxi.py:360-363)
    def integers(self, k, n, site):
        return self.gen.integers(k, size=n)


class ReplayDraws:
    """Per-env pre-decided draws for one step: `site -> array[B]` (or [B,2])."""

    def __init__(self, arrays):
        self.a = arrays

    def uniform(self, n):
        return self.a["uniform"]

    def choice(self, values, mask, site):
        return np.asarray(values)[self.a[site][mask]]

    def normal(self, scale, n, site):
        raise NotImplementedError("per-env normals are taken via normal_masked")

    def normal_masked(self, mask, site):
        return self.a[site][mask]

    def multinomial_argmax(self, ns, p, mask, site):
        return self.a[site][mask]
