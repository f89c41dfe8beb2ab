"""Minimal gymnasium stand-in used ONLY to import the read-only reference when generating golden
fixtures in the survey/build container. Never shipped to the GPU box's
product path; never imported by gym_po_amd."""
import numpy as np
from . import spaces, utils  # noqa: F401
from .spaces import Space  # noqa: F401
from .utils import seeding


class Env:
    _np_random = None
    metadata = {}

    def reset(self, *, seed=None, options=None):
        if seed is not None:
            self._np_random, _ = seeding.np_random(seed)

    @property
    def np_random(self):
        if self._np_random is None:
            self._np_random, _ = seeding.np_random()
        return self._np_random

    @np_random.setter
    def np_random(self, value):
        self._np_random = value
