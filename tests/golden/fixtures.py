"""Golden-fixture helpers shared by the generator (make_golden.py) and the tests.

Fixtures are DATA: seeds, actions, and the reference's outputs (obs / reward / terminated /
truncated per step), RNG transcripts (the values each numpy call returned, in call order) and
final internal state. No reference source is stored.
"""
import json
import os

import numpy as np

GOLDEN_DIR = os.path.dirname(os.path.abspath(__file__))
INDEX = os.path.join(GOLDEN_DIR, "index.json")


def digest(x):
    """Order-sensitive uint64 checksum of an array's values (ints/bools by value, floats by bits)."""
    x = np.ascontiguousarray(x)
    if x.dtype == np.float32:
        v = x.view(np.uint32).astype(np.uint64).ravel()
    elif x.dtype == np.float64:
        v = x.view(np.uint64).ravel()
    else:
        v = x.astype(np.int64).view(np.uint64).ravel()
    w = (np.arange(v.size, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)) | np.uint64(1)
    with np.errstate(over="ignore"):
        return np.uint64((v * w + v).sum(dtype=np.uint64))


def load_index():
    with open(INDEX) as f:
        return json.load(f)


def load_case(name):
    idx = load_index()
    meta = idx["cases"][name]
    data = np.load(os.path.join(GOLDEN_DIR, meta["file"]), allow_pickle=False)
    return meta, data


def step_actions(meta):
    """Regenerate the action sequence a fixture was recorded with."""
    rng = np.random.default_rng(meta["action_seed"])
    T, B = meta["steps"], meta["num_envs"]
    if meta.get("action_kind") == "box2":
        return rng.uniform(-1.0, 1.0, (T, B, 2))
    return rng.integers(0, meta["num_actions"], (T, B))
