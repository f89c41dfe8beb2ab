"""Static map data (extracted from the reference by tests/golden/make_maps.py into data/maps.json).

ROOMS layouts `LAYOUTS` (layouts.py:6-195) as integer room-id grids (wall = -1), `ENDS`/`STARTS`
(layouts.py:197-214), FourRooms `FR_MAP` (msrooms.py:50-66) and the Taxi maps
(extended_taxi.py:26-32, 45-54).
"""
import json
import os

import numpy as np

_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "maps.json")
with open(_PATH) as _f:
    _DATA = json.load(_f)

LAYOUT_GRIDS = {k: np.array(v, dtype=np.int64) for k, v in _DATA["rooms_layouts"].items()}
LAYOUTS = tuple(LAYOUT_GRIDS)
ENDS = {k: tuple(v) for k, v in _DATA["rooms_ends_xy"].items()}
STARTS = {k: tuple(v) for k, v in _DATA["rooms_starts_xy"].items()}
FR_MAP = np.array(_DATA["fourrooms_floor_map"], dtype=np.int64)
TAXI_MAP = tuple(_DATA["taxi_map"])
EXTENDED_TAXI_MAP = tuple(_DATA["extended_taxi_map"])


def layout_grid(layout):
    """np_to_grid(layout_to_np(LAYOUTS[layout])) (layouts.py:217-232)."""
    if layout not in LAYOUT_GRIDS:
        raise AssertionError(f"layout {layout!r} not in {LAYOUTS}")
    return LAYOUT_GRIDS[layout].copy()
