"""Taxi rgb_array rendering: the numpy restatement (oracle/render.py) against frames produced by the reference's
own render path (tests/golden/taxi_render.npz, made by tests/golden/make_render_golden.py with cv2.resize as the
identity: the pre-resize tiled frame plus the text band). CPU only."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gym-po-taxi_amd"))
from oracle import render  # noqa: E402
from gym_po_amd.maps import EXTENDED_TAXI_MAP, TAXI_MAP  # noqa: E402
from gym_po_amd.envs.extended_taxi import convert_str_map_to_walled_np_str, get_locations_from_np_str_map  # noqa: E402

GOLD = np.load(os.path.join(ROOT, "tests", "golden", "taxi_render.npz"))
CASES = {"taxi_n1": (TAXI_MAP, False), "taxi_n5_hansen": (TAXI_MAP, True), "taxi_n9": (TAXI_MAP, False),
         "ext_n3_hansen": (EXTENDED_TAXI_MAP, True), "ext_n10": (EXTENDED_TAXI_MAP, False),
         "taxi_n16_hansen": (TAXI_MAP, True), "ext_n25_hansen": (EXTENDED_TAXI_MAP, True)}


def map_parts(mp):
    desc, tgrid, cc = convert_str_map_to_walled_np_str(mp)
    locs = np.array(get_locations_from_np_str_map(tgrid)).T
    return desc, tgrid, cc, np.concatenate((locs, [[-1, -1]])), locs.shape[0]


@pytest.mark.parametrize("name", sorted(CASES))
def test_tiled_frame_matches_reference(name):
    mp, hansen = CASES[name]
    desc, tgrid, cc, np_locs, nlocs = map_parts(mp)
    states = GOLD[name + "_states"]
    tiled = render.render_tiled(desc, cc, np_locs, nlocs, tgrid.shape[1], states, hansen)
    band = np.zeros((tiled.shape[0], render.TEXT_SPACE, 3), np.uint8)
    np.testing.assert_array_equal(np.concatenate([tiled, band], axis=1), GOLD[name + "_img"])


def test_resize_identity_and_replication():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (7, 11, 3), dtype=np.uint8)
    np.testing.assert_array_equal(render.resize_area_u8(img, 7, 11), img)
    # integer enlargement: INTER_AREA's area coefficients are 0 / 1 everywhere -> pixel replication
    np.testing.assert_array_equal(render.resize_area_u8(img, 14, 33), img.repeat(2, 0).repeat(3, 1))
    with pytest.raises(NotImplementedError):
        render.resize_area_u8(img, 3, 5)
