"""Extract the reference's static map DATA into `gym-po-taxi_amd/gym_po_amd/data/maps.json`.

The maps are data the env needs (like a fixture), not code: ROOMS layouts as integer room-id grids
(wall = -1, exactly `np_to_grid(layout_to_np(LAYOUTS[k]))`, `layouts.py:6-195,217-232`), their
ENDS/STARTS (`layouts.py:197-214`), the FourRooms floor map `FR_MAP` (`msrooms.py:50-66`) and the
Taxi character maps (`extended_taxi.py:26-32,45-54`). Run in the build container only:

    python tests/golden/make_maps.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refload  # noqa: E402

OUT = os.path.join(HERE, "..", "..", "gym-po-taxi_amd", "gym_po_amd", "data", "maps.json")


def main():
    m = refload.load()
    L = m["layouts"]
    rooms = {}
    for k, v in L.LAYOUTS.items():
        g = L.np_to_grid(L.layout_to_np(v))
        rooms[k] = [[int(x) for x in row] for row in g]
    data = {
        "source": "DavidSlayback/gym-po-taxi (reference @ /root/reference), extracted by tests/golden/make_maps.py",
        "rooms_layouts": rooms,
        "rooms_ends_xy": {k: list(v) for k, v in L.ENDS.items()},
        "rooms_starts_xy": {k: list(v) for k, v in L.STARTS.items()},
        "fourrooms_floor_map": [[int(x) for x in row] for row in m["msrooms"].FR_MAP],
        "taxi_map": list(m["extended_taxi"].TAXI_MAP),
        "extended_taxi_map": list(m["extended_taxi"].EXTENDED_TAXI_MAP),
    }
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "w") as f:
        json.dump(data, f, separators=(",", ":"))
    print("wrote", os.path.normpath(OUT))


if __name__ == "__main__":
    main()
