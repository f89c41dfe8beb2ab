"""Golden Taxi frames from the REFERENCE's own render path (extended_taxi.py:289-331 -> str_map_to_img
:121-146 -> tile_images render_utils.py:63-88), run in the build container through refload.

cv2 is not installed: the stub's `resize` is set to the identity and `putText` to a no-op for this run, so
each fixture is the reference's pre-resize tiled frame plus its 20-column text band (the caption is never
drawn: lastaction is None). Inputs are recorded with the outputs.

    python tests/golden/make_render_golden.py      # writes tests/golden/taxi_render.npz
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refload  # noqa: E402

# name: (map, hansen, n_envs, state seed)
CASES = {
    "taxi_n1": ("TAXI_MAP", False, 1, 1),
    "taxi_n5_hansen": ("TAXI_MAP", True, 5, 2),
    "taxi_n9": ("TAXI_MAP", False, 9, 3),
    "ext_n3_hansen": ("EXTENDED_TAXI_MAP", True, 3, 4),
    "ext_n10": ("EXTENDED_TAXI_MAP", False, 10, 5),
    "taxi_n16_hansen": ("TAXI_MAP", True, 16, 6),
    "ext_n25_hansen": ("EXTENDED_TAXI_MAP", True, 25, 7),
}


def main():
    envs = refload.load()
    import cv2  # the stub module refload put on sys.path
    cv2.resize = lambda img, dsize, interpolation=None: img
    cv2.putText = lambda *a, **k: None
    cv2.INTER_AREA, cv2.FONT_HERSHEY_SIMPLEX, cv2.LINE_AA = 3, 0, 16
    et = sys.modules["gym_po.envs.extended_taxi"]
    out = {}
    for name, (mp, hansen, n, seed) in CASES.items():
        env = et.TaxiVecEnv(num_envs=n, map=getattr(et, mp), hansen_obs=hansen)
        rng = np.random.default_rng(seed)
        s = rng.integers(0, env.ns, n)
        # make sure the special placements occur: passenger in the taxi, passenger waiting under the taxi,
        # taxi on its destination
        r, c, p, d = env.decode(s)
        if n >= 3:
            p[0] = env.nlocs
            r[1], c[1] = env.np_locs[p[1] % env.nlocs]
            p[1] = p[1] % env.nlocs
            r[2], c[2] = env.np_locs[d[2]]
        s = env.encode(r, c, p, d)
        env.s = s.astype(int)
        env.lastaction = None
        img = env.render(idx=np.arange(n))
        out[name + "_states"] = s.astype(np.int32)
        out[name + "_img"] = np.asarray(img, np.uint8)
        print(name, img.shape)
    np.savez_compressed(os.path.join(HERE, "taxi_render.npz"), **out)


if __name__ == "__main__":
    main()
