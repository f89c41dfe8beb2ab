"""Taxi rgb_array rendering restated in numpy (TEST INFRASTRUCTURE: only tests/ and tools may import it).

Follows `TaxiVecEnv.render` (extended_taxi.py:289-331), `str_map_to_img` (extended_taxi.py:121-146) and
`tile_images` (render_utils.py:63-88):

- per frame, the bordered char map with 'D' at the destination, 'T' at the taxi, 'P' at a waiting passenger,
  'F' at a taxi carrying the passenger, and "TP" where a waiting passenger shares the taxi's cell — which the
  reference writes into a '<U1' array, so it is stored as 'T' (the TAXI_AND_PASSENGER colour is never used);
- colours from the shared palette (render_utils.py:11-24), every other character LOC;
- Hansen highlight: +64 (uint8, wrapping) on the four orthogonal neighbours of the taxi cell in the bordered map;
- frames tiled on a ceil(sqrt(n)) x ceil(n / ceil(sqrt(n))) grid, zero padding;
- cv2.resize(img, (h * 16, w * 16), INTER_AREA) with (h, w) the bordered map's shape (dsize is (width, height),
  so the frame comes out transposed in aspect), then a 20-column black text band on the right.

The pre-resize frame and the band are pinned against the reference itself (tests/golden/make_render_golden.py,
cv2.resize stubbed as the identity). cv2 is not installed here, so `resize_area_u8` restates OpenCV's generic
(non-IPP) resize for INTER_AREA when at least one axis is enlarged — the linear path with area coefficients and
11-bit fixed point — from its published source: parity unpinned for the resize. The reference's caption
(cv2.putText of the last action) is not drawn.
"""
import numpy as np

CELL_PX = 16
TEXT_SPACE = 20
WALL = (0, 0, 0)
FLOOR = (96, 96, 96)        # gray_mid_dark
TAXI = (128, 128, 0)        # yellow
FULL_TAXI = (0, 128, 0)     # green
PASSENGER = (128, 0, 128)   # purple
FAKE_WALL = (0, 128, 128)   # teal
LOC = (191, 191, 191)       # gray_light
DESTINATION = (0, 0, 128)   # blue
DIRS = ((-1, 0), (1, 0), (0, -1), (0, 1))  # DIRECTIONS_2D_NP[:, :4]: N, S, W, E


def frame_chars(desc, cc, np_locs, nlocs, state, cols):
    """Char map of one env (extended_taxi.py:293-307) for state int `state`."""
    d = state % nlocs
    t = state // nlocs
    p = t % (nlocs + 1)
    t //= nlocs + 1
    r, c = t // cols, t % cols
    img = desc.copy()
    img[cc(*np_locs[d])] = "D"
    tc = cc(r, c)
    img[tc] = "T"
    if p != nlocs:
        pc = cc(*np_locs[p])
        img[pc] = "P"
        if pc == tc:
            img[pc] = "T"  # "TP" truncated by the '<U1' dtype
    else:
        img[tc] = "F"
    return img, tc


def frame_rgb(chars, tc, hansen):
    """str_map_to_img's colouring (extended_taxi.py:126-142) of one frame."""
    h, w = chars.shape
    img = np.empty((h, w, 3), np.uint8)
    lut = {"|": WALL, "P": PASSENGER, "T": TAXI, "F": FULL_TAXI, "D": DESTINATION, " ": FLOOR, ":": FAKE_WALL}
    for y in range(h):
        for x in range(w):
            img[y, x] = lut.get(chars[y, x], LOC)
    if hansen:
        for dy, dx in DIRS:
            img[tc[0] + dy, tc[1] + dx] += np.uint8(64)
    return img


def tile(frames):
    """tile_images (render_utils.py:63-88)."""
    f = np.asarray(frames)
    n, h, w, ch = f.shape
    H = int(np.ceil(np.sqrt(n)))
    W = int(np.ceil(float(n) / H))
    f = np.concatenate([f, np.zeros((H * W - n, h, w, ch), np.uint8)]) if H * W > n else f
    return f.reshape(H, W, h, w, ch).transpose(0, 2, 1, 3, 4).reshape(H * h, W * w, ch)


def render_tiled(desc, cc, np_locs, nlocs, cols, states, hansen):
    """The pre-resize image of `states` (one frame per env, in order)."""
    frames = []
    for s in states:
        chars, tc = frame_chars(desc, cc, np_locs, nlocs, int(s), cols)
        frames.append(frame_rgb(chars, tc, hansen))
    return tile(frames)


def _coeffs(ssize, dsize, clamp):
    """OpenCV resizeGeneric_ coefficient setup for INTER_AREA outside the decimation case: source index and
    (alpha0, alpha1) in 11-bit fixed point (saturate_cast<short>(c * 2048), round to nearest even) per
    destination index. `clamp`: the horizontal setup pins the last source column (fx = 0); the vertical one
    does not (its second row index is clipped instead)."""
    inv_scale = float(dsize) / ssize
    scale = 1.0 / inv_scale
    idx = np.empty(dsize, np.int64)
    a = np.empty((dsize, 2), np.int64)
    for dx in range(dsize):
        sx = int(np.floor(dx * scale))
        fx = np.float32((dx + 1) - (sx + 1) * inv_scale)
        fx = np.float32(0.0) if fx <= 0 else np.float32(fx - np.float32(np.floor(fx)))
        if clamp and sx >= ssize - 1:
            fx, sx = np.float32(0.0), ssize - 1
        idx[dx] = sx
        a[dx, 0] = int(np.rint(np.float32(np.float32(1.0) - fx) * np.float32(2048)))
        a[dx, 1] = int(np.rint(np.float32(fx * np.float32(2048))))
    return idx, a


def resize_area_u8(img, dh, dw):
    """cv2.resize(img, (dw, dh), interpolation=INTER_AREA) for uint8 HxWxC when the resize enlarges at least
    one axis (restated; parity unpinned, see module docstring)."""
    sh, sw, ch = img.shape
    if dh <= sh and dw <= sw and not (dh == sh and dw == sw):
        raise NotImplementedError("INTER_AREA decimation (both axes shrink) is not restated")
    xi, xa = _coeffs(sw, dw, True)
    yi, yb = _coeffs(sh, dh, False)
    src = img.astype(np.int64)
    x1 = np.minimum(xi + 1, sw - 1)
    # horizontal pass: int sums in 11-bit fixed point (HResizeLinear)
    hrow = src[:, xi, :] * xa[None, :, 0, None] + src[:, x1, :] * xa[None, :, 1, None]
    S0, S1 = hrow[np.clip(yi, 0, sh - 1)], hrow[np.clip(yi + 1, 0, sh - 1)]
    b0, b1 = yb[:, 0][:, None, None], yb[:, 1][:, None, None]
    out = (((b0 * (S0 >> 4)) >> 16) + ((b1 * (S1 >> 4)) >> 16) + 2) >> 2  # VResizeLinear<uchar> FixedPtCast
    return np.clip(out, 0, 255).astype(np.uint8)


def render_rgb(desc, cc, np_locs, nlocs, cols, states, hansen):
    """TaxiVecEnv.render(idx=arange(n)) as an rgb array (without the caption)."""
    tiled = render_tiled(desc, cc, np_locs, nlocs, cols, states, hansen)
    h, w = desc.shape
    img = resize_area_u8(tiled, w * CELL_PX, h * CELL_PX)
    return np.concatenate([img, np.zeros((img.shape[0], TEXT_SPACE, 3), np.uint8)], axis=1)
