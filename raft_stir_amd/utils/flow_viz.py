"""Flow visualisation with the Middlebury colour wheel
(reference core/utils/flow_viz.py: ``make_colorwheel``, ``flow_uv_to_colors``,
``flow_to_image`` -- same API, vectorised).

The wheel has 55 hues: red->yellow 15, yellow->green 6, green->cyan 4,
cyan->blue 11, blue->magenta 13, magenta->red 6 (Baker et al., ICCV 2007).
Direction picks the hue (angle of (-u, -v)), magnitude (normalised by the
max radius) the saturation; out-of-range radii are dimmed by 0.75.
"""
from __future__ import annotations

import numpy as np

_SEGMENTS = (15, 6, 4, 11, 13, 6)


def make_colorwheel() -> np.ndarray:
    """(55, 3) float array of RGB wheel colours in [0, 255]."""
    rows = []
    ry, yg, gc, cb, bm, mr = _SEGMENTS

    # each segment ramps one channel up or down while the others stay fixed
    def seg(n, r, g, b):
        t = np.floor(255 * np.arange(n) / n)
        cols = []
        for spec in (r, g, b):
            if spec == "up":
                cols.append(t)
            elif spec == "down":
                cols.append(255 - t)
            else:
                cols.append(np.full(n, float(spec)))
        return np.stack(cols, axis=1)

    rows.append(seg(ry, 255, "up", 0))
    rows.append(seg(yg, "down", 255, 0))
    rows.append(seg(gc, 0, 255, "up"))
    rows.append(seg(cb, 0, "down", 255))
    rows.append(seg(bm, "up", 0, 255))
    rows.append(seg(mr, 255, 0, "down"))
    return np.concatenate(rows, axis=0)


def flow_uv_to_colors(u, v, convert_to_bgr=False):
    """Normalised flow components (H, W) -> uint8 (H, W, 3)."""
    wheel = make_colorwheel()
    ncols = wheel.shape[0]
    rad = np.sqrt(np.square(u) + np.square(v))
    a = np.arctan2(-v, -u) / np.pi
    fk = (a + 1) / 2 * (ncols - 1)
    k0 = np.floor(fk).astype(np.int32)
    k1 = k0 + 1
    k1[k1 == ncols] = 0
    f = (fk - k0)[..., None]
    col = (1 - f) * (wheel[k0] / 255.0) + f * (wheel[k1] / 255.0)
    inside = (rad <= 1)[..., None]
    col = np.where(inside, 1 - rad[..., None] * (1 - col), col * 0.75)
    img = np.floor(255 * col).astype(np.uint8)
    return img[..., ::-1] if convert_to_bgr else img


def flow_to_image(flow_uv, clip_flow=None, convert_to_bgr=False):
    """(H, W, 2) flow -> (H, W, 3) uint8 colour image."""
    assert flow_uv.ndim == 3 and flow_uv.shape[2] == 2, "input flow must have shape [H,W,2]"
    if clip_flow is not None:
        flow_uv = np.clip(flow_uv, 0, clip_flow)
    u, v = flow_uv[..., 0], flow_uv[..., 1]
    rad_max = np.max(np.sqrt(np.square(u) + np.square(v)))
    eps = 1e-5
    return flow_uv_to_colors(u / (rad_max + eps), v / (rad_max + eps), convert_to_bgr)
