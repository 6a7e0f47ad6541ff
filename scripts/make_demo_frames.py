#!/usr/bin/env python
"""Write the procedural demo sequence shipped in demo-frames/.

The reference ships five Sintel frames (reference demo-frames/); this repo
ships a synthetic stand-in of the same size (436 x 1024, RGB PNG) with a
KNOWN motion, so demo.py / rafttoonnx.py run out of the box and a trained
checkpoint can be sanity-checked against the true flow:

  background: smooth multi-octave texture translating by (+3, +1) px / frame
  foreground: a textured disk (radius 90) translating by (-6, +2) px / frame

    python scripts/make_demo_frames.py [--out demo-frames] [--frames 3]
"""
import argparse
import os

import numpy as np
from PIL import Image

H, W = 436, 1024
BG_V = (3.0, 1.0)      # (u, v) px per frame
FG_V = (-6.0, 2.0)
FG_C0 = (560.0, 210.0)  # disk centre (x, y) in frame 0
FG_R = 90.0


def texture(x, y, seed):
    """Smooth RGB texture evaluated at float coordinates (sum of rotated sinusoids)."""
    rng = np.random.default_rng(seed)
    out = np.zeros(x.shape + (3,), np.float64)
    for octave in range(5):
        f = 0.012 * 2.1 ** octave
        for _ in range(3):
            th = rng.uniform(0, np.pi)
            ph = rng.uniform(0, 2 * np.pi, 3)
            amp = 0.55 ** octave
            arg = f * (np.cos(th) * x + np.sin(th) * y)
            out += amp * np.sin(arg[..., None] + ph)
    out -= out.min()
    return 255.0 * out / out.max()


def frame(t):
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float64)
    bg = texture(xx - BG_V[0] * t, yy - BG_V[1] * t, seed=7)
    cx, cy = FG_C0[0] + FG_V[0] * t, FG_C0[1] + FG_V[1] * t
    fg = texture(xx - FG_V[0] * t, yy - FG_V[1] * t, seed=11)
    fg = 0.35 * fg + 0.65 * np.array([230.0, 120.0, 40.0]) * (fg / 255.0)
    d = np.sqrt((xx - cx) ** 2 + (yy - cy) ** 2)
    a = np.clip(FG_R - d + 0.5, 0.0, 1.0)[..., None]  # anti-aliased edge
    return np.clip(np.rint(a * fg + (1 - a) * bg), 0, 255).astype(np.uint8)


def true_flow(t):
    """Forward flow frame t -> t+1 (u, v), [H, W, 2]."""
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float64)
    cx, cy = FG_C0[0] + FG_V[0] * t, FG_C0[1] + FG_V[1] * t
    inside = (xx - cx) ** 2 + (yy - cy) ** 2 <= FG_R ** 2
    flow = np.empty((H, W, 2), np.float32)
    flow[..., 0] = np.where(inside, FG_V[0], BG_V[0])
    flow[..., 1] = np.where(inside, FG_V[1], BG_V[1])
    return flow


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "demo-frames"))
    ap.add_argument("--frames", type=int, default=3)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    for t in range(a.frames):
        Image.fromarray(frame(t)).save(os.path.join(a.out, f"frame_{t + 1:04d}.png"), optimize=True)
    print(f"wrote {a.frames} frames to {a.out}")


if __name__ == "__main__":
    main()
