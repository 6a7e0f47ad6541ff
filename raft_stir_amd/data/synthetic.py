"""Synthetic FlyingChairs-shaped training pairs (no datasets exist offline).

Each sample is (img1, img2, flow, valid) with img in [0, 255] (3 x H x W),
flow 2 x H x W and valid H x W -- exactly the tensors FlowDataset yields
(reference core/datasets.py:81-90).  img1 is smooth random texture; the flow
is a random affine motion plus a few smooth local bumps (|flow| up to ~40 px,
Chairs-like); img2 is img1 backward-warped so that img2(x + flow(x)) ~ img1(x),
which gives a learnable signal (training loss goes down) rather than noise.

Generation runs on whatever device is asked for, so benchmarks can keep a
small pool of batches resident in HBM and never touch the host.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def _smooth_noise(b, c, h, w, scale, gen, device):
    lh, lw = max(2, h // scale), max(2, w // scale)
    base = torch.rand(b, c, lh, lw, generator=gen, device=device)
    return F.interpolate(base, size=(h, w), mode="bicubic", align_corners=False)


def random_flow(b, h, w, gen, device, max_disp=40.0):
    ys = torch.linspace(-1, 1, h, device=device).view(1, h, 1).expand(b, h, w)
    xs = torch.linspace(-1, 1, w, device=device).view(1, 1, w).expand(b, h, w)
    p = (torch.rand(b, 6, generator=gen, device=device) * 2 - 1)
    tx, ty = p[:, 0, None, None] * max_disp * 0.5, p[:, 1, None, None] * max_disp * 0.5
    a, bb = p[:, 2, None, None] * 0.1, p[:, 3, None, None] * 0.1
    rot = p[:, 4, None, None] * 0.1
    zoom = p[:, 5, None, None] * 0.1
    u = tx + (zoom + a) * xs * w / 2 - rot * ys * h / 2
    v = ty + (zoom + bb) * ys * h / 2 + rot * xs * w / 2
    bumps = (_smooth_noise(b, 2, h, w, 32, gen, device) * 2 - 1) * max_disp * 0.25
    return torch.stack([u, v], dim=1) + bumps


def warp(img, flow):
    """Sample img at x + flow(x) (bilinear, border padding)."""
    b, _, h, w = img.shape
    ys, xs = torch.meshgrid(torch.arange(h, device=img.device, dtype=img.dtype),
                            torch.arange(w, device=img.device, dtype=img.dtype), indexing="ij")
    gx = 2 * (xs[None] + flow[:, 0]) / max(w - 1, 1) - 1
    gy = 2 * (ys[None] + flow[:, 1]) / max(h - 1, 1) - 1
    grid = torch.stack([gx, gy], dim=-1)
    return F.grid_sample(img, grid, mode="bilinear", padding_mode="border", align_corners=True)


@torch.no_grad()
def make_batch(batch, height, width, seed=0, device="cpu", max_disp=40.0):
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    tex = (_smooth_noise(batch, 3, height, width, 8, gen, device) * 0.7
           + _smooth_noise(batch, 3, height, width, 2, gen, device) * 0.3) * 255.0
    flow = random_flow(batch, height, width, gen, device, max_disp)
    # img2(x) = img1(x - flow(x)) approximately satisfies img2(x + flow) = img1(x)
    img2 = warp(tex, -flow)
    valid = torch.ones(batch, height, width, device=device)
    return tex.clamp(0, 255), img2.clamp(0, 255), flow, valid


class SyntheticFlowDataset(torch.utils.data.Dataset):
    """Map-style dataset with the FlowDataset item contract, for loaders/tests."""

    def __init__(self, length=1000, size=(368, 496), seed=0, sparse=False):
        self.length = length
        self.size = tuple(size)
        self.seed = seed
        self.sparse = sparse

    def __len__(self):
        return self.length

    def __getitem__(self, idx):
        h, w = self.size
        i1, i2, flow, valid = make_batch(1, h, w, seed=self.seed * 1000003 + idx)
        if self.sparse:
            gen = torch.Generator().manual_seed(idx)
            valid = (torch.rand(1, h, w, generator=gen) < 0.3).float()
            flow = flow * valid[:, None]
        return i1[0], i2[0], flow[0], valid[0]


class DevicePool:
    """A few synthetic batches resident on the device, cycled per step."""

    def __init__(self, n, batch, height, width, device, seed=0):
        self.batches = [make_batch(batch, height, width, seed=seed + k, device=device)
                        for k in range(n)]
        self.i = 0

    def next(self):
        b = self.batches[self.i % len(self.batches)]
        self.i += 1
        return b
