"""Geometric helpers with the reference's API (core/utils/utils.py:26-82)."""
from __future__ import annotations

import numpy as np
import torch

from ..ops.reference import bilinear_sampler, coords_grid as _coords_grid, upflow8  # noqa: F401


def coords_grid(batch, ht, wd, device=None):
    """(B,2,H,W) pixel grid, channel 0 = x, channel 1 = y."""
    return _coords_grid(batch, ht, wd, device=device)


def forward_interpolate(flow):
    """Forward-splat a (2,H,W) flow to warm-start the next frame.

    Nearest-neighbour scattered interpolation of the displaced samples back to
    the grid (reference uses scipy griddata 'nearest'); we use a KD-tree
    query, which is the same nearest-sample rule.
    """
    from scipy.spatial import cKDTree

    flow = flow.detach().cpu().numpy()
    dx, dy = flow[0], flow[1]
    ht, wd = dx.shape
    x0, y0 = np.meshgrid(np.arange(wd), np.arange(ht))
    x1 = (x0 + dx).reshape(-1)
    y1 = (y0 + dy).reshape(-1)
    dxf, dyf = dx.reshape(-1), dy.reshape(-1)
    ok = (x1 > 0) & (x1 < wd) & (y1 > 0) & (y1 < ht)
    if not ok.any():
        return torch.zeros(2, ht, wd, dtype=torch.float32)
    tree = cKDTree(np.stack([x1[ok], y1[ok]], axis=1))
    _, idx = tree.query(np.stack([x0.reshape(-1), y0.reshape(-1)], axis=1), k=1)
    fx = dxf[ok][idx].reshape(ht, wd)
    fy = dyf[ok][idx].reshape(ht, wd)
    return torch.from_numpy(np.stack([fx, fy], axis=0)).float()
