"""Pure-ATen reference implementations (numerics oracles + export path).

Each function is written from the math of the reference,
not from its code, and is what runs on CPU tensors, under TorchScript tracing
and under ONNX export (only standard ops appear in the traced graph).
The HIP kernels in ``csrc/`` are tested against these.

Conventions (reference core/corr.py:29-60, core/utils/utils.py:57-77):
  * coords are pixel coordinates, channel 0 = x, channel 1 = y;
  * bilinear sampling with align_corners=True semantics and zero padding;
  * the lookup window channel k of a level is (i, j) = divmod(k, 2r+1) with
    dx = i - r, dy = j - r  (x-offset-major);
  * pyramid level l is avg_pool2d(2, 2)^l of the level-0 volume over the
    target dims, i.e. floor-sized (55 -> 27 -> 13 -> 6).
"""
from __future__ import annotations

import math
from typing import List

import torch
import torch.nn.functional as F


def coords_grid(batch: int, ht: int, wd: int, device=None, dtype=torch.float32):
    ys = torch.arange(ht, device=device, dtype=dtype).view(ht, 1).expand(ht, wd)
    xs = torch.arange(wd, device=device, dtype=dtype).view(1, wd).expand(ht, wd)
    grid = torch.stack([xs, ys], dim=0)
    return grid.unsqueeze(0).repeat(batch, 1, 1, 1)


def bilinear_sampler(img, coords, mask: bool = False):
    """Sample ``img`` (N,C,H,W) at pixel coords (N,h,w,2) [x, y]."""
    H, W = img.shape[-2:]
    x, y = coords.split([1, 1], dim=-1)
    gx = 2 * x / (W - 1) - 1
    gy = 2 * y / (H - 1) - 1
    out = F.grid_sample(img, torch.cat([gx, gy], dim=-1), align_corners=True)
    if mask:
        m = (gx > -1) & (gy > -1) & (gx < 1) & (gy < 1)
        return out, m.float()
    return out


def corr_volume(fmap1, fmap2):
    """All-pairs correlation (B, H1*W1, H2, W2) = <f1, f2> / sqrt(C)."""
    B, C, H, W = fmap1.shape
    a = fmap1.reshape(B, C, H * W)
    b = fmap2.reshape(B, C, -1)
    corr = torch.matmul(a.transpose(1, 2), b)
    return corr.reshape(B, H * W, fmap2.shape[2], fmap2.shape[3]) / math.sqrt(C)


def corr_pyramid(fmap1, fmap2, num_levels: int = 4) -> List[torch.Tensor]:
    """Level list, each (B*H1*W1, 1, H2_l, W2_l) like reference core/corr.py:13-27."""
    B, C, H, W = fmap1.shape
    vol = corr_volume(fmap1.float(), fmap2.float())
    lvl = vol.reshape(B * H * W, 1, fmap2.shape[2], fmap2.shape[3])
    pyr = [lvl]
    for _ in range(num_levels - 1):
        lvl = F.avg_pool2d(lvl, 2, stride=2)
        pyr.append(lvl)
    return pyr


def _window_delta(r: int, device, dtype):
    d = torch.arange(-r, r + 1, device=device, dtype=dtype)
    # channel k = (dx + r) * (2r+1) + (dy + r): x-offset-major.
    dx = d.view(-1, 1).expand(2 * r + 1, 2 * r + 1)
    dy = d.view(1, -1).expand(2 * r + 1, 2 * r + 1)
    return torch.stack([dx, dy], dim=-1)  # (2r+1, 2r+1, 2) as [x, y]


def corr_lookup(pyramid: List[torch.Tensor], coords, radius: int):
    """Window lookup -> (B, L*(2r+1)^2, H1, W1) fp32."""
    B, _, H, W = coords.shape
    c = coords.permute(0, 2, 3, 1).reshape(B * H * W, 1, 1, 2)
    delta = _window_delta(radius, coords.device, coords.dtype).reshape(
        1, 2 * radius + 1, 2 * radius + 1, 2)
    outs = []
    for lvl, vol in enumerate(pyramid):
        sampled = bilinear_sampler(vol, c / (2 ** lvl) + delta)
        # sampled: (BHW, 1, 2r+1 [rows of grid = dx], 2r+1 [cols = dy])
        outs.append(sampled.reshape(B, H, W, -1))
    out = torch.cat(outs, dim=-1)
    return out.permute(0, 3, 1, 2).contiguous()


def corr_onthefly(fmap1, fmap2, coords, radius: int, num_levels: int = 4):
    """Memory-efficient correlation oracle: pool fmap2, correlate lazily.

    Uses pyramid[l] == corr(f1, avgpool^l(f2)) (linearity), so no
    HW x HW volume is materialised: for each level and each window tap the
    feature of fmap2 is bilinearly sampled and dotted with fmap1.
    """
    B, C, H, W = fmap1.shape
    delta = _window_delta(radius, coords.device, coords.dtype).reshape(-1, 2)
    outs = []
    f2 = fmap2.float()
    f1 = fmap1.float()
    base = coords.permute(0, 2, 3, 1)  # (B,H,W,2)
    for lvl in range(num_levels):
        if lvl > 0:
            f2 = F.avg_pool2d(f2, 2, stride=2)
        taps = []
        for t in range(delta.shape[0]):
            pos = base / (2 ** lvl) + delta[t]
            g = bilinear_sampler(f2, pos)  # (B,C,H,W)
            taps.append((g * f1).sum(dim=1))
        outs.append(torch.stack(taps, dim=1))
    return torch.cat(outs, dim=1) / math.sqrt(C)


def convex_upsample(flow, mask, factor: int = 8):
    """Convex upsampling (reference core/raft.py:72-83).

    flow (N,2,H,W), mask (N,9*f*f,H,W) -> (N,2,f*H,f*W); softmax over the 9
    taps, 3x3 neighbourhood of ``f * flow`` with zero padding.
    """
    N, _, H, W = flow.shape
    m = torch.softmax(mask.view(N, 1, 9, factor, factor, H, W), dim=2)
    nb = F.unfold(factor * flow, [3, 3], padding=1).view(N, 2, 9, 1, 1, H, W)
    up = torch.sum(m * nb, dim=2)  # (N,2,f,f,H,W)
    return up.permute(0, 1, 4, 2, 5, 3).reshape(N, 2, factor * H, factor * W)


def upflow8(flow, mode: str = "bilinear"):
    size = (8 * flow.shape[2], 8 * flow.shape[3])
    return 8 * F.interpolate(flow, size=size, mode=mode, align_corners=True)


def sequence_loss_terms(preds, gt, valid, gamma: float, max_flow: float = 400.0):
    """Weighted L1 over the sequence (reference train.py:47-60)."""
    mag = torch.sum(gt ** 2, dim=1).sqrt()
    v = (valid >= 0.5) & (mag < max_flow)
    n = len(preds)
    loss = 0.0
    for i, p in enumerate(preds):
        w = gamma ** (n - i - 1)
        loss = loss + w * (v[:, None] * (p - gt).abs()).mean()
    return loss, v
