"""Sequence loss and flow metrics (reference train.py:47-72).

loss = sum_i gamma^(N-i-1) * mean(valid * |pred_i - gt|_1), valid = (valid>=0.5) & (|gt| < MAX_FLOW).

Unlike the reference, metrics are returned as device tensors (no ``.item()``
host sync per step); the logger materialises them every SUM_FREQ steps.
"""
from __future__ import annotations

import torch

MAX_FLOW = 400


def sequence_loss(flow_preds, flow_gt, valid, gamma=0.8, max_flow=MAX_FLOW, sync_metrics=True):
    n = len(flow_preds)
    mag = torch.sum(flow_gt ** 2, dim=1).sqrt()
    v = (valid >= 0.5) & (mag < max_flow)
    vf = v[:, None].to(flow_gt.dtype)
    loss = flow_gt.new_zeros(())
    for i, pred in enumerate(flow_preds):
        w = gamma ** (n - i - 1)
        loss = loss + w * (vf * (pred - flow_gt).abs()).mean()
    metrics = flow_metrics(flow_preds[-1].detach(), flow_gt, v)
    if sync_metrics:
        metrics = {k: float(t) for k, t in metrics.items()}
    return loss, metrics


def flow_metrics(pred, gt, valid_mask):
    epe = torch.sum((pred - gt) ** 2, dim=1).sqrt().reshape(-1)
    m = valid_mask.reshape(-1).to(epe.dtype)
    cnt = m.sum().clamp_min(1.0)
    return {
        "epe": (epe * m).sum() / cnt,
        "1px": ((epe < 1).to(epe.dtype) * m).sum() / cnt,
        "3px": ((epe < 3).to(epe.dtype) * m).sum() / cnt,
        "5px": ((epe < 5).to(epe.dtype) * m).sum() / cnt,
    }
