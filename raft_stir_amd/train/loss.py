"""Sequence loss and flow metrics (reference train.py:47-72).

loss = sum_i gamma^(N-i-1) * mean(valid * |pred_i - gt|_1), valid = (valid>=0.5) & (|gt| < MAX_FLOW).

Unlike the reference, metrics are returned as device tensors (no ``.item()``
host sync per step); the logger materialises them every SUM_FREQ steps.

When the predictions are consecutive views of one (N, B, 2, H, W) tensor on
the GPU (the fused training engine returns them that way) the loss and the
metrics are one fused HIP pass forward and the loss gradient one pass
backward (csrc/loss.hip), instead of ~6 ATen kernels per prediction each
way plus ~40 for the metrics.
"""
from __future__ import annotations

import torch

MAX_FLOW = 400


class _SeqLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, preds, gt, valid, gamma, max_flow):
        ctx.save_for_backward(preds, gt, valid)
        ctx.gamma, ctx.max_flow = gamma, max_flow
        loss, metrics = torch.ops.raft_stir.seq_loss(preds, gt, valid, gamma, max_flow)
        ctx.mark_non_differentiable(metrics)
        return loss, metrics

    @staticmethod
    def backward(ctx, g, _gm):
        preds, gt, valid = ctx.saved_tensors
        gp = torch.ops.raft_stir.seq_loss_backward(g.float().reshape(()), preds, gt, valid, ctx.gamma,
                                                   ctx.max_flow)
        return gp, None, None, None, None


def _stacked(flow_preds):
    """The (N, B, 2, H, W) tensor the predictions are consecutive views of, or None."""
    p0 = flow_preds[0]
    base = p0._base
    if base is None or not base.is_contiguous() or base.numel() != len(flow_preds) * p0.numel():
        return None
    for i, p in enumerate(flow_preds):
        if (p._base is not base or not p.is_contiguous() or p.shape != p0.shape
                or p.storage_offset() != base.storage_offset() + i * p0.numel()):
            return None
    return base.view(len(flow_preds), *p0.shape)


def _fused_ok(flow_preds, flow_gt):
    if not flow_gt.is_cuda or flow_preds[0].dtype != torch.float32 or flow_gt.dim() != 4:
        return False
    from ..ops import _ext
    return _ext.use_hip(flow_gt)


def sequence_loss(flow_preds, flow_gt, valid, gamma=0.8, max_flow=MAX_FLOW, sync_metrics=True):
    n = len(flow_preds)
    stacked = _stacked(flow_preds) if _fused_ok(flow_preds, flow_gt) else None
    if stacked is not None:
        gt = flow_gt.float().contiguous()
        vf = valid.float().contiguous()
        # the kernel also forms the last prediction's metrics (flow_metrics' semantics)
        loss, m = _SeqLoss.apply(stacked, gt, vf, float(gamma), float(max_flow))
        metrics = {"epe": m[0], "1px": m[1], "3px": m[2], "5px": m[3]}
        if sync_metrics:
            metrics = {k: float(t) for k, t in metrics.items()}
        return loss, metrics
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
