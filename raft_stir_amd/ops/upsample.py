"""Convex x8 upsampling op (csrc/convex_upsample.hip on GPU, ATen on CPU)."""
from __future__ import annotations

import torch

from . import _ext
from . import reference as ref
from .corr import to_nhwc


class _ConvexUp(torch.autograd.Function):
    @staticmethod
    def forward(ctx, flow, mask_nhwc):
        ctx.save_for_backward(flow, mask_nhwc)
        return torch.ops.raft_stir.convex_upsample(flow, mask_nhwc)

    @staticmethod
    def backward(ctx, dup):
        flow, mask = ctx.saved_tensors
        dflow, dmask = torch.ops.raft_stir.convex_upsample_backward(flow, mask, dup.contiguous())
        return dflow, dmask


def convex_upsample(flow: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """flow (N,2,H,W), mask (N,576,H,W) -> (N,2,8H,8W) fp32."""
    if _ext.use_hip(flow):
        m = to_nhwc(mask)
        if m.dtype not in (torch.float32, torch.bfloat16):
            m = m.float()
        return _ConvexUp.apply(flow.float().contiguous(), m)
    return ref.convex_upsample(flow, mask.to(flow.dtype))


def upflow8(flow: torch.Tensor) -> torch.Tensor:
    return ref.upflow8(flow)
