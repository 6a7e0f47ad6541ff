"""Fused channels-last normalisation + activation for the encoders.

``norm_act(norm, x, relu=True, residual=None)`` computes, with the semantics of
reference core/extractor.py (``relu(norm(x))``; residual blocks
``relu(skip + relu(norm(conv(y))))``):

    y = norm(x); if relu: y = relu(y); if residual is not None: y = relu(residual + y)

On GPU tensors with an InstanceNorm2d (no affine, no running stats -- the
reference fnet) or BatchNorm2d (the reference cnet; training mode uses batch
statistics and updates the running buffers exactly like nn.BatchNorm2d, eval
mode uses the running buffers) it runs csrc/norm.hip directly on the NHWC
memory of a channels_last activation: no NCHW round-trip copies, one stats
pass + one fused apply pass forward, one reduction + one apply pass backward.
Everything else (CPU, export, GroupNorm, identity) takes the composite path.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _ext
from . import enc_conv
from . import fp32conv

_CL = torch.channels_last
_FOLD_BIAS = os.environ.get("RS_FOLD_BIAS", "1") != "0"


def _nhwc(x):
    return x.permute(0, 2, 3, 1)


class _NormAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, res, mean, rstd, relu, batch_stats, bias=None):
        xn = _nhwc(x)
        rn = _nhwc(res) if res is not None else None
        y = torch.ops.raft_stir.norm_act(xn, mean, rstd, gamma, beta, rn, relu)
        ctx.save_for_backward(x, gamma, beta, res, mean, rstd)
        ctx.relu, ctx.batch_stats = relu, batch_stats
        ctx.bias_meta = (bias.shape, bias.dtype) if bias is not None else None
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        x, gamma, beta, res, mean, rstd = ctx.saved_tensors
        dyn = _nhwc(dy.contiguous(memory_format=_CL)).to(x.dtype)
        rn = _nhwc(res) if res is not None else None
        dx, dres, s1, s2, s12 = torch.ops.raft_stir.norm_act_backward(
            dyn, _nhwc(x), mean, rstd, gamma, beta, rn, ctx.relu, ctx.batch_stats)
        want_g = gamma is not None and ctx.needs_input_grad[1]
        want_b = beta is not None and ctx.needs_input_grad[2]
        if want_g and want_b:
            d = s12.sum(1)  # (2, C): one reduction for dbeta and dgamma (s1 = s12[0], s2 = s12[1])
            dbeta, dgamma = d[0], d[1]
        else:
            dgamma = s2.sum(0) if want_g else None
            dbeta = s1.sum(0) if want_b else None
        dres_out = dres.permute(0, 3, 1, 2) if res is not None else None
        dbias = None
        if ctx.bias_meta is not None and ctx.needs_input_grad[8]:
            shape, dtype = ctx.bias_meta
            if ctx.batch_stats:
                # a per-channel constant is removed by the batch/instance
                # mean: its gradient is exactly zero
                dbias = torch.zeros(shape, dtype=dtype, device=dy.device)
            else:  # running statistics: d pre / d bias = gamma * rstd
                g = gamma.float() if gamma is not None else 1.0
                dbias = (s1.sum(0) * g * rstd.reshape(-1)).to(dtype)
        return dx.permute(0, 3, 1, 2), dgamma, dbeta, dres_out, None, None, None, None, dbias


def _hip_ok(norm, x, residual):
    if not _ext.use_hip(x) or x.dim() != 4:
        return False
    if x.dtype not in (torch.float32, torch.bfloat16):
        return False
    if not x.is_contiguous(memory_format=_CL):
        return False
    if residual is not None and (residual.dtype != x.dtype or residual.shape != x.shape):
        return False
    C = x.shape[1]
    vn = 8 if x.dtype == torch.bfloat16 else 4
    if C % vn or C // vn > 256:
        return False
    if isinstance(norm, nn.InstanceNorm2d):
        return not norm.affine and not norm.track_running_stats
    if isinstance(norm, nn.BatchNorm2d):
        return norm.affine and norm.track_running_stats and norm.momentum is not None
    return False


def norm_act(norm: nn.Module, x: torch.Tensor, relu: bool = True, residual=None, bias=None):
    """``bias``: the producing convolution's bias, folded into the statistics
    (see :func:`conv_norm_act`); None if already applied."""
    if not _hip_ok(norm, x, residual):
        if bias is not None:
            x = x + bias.to(x.dtype).view(1, -1, 1, 1)
        y = norm(x)
        if relu:
            y = F.relu(y)
        if residual is not None:
            y = F.relu(residual + y)
        return y
    if residual is not None:
        residual = residual.contiguous(memory_format=_CL)
    xn = _nhwc(x)
    if isinstance(norm, nn.InstanceNorm2d):
        with torch.no_grad():  # the stats' gradient is part of _NormAct.backward
            mean, rstd = torch.ops.raft_stir.norm_stats(xn, True, norm.eps)
        return _NormAct.apply(x, None, None, residual, mean, rstd, relu, True, bias)
    # BatchNorm2d
    batch_stats = norm.training
    if batch_stats:
        with torch.no_grad():
            mean, rstd = torch.ops.raft_stir.norm_stats(xn, False, norm.eps)
            n = x.numel() // x.shape[1]
            rm, rv = norm.running_mean, norm.running_var
            if rm.dtype == torch.float32 and rv.dtype == torch.float32 and rm.is_contiguous() and rv.is_contiguous():
                # one fused launch (csrc/norm.hip bn_running_kernel)
                torch.ops.raft_stir.bn_running_update(
                    mean.reshape(-1), rstd.reshape(-1), None if bias is None else bias.detach().float().contiguous(),
                    rm, rv, norm.num_batches_tracked, norm.eps, norm.momentum, n)
            else:
                var = (rstd.reshape(-1).pow(-2) - norm.eps).clamp_min(0)
                unbiased = var * (n / max(n - 1, 1))
                m = norm.momentum
                bmean = mean.reshape(-1) if bias is None else mean.reshape(-1) + bias.detach().float()
                rm.mul_(1 - m).add_(bmean, alpha=m)
                rv.mul_(1 - m).add_(unbiased, alpha=m)
                norm.num_batches_tracked.add_(1)
    else:
        mean = norm.running_mean.float().reshape(1, -1)
        if bias is not None:  # gamma * (x + b - mean) * rstd + beta
            mean = mean - bias.detach().float().reshape(1, -1)
        rstd = torch.rsqrt(norm.running_var.float() + norm.eps).reshape(1, -1)
    return _NormAct.apply(x, norm.weight, norm.bias, residual, mean.contiguous(), rstd.contiguous(),
                          relu, batch_stats, bias)


def _norm_kind_ok(norm):
    if isinstance(norm, nn.InstanceNorm2d):
        return not norm.affine and not norm.track_running_stats
    if isinstance(norm, nn.BatchNorm2d):
        return norm.affine and norm.track_running_stats and norm.momentum is not None
    return False


def conv_norm_act(conv: nn.Conv2d, norm: nn.Module, x: torch.Tensor, relu: bool = True, residual=None):
    """``norm_act(norm, conv(x), relu, residual)``.  On the GPU path the conv
    runs without its bias and the bias is folded into the normalisation
    (instance / train-mode batch norm remove it exactly; eval-mode batch norm
    shifts its running mean by it): no bias-add pass over the conv output
    forward and no bias-gradient reduction over it backward."""
    if conv.bias is None or not _FOLD_BIAS or not _ext.use_hip(x) or not _norm_kind_ok(norm):
        return norm_act(norm, conv(x), relu, residual)
    if enc_conv.eligible(conv, x):  # stride-1 3x3 on the hand-written implicit-GEMM kernels
        return norm_act(norm, enc_conv.conv3x3(conv, x), relu, residual, bias=conv.bias)
    if enc_conv.eligible_geo(conv, x):  # stride-2 3x3 / 1x1 (strided geometry of the same kernels)
        return norm_act(norm, enc_conv.conv_geo(conv, x, bias=False), relu, residual, bias=conv.bias)
    y = fp32conv.conv2d(x, conv.weight, None, conv.stride, conv.padding, conv.dilation, conv.groups)
    return norm_act(norm, y, relu, residual, bias=conv.bias)


def conv_pair_norm_act(conv1: nn.Conv2d, norm1: nn.Module, down: nn.Conv2d, norm_d: nn.Module, x: torch.Tensor):
    """(norm_act(norm1, conv1(x)), norm_act(norm_d, down(x), relu=False)) for a
    residual block's stride-2 first conv and its stride-2 1x1 shortcut: on the
    GPU path both convs are one autograd node (ops/enc_conv.py conv_pair) whose
    backward produces ONE input gradient (the shortcut's term fused into the
    3x3's (0, 0) phase) instead of two dgrads and an add."""
    fold = (conv1.bias is not None and down.bias is not None and _FOLD_BIAS and _ext.use_hip(x)
            and _norm_kind_ok(norm1) and _norm_kind_ok(norm_d))
    if fold and enc_conv.pair_eligible(conv1, down, x):
        y1, yd = enc_conv.conv_pair(conv1, down, x)
        return (norm_act(norm1, y1, True, None, bias=conv1.bias),
                norm_act(norm_d, yd, False, None, bias=down.bias))
    return conv_norm_act(conv1, norm1, x), conv_norm_act(down, norm_d, x, relu=False)
