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

import weakref

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _ext
from . import enc_conv
from . import fp32conv
from ..runtime import weights

_CL = torch.channels_last
_FOLD_BIAS = True


def _nhwc(x):
    return x.permute(0, 2, 3, 1)


class _NormAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, res, mean, rstd, relu, batch_stats, bias=None, sink=None):
        xn = _nhwc(x)
        rn = _nhwc(res) if res is not None else None
        y = torch.ops.raft_stir.norm_act(xn, mean, rstd, gamma, beta, rn, relu)
        ctx.save_for_backward(x, gamma, beta, res, mean, rstd)
        ctx.relu, ctx.batch_stats = relu, batch_stats
        ctx.sink = sink
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
            # (2, C): dbeta and dgamma (s1 = s12[0], s2 = s12[1]); batch statistics
            # have one group -- a view, no reduction launch
            d = s12[:, 0] if s12.shape[1] == 1 else s12.sum(1)
            dbeta, dgamma = d[0], d[1]
        else:
            dgamma = s2.sum(0) if want_g else None
            dbeta = s1.sum(0) if want_b else None
        dres_out = dres.permute(0, 3, 1, 2) if res is not None else None
        if res is not None and ctx.sink is not None and ctx.sink.armed:
            # the block's first conv adds it into its input gradient (enc_conv.GradSink)
            ctx.sink.dres, dres_out = dres, None
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
        return dx.permute(0, 3, 1, 2), dgamma, dbeta, dres_out, None, None, None, None, dbias, None


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


def _cached(norm: nn.Module, name: str, srcs, compute):
    """Per-module cache of tensors derived from ``srcs`` (eval-mode BatchNorm
    constants).  Keyed on the weight generation and the sources' version
    counters; a stale entry is recomputed INTO its existing storage, so hipGraphs
    captured with it stay valid (runtime/weights.py refresh_all re-runs every
    entry through the registered refresher)."""
    key = (weights.generation(),) + tuple((t.data_ptr(), t._version) for t in srcs) + (norm.eps,)
    hit = norm.__dict__.get(name)
    if hit is not None and hit[0] == key:
        return hit[2]
    with torch.no_grad():
        vals = compute()
        if hit is not None and all(a.shape == b.shape for a, b in zip(hit[2], vals)):
            for a, b in zip(hit[2], vals):
                a.copy_(b)
            vals = hit[2]
    norm.__dict__[name] = (key, (srcs, compute), vals)
    _LIVE.add(norm)
    return vals


_LIVE = weakref.WeakSet()


def _refresh_cached() -> None:
    for norm in list(_LIVE):
        for name in ("_rs_affine", "_rs_moments"):
            hit = norm.__dict__.get(name)
            if hit is not None:
                srcs, compute = hit[1]
                norm.__dict__[name] = (None,) + hit[1:]
                _cached(norm, name, srcs, compute)


weights.register_refresher(_refresh_cached)


def _eval_affine(norm: nn.BatchNorm2d, bias):
    """Eval-mode BatchNorm (+ the folded conv bias) as per-channel (scale,
    shift), padded to a multiple of 4 channels: y = x_nobias * scale + shift."""
    srcs = [norm.running_mean, norm.running_var, norm.weight, norm.bias] + ([bias] if bias is not None else [])

    def compute():
        C = norm.running_mean.numel()
        scale = norm.weight.detach().float() * torch.rsqrt(norm.running_var.float() + norm.eps)
        mean = norm.running_mean.float() - (bias.detach().float() if bias is not None else 0.0)
        shift = norm.bias.detach().float() - mean * scale
        pad = (-C) % 4
        sc = torch.zeros(C + pad, device=scale.device, dtype=torch.float32)
        sh = torch.zeros(C + pad, device=scale.device, dtype=torch.float32)
        sc[:C] = scale
        sh[:C] = shift
        return sc, sh
    return _cached(norm, "_rs_affine", srcs, compute)


def _eval_fused_ok(conv: nn.Conv2d, norm: nn.Module, x: torch.Tensor, residual) -> bool:
    """Eval-mode BatchNorm with nothing to differentiate: the whole norm ->
    ReLU (-> residual add -> ReLU) chain goes into the conv epilogue."""
    if not isinstance(norm, nn.BatchNorm2d) or norm.training or not _norm_kind_ok(norm):
        return False
    if torch.is_grad_enabled() and (x.requires_grad or conv.weight.requires_grad or norm.weight.requires_grad
                                    or norm.bias.requires_grad
                                    or (residual is not None and residual.requires_grad)):
        return False
    if residual is not None and (residual.shape != x.shape[:1] + residual.shape[1:] or residual.dtype != x.dtype
                                 or not residual.is_contiguous(memory_format=_CL)):
        return False
    if x.dtype == torch.float32:
        return enc_conv.eligible_f32(conv, x, residual)
    if enc_conv.eligible(conv, x):
        return True
    return residual is None and enc_conv.eligible_geo(conv, x)


def norm_act(norm: nn.Module, x: torch.Tensor, relu: bool = True, residual=None, bias=None, res_sink=None):
    """``bias``: the producing convolution's bias, folded into the statistics
    (see :func:`conv_norm_act`); None if already applied.  ``res_sink``: see
    :func:`conv_norm_act`."""
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

    def batch_moments(per_sample):
        with torch.no_grad():  # the stats' gradient is part of _NormAct.backward
            return torch.ops.raft_stir.norm_stats(xn, per_sample, norm.eps)
    if isinstance(norm, nn.InstanceNorm2d):
        mean, rstd = batch_moments(True)
        return _NormAct.apply(x, None, None, residual, mean, rstd, relu, True, bias, res_sink)
    # BatchNorm2d
    batch_stats = norm.training
    if batch_stats:
        n = x.numel() // x.shape[1]
        rm, rv = norm.running_mean, norm.running_var
        if rm.dtype == torch.float32 and rv.dtype == torch.float32 and rm.is_contiguous() and rv.is_contiguous():
            # the running update rides on the statistics finalize (csrc/norm.hip finalize_kernel)
            with torch.no_grad():
                nbt = norm.num_batches_tracked
                mean, rstd = torch.ops.raft_stir.norm_stats(
                    xn, False, norm.eps, rm, rv, nbt if nbt is not None and nbt.dtype == torch.long else None,
                    None if bias is None else bias.detach().float().contiguous(), norm.momentum, n)
                # a custom mutable op does not bump the version counters: do it
                # here so the eval-mode caches keyed on them (_cached) go stale
                torch.autograd.graph.increment_version([rm, rv])
        else:
            mean, rstd = batch_moments(False)
            with torch.no_grad():
                var = (rstd.reshape(-1).pow(-2) - norm.eps).clamp_min(0)
                unbiased = var * (n / max(n - 1, 1))
                m = norm.momentum
                bmean = mean.reshape(-1) if bias is None else mean.reshape(-1) + bias.detach().float()
                rm.mul_(1 - m).add_(bmean, alpha=m)
                rv.mul_(1 - m).add_(unbiased, alpha=m)
                norm.num_batches_tracked.add_(1)
    else:
        mean, rstd = _eval_moments(norm, bias)
    return _NormAct.apply(x, norm.weight, norm.bias, residual, mean.contiguous(), rstd.contiguous(),
                          relu, batch_stats, bias, res_sink)


def _eval_moments(norm: nn.BatchNorm2d, bias):
    """(running mean - conv bias, rsqrt(running var + eps)) as (1, C) fp32,
    cached on the module (:func:`_cached`)."""
    srcs = [norm.running_mean, norm.running_var] + ([bias] if bias is not None else [])

    def compute():
        mean = norm.running_mean.float().reshape(1, -1)
        if bias is not None:  # gamma * (x + b - mean) * rstd + beta
            mean = mean - bias.detach().float().reshape(1, -1)
        rstd = torch.rsqrt(norm.running_var.float() + norm.eps).reshape(1, -1)
        return mean.contiguous(), rstd.contiguous()
    return _cached(norm, "_rs_moments", srcs, compute)


def _norm_kind_ok(norm):
    if isinstance(norm, nn.InstanceNorm2d):
        return not norm.affine and not norm.track_running_stats
    if isinstance(norm, nn.BatchNorm2d):
        return norm.affine and norm.track_running_stats and norm.momentum is not None
    return False


def conv_norm_act(conv: nn.Conv2d, norm: nn.Module, x: torch.Tensor, relu: bool = True, residual=None,
                  grad_sink=None, res_sink=None):
    """``norm_act(norm, conv(x), relu, residual)``.  On the GPU path the conv
    runs without its bias and the bias is folded into the normalisation
    (instance / train-mode batch norm remove it exactly; eval-mode batch norm
    shifts its running mean by it): no bias-add pass over the conv output
    forward and no bias-gradient reduction over it backward.  ``grad_sink`` /
    ``res_sink``: an enc_conv.GradSink shared by a residual block's first conv
    (absorbs the skip gradient in its input gradient) and its second norm
    (hands the skip gradient over instead of returning it)."""
    if enc_conv.sconv_eligible(conv, x, residual):  # narrow channels (RAFT-small encoders), inference
        if isinstance(norm, nn.Sequential) and len(norm) == 0:  # norm_fn 'none': all in the conv epilogue
            return enc_conv.sconv(conv, x, True, relu, residual)
        if _norm_kind_ok(norm) and _FOLD_BIAS:
            return norm_act(norm, enc_conv.sconv(conv, x, False), relu, residual, bias=conv.bias)
        return norm_act(norm, enc_conv.sconv(conv, x, True), relu, residual)
    if enc_conv.sconv_train_eligible(conv, x):  # narrow channels (RAFT-small encoders), training
        fold = conv.bias is not None and _norm_kind_ok(norm)
        return norm_act(norm, enc_conv.sconv_train(conv, x, bias=not fold), relu, residual,
                        bias=conv.bias if fold else None)
    if conv.bias is None or not _FOLD_BIAS or not _ext.use_hip(x) or not _norm_kind_ok(norm):
        if residual is None and conv.bias is not None and _ext.use_hip(x) and enc_conv.stem_eligible(conv, x):
            # the 7x7 stem ahead of a norm that cannot absorb the bias (RAFT-small's
            # norm_fn 'none' context encoder): the bias as a separate add
            y = enc_conv.stem(conv, x)
            return norm_act(norm, y + conv.bias.to(y.dtype).view(1, -1, 1, 1), relu, residual)
        if _ext.use_hip(x) and enc_conv.eligible_geo(conv, x):  # e.g. RAFT-small's wide shortcut ahead of norm_fn 'none'
            return norm_act(norm, enc_conv.conv_geo(conv, x), relu, residual)
        return norm_act(norm, conv(x), relu, residual)
    if residual is None and enc_conv.stem_eligible(conv, x):  # the 7x7 / stride-2 stem (csrc/stem.hip)
        if isinstance(norm, nn.BatchNorm2d) and not norm.training and not (
                torch.is_grad_enabled() and (conv.weight.requires_grad or norm.weight.requires_grad
                                             or norm.bias.requires_grad)):
            sc, sh = _eval_affine(norm, conv.bias)
            return enc_conv.stem_norm(conv, x, sc, sh, relu)
        return norm_act(norm, enc_conv.stem(conv, x), relu, residual, bias=conv.bias)
    if enc_conv.eligible_f32_train(conv, x):  # fp32 training on the split-bf16 F32 tiles
        return norm_act(norm, enc_conv.conv_f32_train(conv, x, bias=False), relu, residual, bias=conv.bias)
    if _eval_fused_ok(conv, norm, x, residual):  # eval BatchNorm: everything in the conv epilogue
        sc, sh = _eval_affine(norm, conv.bias)
        return enc_conv.conv_norm(conv, x, sc, sh, relu, residual)
    if enc_conv.eligible_f32(conv, x):  # fp32 inference on the split-bf16 F32 tiles
        return norm_act(norm, enc_conv.conv_f32(conv, x, bias=False), relu, residual, bias=conv.bias)
    if enc_conv.eligible(conv, x):  # stride-1 3x3 on the hand-written implicit-GEMM kernels
        return norm_act(norm, enc_conv.conv3x3(conv, x, sink=grad_sink), relu, residual, bias=conv.bias,
                        res_sink=res_sink)
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
    if fold and x.dtype == torch.float32:  # fp32: each conv on its own F32 path (inference or training)
        return conv_norm_act(conv1, norm1, x), conv_norm_act(down, norm_d, x, relu=False)
    if fold and enc_conv.pair_eligible(conv1, down, x):
        if _eval_fused_ok(conv1, norm1, x, None) and _eval_fused_ok(down, norm_d, x, None):
            sc1, sh1 = _eval_affine(norm1, conv1.bias)
            scd, shd = _eval_affine(norm_d, down.bias)
            return (enc_conv.conv_norm(conv1, x, sc1, sh1, True),
                    enc_conv.conv_norm(down, x, scd, shd, False))
        y1, yd = enc_conv.conv_pair(conv1, down, x)
        return (norm_act(norm1, y1, True, None, bias=conv1.bias),
                norm_act(norm_d, yd, False, None, bias=down.bias))
    return conv_norm_act(conv1, norm1, x), conv_norm_act(down, norm_d, x, relu=False)
