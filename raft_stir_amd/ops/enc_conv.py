"""Stride-1 3x3 encoder convolutions on the hand-written implicit-GEMM kernels.

The residual blocks of the feature / context encoders (reference
core/extractor.py:6-56, 118-192) spend most of the encoder FLOPs in stride-1
3x3 convolutions at 1/2, 1/4 and 1/8 resolution (64, 96, 128 channels).  On
the GPU bf16 path they run here instead of MIOpen:

  forward : csrc/enc_halo.hip (halo tiles, the block's weights
            resident in LDS) for 64 / 96 input channels, else the csrc/conv.hip
            implicit GEMM (NHWC, buffer-DMA tiles)
  dgrad   : the same kernels on dY with the transposed, spatially flipped
            weight (a stride-1 'same' conv's input gradient is a conv)
  wgrad   : csrc/conv_wgrad.hip (split-K over pixels, fp32 accumulation);
            96 input channels as two overlapping 64-channel segments

Measured on MI355X at the Chairs training shape (scripts/bench_encoder_conv.py):
fwd + dgrad + wgrad of one conv per shape 2.01 ms (MIOpen) -> 1.35 ms.
The bias is folded into the following normalisation (ops/norm.py), so these
convolutions have none.
"""
from __future__ import annotations

import os
import weakref

import torch
import torch.nn as nn

from . import _ext, wpack
from .conv import (EPI_BIAS, EPI_NORM, choose_tile_f32, conv_fused, frag32_eligible, frag_weight, frag_weight_split,
                   pack_weight, pad_to)

_ENABLED = os.environ.get("RS_ENC_CONV", "1") != "0"
_CL = torch.channels_last


def choose_enc_tile(P: int, cin: int, cout: int) -> int:
    """Kernel variant for a stride-1 3x3 conv reading ``cin`` and writing
    ``cout`` channels over P pixels (scripts/bench_encoder_conv.py)."""
    if cin % 64 or cout % 64:
        return 4                   # 128x64 register-staged tile, 32-deep K steps
    if cout <= 64:
        return 17                  # 64 co x 64 px buffer-DMA tile (1/2-res 64->64: 125 vs 140 us for
                                   # the 128-px tile 21, profiles/r2/enc_conv_tiles.txt)
    return 16 if P >= 40000 else 17


_WGRAD_DMA = True
_HALO = True


def _halo_ok(cin: int, cout: int) -> bool:
    """csrc/enc_halo.hip (halo tiles, weights resident in LDS) has
    this conv: 64 input channels with a multiple of 64 outputs, or 96 inputs
    with a multiple of 32 (the encoders' layer1 / layer2 3x3 convs; layer3's
    128-channel convs measured faster on the implicit-GEMM tiles,
    profiles/r2/enc_halo_bench.txt, and the 128-channel halo variant was
    removed)."""
    if not _HALO:
        return False
    if cin == 64:
        return cout % 64 == 0
    return cin == 96 and cout % 32 == 0


# csrc/conv_v3.h weight-streaming tiles for the encoder 3x3 convs where they
# measured faster than the halo / implicit-GEMM kernels (scripts/bench_enc_v3.py,
# profiles/r5/README.md: forward 364 -> 255 us over the six fnet / cnet shapes;
# the 1/2-res 64 -> 64 conv of fnet's 16 images stays on csrc/enc_halo.hip).
# 96 channels are read as two overlapping 64-channel windows, [0, 64) and
# [32, 96), with zero weights on the duplicated half.
_V3 = True
# 64 -> 64 convs with at least this many pixels stay on the halo kernel: both
# encoders' 1/2-res convs at the training shape (fnet 730k, cnet 365k pixels;
# cnet on the halo kernel: 431.5 / 431.0 vs 429.7 / 429.2 pairs/s with v3 tile
# 65, profiles/r6/ab_halo_cnet_s10.txt -- and its backward gets the halo
# kernel's skip-gradient accumulation).  RS_HALO_MIN_P: A/B of the crossover
_HALO_MIN_P = int(os.environ.get("RS_HALO_MIN_P", "300000"))


def _v3_tile(P: int, cin: int, cout: int):
    if not _V3 or cin % 32 or cin < 64 or cout % 32:
        return None
    if cin == 64 and cout == 64 and P >= _HALO_MIN_P:
        return None
    # (tile 68, the 8-wave 64 x 384-px tile, wins the isolated cnet 1/2-res
    # conv but costs 131 vs 91 us per call inside the training step, where it
    # co-runs with fnet: profiles/r5/train_kernel_stats_s18_*.csv)
    return 65 if cout <= 64 else 61


def _v3_windows(cin: int):
    """(channel windows of the input, pack_weight segment spec) for the v3 tiles."""
    if cin % 64 == 0:
        return [(0, cin)], [(cin, [(0, cin, 0)])]
    return [(0, 64), (cin - 64, 64)], [(64, [(0, 64, 0)]), (64, [(64, cin - 64, 128 - cin)])]


def _v3_weight(weight: torch.Tensor, dgrad: bool) -> torch.Tensor:
    cout, cin = weight.shape[:2]
    k_in, k_out = (cout, cin) if dgrad else (cin, cout)
    _, wsegs = _v3_windows(k_in)

    def layout(ws):
        w = ws[0].transpose(0, 1).flip(2, 3) if dgrad else ws[0]
        return frag_weight(pack_weight(w, wsegs, pad_to(k_out, 128), _F32))
    return wpack.packed(("v3", id(weight), dgrad), [weight], layout)


def _conv3x3_v3(xn, weight, k_in, k_out, out, tile, dgrad):
    wins, _ = _v3_windows(k_in)
    wf = _v3_weight(weight, dgrad)
    conv_fused([(xn, o, c) for o, c in wins], wf, None, 3, 3, k_out, EPI_BIAS, out, 0, tile=tile, wf=wf)


def _conv3x3_into(xn, wp, cin, cout, out, P):
    if _halo_ok(cin, cout):
        torch.ops.raft_stir.conv3x3_halo(xn, wp, out, cin, cout)
    else:
        conv_fused([(xn, 0, cin)], wp, None, 3, 3, cout, EPI_BIAS, out, 0, tile=choose_enc_tile(P, cin, cout))


def _wgrad_covers(cin: int, cout: int) -> bool:
    """csrc/conv_wgrad.hip handles this conv's weight gradient: input
    channels in 64-wide segments (a multiple of 32 >= 64 via overlapping
    segments); the buffer-DMA kernel range-checks the dY rows of a partial
    128-channel M tile, the register-staged one needs whole tiles."""
    if cin % 32 or cin < 64 or cout % 32:
        return False
    if _WGRAD_DMA:
        return True
    return cin % 64 == 0 and cout % 64 == 0 and (cout <= 64 or cout % 128 == 0)


def eligible(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    if not _ENABLED or x.dtype != torch.bfloat16 or x.dim() != 4 or not _ext.use_hip(x):
        return False
    if conv.kernel_size != (3, 3) or conv.stride != (1, 1) or conv.padding != (1, 1):
        return False
    if conv.dilation != (1, 1) or conv.groups != 1 or conv.padding_mode != "zeros":
        return False
    cin, cout = conv.in_channels, conv.out_channels
    if cin % 32 or cout % 32 or not x.is_contiguous(memory_format=_CL):
        return False
    return x.numel() * 2 < (1 << 31)


def _nhwc(t: torch.Tensor) -> torch.Tensor:
    t = t.contiguous(memory_format=_CL)
    return t.permute(0, 2, 3, 1)


# Packed bf16 weights: every layout is a static index map into the source
# parameters, all repacked together in three kernels after each optimizer
# step (ops/wpack.py).
_F32 = torch.float32


def _packed(weight: torch.Tensor, dgrad: bool) -> torch.Tensor:
    cout, cin = weight.shape[:2]
    if dgrad:
        return wpack.packed(("s1_dgrad", id(weight)), [weight], lambda ws: pack_weight(
            ws[0].transpose(0, 1).flip(2, 3), [(cout, [(0, cout, 0)])], pad_to(cin, 128), _F32))
    return _fwd_weight(weight)


# ----------------------------------------------------------- deferred wgrads
# During a training forward RAFT.forward hands the encoder conv weights to the
# convs as VIEWS produced by a DeferGrads node created before the encoders
# (models/fused_train.py).  A conv fed such a view launches its weight
# gradient on the deferred-gradient stream and returns at once, so the
# encoder's dgrad chain (the critical path of the backward) does not wait for
# the weight-gradient GEMMs; DeferGrads.backward, which autograd runs last,
# joins that stream before the gradients reach AccumulateGrad / DDP.
_DEFER = {"stream": None, "views": {}}


class defer_weights:
    """Route ``views`` ({id(param): view}) into the encoder convs, with their
    weight gradients on ``stream``."""

    def __init__(self, stream, views):
        self.stream, self.views = stream, views

    def __enter__(self):
        self.prev = (_DEFER["stream"], _DEFER["views"])
        _DEFER["stream"], _DEFER["views"] = self.stream, self.views

    def __exit__(self, *exc):
        _DEFER["stream"], _DEFER["views"] = self.prev


class _Hold:
    """A parameter passed to an autograd Function without an autograd edge
    (its packed layouts are keyed on the parameter, not on the view)."""
    __slots__ = ("p",)

    def __init__(self, p):
        self.p = p


def _weight_in(param):
    """(autograd input for the weight, deferred-gradient stream or None)."""
    v = _DEFER["views"].get(id(param))
    return (param, None) if v is None else (v, _DEFER["stream"])


def _wgrad_on(stream, fn, inputs):
    """Run ``fn()`` (-> tuple of gradients) on ``stream`` when deferred."""
    if stream is None:
        return fn()
    cur = torch.cuda.current_stream(inputs[0].device)
    stream.wait_stream(cur)
    for t in inputs:
        t.record_stream(stream)
    with torch.cuda.stream(stream):
        out = fn()
    for g in out:
        if g is not None:
            g.record_stream(cur)
    return out


class GradSink:
    """Hands a residual block's skip-path gradient (produced by the second
    normalisation's backward, ops/norm.py _NormAct) to the block's first conv,
    whose input-gradient kernel adds it in its epilogue (conv3x3_halo
    accumulate): no separate add over the block input's gradient.  ``armed``
    is set by a first conv that will consume it; unarmed, the norm returns
    the skip gradient to autograd as usual."""
    __slots__ = ("armed", "dres")

    def __init__(self):
        self.armed = False
        self.dres = None


class _Conv3x3(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, hold, wstream, sink=None):
        weight = hold.p
        ctx.param, ctx.wstream = weight, wstream
        xn = _nhwc(x)
        N, H, W, cin = xn.shape
        cout = weight.shape[0]
        P = N * H * W
        out = torch.empty(N, H, W, cout, device=x.device, dtype=torch.bfloat16)
        t = _v3_tile(P, cin, cout)
        if t is not None:
            _conv3x3_v3(xn, weight, cin, cout, out, t, False)
        else:
            _conv3x3_into(xn, _packed(weight, False), cin, cout, out, P)
        ctx.save_for_backward(x)
        # the skip gradient is added in the halo kernel's dgrad epilogue only
        # (an out += v kind in the v2 / v3 tiles' shared epilogue slowed every
        # conv on them by 1-7%: profiles/r5/infer_kernel_stats_s21_*.csv)
        ctx.sink = sink if sink is not None and _halo_ok(cout, cin) and _v3_tile(P, cout, cin) is None else None
        if ctx.sink is not None:
            ctx.sink.armed = True
        return out.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        x, = ctx.saved_tensors
        weight = ctx.param
        xn = _nhwc(x)
        N, H, W, cin = xn.shape
        cout = weight.shape[0]
        P = N * H * W
        dyn = _nhwc(dy.to(torch.bfloat16))
        dx = dw = None
        if ctx.needs_input_grad[0]:
            sink = ctx.sink
            td = _v3_tile(P, cout, cin)
            if sink is not None and sink.dres is not None:
                # dX = skip gradient + dgrad, accumulated in the halo kernel's epilogue
                dxn, sink.dres = sink.dres, None
                torch.ops.raft_stir.conv3x3_halo(dyn, _packed(weight, True), dxn, cout, cin, accumulate=True)
            else:
                dxn = torch.empty(N, H, W, cin, device=x.device, dtype=torch.bfloat16)
                if td is not None:
                    _conv3x3_v3(dyn, weight, cout, cin, dxn, td, True)
                else:
                    _conv3x3_into(dyn, _packed(weight, True), cout, cin, dxn, P)
            dx = dxn.permute(0, 3, 1, 2)
        if ctx.needs_input_grad[1]:
            dw, = _wgrad_on(ctx.wstream, lambda: (_wgrad3x3(dyn, x, xn, weight, cin, cout, P),), [dyn, x])
        return dx, dw, None, None, None


# csrc/enc_wgrad.hip: all nine taps of a 64 x 64 channel slice per block over
# halo tiles (deterministic); every encoder 3x3 stride-1 conv (64 / 96 / 128
# channels; 96 as two overlapping 64-channel blocks)
_ENC_WGRAD = True


def _enc_wgrad_op(dy, x):
    return torch.ops.raft_stir.enc_wgrad(dy, x)


def _wgrad3x3(dyn, x, xn, weight, cin, cout, P):
    if _ENC_WGRAD and cin % 32 == 0 and cout % 32 == 0 and min(cin, cout) >= 64:
        return _enc_wgrad_op(dyn, xn).to(weight.dtype)
    if _wgrad_covers(cin, cout):
        # the kernel tiles input channels in 64-wide segments: an odd
        # multiple of 32 (96) is covered by two OVERLAPPING segments,
        # [0, cin-32) and [cin-64, cin), whose dW columns are spliced
        segs = [(0, cin)] if cin % 64 == 0 else [(0, cin - 32), (cin - 64, 64)]
        ktot = sum(c for _, c in segs)
        acc = torch.zeros(pad_to(cout, 128), 9, ktot, device=x.device, dtype=torch.float32)
        torch.ops.raft_stir.conv_wgrad(dyn, 0, cout, [xn] * len(segs), [o for o, _ in segs],
                                       [c for _, c in segs], [P] * len(segs), 3, 3, acc, None, 0)
        acc = acc[:cout]
        if len(segs) > 1:
            acc = torch.cat([acc[..., :cin - 32], acc[..., cin:cin + 32]], -1)
        return acc.view(cout, 3, 3, cin).permute(0, 3, 1, 2).to(weight.dtype)
    # channel counts the wgrad kernel does not tile: MIOpen
    return torch.ops.aten.convolution_backward(
        dyn.permute(0, 3, 1, 2), x, weight.to(torch.bfloat16), None, [1, 1], [1, 1], [1, 1], False,
        [0, 0], 1, [False, True, False])[1].to(weight.dtype)


def conv3x3(conv: nn.Conv2d, x: torch.Tensor, sink=None) -> torch.Tensor:
    """conv(x) without its bias (see :func:`eligible`); ``sink``: a
    :class:`GradSink` whose skip gradient the input gradient absorbs."""
    w, st = _weight_in(conv.weight)
    return _Conv3x3.apply(x, w, _Hold(conv.weight), st, sink)


# ------------------------------------------------------------------- 7x7 stem
# The encoders' 7x7 / stride-2 stem (3 -> 64 / 32 channels) on csrc/stem.hip:
# forward (bf16 under autocast, split-bf16 for fp32 inference) with the shared
# conv epilogues (bias, eval-BN scale / shift + ReLU) and a
# deterministic MFMA weight gradient; the image needs no input gradient.
# Every mode runs here: bf16 training (forward + weight gradient), fp32
# training (split-bf16 forward, three-product split weight gradient), bf16 /
# fp32 inference, both encoders and RAFT-small's 32-channel stem
# (scripts/bench_stem.py).
_STEM = True


def _stem_layout(ws):
    w = ws[0]
    cout = w.shape[0]
    t = w.permute(0, 2, 3, 1).reshape(cout, 7, 21)  # [co][ky][kx * 3 + ci]
    out = torch.zeros(64, 7, 32, dtype=t.dtype, device=t.device)
    out[:cout, :, :21] = t
    return out


def stem_eligible(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    if not (_ENABLED and _STEM) or not _ext.use_hip(x) or x.dim() != 4:
        return False
    if conv.kernel_size != (7, 7) or conv.stride != (2, 2) or conv.padding != (3, 3) or conv.in_channels != 3:
        return False
    if conv.dilation != (1, 1) or conv.groups != 1 or conv.padding_mode != "zeros":
        return False
    if conv.out_channels > 64 or conv.out_channels % 8 or x.requires_grad:
        return False
    if x.dtype not in (torch.float32, torch.bfloat16) or not x.is_contiguous(memory_format=_CL):
        return False
    return x.numel() * 4 < (1 << 31)


def _stem_out(conv, x):
    N, _, H, W = x.shape
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    f32 = not torch.is_autocast_enabled("cuda") and x.dtype == torch.float32
    out = torch.empty(N, Ho, Wo, conv.out_channels, device=x.device,
                      dtype=torch.float32 if f32 else torch.bfloat16)
    w = (wpack.packed_split if f32 else wpack.packed)(("stem", id(conv.weight)), [conv.weight], _stem_layout)
    return out, w


class _Stem(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, hold, wstream):
        conv = hold.p
        out, wp = _stem_out(conv, x)
        torch.ops.raft_stir.stem_conv(_nhwc(x), wp, None, out, conv.out_channels, 0)
        ctx.save_for_backward(x)
        ctx.param, ctx.wstream = conv.weight, wstream
        return out.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        x, = ctx.saved_tensors
        weight = ctx.param
        dw = None
        if ctx.needs_input_grad[1]:
            if x.dtype == torch.float32 and dy.dtype == torch.float32:
                # fp32 training: split-bf16 operands, dW = dYh.Xh + dYh.Xl + dYl.Xh
                xh, xl = _split(_nhwc(x))
                dh, dl = _split(_nhwc(dy.contiguous(memory_format=_CL)))

                def wgrad():
                    g = torch.empty(weight.shape, device=dy.device, dtype=torch.float32)
                    t = torch.empty_like(g)
                    torch.ops.raft_stir.stem_wgrad(xh, dh, weight.shape[0], g)
                    torch.ops.raft_stir.stem_wgrad(xl, dh, weight.shape[0], t)
                    g += t
                    torch.ops.raft_stir.stem_wgrad(xh, dl, weight.shape[0], t)
                    g += t
                    return (g.to(weight.dtype),)
                dw, = _wgrad_on(ctx.wstream, wgrad, [dh, dl, xh, xl])
            else:
                dyn = _nhwc(dy.to(torch.bfloat16))

                def wgrad():
                    g = torch.empty(weight.shape, device=dy.device, dtype=torch.float32)
                    torch.ops.raft_stir.stem_wgrad(_nhwc(x), dyn, weight.shape[0], g)
                    return (g.to(weight.dtype),)
                dw, = _wgrad_on(ctx.wstream, wgrad, [dyn, x])
        return None, dw, None, None


def stem(conv: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    """conv(x) without its bias (:func:`stem_eligible`)."""
    w, st = _weight_in(conv.weight)
    return _Stem.apply(x, w, _Hold(conv), st)


@torch.no_grad()
def stem_norm(conv: nn.Conv2d, x: torch.Tensor, scale, shift, relu: bool) -> torch.Tensor:
    """Inference: ``[relu](conv_nobias(x) * scale + shift)`` (eval BatchNorm in the epilogue)."""
    out, wp = _stem_out(conv, x)
    torch.ops.raft_stir.stem_conv(_nhwc(x), wp, shift, out, conv.out_channels, EPI_NORM, scale, bool(relu))
    return out.permute(0, 3, 1, 2)


# ------------------------------------------------------------- fp32 inference
# fp32 (the reference's default inference precision) on the split-bf16 F32
# tiles of csrc/conv.hip: every stride-1 / stride-2 3x3 and 1x1 encoder conv,
# no autograd (fp32 training keeps the module graph).  Weights in the split
# [wh | wl] layout through the same packed-weight registry (wpack.packed_split).
_F32_ENC = True


def _split_weight(weight: torch.Tensor) -> torch.Tensor:
    cout, cin = weight.shape[:2]
    return wpack.packed_split(("fwd", id(weight)), [weight], lambda ws: pack_weight(
        ws[0], [(cin, [(0, cin, 0)])], pad_to(cout, 128), _F32))


# stride-1 3x3 fp32 convs (forward and input gradient) on the fp32
# weight-streaming tiles (csrc/conv_v3f.hip): the split weight is tagged with
# its [frag(wh); frag(wl)] copy, recomputed at every call from the registry's
# current split weight (a few small permute kernels; the registry refreshes
# the split weight in place, so a cached copy could go stale)
_V3F_ENC = True


def _tag_frag32(ws: torch.Tensor, cin: int, cout: int) -> torch.Tensor:
    # whole output blocks only: 128-output convs on tiles 81-83, 64-output ones
    # on tile 84 (on the 128-row tiles half the block was wasted: 276 us per
    # call vs 373 on the register tile 6, gpurun_out/r6s27)
    if _V3F_ENC and cin % 64 == 0 and cout % 64 == 0 and frag32_eligible(ws, 3, 3):
        ws._rs_frag32 = frag_weight_split(ws)
    return ws


def eligible_f32(conv: nn.Conv2d, x: torch.Tensor, residual=None) -> bool:
    """fp32 inference conv on the F32 tiles: 3x3 (stride 1 / 2, pad 1) or 1x1
    (stride 1 / 2), channel counts multiples of 32, nothing to differentiate."""
    if not (_ENABLED and _F32_ENC) or x.dtype != torch.float32 or x.dim() != 4 or not _ext.use_hip(x):
        return False
    if torch.is_autocast_enabled("cuda"):
        return False
    if torch.is_grad_enabled() and (x.requires_grad or conv.weight.requires_grad
                                    or (conv.bias is not None and conv.bias.requires_grad)
                                    or (residual is not None and residual.requires_grad)):
        return False
    k, s, p = conv.kernel_size, conv.stride, conv.padding
    if conv.dilation != (1, 1) or conv.groups != 1 or conv.padding_mode != "zeros" or isinstance(p, str):
        return False
    if not ((k == (3, 3) and p == (1, 1) and s in ((1, 1), (2, 2))) or (k == (1, 1) and p == (0, 0) and s in ((1, 1), (2, 2)))):
        return False
    if conv.in_channels % 32 or conv.out_channels % 4 or not x.is_contiguous(memory_format=_CL):
        return False
    if residual is not None and (k != (3, 3) or s != (1, 1)):
        return False
    return x.numel() * 4 < (1 << 31)


@torch.no_grad()
def conv_f32(conv: nn.Conv2d, x: torch.Tensor, bias: bool = True, scale=None, shift=None,
             relu: bool = False, residual=None) -> torch.Tensor:
    """fp32 ``conv(x)`` (:func:`eligible_f32`) with the optional eval-BN
    ``scale`` / ``shift`` epilogue (+ ReLU, + residual; the conv bias must
    already be folded into shift)."""
    xn = _nhwc(x)
    N, H, W, cin = xn.shape
    cout = conv.out_channels
    kh, kw = conv.kernel_size
    pad, stride = conv.padding, conv.stride
    wp = _split_weight(conv.weight)
    norm = scale is not None
    b = shift if norm else (conv.bias.detach().float().contiguous() if (bias and conv.bias is not None) else None)
    if stride == (1, 1) and (kh, kw) == (3, 3):
        out = torch.empty(N, H, W, cout, device=x.device, dtype=torch.float32)
        rn = _nhwc(residual) if residual is not None else None
        wp = _tag_frag32(wp, cin, cout)
        conv_fused([(xn, 0, cin)], wp, b, 3, 3, cout, EPI_NORM if norm else EPI_BIAS, out, 0,
                   hd=int(bool(relu)), aux1=rn, tile=None, nscale=scale)
        return out.permute(0, 3, 1, 2)
    Ho = (H + 2 * pad[0] - kh) // stride[0] + 1
    Wo = (W + 2 * pad[1] - kw) // stride[1] + 1
    out = torch.empty(N, Ho, Wo, cout, device=x.device, dtype=torch.float32)
    torch.ops.raft_stir.conv_geo([xn], [0], [cin], wp, b, kh, kw, pad[0], pad[1], stride[0], stride[1], Ho, Wo,
                                 cout, out, 0, 1, 1, 0, 0, choose_tile_f32(N * Ho * Wo, cout, geo=True), scale,
                                 bool(relu))
    return out.permute(0, 3, 1, 2)


# -------------------------------------------------------------- fp32 training
# fp32 encoder convs in TRAINING (the reference's default precision,
# /root/reference/train_standard.sh) on the same split-bf16 F32 tiles:
#   forward : conv_f32 (above);
#   dgrad   : stride 1 -- the conv of dY with the flipped, transposed weight;
#             stride 2 / 1x1 -- the phase-split dgrad of conv_geo -- both on
#             the F32 tiles with split-packed weights, fp32 in and out;
#   wgrad   : three bf16 MFMA GEMMs over split operands, dYh.Xh + dYl.Xh +
#             dYh.Xl (csrc/split.hip, then enc_wgrad / conv_wgrad_strided):
#             ~2^-16 relative, the same scheme as the fused update block;
#   bias    : column sum of dY in fp32 (the projection head only; the other
#             convs' biases fold into their normalisation).
_F32_TRAIN = True


def _f32_shape_ok(conv: nn.Conv2d) -> bool:
    k, s, p = conv.kernel_size, conv.stride, conv.padding
    if conv.dilation != (1, 1) or conv.groups != 1 or conv.padding_mode != "zeros" or isinstance(p, str):
        return False
    return (k == (3, 3) and p == (1, 1) and s in ((1, 1), (2, 2))) or (k == (1, 1) and p == (0, 0) and s in ((1, 1), (2, 2)))


def eligible_f32_train(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    """fp32 training conv on the F32 tiles (see above): the eligible_f32
    shapes, input and output channels multiples of 32 (>= 64 for the weight
    gradient kernels), something to differentiate."""
    if not (_ENABLED and _F32_ENC and _F32_TRAIN and _GEO_SCOPE[0]) or x.dtype != torch.float32 or x.dim() != 4:
        return False
    if not _ext.use_hip(x) or torch.is_autocast_enabled("cuda") or not torch.is_grad_enabled():
        return False
    if not (x.requires_grad or conv.weight.requires_grad or (conv.bias is not None and conv.bias.requires_grad)):
        return False
    if conv.weight.dtype != torch.float32 or not _f32_shape_ok(conv):
        return False
    cin, cout = conv.in_channels, conv.out_channels
    if cin % 32 or cout % 32 or min(cin, cout) < 64 or not x.is_contiguous(memory_format=_CL):
        return False
    return x.numel() * 4 < (1 << 31)


def _split(t: torch.Tensor):
    """(hi, lo) bf16 of a contiguous fp32 tensor (csrc/split.hip)."""
    t = t.contiguous()
    if t.data_ptr() % 16 == 0:
        hi, lo = torch.ops.raft_stir.split_bf16(t)
        return hi, lo
    hi = t.to(torch.bfloat16)
    return hi, (t - hi.float()).to(torch.bfloat16)


def _split_dgrad_weight(weight: torch.Tensor) -> torch.Tensor:
    cout, cin = weight.shape[:2]
    return wpack.packed_split(("s1_dgrad", id(weight)), [weight], lambda ws: pack_weight(
        ws[0].transpose(0, 1).flip(2, 3), [(cout, [(0, cout, 0)])], pad_to(cin, 128), _F32))


def _f32_wgrad(conv: nn.Conv2d, dyn, x, want_w: bool, want_b: bool):
    weight = conv.weight
    dw = db = None
    if want_w:
        dyh, dyl = _split(dyn)
        xh, xl = _split(_nhwc(x))
        cin, cout = conv.in_channels, conv.out_channels
        if conv.kernel_size == (3, 3) and conv.stride == (1, 1):
            P = xh.shape[0] * xh.shape[1] * xh.shape[2]
            f = lambda d, xx: _wgrad3x3(d, xx.permute(0, 3, 1, 2), xx, weight, cin, cout, P)
        else:
            f = lambda d, xx: _conv_geo_wgrad(d, xx.permute(0, 3, 1, 2), weight, tuple(conv.stride), False)[0]
        dw = f(dyh, xh) + f(dyl, xh) + f(dyh, xl)
    if want_b:
        db = dyn.sum((0, 1, 2)).to(conv.bias.dtype)
    return dw, db


class _ConvF32(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, hold, wstream):
        conv = hold.p
        out = conv_f32(conv, x, bias=bias is not None)
        ctx.save_for_backward(x)
        ctx.conv, ctx.wstream, ctx.has_bias = conv, wstream, bias is not None
        return out

    @staticmethod
    def backward(ctx, dy):
        x, = ctx.saved_tensors
        conv = ctx.conv
        dyn = _nhwc(dy.float().contiguous(memory_format=_CL))
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            if conv.kernel_size == (3, 3) and conv.stride == (1, 1):
                N, H, W, cout = dyn.shape
                dxn = torch.empty(N, H, W, conv.in_channels, device=dy.device, dtype=torch.float32)
                wd = _tag_frag32(_split_dgrad_weight(conv.weight), cout, conv.in_channels)
                conv_fused([(dyn, 0, cout)], wd, None, 3, 3, conv.in_channels, EPI_BIAS, dxn, 0, tile=None)
                dx = dxn.permute(0, 3, 1, 2)
            else:
                dx = _conv_geo_dgrad([dyn], [conv.weight], x.shape, tuple(conv.stride), tuple(conv.padding),
                                     f32=True).permute(0, 3, 1, 2)
        want_w = ctx.needs_input_grad[1]
        want_b = ctx.has_bias and ctx.needs_input_grad[2]
        if want_w or want_b:
            dw, db = _wgrad_on(ctx.wstream, lambda: _f32_wgrad(conv, dyn, x, want_w, want_b), [dyn, x])
        return dx, dw, db, None, None


def conv_f32_train(conv: nn.Conv2d, x: torch.Tensor, bias: bool = True) -> torch.Tensor:
    """fp32 training ``conv(x)`` (:func:`eligible_f32_train`); ``bias=False``
    drops the conv bias (folded into the following normalisation)."""
    w, st = _weight_in(conv.weight)
    b = conv.bias if (bias and conv.bias is not None) else None
    if b is not None and st is not None:
        b = _DEFER["views"].get(id(conv.bias), b)
    return _ConvF32.apply(x, w, b, _Hold(conv), st)


def conv_norm(conv: nn.Conv2d, x: torch.Tensor, scale, shift, relu: bool, residual=None) -> torch.Tensor:
    """Inference (no autograd): ``[relu](conv_nobias(x) * scale + shift)``, then
    ``relu(. + residual)`` -- an eval-mode BatchNorm (scale / shift per output
    channel, the conv bias folded into shift: ops/norm.py) and the block's
    activations in the conv epilogue.  Stride-1 3x3 convs (:func:`eligible`) and
    strided / 1x1 ones (:func:`eligible_geo`, no residual); fp32 inputs on the
    F32 tiles (:func:`eligible_f32`)."""
    if x.dtype == torch.float32:
        return conv_f32(conv, x, scale=scale, shift=shift, relu=relu, residual=residual)
    xn = _nhwc(x)
    N, H, W, cin = xn.shape
    cout = conv.out_channels
    rn = _nhwc(residual) if residual is not None else None
    if conv.stride == (1, 1) and conv.kernel_size == (3, 3):
        wp = _packed(conv.weight, False)
        out = torch.empty(N, H, W, cout, device=x.device, dtype=torch.bfloat16)
        if _halo_ok(cin, cout):
            torch.ops.raft_stir.conv3x3_halo(xn, wp, out, cin, cout, scale, shift, rn, bool(relu))
        else:
            conv_fused([(xn, 0, cin)], wp, shift, 3, 3, cout, EPI_NORM, out, 0, hd=int(bool(relu)), aux1=rn,
                       tile=choose_enc_tile(N * H * W, cin, cout), nscale=scale)
        return out.permute(0, 3, 1, 2)
    assert residual is None, "conv_norm: the strided / 1x1 convs have no residual input"
    kh, kw = conv.kernel_size
    pad, stride = conv.padding, conv.stride
    Ho = (H + 2 * pad[0] - kh) // stride[0] + 1
    Wo = (W + 2 * pad[1] - kw) // stride[1] + 1
    out = torch.empty(N, Ho, Wo, cout, device=x.device, dtype=torch.bfloat16)
    torch.ops.raft_stir.conv_geo([xn], [0], [cin], _fwd_weight(conv.weight), shift, kh, kw, pad[0], pad[1],
                                 stride[0], stride[1], Ho, Wo, cout, out, 0, 1, 1, 0, 0, _geo_tile(cout, [cin]),
                                 scale, bool(relu))
    return out.permute(0, 3, 1, 2)


# ----------------------------------------------------------------- strided / 1x1
# The rest of the encoder convolutions (reference core/extractor.py:10, 44, 65,
# 103, 144): the stride-2 3x3 first conv of stages 2 and 3, the stride-2 1x1
# downsample shortcut beside it, and the 1x1 projection head.  All on
# csrc/conv.hip's register-staged implicit GEMM in its strided geometry
# (torch.ops.raft_stir.conv_geo) and csrc/conv_wgrad.hip's strided weight
# gradient (conv_wgrad_strided):
#
#   forward : GEMM pixel (y, x) reads input (y*S + ky - P, x*S + kx - P)
#   dgrad   : split by the PARITY of the input pixel (phase r = i mod S): only
#             taps k = (r + P) mod S contribute, each from dY at offset
#             d = (r + P - k) / S, so every phase is a dense stride-1 conv of
#             dY with a 1x1 / 1x2 / 2x1 / 2x2 sub-kernel whose outputs land on
#             every S-th input pixel (no zero-tap MACs, no col2im, no atomics);
#             the 1x1 shortcut only has the (0, 0) phase and is fused into the
#             3x3's (0, 0) phase as a second K segment (conv_pair)
#   wgrad   : split-K MFMA over dY pixels with strided X rows
_GEO = True
_GEO_SCOPE = [True]  # per-encoder switch (geo_scope): off for RAFT-small's encoder (its narrow convs run on sconv)
# ... except its convs with >= _WIDE_GEO input AND output channels (the 1x1
# projection 96 -> 128 / 160 and layer 3's 64 -> 96 stride-2 shortcut): the
# VALU weight gradient of the projection took 249 / 387 us per call
# (profiles/r6/README.md); RS_WIDE_GEO=0 keeps every RAFT-small conv on sconv
_WIDE_GEO = int(os.environ.get("RS_WIDE_GEO", "64"))


def _wide(conv: nn.Conv2d) -> bool:
    return _WIDE_GEO > 0 and conv.in_channels >= _WIDE_GEO and conv.out_channels >= _WIDE_GEO


class geo_scope:
    """Enable / disable the strided-geometry path inside a block (set by the
    encoder: RAFT-small's narrow 32-96-channel bottleneck convs run on the
    csrc/sconv.hip / sconv_train.hip kernels instead -- the geometry tiles
    measured 602 vs 657 pairs/s there -- while full RAFT uses them)."""

    def __init__(self, on: bool):
        self.on = on

    def __enter__(self):
        self.prev = _GEO_SCOPE[0]
        _GEO_SCOPE[0] = self.on

    def __exit__(self, *exc):
        _GEO_SCOPE[0] = self.prev


def _geo_ok(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    if not (_ENABLED and _GEO and (_GEO_SCOPE[0] or _wide(conv))) or x.dtype != torch.bfloat16 or x.dim() != 4 \
            or not _ext.use_hip(x):
        return False
    k, s, p = conv.kernel_size, conv.stride, conv.padding
    if conv.dilation != (1, 1) or conv.groups != 1 or conv.padding_mode != "zeros" or isinstance(p, str):
        return False
    shape_ok = (k == (3, 3) and s == (2, 2) and p == (1, 1)) or (k == (1, 1) and p == (0, 0) and s in ((1, 1), (2, 2)))
    cin, cout = conv.in_channels, conv.out_channels
    return (shape_ok and cin % 32 == 0 and cin >= 64 and cout % 32 == 0 and x.is_contiguous(memory_format=_CL)
            and x.numel() * 2 < (1 << 31))


def eligible_geo(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    """Strided 3x3 / strided or plain 1x1 encoder conv on the HIP kernels."""
    return _geo_ok(conv, x)


def _phase_taps(k: int, s: int, p: int, r: int):
    """Taps k' (ascending dY offset d) feeding input phase r: [(d, k'), ...]."""
    return sorted(((r + p - kk) // s, kk) for kk in range(k) if (r + p - kk) % s == 0)


def _fwd_weight(weight):
    cout, cin = weight.shape[:2]
    return wpack.packed(("fwd", id(weight)), [weight],
                        lambda ws: pack_weight(ws[0], [(cin, [(0, cin, 0)])], pad_to(cout, 128), _F32))


def _phase_weight(weights, ry, rx, strides, pads, f32=False):
    """Packed dgrad weight of phase (ry, rx) of one strided conv:
    [pad128(Cin)][kh' * kw'][Cout] (``f32``: the split [wh | wl] form)."""
    assert len(weights) == 1, "several convs share a phase weight through _pair_phase_weight"
    w0 = weights[0]
    cout, cin, kh, kw = w0.shape
    ty = _phase_taps(kh, strides[0], pads[0], ry)
    tx = _phase_taps(kw, strides[1], pads[1], rx)

    def layout(ws):
        sub = ws[0][:, :, [k for _, k in ty]][:, :, :, [k for _, k in tx]]  # [cout, cin, kh', kw']
        return pack_weight(sub.transpose(0, 1), [(cout, [(0, cout, 0)])], pad_to(cin, 128), _F32)
    pk = wpack.packed_split if f32 else wpack.packed
    return pk(("phase", id(w0), ry, rx, tuple(strides), tuple(pads)), [w0], layout)


def _geo_tile(cout: int, chans) -> int:
    k64 = all(c % 64 == 0 for c in chans)
    if cout > 64:
        return 7 if k64 else 4
    return 6 if k64 else 3


def _conv_geo_fwd(x, weight, bias, stride, pad):
    xn = _nhwc(x)
    N, Hi, Wi, cin = xn.shape
    cout, _, kh, kw = weight.shape
    Ho = (Hi + 2 * pad[0] - kh) // stride[0] + 1
    Wo = (Wi + 2 * pad[1] - kw) // stride[1] + 1
    out = torch.empty(N, Ho, Wo, cout, device=x.device, dtype=torch.bfloat16)
    b = None if bias is None else bias.detach().float().contiguous()
    torch.ops.raft_stir.conv_geo([xn], [0], [cin], _fwd_weight(weight), b, kh, kw, pad[0], pad[1], stride[0],
                                 stride[1], Ho, Wo, cout, out, 0, 1, 1, 0, 0, _geo_tile(cout, [cin]))
    return out


def _conv_geo_dgrad(dys, weights, x_shape, stride, pad, f32=False):
    """dX (NHWC bf16; ``f32``: fp32 on the split-bf16 F32 tiles) of convs
    sharing the input: sum over ``weights`` of their input gradients from
    ``dys`` (NHWC output gradients of the same dtype)."""
    N, cin, Hi, Wi = x_shape
    kh, kw = weights[0].shape[2:]
    Ho, Wo = dys[0].shape[1:3]
    sy, sx = stride
    phases = []
    for ry in range(sy):
        for rx in range(sx):
            use = [i for i, w in enumerate(weights)
                   if _phase_taps(w.shape[2], sy, pad[0], ry) and _phase_taps(w.shape[3], sx, pad[1], rx)]
            phases.append((ry, rx, use))
    full = all(len(u) > 0 for _, _, u in phases)
    dx = (torch.empty if full else torch.zeros)(N, Hi, Wi, cin, device=dys[0].device,
                                                dtype=torch.float32 if f32 else torch.bfloat16)
    for ry, rx, use in phases:
        if not use:
            continue
        mh, mw = -(-(Hi - ry) // sy), -(-(Wi - rx) // sx)
        if mh <= 0 or mw <= 0:
            continue
        ws = [weights[i] for i in use]
        ty = _phase_taps(ws[0].shape[2], sy, pad[0], ry)
        tx = _phase_taps(ws[0].shape[3], sx, pad[1], rx)
        for w in ws[1:]:  # fused K segments must share the sub-kernel
            assert _phase_taps(w.shape[2], sy, pad[0], ry) == ty and _phase_taps(w.shape[3], sx, pad[1], rx) == tx
        wp = _phase_weight(ws, ry, rx, stride, pad, f32)
        chans = [weights[i].shape[0] for i in use]
        tile = choose_tile_f32(N * mh * mw, cin, geo=True) if f32 else _geo_tile(cin, chans)
        torch.ops.raft_stir.conv_geo([dys[i] for i in use], [0] * len(use), chans, wp, None, len(ty), len(tx),
                                     -ty[0][0], -tx[0][0], 1, 1, mh, mw, cin, dx, 0, sy, sx, ry, rx, tile)
    return dx


def _conv_geo_wgrad(dy, x, weight, stride, want_bias):
    """(dW, db) of a strided / 1x1 conv: split-K MFMA over dY pixels."""
    xn = _nhwc(x)
    cin = xn.shape[3]
    cout, _, kh, kw = weight.shape
    segs = [(0, cin)] if cin % 64 == 0 else [(0, cin - 32), (cin - 64, 64)]
    ktot = sum(c for _, c in segs)
    acc = torch.zeros(pad_to(cout, 128), kh * kw, ktot, device=x.device, dtype=torch.float32)
    db = torch.zeros(cout, device=x.device, dtype=torch.float32) if want_bias else None
    torch.ops.raft_stir.conv_wgrad_strided(dy, cout, [xn] * len(segs), [o for o, _ in segs], [c for _, c in segs],
                                           kh, kw, stride[0], stride[1], acc, db)
    acc = acc[:cout]
    if len(segs) > 1:
        acc = torch.cat([acc[..., :cin - 32], acc[..., cin:cin + 32]], -1)
    dw = acc.view(cout, kh, kw, cin).permute(0, 3, 1, 2).to(weight.dtype)
    return dw, (db.to(weight.dtype) if db is not None else None)


class _ConvGeo(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, stride, pad, hold, wstream):
        weight = hold.p
        out = _conv_geo_fwd(x, weight, bias, stride, pad)
        ctx.save_for_backward(x)
        ctx.param, ctx.wstream = weight, wstream
        ctx.stride, ctx.pad, ctx.has_bias = stride, pad, bias is not None
        return out.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        x, = ctx.saved_tensors
        weight = ctx.param
        dyn = _nhwc(dy.to(torch.bfloat16))
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = _conv_geo_dgrad([dyn], [weight], x.shape, ctx.stride, ctx.pad).permute(0, 3, 1, 2)
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            want_b = ctx.has_bias and ctx.needs_input_grad[2]
            dw, db = _wgrad_on(ctx.wstream, lambda: _conv_geo_wgrad(dyn, x, weight, ctx.stride, want_b), [dyn, x])
        return dx, dw, db, None, None, None, None


def conv_geo(conv: nn.Conv2d, x: torch.Tensor, bias: bool = True) -> torch.Tensor:
    """conv(x) on the HIP kernels (see :func:`eligible_geo`); ``bias=False``
    drops the conv's bias (folded into a following normalisation)."""
    b = conv.bias if bias else None
    w, st = _weight_in(conv.weight)
    if b is not None and st is not None:
        b = _DEFER["views"].get(id(conv.bias), b)
    return _ConvGeo.apply(x, w, b, tuple(conv.stride), tuple(conv.padding), _Hold(conv.weight), st)


class _ConvPair(torch.autograd.Function):
    """The stride-2 3x3 conv and the stride-2 1x1 shortcut of a residual
    block's first conv (both read the block input, no biases): one input
    gradient, with the shortcut's term fused into the 3x3's (0, 0) phase."""

    @staticmethod
    def forward(ctx, x, w1, wd, stride, holds, wstream):
        w1, wd = holds.p
        y1 = _conv_geo_fwd(x, w1, None, stride, (1, 1))
        yd = _conv_geo_fwd(x, wd, None, stride, (0, 0))
        ctx.save_for_backward(x)
        ctx.params, ctx.wstream = (w1, wd), wstream
        ctx.stride = stride
        return y1.permute(0, 3, 1, 2), yd.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy1, dyd):
        x, = ctx.saved_tensors
        w1, wd = ctx.params
        s = ctx.stride
        d1 = _nhwc(dy1.to(torch.bfloat16))
        dd = _nhwc(dyd.to(torch.bfloat16))
        dx = dw1 = dwd = None
        if ctx.needs_input_grad[0]:
            dx = _pair_dgrad(d1, dd, w1, wd, x.shape, s).permute(0, 3, 1, 2)
        n1, n2 = ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        if n1 or n2:
            dw1, dwd = _wgrad_on(ctx.wstream, lambda: (_conv_geo_wgrad(d1, x, w1, s, False)[0] if n1 else None,
                                                       _conv_geo_wgrad(dd, x, wd, s, False)[0] if n2 else None),
                                 [d1, dd, x])
        return dx, dw1, dwd, None, None, None


def _pair_dgrad(d1, dd, w1, wd, x_shape, stride):
    N, cin, Hi, Wi = x_shape
    dx = torch.empty(N, Hi, Wi, cin, device=d1.device, dtype=torch.bfloat16)
    sy, sx = stride
    for ry in range(sy):
        for rx in range(sx):
            mh, mw = -(-(Hi - ry) // sy), -(-(Wi - rx) // sx)
            ty = _phase_taps(3, sy, 1, ry)
            tx = _phase_taps(3, sx, 1, rx)
            shortcut = bool(_phase_taps(1, sy, 0, ry) and _phase_taps(1, sx, 0, rx))
            if shortcut:  # (0, 0): the centre tap of the 3x3 and the 1x1, as two K segments
                assert len(ty) == 1 and len(tx) == 1 and ty[0][0] == 0 and tx[0][0] == 0
                ws, dys = [w1, wd], [d1, dd]
            else:
                ws, dys = [w1], [d1]
            wp = _pair_phase_weight(ws, ry, rx, stride)
            chans = [w.shape[0] for w in ws]
            torch.ops.raft_stir.conv_geo(dys, [0] * len(ws), chans, wp, None, len(ty), len(tx), -ty[0][0],
                                         -tx[0][0], 1, 1, mh, mw, cin, dx, 0, sy, sx, ry, rx, _geo_tile(cin, chans))
    return dx


def _pair_phase_weight(ws, ry, rx, stride):
    """Phase (ry, rx) dgrad weight of the 3x3/s2 conv, with the 1x1/s2
    shortcut appended as a second K segment on the (0, 0) phase."""
    cout, cin = ws[0].shape[:2]
    ty = _phase_taps(3, stride[0], 1, ry)
    tx = _phase_taps(3, stride[1], 1, rx)

    def layout(ts):
        blocks = [ts[0][:, :, [k for _, k in ty]][:, :, :, [k for _, k in tx]].transpose(0, 1)]
        if len(ts) > 1:  # the 1x1 shortcut: the same 1x1 sub-kernel (centre tap)
            blocks.append(ts[1].transpose(0, 1))
        segs, o = [], 0
        for t in ts:
            segs.append((t.shape[0], [(o, t.shape[0], 0)]))
            o += t.shape[0]
        return pack_weight(torch.cat(blocks, 1), segs, pad_to(cin, 128), _F32)
    return wpack.packed(("pair", id(ws[0]), ry, rx, len(ws)), list(ws), layout)


def pair_eligible(conv1: nn.Conv2d, down: nn.Conv2d, x: torch.Tensor) -> bool:
    return (_geo_ok(conv1, x) and _geo_ok(down, x) and conv1.kernel_size == (3, 3) and conv1.stride == (2, 2)
            and down.kernel_size == (1, 1) and down.stride == (2, 2) and down.out_channels == conv1.out_channels)


def conv_pair(conv1: nn.Conv2d, down: nn.Conv2d, x: torch.Tensor):
    """(conv1(x), down(x)) without biases (both folded into their norms)."""
    w1, st = _weight_in(conv1.weight)
    wd, _ = _weight_in(down.weight)
    return _ConvPair.apply(x, w1, wd, tuple(conv1.stride), _Hold((conv1.weight, down.weight)), st)


# ------------------------------------------------------- narrow-channel convs
# RAFT-small's encoders (reference core/extractor.py:60-116, :195-267) run
# 1x1 / 3x3 convs of 8-96 channels; at inference they go to csrc/sconv.hip
# (VALU, fp32 accumulation, bias / ReLU / residual in the epilogue, bf16 or
# fp32 NHWC) instead of MIOpen + a bias kernel + an autocast weight cast.
_SCONV = True


def sconv_eligible(conv: nn.Conv2d, x: torch.Tensor, residual=None) -> bool:
    """Inside RAFT-small's encoder only (the scope where geo_scope(False) keeps
    the MFMA strided paths off): full RAFT's 64-128-channel convs stay on the
    MFMA kernels (and so do RAFT-small's wide convs, :func:`_wide`)."""
    if not (_ENABLED and _SCONV) or _GEO_SCOPE[0] or x.dim() != 4 or not _ext.use_hip(x) or _geo_ok(conv, x):
        return False
    if x.dtype not in (torch.bfloat16, torch.float32) or not x.is_contiguous(memory_format=_CL):
        return False
    if x.dtype == torch.float32 and torch.is_autocast_enabled("cuda"):
        return False  # autocast would have run this conv in bf16
    if torch.is_grad_enabled() and (x.requires_grad or conv.weight.requires_grad
                                    or (conv.bias is not None and conv.bias.requires_grad)
                                    or (residual is not None and residual.requires_grad)):
        return False  # inference only (no backward kernels)
    k, s, p = conv.kernel_size, conv.stride, conv.padding
    if k not in ((1, 1), (3, 3)) or isinstance(p, str) or p != (k[0] // 2, k[1] // 2):
        return False
    if s not in ((1, 1), (2, 2)) or conv.dilation != (1, 1) or conv.groups != 1 or conv.padding_mode != "zeros":
        return False
    cin, cout = conv.in_channels, conv.out_channels
    if cin % 8 or cout % 8 or min(4, cout // 8) * 8 * k[0] * k[1] * cin > 16384:
        return False
    if residual is not None and (residual.dtype != x.dtype or not residual.is_contiguous(memory_format=_CL)):
        return False
    return x.numel() * x.element_size() < (1 << 31)


def _sconv_weight(conv: nn.Conv2d) -> torch.Tensor:
    """fp32 [Cout, KH, KW, Cin], cached per weight version (runtime/weights.py
    generation + the parameter's version counter)."""
    from ..runtime import weights
    w = conv.weight
    key = (weights.generation(), w.data_ptr(), w._version)
    hit = conv.__dict__.get("_rs_sconv_w")
    if hit is not None and hit[0] == key:
        return hit[1]
    with torch.no_grad():
        t = w.detach().float().permute(0, 2, 3, 1).contiguous()
        if hit is not None and hit[1].shape == t.shape:
            hit[1].copy_(t)  # in place: hipGraphs captured with the old tensor stay valid
            t = hit[1]
    conv.__dict__["_rs_sconv_w"] = (key, t)
    _SCONV_LIVE.add(conv)
    return t


_SCONV_LIVE = weakref.WeakSet()


def _refresh_sconv() -> None:
    """runtime/weights.py refresh_all: rewrite every live permuted sconv weight
    in place, so GraphedInference replays of RAFT-small's encoders see the
    current parameters (the captured graph holds the cached tensor)."""
    for conv in list(_SCONV_LIVE):
        hit = conv.__dict__.get("_rs_sconv_w")
        if hit is not None:
            conv.__dict__["_rs_sconv_w"] = (None, hit[1])
            _sconv_weight(conv)


def _register_sconv_refresher():
    from ..runtime import weights
    weights.register_refresher(_refresh_sconv)


_register_sconv_refresher()


def sconv_train_eligible(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    """Training form of the narrow-channel path, inside RAFT-small's encoder
    (geo_scope(False)): forward and input gradient on csrc/sconv.hip, weight
    gradient on csrc/sconv_train.hip.  bf16 under autocast or fp32 without it
    (the wide convs go to the MFMA geometry path, :func:`_wide`)."""
    if not (_ENABLED and _SCONV) or _GEO_SCOPE[0] or x.dim() != 4 or not _ext.use_hip(x) or _geo_ok(conv, x):
        return False
    if not torch.is_grad_enabled() or not (x.requires_grad or conv.weight.requires_grad):
        return False
    ac = torch.is_autocast_enabled("cuda")
    if not ((ac and x.dtype == torch.bfloat16) or (not ac and x.dtype == torch.float32)):
        return False
    if not x.is_contiguous(memory_format=_CL) or conv.weight.dtype != torch.float32:
        return False
    k, s, p = conv.kernel_size, conv.stride, conv.padding
    if k not in ((1, 1), (3, 3)) or isinstance(p, str) or p != (k[0] // 2, k[1] // 2):
        return False
    if s not in ((1, 1), (2, 2)) or conv.dilation != (1, 1) or conv.groups != 1 or conv.padding_mode != "zeros":
        return False
    cin, cout = conv.in_channels, conv.out_channels
    taps = k[0] * k[1]
    if cin % 8 or cout % 8 or min(4, cout // 8) * 8 * taps * cin > 16384 or min(4, cin // 8) * 8 * taps * cout > 16384:
        return False
    return x.numel() * x.element_size() < (1 << 31)


def _sconv_dgrad_weight(weight: torch.Tensor) -> torch.Tensor:
    """The input-gradient conv's weight: flipped and transposed, fp32 [Cin, KH, KW, Cout]."""
    return weight.detach().float().permute(1, 2, 3, 0).flip(1, 2).contiguous()


class _SConvTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, stride, pad, hold):
        conv = hold.p
        xn = _nhwc(x)
        N, H, W, _ = xn.shape
        kh, kw = conv.kernel_size
        Ho, Wo = (H + 2 * pad - kh) // stride + 1, (W + 2 * pad - kw) // stride + 1
        out = torch.empty(N, Ho, Wo, conv.out_channels, device=x.device, dtype=x.dtype)
        b = bias.detach().float().contiguous() if bias is not None else None
        torch.ops.raft_stir.sconv(xn, _sconv_weight(conv), b, stride, pad, False, out, 0, None)
        ctx.save_for_backward(x)
        ctx.conv, ctx.stride, ctx.pad, ctx.has_bias = conv, stride, pad, bias is not None
        return out.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        x, = ctx.saved_tensors
        conv, s, p = ctx.conv, ctx.stride, ctx.pad
        xn = _nhwc(x)
        N, H, W, cin = xn.shape
        kh, kw = conv.kernel_size
        dyn = _nhwc(dy.to(x.dtype).contiguous(memory_format=_CL))
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            src = dyn
            if s != 1:  # the transposed stride: dY on every s-th input pixel, zeros between
                src = torch.zeros(N, H, W, dyn.shape[3], device=dy.device, dtype=dyn.dtype)
                src[:, ::s, ::s] = dyn
            dxn = torch.empty(N, H, W, cin, device=dy.device, dtype=x.dtype)
            torch.ops.raft_stir.sconv(src, _sconv_dgrad_weight(conv.weight), None, 1, kh // 2 if s == 1 else p,
                                      False, dxn, 0, None)
            dx = dxn.permute(0, 3, 1, 2)
        if ctx.needs_input_grad[1]:
            g = torch.empty(conv.out_channels, kh, kw, cin, device=dy.device, dtype=torch.float32)
            torch.ops.raft_stir.sconv_wgrad(dyn, xn, kh, kw, s, p, g)
            dw = g.permute(0, 3, 1, 2).to(conv.weight.dtype)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = dyn.float().sum((0, 1, 2)).to(conv.bias.dtype)
        return dx, dw, db, None, None, None


def sconv_train(conv: nn.Conv2d, x: torch.Tensor, bias: bool = True) -> torch.Tensor:
    """conv(x) [+ bias] with autograd on the narrow-channel kernels (:func:`sconv_train_eligible`)."""
    b = conv.bias if bias else None
    return _SConvTrain.apply(x, conv.weight, b, conv.stride[0], conv.padding[0], _Hold(conv))


def sconv(conv: nn.Conv2d, x: torch.Tensor, bias: bool = True, relu: bool = False, residual=None) -> torch.Tensor:
    """[relu](conv(x) [+ bias]) [then relu(. + residual)] on csrc/sconv.hip;
    channels_last in and out (see :func:`sconv_eligible`)."""
    xn = _nhwc(x)
    N, H, W, _ = xn.shape
    kh, kw = conv.kernel_size
    s, p = conv.stride[0], conv.padding[0]
    Ho, Wo = (H + 2 * p - kh) // s + 1, (W + 2 * p - kw) // s + 1
    cout = conv.out_channels
    out = torch.empty(N, Ho, Wo, cout, device=x.device, dtype=x.dtype)
    b = conv.bias.detach().float().contiguous() if (bias and conv.bias is not None) else None
    rn = _nhwc(residual).contiguous() if residual is not None else None
    torch.ops.raft_stir.sconv(xn, _sconv_weight(conv), b, s, p, bool(relu), out, 0, rn)
    return out.permute(0, 3, 1, 2)
