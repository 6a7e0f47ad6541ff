"""Stride-1 3x3 encoder convolutions on the hand-written implicit-GEMM kernels.

The residual blocks of the feature / context encoders (reference
core/extractor.py:6-56, 118-192) spend most of the encoder FLOPs in stride-1
3x3 convolutions at 1/2, 1/4 and 1/8 resolution (64, 96, 128 channels).  On
the GPU bf16 path they run here instead of MIOpen:

  forward : csrc/conv.hip implicit GEMM (NHWC, buffer-DMA tiles)
  dgrad   : the same kernel on dY with the transposed, spatially flipped
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

from . import _ext
from .conv import EPI_BIAS, conv_fused, pack_weight, pad_to

_ENABLED = os.environ.get("RS_ENC_CONV", "1") != "0"
_CL = torch.channels_last


def choose_enc_tile(P: int, cin: int, cout: int) -> int:
    """Kernel variant for a stride-1 3x3 conv reading ``cin`` and writing
    ``cout`` channels over P pixels (scripts/bench_encoder_conv.py)."""
    if cin % 64 or cout % 64:
        return 4                   # 128x64 register-staged tile, 32-deep K steps
    if cout <= 64:
        return 21                  # 64 co x 128 px buffer-DMA tile
    return 16 if P >= 40000 else 17


_WGRAD_DMA = os.environ.get("RS_WGRAD_DMA", "1") != "0"


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


# Packed bf16 weights per (parameter, layout), repacked when the parameter
# changes (optimizer step / load_state_dict bump its version).  A repack is
# copied into the previous storage so a captured hipGraph keeps reading the
# live tensor; no packing kernels run inside a graph replay.  Entries hold a
# weak reference to their parameter and are dropped when it dies, so a new
# parameter that reuses a dead one's id() never sees its packed copy.
_PACKED = {}


def _packed(weight: torch.Tensor, dgrad: bool) -> torch.Tensor:
    key = (id(weight), dgrad)
    ver = (weight.data_ptr(), weight._version, weight.device, tuple(weight.shape))
    ent = _PACKED.get(key)
    if ent is not None and ent[0]() is weight and ent[1] == ver:
        return ent[2]
    cout, cin = weight.shape[:2]
    if dgrad:
        new = pack_weight(weight.transpose(0, 1).flip(2, 3), [(cout, [(0, cout, 0)])], pad_to(cin, 128))
    else:
        new = pack_weight(weight, [(cin, [(0, cin, 0)])], pad_to(cout, 128))
    if ent is not None and ent[0]() is weight and ent[2].shape == new.shape and ent[2].device == new.device:
        ent[2].copy_(new)
        new = ent[2]
    ref = weakref.ref(weight, lambda _r, k=key: _PACKED.pop(k, None))
    _PACKED[key] = (ref, ver, new)
    return new


class _Conv3x3(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight):
        xn = _nhwc(x)
        N, H, W, cin = xn.shape
        cout = weight.shape[0]
        P = N * H * W
        wp = _packed(weight, False)
        out = torch.empty(N, H, W, cout, device=x.device, dtype=torch.bfloat16)
        conv_fused([(xn, 0, cin)], wp, None, 3, 3, cout, EPI_BIAS, out, 0, tile=choose_enc_tile(P, cin, cout))
        ctx.save_for_backward(x, weight)
        return out.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        xn = _nhwc(x)
        N, H, W, cin = xn.shape
        cout = weight.shape[0]
        P = N * H * W
        dyn = _nhwc(dy.to(torch.bfloat16))
        dx = dw = None
        if ctx.needs_input_grad[0]:
            wd = _packed(weight, True)
            dxn = torch.empty(N, H, W, cin, device=x.device, dtype=torch.bfloat16)
            conv_fused([(dyn, 0, cout)], wd, None, 3, 3, cin, EPI_BIAS, dxn, 0, tile=choose_enc_tile(P, cout, cin))
            dx = dxn.permute(0, 3, 1, 2)
        if ctx.needs_input_grad[1]:
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
                dw = acc.view(cout, 3, 3, cin).permute(0, 3, 1, 2).to(weight.dtype)
            else:  # channel counts the wgrad kernel does not tile: MIOpen
                dw = torch.ops.aten.convolution_backward(
                    dyn.permute(0, 3, 1, 2), x, weight.to(torch.bfloat16), None, [1, 1], [1, 1], [1, 1], False,
                    [0, 0], 1, [False, True, False])[1].to(weight.dtype)
        return dx, dw


def conv3x3(conv: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    """conv(x) without its bias (see :func:`eligible`)."""
    return _Conv3x3.apply(x, conv.weight)
