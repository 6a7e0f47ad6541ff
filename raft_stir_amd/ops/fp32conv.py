"""fp32 GPU convolutions with a measured per-shape memory-format choice.

The bf16 path runs the update block on the hand-written kernels (ops/conv.py);
fp32 (the reference's default evaluation / export precision, evaluate.py and
rafttoonnx.py run without --mixed_precision) stays on MIOpen.  MIOpen's fp32
solvers differ by an order of magnitude between layouts, and in BOTH
directions (scripts/fp32_conv_probe.py, MI355X):

  RAFT-small ConvGRU 3x3 242->192 at 64x80     NCHW  53 us   NHWC 297 us
  whole RAFT-small 512x640 graphed (12 iters)  NCHW 7.0 ms   NHWC 11.6 ms
  whole RAFT 1088x436 graphed (12 iters)       NCHW 20.7 ms  NHWC 13.7 ms

so the first fp32 call of each (input shape, weight shape, conv params) times
both layouts (a few back-to-back runs each, outside any graph capture) and
every later call -- including hipGraph captures -- uses the faster one.  The
activations stay channels_last between convolutions (the HIP kernels read
NHWC); an NCHW conv converts its input and hands back a channels_last output,
and those copies are part of what is timed.

RS_FP32_LAYOUT=nchw|nhwc forces one layout (no timing).
"""
from __future__ import annotations

import os
from typing import Dict, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

_CL = torch.channels_last
_FORCE = os.environ.get("RS_FP32_LAYOUT", "").lower()
_CHOICE: Dict[Tuple, bool] = {}   # key -> True: run NCHW


def active(x: torch.Tensor) -> bool:
    """fp32 conv on the GPU outside autocast: layout-tuned."""
    return x.is_cuda and x.dtype == torch.float32 and not torch.is_autocast_enabled("cuda")


def _run(x, w, b, stride, padding, dilation, groups, nchw: bool):
    if nchw:
        y = F.conv2d(x.contiguous(), w.contiguous(), b, stride, padding, dilation, groups)
        return y.contiguous(memory_format=_CL)
    return F.conv2d(x.contiguous(memory_format=_CL), w.contiguous(memory_format=_CL), b, stride, padding,
                    dilation, groups)


def _time(fn, reps: int = 3) -> float:
    fn()  # first call: MIOpen solution search / kernel load
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e)


def choose(x, w, b, stride, padding, dilation, groups) -> bool:
    if _FORCE in ("nchw", "nhwc"):
        return _FORCE == "nchw"
    key = (tuple(x.shape), tuple(w.shape), b is not None, tuple(stride), tuple(padding), tuple(dilation), groups,
           x.device)
    c = _CHOICE.get(key)
    if c is not None:
        return c
    if torch.cuda.is_current_stream_capturing():
        return False  # untuned shape inside a capture: no timing possible, keep NHWC
    with torch.no_grad():
        t_nchw = _time(lambda: _run(x, w, b, stride, padding, dilation, groups, True))
        t_nhwc = _time(lambda: _run(x, w, b, stride, padding, dilation, groups, False))
    c = _CHOICE[key] = t_nchw < t_nhwc
    return c


def _pair(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (v, v)


def conv2d(x, w, b=None, stride=1, padding=0, dilation=1, groups=1):
    """F.conv2d with the tuned layout for fp32 GPU inputs; channels_last out."""
    if not active(x):
        return F.conv2d(x, w, b, stride, padding, dilation, groups)
    stride, padding, dilation = _pair(stride), _pair(padding), _pair(dilation)
    return _run(x, w, b, stride, padding, dilation, groups, choose(x, w, b, stride, padding, dilation, groups))


def conv_module(conv: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    """``conv(x)`` through :func:`conv2d` (zero padding only)."""
    if not active(x) or conv.padding_mode != "zeros" or isinstance(conv.padding, str):
        return conv(x)
    return conv2d(x, conv.weight, conv.bias, conv.stride, conv.padding, conv.dilation, conv.groups)


def conv_backward(dy, x, w, stride, padding, dilation=(1, 1), groups=1, mask=(True, True, True)):
    """aten.convolution_backward in the layout chosen for the forward of the
    same shape (NHWC if that forward was never tuned); channels_last dx."""
    stride, padding, dilation = _pair(stride), _pair(padding), _pair(dilation)
    nchw = False
    if active(x):
        if _FORCE in ("nchw", "nhwc"):
            nchw = _FORCE == "nchw"
        else:
            key = (tuple(x.shape), tuple(w.shape), True, stride, padding, dilation, groups, x.device)
            nchw = _CHOICE.get(key, False)
    fmt = torch.contiguous_format if nchw else _CL
    dx, dw, db = torch.ops.aten.convolution_backward(
        dy.contiguous(memory_format=fmt), x.contiguous(memory_format=fmt), w.contiguous(memory_format=fmt),
        [w.shape[0]], list(stride), list(padding), list(dilation), False, [0, 0], groups, list(mask))
    if dx is not None:
        dx = dx.contiguous(memory_format=_CL)
    return dx, dw, db
