"""Fused ConvGRU pass (one autograd node per GRU pass).

Forward (channels_last, compute dtype = autocast dtype or the input dtype):
    zr   = conv(cat[h, x], [Wz; Wr])          # ONE conv, 2*hdim outputs
    z, r, rhx = gate_zr(zr, h, x)             # HIP: sigmoid, r*h, [r*h | x]
    q    = conv(rhx, Wq)
    h', q~ = gate_q(q, z, h)                  # HIP: tanh + (1-z)h + z q~
Backward (hand-written chain; HIP kernels for every elementwise stage and
``aten.convolution_backward`` for the dgrad/wgrad pairs):
    dq, dz_pre, dh_d = bwd_q(dh', z, h, q~)
    drhx, dWq, dbq   = conv_bwd(dq; rhx, Wq)
    dr_pre           = bwd_r(drhx, h, r)         (written into dzr[:, hd:])
    dhx, dWzr, dbzr  = conv_bwd([dz_pre | dr_pre]; hx, Wzr)
    dh, dx           = bwd_fin(dh_d, drhx, r, dhx)
Reference semantics: core/update.py:16-60.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _ext
from . import fp32conv
from .corr import to_nhwc, from_nhwc

_CL = torch.channels_last
def fused_available(h: torch.Tensor) -> bool:
    return _ext.use_hip(h)


def _conv_bwd(dy, x, w, padding):
    return fp32conv.conv_backward(dy, x, w, (1, 1), padding)


class _GRUPass(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, x, wzr, bzr, wq, bq, padding):
        # h: (B,hd,H,W), x: (B,cin,H,W) channels_last, same dtype
        hx = torch.cat([h, x], dim=1).contiguous(memory_format=_CL)
        zr = fp32conv.conv2d(hx, wzr, bzr, 1, padding)
        hn_ = to_nhwc(h)
        z, r, rhx = torch.ops.raft_stir.gru_gate_zr(to_nhwc(zr), hn_, to_nhwc(x))
        q = fp32conv.conv2d(from_nhwc(rhx), wq, bq, 1, padding)
        hn, qt = torch.ops.raft_stir.gru_gate_q(to_nhwc(q), z, hn_)
        ctx.padding = padding
        ctx.save_for_backward(hx, rhx, wzr, wq, hn_, z, r, qt)
        return from_nhwc(hn)

    @staticmethod
    def backward(ctx, dhn):
        hx, rhx, wzr, wq, h, z, r, qt = ctx.saved_tensors
        pad = ctx.padding
        dq, dzr, dh_d = torch.ops.raft_stir.gru_bwd_q(to_nhwc(dhn).to(h.dtype), z, h, qt)
        drhx, dwq, dbq = _conv_bwd(from_nhwc(dq), from_nhwc(rhx), wq, pad)
        drhx = to_nhwc(drhx)
        torch.ops.raft_stir.gru_bwd_r(drhx, h, r, dzr)
        dhx, dwzr, dbzr = _conv_bwd(from_nhwc(dzr), hx, wzr, pad)
        dh, dx = torch.ops.raft_stir.gru_bwd_fin(dh_d, drhx, r, to_nhwc(dhx))
        return from_nhwc(dh), from_nhwc(dx), dwzr, dbzr, dwq, dbq, None


def _compute_dtype(h):
    if torch.is_autocast_enabled("cuda"):
        return torch.get_autocast_dtype("cuda")
    return h.dtype if h.dtype in (torch.float32, torch.bfloat16) else torch.float32


_WCACHE = {}


def begin_forward():
    """Called once per RAFT forward: the fused/cast GRU weights are built once
    per forward (they are nodes of this forward's autograd graph, so their
    gradients accumulate over the iterations and flow back once)."""
    _WCACHE.clear()


def _weights(convz, convr, convq, dt):
    # keyed on the parameters' storage and version counters too: a module
    # used outside RAFT.forward (no begin_forward) or a new module reusing a
    # freed one's id must never see stale weights
    ps = (convz.weight, convz.bias, convr.weight, convr.bias, convq.weight, convq.bias)
    from ..runtime.weights import generation
    key = (id(convz), dt, generation()) + tuple((p.data_ptr(), p._version) for p in ps)
    w = _WCACHE.get(key)
    if w is None:
        if len(_WCACHE) > 32:
            _WCACHE.clear()
        wzr = torch.cat([convz.weight, convr.weight], dim=0).to(dt).contiguous(memory_format=_CL)
        bzr = torch.cat([convz.bias, convr.bias], dim=0).to(dt)
        wq = convq.weight.to(dt).contiguous(memory_format=_CL)
        bq = convq.bias.to(dt)
        w = _WCACHE[key] = (wzr, bzr, wq, bq)
    return w


def gru_pass(h, x, convz, convr, convq):
    dt = _compute_dtype(h)
    wzr, bzr, wq, bq = _weights(convz, convr, convq, dt)
    h = h.to(dt).contiguous(memory_format=_CL)
    x = x.to(dt).contiguous(memory_format=_CL)
    with torch.autocast("cuda", enabled=False):
        return _GRUPass.apply(h, x, wzr, bzr, wq, bq, tuple(convz.padding))
