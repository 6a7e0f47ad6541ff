"""Both encoders of a bf16 training step as ONE scheduled autograd node.

Reference semantics: core/extractor.py:6-56 (ResidualBlock: conv3x3 ->
norm1 -> ReLU -> conv3x3 -> norm2 -> ReLU, + identity or (1x1/s2 conv ->
norm3) shortcut, ReLU) and :118-192 (BasicEncoder: 7x7/s2 stem -> norm1 ->
ReLU, layer1-3, 1x1 projection), fnet with instance norm on both images,
cnet with batch norm (train-mode statistics, running-buffer update) on
image1 -- reference core/raft.py:95-110.

Per-module autograd (ops/enc_conv.py + ops/norm.py) runs every conv and
every normalisation as its own Function: ~6.9 ms of host enqueue per step
for ~6.4 ms of GPU work (profiles/r6/README.md, scripts/bench_encoders.py),
and the normalisation chains cannot be restructured across Function
boundaries.  Here a plan of the two encoders is built once and
``FusedEncoders.run`` / ``EncoderFn`` run

  forward  : fnet stage k on the main HIP stream, cnet stage k on the side
             stream, k = stem, six residual blocks, head -- every conv and
             norm kernel called directly on NHWC buffers;
  backward : the hand-written reverse of the same plan on the same streams
             (fnet on main, cnet on side), weight gradients with their dgrads.

Normalisation layout per residual block (bias folded away: a per-channel
constant before instance / train-mode batch norm has no effect and a zero
gradient):

  stride 1:  a1 = conv1(y)      y1 = relu(n1(a1))
             a2 = conv2(y1)     out = relu(y + relu(n2(a2)))
  stride 2:  a1, d = conv3x3/s2(y), conv1x1/s2(y)
             a2 = conv2(relu(n1(a1)))
             out = relu(n3(d) + relu(n2(a2)))   -- n3 applied inside the
             output pass (csrc/norm.hip apply with an affine residual), r
             never materialised

The backward takes the skip-path gradient as a SECOND upstream gradient of
the previous normalisation (the kernels add the two on the fly), so no
gradient is ever summed in a separate pass, and the downsample norm's
gradient statistics come out of the output pass's backward.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from ..ops import _ext, wpack
from ..ops import enc_conv as E
from .extractor import BasicEncoder, ResidualBlock

R = torch.ops.raft_stir
_CL = torch.channels_last
ENABLED = os.environ.get("RS_FUSED_ENC", "1") != "0"  # A/B switch: 0 = per-module autograd path
_BF = torch.bfloat16


def _nchw(t):
    return t.permute(0, 3, 1, 2)


class _Norm:
    """One normalisation layer of the plan: instance norm (per-sample
    statistics) or train-mode BatchNorm (batch statistics + running update)."""

    def __init__(self, norm: nn.Module, conv_bias):
        self.m = norm
        self.inst = isinstance(norm, nn.InstanceNorm2d)
        self.bias = conv_bias  # the producing conv's bias (folded: running mean only)

    @staticmethod
    def ok(norm) -> bool:
        if isinstance(norm, nn.InstanceNorm2d):
            return not norm.affine and not norm.track_running_stats
        if isinstance(norm, nn.BatchNorm2d):
            return norm.affine and norm.track_running_stats and norm.momentum is not None and norm.training
        return False

    def params(self):
        return [] if self.inst else [self.m.weight, self.m.bias]

    @property
    def gamma(self):
        return None if self.inst else self.m.weight

    @property
    def beta(self):
        return None if self.inst else self.m.bias

    def stats(self, xn):
        """(mean, rstd) of a raw NHWC conv output; BatchNorm also updates its
        running buffers (the conv bias shifts the running mean only)."""
        m = self.m
        if self.inst:
            return R.norm_stats(xn, True, m.eps)
        n = xn.numel() // xn.shape[3]
        nbt = m.num_batches_tracked
        mean, rstd = R.norm_stats(xn, False, m.eps, m.running_mean, m.running_var,
                                  nbt if nbt is not None and nbt.dtype == torch.long else None,
                                  None if self.bias is None else self.bias.detach().float().contiguous(),
                                  m.momentum, n)
        torch.autograd.graph.increment_version([m.running_mean, m.running_var])
        return mean, rstd

    def param_grads(self, s12):
        """(dgamma, dbeta) from the backward's (2, G, C) per-group sums."""
        if self.inst:
            return []
        d = s12[:, 0] if s12.shape[1] == 1 else s12.sum(1)
        return [d[1], d[0]]


class _Plan:
    """Static description of one BasicEncoder for the fused engine."""

    def __init__(self, enc: BasicEncoder):
        self.enc = enc
        self.stem = (enc.conv1, _Norm(enc.norm1, enc.conv1.bias))
        self.blocks = []
        for layer in (enc.layer1, enc.layer2, enc.layer3):
            for blk in layer:
                d = None
                if blk.downsample is not None:
                    d = (blk.downsample[0], _Norm(blk.norm3, blk.downsample[0].bias))
                self.blocks.append((blk, _Norm(blk.norm1, blk.conv1.bias), _Norm(blk.norm2, blk.conv2.bias), d))
        self.head = enc.conv2
        # parameters in the order the Function receives (and returns gradients for) them
        ps = [self.stem[0].weight, self.stem[0].bias, *self.stem[1].params()]
        for blk, n1, n2, d in self.blocks:
            ps += [blk.conv1.weight, blk.conv1.bias, *n1.params(), blk.conv2.weight, blk.conv2.bias, *n2.params()]
            if d is not None:
                ps += [d[0].weight, d[0].bias, *d[1].params()]
        ps += [self.head.weight, self.head.bias]
        self.params = ps

    @staticmethod
    def ok(enc) -> bool:
        if not isinstance(enc, BasicEncoder) or not enc.training or enc.dropout is not None or not enc.hip_geo:
            return False
        if not _Norm.ok(enc.norm1) or enc.conv1.bias is None or enc.conv2.bias is None:
            return False
        for layer in (enc.layer1, enc.layer2, enc.layer3):
            for blk in layer:
                if not isinstance(blk, ResidualBlock) or not (_Norm.ok(blk.norm1) and _Norm.ok(blk.norm2)):
                    return False
                if blk.conv1.bias is None or blk.conv2.bias is None:
                    return False
                if blk.downsample is not None and (not _Norm.ok(blk.norm3) or blk.downsample[0].bias is None
                                                   or blk.conv1.stride != (2, 2)):
                    return False
                if blk.downsample is None and blk.conv1.stride != (1, 1):
                    return False
        return True


# ------------------------------------------------------------------ conv steps
def _conv3x3(xn, weight, cout):
    N, H, W, cin = xn.shape
    out = torch.empty(N, H, W, cout, device=xn.device, dtype=_BF)
    t = E._v3_tile(N * H * W, cin, cout)
    if t is not None:
        E._conv3x3_v3(xn, weight, cin, cout, out, t, False)
    else:
        E._conv3x3_into(xn, E._packed(weight, False), cin, cout, out, N * H * W)
    return out


def _dgrad3x3(dyn, weight, cin, acc=None):
    """dX of a stride-1 3x3 conv; ``acc`` (NHWC bf16): dX is ADDED to it in the
    halo kernel's epilogue when that kernel serves the shape, else None is
    returned for the caller to pass ``acc`` on as a second gradient."""
    N, H, W, cout = dyn.shape
    P = N * H * W
    td = E._v3_tile(P, cout, cin)
    if acc is not None and td is None and E._halo_ok(cout, cin):
        R.conv3x3_halo(dyn, E._packed(weight, True), acc, cout, cin, accumulate=True)
        return acc, True
    dx = torch.empty(N, H, W, cin, device=dyn.device, dtype=_BF)
    if td is not None:
        E._conv3x3_v3(dyn, weight, cout, cin, dx, td, True)
    else:
        E._conv3x3_into(dyn, E._packed(weight, True), cout, cin, dx, P)
    return dx, False


def _wgrad3x3(dyn, xn, weight):
    cout, cin = weight.shape[:2]
    N, H, W, _ = xn.shape
    return E._wgrad3x3(dyn, _nchw(xn), xn, weight, cin, cout, N * H * W)


class _EncState:
    """Saved activations of one encoder's forward."""
    __slots__ = ("x", "a0", "st0", "y0", "blocks", "ylast", "out")


def _stem_fwd(plan, x):
    conv, n0 = plan.stem
    xn = E._nhwc(x)
    N, H, W, _ = xn.shape
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    a0 = torch.empty(N, Ho, Wo, conv.out_channels, device=x.device, dtype=_BF)
    wp = wpack.packed(("stem", id(conv.weight)), [conv.weight], E._stem_layout)
    R.stem_conv(xn, wp, None, a0, conv.out_channels, 0)
    st0 = n0.stats(a0)
    y0 = R.norm_act(a0, st0[0], st0[1], n0.gamma, n0.beta, None, True)
    return a0, st0, y0


def _block_fwd(blk, n1, n2, d, y):
    cout = blk.conv1.out_channels
    if d is None:
        a1 = _conv3x3(y, blk.conv1.weight, cout)
        dd = st3 = None
    else:
        yc = _nchw(y)
        a1 = E._conv_geo_fwd(yc, blk.conv1.weight, None, tuple(blk.conv1.stride), (1, 1))
        dd = E._conv_geo_fwd(yc, d[0].weight, None, tuple(d[0].stride), (0, 0))
        st3 = d[1].stats(dd)
    st1 = n1.stats(a1)
    y1 = R.norm_act(a1, st1[0], st1[1], n1.gamma, n1.beta, None, True)
    a2 = _conv3x3(y1, blk.conv2.weight, cout)
    st2 = n2.stats(a2)
    if d is None:
        out = R.norm_act(a2, st2[0], st2[1], n2.gamma, n2.beta, y, True)
    else:  # relu(relu(n2(a2)) + n3(d)): the shortcut's norm inside the output pass
        out = R.norm_act(a2, st2[0], st2[1], n2.gamma, n2.beta, dd, True, st3[0], st3[1], d[1].gamma, d[1].beta)
    return out, (y, a1, st1, y1, a2, st2, dd, st3)


def _head_fwd(plan, y):
    h = plan.head
    return E._conv_geo_fwd(_nchw(y), h.weight, h.bias, (1, 1), (0, 0))


def _enc_stages(plan):
    """The forward as a list of stage callables over a shared state (so two
    encoders can be issued stage-interleaved on two streams)."""
    def stem(s, x):
        s.x = x
        s.a0, s.st0, s.y0 = _stem_fwd(plan, x)
        s.blocks = []
        return s.y0

    def block(i):
        def run(s, y):
            blk, n1, n2, d = plan.blocks[i]
            out, saved = _block_fwd(blk, n1, n2, d, y)
            s.blocks.append(saved)
            return out
        return run

    def head(s, y):
        s.ylast = y
        return _head_fwd(plan, y)
    return [stem] + [block(i) for i in range(len(plan.blocks))] + [head]


# ------------------------------------------------------------------ backward
def _norm_bwd(n, dy, xn, st, relu, res=None, dy2=None, rn=None, rst=None):
    """(dx, dres, [param grads], [residual-norm param grads]) of
    y = [relu](n(x)) [then relu(. + res)], upstream gradient dy (+ dy2);
    ``rn`` / ``rst``: the residual is raw and normalised by that norm / those
    statistics (dres is then the raw residual's gradient)."""
    if rn is None:
        out = R.norm_act_backward(dy, xn, st[0], st[1], n.gamma, n.beta, res, relu, True, dy2)
        return out[0], (out[1] if res is not None else None), n.param_grads(out[4]), []
    out = R.norm_act_backward(dy, xn, st[0], st[1], n.gamma, n.beta, res, relu, True, dy2,
                              rst[0], rst[1], rn.gamma, rn.beta)
    return out[0], out[1], n.param_grads(out[4]), rn.param_grads(out[5])


def _enc_bwd_stages(plan, s, grads):
    """Backward stages in reverse order; each returns the gradient of its input.
    ``grads``: dict param -> gradient (filled in)."""
    zero_bias = lambda conv: torch.zeros_like(conv.bias)

    def head(gpair):
        h = plan.head
        gn = E._nhwc(gpair[0].to(_BF))
        y = s.ylast
        dy = E._conv_geo_dgrad([gn], [h.weight], _nchw(y).shape, (1, 1), (0, 0))
        dw, db = E._conv_geo_wgrad(gn, _nchw(y), h.weight, (1, 1), True)
        grads[h.weight], grads[h.bias] = dw, db
        return dy, None

    def block(i):
        def run(gpair):
            g, g2 = gpair  # g2: the skip gradient of the next block, added inside the norm kernels
            blk, n1, n2, d = plan.blocks[i]
            y, a1, st1, y1, a2, st2, dd_raw, st3 = s.blocks[i]
            if d is None:
                da2, dres, pg2, _ = _norm_bwd(n2, g, a2, st2, True, y, g2)
            else:  # dres: the gradient of the raw shortcut conv output, through its norm
                da2, dres, pg2, pg3 = _norm_bwd(n2, g, a2, st2, True, dd_raw, g2, d[1], st3)
            dy1, _ = _dgrad3x3(da2, blk.conv2.weight, blk.conv2.in_channels)
            grads[blk.conv2.weight] = _wgrad3x3(da2, y1, blk.conv2.weight)
            grads[blk.conv2.bias] = zero_bias(blk.conv2)
            for p, gp in zip(n2.params(), pg2):
                grads[p] = gp
            da1, _, pg1, _ = _norm_bwd(n1, dy1, a1, st1, True)
            grads[blk.conv1.bias] = zero_bias(blk.conv1)
            for p, gp in zip(n1.params(), pg1):
                grads[p] = gp
            if d is None:
                dy, fused = _dgrad3x3(da1, blk.conv1.weight, blk.conv1.in_channels, acc=dres)
                grads[blk.conv1.weight] = _wgrad3x3(da1, y, blk.conv1.weight)
                return dy, (None if fused else dres)
            ddn = dres
            for p, gp in zip(d[1].params(), pg3):
                grads[p] = gp
            grads[d[0].bias] = zero_bias(d[0])
            stride = tuple(blk.conv1.stride)
            dy = E._pair_dgrad(da1, ddn, blk.conv1.weight, d[0].weight, _nchw(y).shape, stride)
            grads[blk.conv1.weight] = E._conv_geo_wgrad(da1, _nchw(y), blk.conv1.weight, stride, False)[0]
            grads[d[0].weight] = E._conv_geo_wgrad(ddn, _nchw(y), d[0].weight, stride, False)[0]
            return dy, None
        return run

    def stem(gpair):
        g, g2 = gpair
        conv, n0 = plan.stem
        da0, _, pg0, _ = _norm_bwd(n0, g, s.a0, s.st0, True, None, g2)
        for p, gp in zip(n0.params(), pg0):
            grads[p] = gp
        gw = torch.empty(conv.weight.shape, device=g.device, dtype=torch.float32)
        R.stem_wgrad(E._nhwc(s.x), da0, conv.weight.shape[0], gw)
        grads[conv.weight] = gw.to(conv.weight.dtype)
        grads[conv.bias] = zero_bias(conv)
        return None, None
    return [head] + [block(i) for i in reversed(range(len(plan.blocks)))] + [stem]


class EncoderFn(torch.autograd.Function):
    """One encoder as one autograd node.  Its forward was already run
    (FusedEncoders.run issues both encoders' forwards stage-interleaved on
    two streams); this node hands out the output and owns the backward,
    which autograd runs on the stream of the forward (main for fnet, side for
    cnet) as soon as THIS encoder's gradient is ready: cnet's backward
    starts right after the update loop's and overlaps the correlation
    backward that fnet's waits for."""

    @staticmethod
    def forward(ctx, plan, state, x, *params):
        ctx.plan, ctx.state = plan, state
        out = state.out
        state.out = None
        return _nchw(out)

    @staticmethod
    def backward(ctx, g):
        plan, s = ctx.plan, ctx.state
        if g is None:
            g = _nchw(torch.zeros(s.ylast.shape[:3] + (plan.head.out_channels,), device=s.ylast.device))
        grads = {}
        cur = (g, None)
        for stage in _enc_bwd_stages(plan, s, grads):
            cur = stage(cur)
        ctx.state = None
        return (None, None, None, *[grads[p] for p in plan.params])


class FusedEncoders:
    """The engine: plans of both encoders, cached on the RAFT module."""

    def __init__(self, model):
        self.model = model
        self.fplan, self.cplan = _Plan(model.fnet), _Plan(model.cnet)
        self.params = self.fplan.params + self.cplan.params

    @staticmethod
    def eligible(model, x) -> bool:
        return (ENABLED and x.is_cuda and _ext.use_hip(x) and torch.is_grad_enabled() and torch.is_autocast_enabled("cuda")
                and torch.get_autocast_dtype("cuda") == torch.bfloat16 and x.dtype == torch.float32
                and x.is_contiguous(memory_format=_CL) and _Plan.ok(model.fnet) and _Plan.ok(model.cnet)
                and not torch.jit.is_tracing())

    def run(self, xf, xc, side):
        """(fnet(xf), cnet(xc)): both forwards issued stage by stage on the
        main and ``side`` streams, then one :class:`EncoderFn` node per
        encoder (cnet's created under ``side``).  The caller joins ``side``
        before the main stream reads cnet's output."""
        main = torch.cuda.current_stream(xf.device)
        sf, sc = _EncState(), _EncState()
        ff, fc = _enc_stages(self.fplan), _enc_stages(self.cplan)
        side.wait_stream(main)
        xc.record_stream(side)
        with torch.no_grad():
            of, oc = xf, xc
            for k in range(max(len(ff), len(fc))):
                if k < len(ff):
                    of = ff[k](sf, of)
                if k < len(fc):
                    with torch.cuda.stream(side):
                        oc = fc[k](sc, oc)
        sf.out, sc.out = of, oc
        f = EncoderFn.apply(self.fplan, sf, xf, *self.fplan.params)
        with torch.cuda.stream(side):
            c = EncoderFn.apply(self.cplan, sc, xc, *self.cplan.params)
        return f, c
