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
boundaries.  Here a plan of the two encoders is built once and each
encoder STAGE (stem, six residual blocks, head) is one autograd node
(``_StageFn``):

  forward  : fnet stage k on the main HIP stream, cnet stage k on the side
             stream -- every conv and norm kernel called directly on NHWC
             buffers;
  backward : the hand-written reverse of each stage on the same stream,
             weight gradients with their dgrads; autograd interleaves the
             two encoders' stages as their gradients become ready (a single
             node per encoder serialised them: cnet's whole backward was
             issued before fnet's could start).

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

import contextlib
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
# (Statistics written by the conv epilogues instead of a separate pass were
# measured slower: the v3 / halo convs run 1-2 waves per SIMD, where the
# epilogue's extra VALU work and LDS transposition are not hidden -- +12-15 %
# per conv against a 9-24 us statistics pass; branch exp/epilogue-stats,
# profiles/r6/README.md.)
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


class _Stage:
    """One stage of one encoder (stem, a residual block or the head): its
    forward, its backward and its parameters.  ``sink`` is shared by the
    stages of one encoder: a residual block's backward leaves the skip-path
    gradient of its input there for the previous stage's backward, which
    takes it as the second upstream gradient of its output normalisation
    (no separate add pass, and the autograd edge carries only the conv
    input gradient)."""

    def __init__(self, plan, kind, index, sink):
        self.plan, self.kind, self.i, self.sink = plan, kind, index, sink
        if kind == "stem":
            conv, n0 = plan.stem
            self.params = [conv.weight, conv.bias, *n0.params()]
        elif kind == "head":
            self.params = [plan.head.weight, plan.head.bias]
        else:
            blk, n1, n2, d = plan.blocks[index]
            self.params = [blk.conv1.weight, blk.conv1.bias, *n1.params(), blk.conv2.weight, blk.conv2.bias,
                           *n2.params()]
            if d is not None:
                self.params += [d[0].weight, d[0].bias, *d[1].params()]
        self.saved = None

    # ------------------------------------------------------------- forward
    def forward(self, x):
        if self.kind == "stem":
            a0, st0, y0 = _stem_fwd(self.plan, x)
            self.saved = (x, a0, st0)
            return y0
        if self.kind == "head":
            self.saved = (x,)
            return _head_fwd(self.plan, x)
        blk, n1, n2, d = self.plan.blocks[self.i]
        out, self.saved = _block_fwd(blk, n1, n2, d, x)
        return out

    # ------------------------------------------------------------ backward
    def _zero_bias(self, bias):
        """The exactly-zero gradient of a conv bias folded into a batch /
        instance norm: disjoint slices of ONE zeroed buffer per encoder and
        step (one fill instead of one per bias; distinct memory per
        parameter, so AccumulateGrad may keep them as .grad)."""
        buf = self.sink.get("zb")
        if buf is None or buf[1] + bias.numel() > buf[0].numel():
            n = sum(c.bias.numel() for c in self.plan.enc.modules() if isinstance(c, nn.Conv2d))
            buf = [torch.zeros(n, device=bias.device, dtype=bias.dtype), 0]
            self.sink["zb"] = buf
        t = buf[0][buf[1]:buf[1] + bias.numel()].view_as(bias)
        buf[1] += bias.numel()
        return t

    def backward(self, g):
        """(input gradient, {param: gradient}); g: this stage's output gradient."""
        grads = {}
        g = g.contiguous()
        g2 = self.sink.pop(self.i, None)  # the next block's skip gradient of this output
        zb = self._zero_bias
        if self.kind == "head":
            h, (y,) = self.plan.head, self.saved
            gn = g.to(_BF)
            dy = E._conv_geo_dgrad([gn], [h.weight], _nchw(y).shape, (1, 1), (0, 0))
            grads[h.weight], grads[h.bias] = E._conv_geo_wgrad(gn, _nchw(y), h.weight, (1, 1), True)
            return dy, grads
        if self.kind == "stem":
            conv, n0 = self.plan.stem
            x, a0, st0 = self.saved
            da0, _, pg0, _ = _norm_bwd(n0, g, a0, st0, True, None, g2)
            grads.update(zip(n0.params(), pg0))
            gw = torch.empty(conv.weight.shape, device=g.device, dtype=torch.float32)
            R.stem_wgrad(E._nhwc(x), da0, conv.weight.shape[0], gw)
            grads[conv.weight] = gw.to(conv.weight.dtype)
            grads[conv.bias] = zb(conv.bias)
            return None, grads
        blk, n1, n2, d = self.plan.blocks[self.i]
        y, a1, st1, y1, a2, st2, dd_raw, st3 = self.saved
        if d is None:
            da2, dres, pg2, _ = _norm_bwd(n2, g, a2, st2, True, y, g2)
        else:  # dres: the gradient of the raw shortcut conv output, through its norm
            da2, dres, pg2, pg3 = _norm_bwd(n2, g, a2, st2, True, dd_raw, g2, d[1], st3)
            grads.update(zip(d[1].params(), pg3))
        grads.update(zip(n2.params(), pg2))
        dy1, _ = _dgrad3x3(da2, blk.conv2.weight, blk.conv2.in_channels)
        grads[blk.conv2.weight] = _wgrad3x3(da2, y1, blk.conv2.weight)
        grads[blk.conv2.bias] = zb(blk.conv2.bias)
        da1, _, pg1, _ = _norm_bwd(n1, dy1, a1, st1, True)
        grads.update(zip(n1.params(), pg1))
        grads[blk.conv1.bias] = zb(blk.conv1.bias)
        if d is None:
            dy, fused = _dgrad3x3(da1, blk.conv1.weight, blk.conv1.in_channels, acc=dres)
            grads[blk.conv1.weight] = _wgrad3x3(da1, y, blk.conv1.weight)
            if not fused:
                self.sink[self.i - 1] = dres
            return dy, grads
        grads[d[0].bias] = zb(d[0].bias)
        stride = tuple(blk.conv1.stride)
        dy = E._pair_dgrad(da1, dres, blk.conv1.weight, d[0].weight, _nchw(y).shape, stride)
        grads[blk.conv1.weight] = E._conv_geo_wgrad(da1, _nchw(y), blk.conv1.weight, stride, False)[0]
        grads[d[0].weight] = E._conv_geo_wgrad(dres, _nchw(y), d[0].weight, stride, False)[0]
        return dy, grads


class _StageFn(torch.autograd.Function):
    """One encoder stage as one autograd node; autograd runs its backward on
    the stream of its forward (fnet: main, cnet: side) and interleaves the two
    encoders' stage nodes by creation order, as soon as each gradient is
    ready (cnet's backward starts right after the update loop's and overlaps
    the correlation backward that fnet's waits for)."""

    @staticmethod
    def forward(ctx, stage, x, *params):
        ctx.stage = stage
        return stage.forward(x)

    @staticmethod
    def backward(ctx, g):
        stage = ctx.stage
        dx, grads = stage.backward(g)
        stage.saved = None
        ctx.stage = None
        return (None, dx, *[grads[p] for p in stage.params])


class FusedEncoders:
    """The engine: plans of both encoders, cached on the RAFT module."""

    def __init__(self, model):
        self.model = model
        self.fplan, self.cplan = _Plan(model.fnet), _Plan(model.cnet)
        self.params = self.fplan.params + self.cplan.params

    @staticmethod
    def eligible(model, x) -> bool:
        return (ENABLED and x.is_cuda and _ext.use_hip(x) and torch.is_grad_enabled()
                and torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16
                and x.dtype == torch.float32 and x.is_contiguous(memory_format=_CL)
                and _Plan.ok(model.fnet) and _Plan.ok(model.cnet) and not torch.jit.is_tracing())

    @staticmethod
    def _stages(plan):
        sink = {}
        n = len(plan.blocks)
        return ([_Stage(plan, "stem", -1, sink)] + [_Stage(plan, "block", i, sink) for i in range(n)]
                + [_Stage(plan, "head", n, sink)])

    def run(self, xf, xc, side):
        """(fnet(xf), cnet(xc)) as NCHW views of channels-last bf16: stage k of
        fnet on the current stream, then stage k of cnet on ``side`` (None:
        the single-stream schedule, same kernels in the same order).  The
        caller joins ``side`` before the main stream reads cnet's output."""
        ff, fc = self._stages(self.fplan), self._stages(self.cplan)
        on_side = torch.cuda.stream(side) if side is not None else contextlib.nullcontext()
        if side is not None:
            side.wait_stream(torch.cuda.current_stream(xf.device))
            xc.record_stream(side)
        of, oc = xf, xc
        for sf, sc in zip(ff, fc):
            of = _StageFn.apply(sf, of, *sf.params)
            with on_side:
                oc = _StageFn.apply(sc, oc, *sc.params)
        return _nchw(of), _nchw(oc)
