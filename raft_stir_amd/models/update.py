"""Update operator: motion encoder, convolutional GRU, flow and mask heads.

Parity with reference core/update.py:
  * FlowHead (:6-14): 3x3 conv -> ReLU -> 3x3 conv to 2 channels.
  * ConvGRU (:16-31, RAFT-small): 3x3 z/r/q gates.
  * SepConvGRU (:33-60, full RAFT): a 1x5 pass then a 5x1 pass.
  * SmallMotionEncoder (:62-77) / BasicMotionEncoder (:79-97).
  * SmallUpdateBlock (:99-112) / BasicUpdateBlock (:114-136, mask x0.25).

Module/parameter names are identical to the reference's so checkpoints load.

GPU path: each GRU pass is a single autograd node
(:func:`raft_stir_amd.ops.gru.gru_pass`) that runs the z|r convolution as ONE
conv with concatenated weights (N = 2*hdim), applies the sigmoid gates and
``r*h`` in a fused HIP kernel, runs the q convolution and finishes with a fused
tanh + GRU-blend kernel; its backward is hand-written (fused gate-gradient
kernels + conv dgrad/wgrad). The CPU path is the plain composite below; it is
the numerics oracle and the path traced for TorchScript/ONNX export.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import gru as gru_ops
from ..ops.fp32conv import conv_module as _cv


class FlowHead(nn.Module):
    def __init__(self, input_dim=128, hidden_dim=256):
        super().__init__()
        self.conv1 = nn.Conv2d(input_dim, hidden_dim, 3, padding=1)
        self.conv2 = nn.Conv2d(hidden_dim, 2, 3, padding=1)
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        return _cv(self.conv2, self.relu(_cv(self.conv1, x)))


def _gru_step_reference(convz, convr, convq, h, x):
    hx = torch.cat([h, x], dim=1)
    z = torch.sigmoid(convz(hx))
    r = torch.sigmoid(convr(hx))
    q = torch.tanh(convq(torch.cat([r * h, x], dim=1)))
    return (1 - z) * h + z * q


def _gru_step(convz, convr, convq, h, x, fused):
    if fused and gru_ops.fused_available(h):
        return gru_ops.gru_pass(h, x, convz, convr, convq)
    return _gru_step_reference(convz, convr, convq, h, x)


class ConvGRU(nn.Module):
    def __init__(self, hidden_dim=128, input_dim=192 + 128):
        super().__init__()
        cin = hidden_dim + input_dim
        self.convz = nn.Conv2d(cin, hidden_dim, 3, padding=1)
        self.convr = nn.Conv2d(cin, hidden_dim, 3, padding=1)
        self.convq = nn.Conv2d(cin, hidden_dim, 3, padding=1)
        self.fused = True

    def forward(self, h, x):
        return _gru_step(self.convz, self.convr, self.convq, h, x, self.fused)


class SepConvGRU(nn.Module):
    def __init__(self, hidden_dim=128, input_dim=192 + 128):
        super().__init__()
        cin = hidden_dim + input_dim
        for axis, (k, p) in (("1", ((1, 5), (0, 2))), ("2", ((5, 1), (2, 0)))):
            for gate in "zrq":
                setattr(self, f"conv{gate}{axis}", nn.Conv2d(cin, hidden_dim, k, padding=p))
        self.fused = True

    def forward(self, h, x):
        h = _gru_step(self.convz1, self.convr1, self.convq1, h, x, self.fused)  # horizontal
        h = _gru_step(self.convz2, self.convr2, self.convq2, h, x, self.fused)  # vertical
        return h


class SmallMotionEncoder(nn.Module):
    def __init__(self, corr_planes):
        super().__init__()
        self.convc1 = nn.Conv2d(corr_planes, 96, 1, padding=0)
        self.convf1 = nn.Conv2d(2, 64, 7, padding=3)
        self.convf2 = nn.Conv2d(64, 32, 3, padding=1)
        self.conv = nn.Conv2d(128, 80, 3, padding=1)

    def forward(self, flow, corr):
        c = F.relu(_cv(self.convc1, corr))
        f = F.relu(_cv(self.convf2, F.relu(_cv(self.convf1, flow))))
        out = F.relu(_cv(self.conv, torch.cat([c, f], dim=1)))
        return torch.cat([out, flow.to(out.dtype)], dim=1)


class BasicMotionEncoder(nn.Module):
    def __init__(self, corr_planes):
        super().__init__()
        self.convc1 = nn.Conv2d(corr_planes, 256, 1, padding=0)
        self.convc2 = nn.Conv2d(256, 192, 3, padding=1)
        self.convf1 = nn.Conv2d(2, 128, 7, padding=3)
        self.convf2 = nn.Conv2d(128, 64, 3, padding=1)
        self.conv = nn.Conv2d(64 + 192, 128 - 2, 3, padding=1)

    def forward(self, flow, corr):
        c = F.relu(_cv(self.convc2, F.relu(_cv(self.convc1, corr))))
        f = F.relu(_cv(self.convf2, F.relu(_cv(self.convf1, flow))))
        out = F.relu(_cv(self.conv, torch.cat([c, f], dim=1)))
        return torch.cat([out, flow.to(out.dtype)], dim=1)


def _planes(cfg_or_args):
    levels = getattr(cfg_or_args, "corr_levels")
    radius = getattr(cfg_or_args, "corr_radius")
    return levels * (2 * radius + 1) ** 2


class SmallUpdateBlock(nn.Module):
    def __init__(self, args, hidden_dim=96):
        super().__init__()
        self.encoder = SmallMotionEncoder(_planes(args))
        self.gru = ConvGRU(hidden_dim=hidden_dim, input_dim=82 + 64)
        self.flow_head = FlowHead(hidden_dim, hidden_dim=128)

    def forward(self, net, inp, corr, flow):
        motion = self.encoder(flow, corr)
        net = self.gru(net, torch.cat([inp, motion], dim=1))
        return net, None, self.flow_head(net)


class BasicUpdateBlock(nn.Module):
    def __init__(self, args, hidden_dim=128, input_dim=128):
        super().__init__()
        self.args = args
        self.encoder = BasicMotionEncoder(_planes(args))
        self.gru = SepConvGRU(hidden_dim=hidden_dim, input_dim=128 + hidden_dim)
        self.flow_head = FlowHead(hidden_dim, hidden_dim=256)
        self.mask = nn.Sequential(
            nn.Conv2d(128, 256, 3, padding=1),
            nn.ReLU(inplace=True),
            nn.Conv2d(256, 64 * 9, 1, padding=0))

    def forward(self, net, inp, corr, flow, upsample=True):
        motion = self.encoder(flow, corr)
        net = self.gru(net, torch.cat([inp, motion], dim=1))
        delta = self.flow_head(net)
        # 0.25 scale balances the mask gradients (reference core/update.py:134)
        mask = 0.25 * _cv(self.mask[2], F.relu(_cv(self.mask[0], net))) if upsample else None
        return net, mask, delta
