"""Feature and context encoders (1/8 resolution).

Behavioural parity with reference core/extractor.py:
  * BasicEncoder (full RAFT, core/extractor.py:118-192): 7x7/s2 stem -> 64ch,
    three stages of two residual blocks (64, 96/s2, 128/s2), 1x1 projection.
  * SmallEncoder (RAFT-small, core/extractor.py:195-267): 7x7/s2 stem -> 32ch,
    bottleneck stages (32, 64/s2, 96/s2), 1x1 projection.
  * A list/tuple input is run as one concatenated batch and split back
    (core/extractor.py:170-190), which matters for instance norm only in that
    it is per-sample (identical to two separate calls).

Parameter/buffer names are kept identical so reference ``.pth`` files load
unchanged (including the aliased ``normK`` / ``downsample.1`` pair that the
reference creates by registering the same norm module twice).

MI355X notes: the encoders run once per image pair; on the GPU bf16 path
their 3x3 (stride 1 and 2) and 1x1 convolutions run on the hand-written
implicit-GEMM kernels (ops/enc_conv.py; fp32 -- inference and training -- on
the split-bf16 F32 tiles; the 7x7 stem runs on csrc/stem.hip, forward and
weight gradient; RAFT-small's narrow bottleneck convs run on csrc/sconv.hip
and csrc/sconv_train.hip), and every
norm -> ReLU (-> residual add -> ReLU) chain is one fused NHWC pass of
csrc/norm.hip (ops/norm.py) instead of PyTorch's instance_norm, which would
copy each channels_last map to NCHW and back.  NHWC also keeps the 1x1
projection's output directly usable as the K-contiguous operand of the
correlation MFMA GEMM (csrc/corr_volume.hip).
"""
from __future__ import annotations


import torch
import torch.nn as nn

from ..ops import enc_conv
from ..ops.fp32conv import conv_module
from ..ops.norm import conv_norm_act, conv_pair_norm_act


# the residual blocks' skip gradient is added in the first conv's
# input-gradient epilogue (ops/enc_conv.py GradSink) instead of a separate add
_RES_SINK = True


def make_norm(kind: str, channels: int, groups: int) -> nn.Module:
    table = {
        "group": lambda: nn.GroupNorm(num_groups=groups, num_channels=channels),
        "batch": lambda: nn.BatchNorm2d(channels),
        "instance": lambda: nn.InstanceNorm2d(channels),
        "none": lambda: nn.Sequential(),
    }
    if kind not in table:
        raise ValueError(f"unknown norm_fn {kind!r}")
    return table[kind]()


class ResidualBlock(nn.Module):
    """Two 3x3 convs + norm/ReLU with identity or strided 1x1 shortcut."""

    def __init__(self, in_planes, planes, norm_fn="group", stride=1):
        super().__init__()
        g = planes // 8
        self.conv1 = nn.Conv2d(in_planes, planes, 3, padding=1, stride=stride)
        self.conv2 = nn.Conv2d(planes, planes, 3, padding=1)
        self.relu = nn.ReLU(inplace=True)
        self.norm1 = make_norm(norm_fn, planes, g)
        self.norm2 = make_norm(norm_fn, planes, g)
        self.downsample = None
        if stride != 1:
            self.norm3 = make_norm(norm_fn, planes, g)
            self.downsample = nn.Sequential(
                nn.Conv2d(in_planes, planes, 1, stride=stride), self.norm3)

    def forward(self, x):
        sink = None
        if self.downsample is None:
            # the skip gradient goes straight into conv1's input-gradient epilogue
            sink = enc_conv.GradSink() if (x.is_cuda and _RES_SINK) else None
            y, skip = conv_norm_act(self.conv1, self.norm1, x, grad_sink=sink), x
        else:
            y, skip = conv_pair_norm_act(self.conv1, self.norm1, self.downsample[0], self.norm3, x)
        # relu(skip + relu(norm2(conv2(y)))) as one fused pass on GPU
        return conv_norm_act(self.conv2, self.norm2, y, relu=True, residual=skip, res_sink=sink)


class BottleneckBlock(nn.Module):
    """1x1 reduce (planes/4) -> 3x3 (stride) -> 1x1 expand, with shortcut."""

    def __init__(self, in_planes, planes, norm_fn="group", stride=1):
        super().__init__()
        q = planes // 4
        g = planes // 8
        self.conv1 = nn.Conv2d(in_planes, q, 1, padding=0)
        self.conv2 = nn.Conv2d(q, q, 3, padding=1, stride=stride)
        self.conv3 = nn.Conv2d(q, planes, 1, padding=0)
        self.relu = nn.ReLU(inplace=True)
        self.norm1 = make_norm(norm_fn, q, g)
        self.norm2 = make_norm(norm_fn, q, g)
        self.norm3 = make_norm(norm_fn, planes, g)
        self.downsample = None
        if stride != 1:
            self.norm4 = make_norm(norm_fn, planes, g)
            self.downsample = nn.Sequential(
                nn.Conv2d(in_planes, planes, 1, stride=stride), self.norm4)

    def forward(self, x):
        y = conv_norm_act(self.conv1, self.norm1, x)
        y = conv_norm_act(self.conv2, self.norm2, y)
        skip = x if self.downsample is None else conv_norm_act(self.downsample[0], self.norm4, x, relu=False)
        return conv_norm_act(self.conv3, self.norm3, y, relu=True, residual=skip)


class _Encoder(nn.Module):
    """Shared stem/stage/projection skeleton for both encoder sizes."""

    block_cls = ResidualBlock
    stem_dim = 64
    stage_dims = (64, 96, 128)
    hip_geo = True  # strided / 1x1 convs on the HIP kernels (ops/enc_conv.py geo_scope)

    def __init__(self, output_dim=128, norm_fn="batch", dropout=0.0):
        super().__init__()
        self.norm_fn = norm_fn
        self.norm1 = make_norm(norm_fn, self.stem_dim, 8)
        self.conv1 = nn.Conv2d(3, self.stem_dim, kernel_size=7, stride=2, padding=3)
        self.relu1 = nn.ReLU(inplace=True)
        self.in_planes = self.stem_dim
        d1, d2, d3 = self.stage_dims
        self.layer1 = self._stage(d1, 1)
        self.layer2 = self._stage(d2, 2)
        self.layer3 = self._stage(d3, 2)
        self._build_head(d3, output_dim, dropout)
        self._init_weights()

    def _build_head(self, in_dim, output_dim, dropout):
        raise NotImplementedError

    def _stage(self, dim, stride):
        first = self.block_cls(self.in_planes, dim, self.norm_fn, stride=stride)
        second = self.block_cls(dim, dim, self.norm_fn, stride=1)
        self.in_planes = dim
        return nn.Sequential(first, second)

    def _init_weights(self):
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.InstanceNorm2d, nn.GroupNorm)):
                if m.weight is not None:
                    nn.init.constant_(m.weight, 1)
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)

    def stage_fns(self):
        """The forward as a list of callables: stem, each residual block, head.
        RAFT.forward runs two encoders stage-by-stage in lockstep on two HIP
        streams, so the HOST issues both chains interleaved -- and, because
        autograd replays nodes by creation order, so does the backward (a
        whole encoder issued first left the other stream idle for its ~2 ms
        of host issue time, profiles/r2/train_streams.txt)."""
        fns = [lambda x: conv_norm_act(self.conv1, self.norm1, x)]
        for layer in (self.layer1, self.layer2, self.layer3):
            fns.extend(layer)
        if not self.hip_geo:
            fns = [self._no_geo(f) for f in fns]

        def head(x):
            x = self._head_conv(x)
            if self.training and self.dropout is not None:
                x = self.dropout(x)
            return x
        fns.append(head if self.hip_geo else self._no_geo(head))
        return fns

    @staticmethod
    def _no_geo(fn):
        def run(x):
            with enc_conv.geo_scope(False):
                return fn(x)
        return run

    def _head_conv(self, x):
        """1x1 projection (with bias): HIP implicit GEMM on the GPU bf16 path
        and on the split-bf16 F32 tiles for fp32 inference."""
        if enc_conv.eligible_f32(self.conv2, x):
            return enc_conv.conv_f32(self.conv2, x)
        if enc_conv.eligible_f32_train(self.conv2, x):  # fp32 training (split-bf16 F32 tiles)
            return enc_conv.conv_f32_train(self.conv2, x)
        if not self.hip_geo and enc_conv.sconv_eligible(self.conv2, x):  # RAFT-small inference
            return enc_conv.sconv(self.conv2, x)
        if not self.hip_geo and enc_conv.sconv_train_eligible(self.conv2, x):  # RAFT-small training
            return enc_conv.sconv_train(self.conv2, x)
        if enc_conv.eligible_geo(self.conv2, x):
            return enc_conv.conv_geo(self.conv2, x)
        return conv_module(self.conv2, x)

    def forward(self, x):
        pair = isinstance(x, (list, tuple))
        if pair:
            n = x[0].shape[0]
            x = torch.cat(list(x), dim=0)
        with enc_conv.geo_scope(self.hip_geo):
            x = conv_norm_act(self.conv1, self.norm1, x)
            x = self.layer3(self.layer2(self.layer1(x)))
            x = self._head_conv(x)
        if self.training and self.dropout is not None:
            x = self.dropout(x)
        if pair:
            return torch.split(x, [n, n], dim=0)
        return x


class BasicEncoder(_Encoder):
    block_cls = ResidualBlock
    stem_dim = 64
    stage_dims = (64, 96, 128)

    def _build_head(self, in_dim, output_dim, dropout):
        self.conv2 = nn.Conv2d(in_dim, output_dim, kernel_size=1)
        self.dropout = nn.Dropout2d(p=dropout) if dropout > 0 else None


class SmallEncoder(_Encoder):
    block_cls = BottleneckBlock
    stem_dim = 32
    stage_dims = (32, 64, 96)
    hip_geo = False

    def _build_head(self, in_dim, output_dim, dropout):
        self.dropout = nn.Dropout2d(p=dropout) if dropout > 0 else None
        self.conv2 = nn.Conv2d(in_dim, output_dim, kernel_size=1)
