"""Correlation ops: all-pairs volume + pyramid, window lookup, on-the-fly.

GPU tensors run the hand-written HIP kernels (csrc/corr_volume.hip,
csrc/corr_lookup.hip, csrc/corr_onthefly.hip); CPU tensors and export run
the ATen oracles of ops/reference.py.

Autograd design for the all-pairs path (training).  The reference
differentiates through ``grid_sample`` per level per iteration (a dense,
zero-filled pyramid gradient each time) and then through
``avg_pool2d`` and ``bmm``.  Here:

* :class:`_CorrVolume` builds the whole pyramid in one kernel and returns a
  0-d *token*; the pyramid itself lives in a :class:`CorrState` that the
  lookups read.
* every :class:`_CorrLookup` backward accumulates its cell gradients straight
  into ONE pyramid-shaped fp32 buffer owned by the state (own-row writes, no
  atomics) and returns a zero token gradient;
* when autograd reaches the volume node (after all lookups, by topology) it
  folds the pyramid gradient into level 0 (avg-pool backward + 1/sqrt(C)) and
  issues the two GEMMs  df1 = G f2,  df2 = G^T f1  once per step, both in one
  MFMA launch (csrc/corr_bwd.hip; split-bf16 operands for fp32 features).
"""
from __future__ import annotations

import math
from typing import List, Optional

import torch
import torch.nn.functional as F

from . import _ext
from . import reference as ref


class CorrState:
    __slots__ = ("pyr", "gpyr", "levels", "radius", "scale", "shape", "pyr_bf16", "feats", "early")

    def __init__(self, levels: int, radius: int, pyr_bf16: bool = False):
        self.pyr: Optional[List[torch.Tensor]] = None
        self.gpyr: Optional[List[torch.Tensor]] = None
        self.levels = levels
        self.radius = radius
        self.scale = 1.0
        self.shape = None
        self.pyr_bf16 = pyr_bf16  # bf16 pyramid storage (RAFTConfig.corr_dtype)
        self.feats = None  # (f1, f2) of the volume, for volume_backward ahead of autograd
        self.early = None  # (df1, df2) computed early by the training engine (see early_backward)

    def early_backward(self) -> bool:
        """Run the volume backward NOW (the fused training engine calls this on
        the main stream as soon as the last lookup backward is joined, before
        it issues the weight gradients): the fold and the feature-gradient
        GEMMs then run while the host issues the weight gradients, unpacks
        them and walks autograd, instead of after it (a 0.68 ms idle gap on
        the main queue, profiles/r6/train_streams_engine_s5.txt).  The
        volume node returns the stored result."""
        if self.gpyr is None or self.feats is None or self.early is not None:
            return False
        self.early = _volume_backward(self, *self.feats)
        return True

    def zero_grads(self) -> List[torch.Tensor]:
        """Dense fp32 gradient pyramid (contiguous rows), whatever the storage of pyr."""
        return [torch.zeros(p.shape, device=p.device, dtype=torch.float32) for p in self.pyr]


def to_nhwc(x: torch.Tensor) -> torch.Tensor:
    """(B,C,H,W) -> contiguous (B,H,W,C) (free when x is channels_last)."""
    return x.permute(0, 2, 3, 1).contiguous()


def from_nhwc(x: torch.Tensor) -> torch.Tensor:
    """contiguous (B,H,W,C) -> (B,C,H,W) view with channels_last strides."""
    return x.permute(0, 3, 1, 2)


def _fused_bwd_ok(gpyr, B, N1, H2, W2, C, bf16, f32) -> bool:
    """The preconditions of torch.ops.raft_stir.corr_volume_backward
    (csrc/ops.cpp), checked here so shapes it refuses (large batches or grids)
    take the fold + library-GEMM fallback instead of raising."""
    if C % 128 or not (bf16 or f32):
        return False
    Ep = -(-(H2 * W2) // 64) * 64  # csrc/corr_bwd.hip corr_bwd_pitch (BK = 64)
    coarse = sum(g.shape[2] * g.shape[3] for g in gpyr[1:])
    row_fold = Ep <= 6144 and coarse <= 4096  # csrc/corr_lookup.hip pyr_fold_rows_kernel
    g0 = gpyr[0]
    if not (row_fold or (bf16 and g0.stride(1) % 4 == 0 and g0.data_ptr() % 16 == 0)):
        return False
    return B * N1 * Ep * 2 < 2 ** 31 and B * max(N1, H2 * W2) * C * 2 < 2 ** 31


class _CorrVolume(torch.autograd.Function):
    @staticmethod
    def forward(ctx, f1, f2, state: CorrState):
        # f1: (B,N1,C), f2: (B,H2,W2,C) contiguous, fp32 or bf16
        state.scale = 1.0 / math.sqrt(f1.shape[-1])
        bf16 = state.pyr_bf16 and f1.dtype == torch.bfloat16
        state.pyr = list(torch.ops.raft_stir.corr_volume(f1, f2, state.levels, state.scale, bf16))
        state.shape = (f1.shape, f2.shape)
        state.feats = (f1, f2) if (ctx.needs_input_grad[0] or ctx.needs_input_grad[1]) else None
        state.early = None
        ctx.state = state
        ctx.save_for_backward(f1, f2)
        return f1.new_zeros((), dtype=torch.float32)

    @staticmethod
    def backward(ctx, _dtoken):
        state: CorrState = ctx.state
        f1, f2 = ctx.saved_tensors
        if state.early is not None:
            df1, df2 = state.early
        elif state.gpyr is None:
            return None, None, None
        else:
            df1, df2 = _volume_backward(state, f1, f2)
        state.gpyr = state.pyr = state.feats = state.early = None
        return df1, df2, None


def _volume_backward(state: CorrState, f1, f2):
    """(df1, df2) of the all-pairs volume from the gradient pyramid state.gpyr."""
    B, N1, C = f1.shape
    _, H2, W2, _ = f2.shape
    bf16 = f1.dtype == torch.bfloat16 and f2.dtype == torch.bfloat16
    f32 = f1.dtype == torch.float32 and f2.dtype == torch.float32
    if _fused_bwd_ok(state.gpyr, B, N1, H2, W2, C, bf16, f32):
        # csrc/corr_bwd.hip: one fold pass into a padded bf16 G, then both
        # feature-gradient GEMMs in one MFMA launch (deterministic); fp32
        # features: split-bf16 operands, three K passes, fp32 gradients
        df1, df2 = torch.ops.raft_stir.corr_volume_backward(state.gpyr, f1.contiguous(), f2.contiguous(),
                                                           state.scale)
    elif bf16:
        # other channel counts: bf16 library GEMMs on the folded gradient
        G = torch.empty(B, N1, H2 * W2, device=f1.device, dtype=torch.bfloat16)
        torch.ops.raft_stir.pyr_grad_fold_bf16(state.gpyr, state.scale, G)
        df1 = torch.bmm(G, f2.reshape(B, H2 * W2, C))
        df2 = torch.bmm(G.transpose(1, 2), f1)
    else:
        torch.ops.raft_stir.pyr_grad_fold(state.gpyr, state.scale)
        G = state.gpyr[0].view(B, N1, H2 * W2)
        df1 = torch.bmm(G, f2.reshape(B, H2 * W2, C).float())
        df2 = torch.bmm(G.transpose(1, 2), f1.float())
    return df1.to(f1.dtype), df2.view(B, H2, W2, C).to(f2.dtype)


class _CorrLookup(torch.autograd.Function):
    @staticmethod
    def forward(ctx, token, coords, state: CorrState, out_bf16: bool):
        ctx.state = state
        ctx.save_for_backward(coords)
        return torch.ops.raft_stir.corr_lookup(state.pyr, coords, state.radius, out_bf16)

    @staticmethod
    def backward(ctx, dout):
        state: CorrState = ctx.state
        (coords,) = ctx.saved_tensors
        if state.gpyr is None:
            state.gpyr = state.zero_grads()
        torch.ops.raft_stir.corr_lookup_backward(state.gpyr, coords, state.radius,
                                                 dout.contiguous())
        return coords.new_zeros(()), None, None, None


class AllPairsCorr:
    """All-pairs correlation pyramid + lookup (reference CorrBlock semantics).

    Built from NCHW (ideally channels_last) feature maps. ``__call__(coords)``
    returns (B, levels*(2r+1)^2, H, W); on GPU the result is a channels_last
    view in ``out_dtype``.
    """

    def __init__(self, fmap1, fmap2, num_levels=4, radius=4, out_dtype=torch.float32, pyr_dtype=torch.float32):
        self.num_levels = num_levels
        self.radius = radius
        self.out_dtype = out_dtype
        self.hip = _ext.use_hip(fmap1)
        if self.hip:
            f1 = to_nhwc(fmap1)
            B, H, W, C = f1.shape
            f2 = to_nhwc(fmap2.to(f1.dtype))
            if f1.dtype not in (torch.float32, torch.bfloat16):
                f1, f2 = f1.float(), f2.float()
            # bf16 pyramid storage needs bf16 feature maps (autocast); fp32 otherwise
            self.state = CorrState(num_levels, radius, pyr_bf16=pyr_dtype == torch.bfloat16)
            self.token = _CorrVolume.apply(f1.view(B, H * W, C), f2, self.state)
        else:
            self.pyramid = ref.corr_pyramid(fmap1, fmap2, num_levels)

    @property
    def corr_pyramid(self):
        if self.hip:
            B = self.state.shape[0][0]
            return [p.reshape(-1, 1, p.shape[2], p.shape[3]) for p in self.state.pyr]
        return self.pyramid

    def __call__(self, coords):
        if self.hip:
            out = _CorrLookup.apply(self.token, coords.float().contiguous(), self.state,
                                    self.out_dtype == torch.bfloat16)
            return from_nhwc(out)
        return ref.corr_lookup(self.pyramid, coords, self.radius).to(self.out_dtype)


class _CorrOTF(torch.autograd.Function):
    @staticmethod
    def forward(ctx, coords, radius, scale, out_bf16, f1, *f2s):
        ctx.radius, ctx.scale = radius, scale
        ctx.save_for_backward(coords, f1, *f2s)
        return torch.ops.raft_stir.corr_otf(f1, list(f2s), coords, radius, scale, out_bf16)

    @staticmethod
    def backward(ctx, dout):
        coords, f1, *f2s = ctx.saved_tensors
        grads = torch.ops.raft_stir.corr_otf_backward(f1, list(f2s), coords, ctx.radius,
                                                      ctx.scale, dout.contiguous())
        df1 = grads[0].to(f1.dtype)
        df2 = [g.to(f.dtype) for g, f in zip(grads[1:], f2s)]
        return (None, None, None, None, df1, *df2)


class OnTheFlyCorr:
    """Memory-efficient correlation (reference AlternateCorrBlock semantics,
    core/corr.py:63-91) -- O(HW*C) memory, recomputed every iteration, and
    (unlike the reference) differentiable."""

    def __init__(self, fmap1, fmap2, num_levels=4, radius=4, out_dtype=torch.float32):
        self.num_levels = num_levels
        self.radius = radius
        self.out_dtype = out_dtype
        self.hip = _ext.use_hip(fmap1)
        self.fmap1, self.fmap2 = fmap1, fmap2
        if self.hip:
            dt = torch.bfloat16 if fmap1.dtype == torch.bfloat16 else torch.float32
            f1 = fmap1.to(dt).contiguous(memory_format=torch.channels_last)
            f2 = fmap2.to(dt).contiguous(memory_format=torch.channels_last)
            levels = [f2]
            for _ in range(num_levels - 1):
                levels.append(F.avg_pool2d(levels[-1], 2, stride=2))
            self.f1 = to_nhwc(f1)
            self.f2s = [to_nhwc(t) for t in levels]
            self.scale = 1.0 / math.sqrt(fmap1.shape[1])

    def __call__(self, coords):
        if self.hip:
            out = _CorrOTF.apply(coords.float().contiguous(), self.radius, self.scale,
                                 self.out_dtype == torch.bfloat16, self.f1, *self.f2s)
            return from_nhwc(out)
        return ref.corr_onthefly(self.fmap1, self.fmap2, coords, self.radius,
                                 self.num_levels).to(self.out_dtype)
