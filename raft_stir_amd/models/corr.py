"""Correlation blocks with the reference's public API.

``CorrBlock(fmap1, fmap2, num_levels=4, radius=4)`` and
``AlternateCorrBlock(...)`` keep the constructor / ``__call__(coords)``
contract of reference core/corr.py:12-91; the work is done by
:mod:`raft_stir_amd.ops.corr` (MFMA GEMM + fused pyramid + HIP lookup on GPU,
ATen oracle on CPU).
"""
from __future__ import annotations

import torch

from ..ops.corr import AllPairsCorr, OnTheFlyCorr
from ..ops import reference as ref


class CorrBlock(AllPairsCorr):
    def __init__(self, fmap1, fmap2, num_levels=4, radius=4, out_dtype=torch.float32, pyr_dtype=torch.float32):
        super().__init__(fmap1, fmap2, num_levels=num_levels, radius=radius, out_dtype=out_dtype,
                         pyr_dtype=pyr_dtype)

    @staticmethod
    def corr(fmap1, fmap2):
        """(B, H, W, 1, H, W) all-pairs volume / sqrt(C) (reference core/corr.py:52-60)."""
        B, C, H, W = fmap1.shape
        return ref.corr_volume(fmap1, fmap2).view(B, H, W, 1, H, W)


class AlternateCorrBlock(OnTheFlyCorr):
    def __init__(self, fmap1, fmap2, num_levels=4, radius=4, out_dtype=torch.float32):
        super().__init__(fmap1, fmap2, num_levels=num_levels, radius=radius, out_dtype=out_dtype)
