"""Deterministic training mode (bitwise-reproducible steps on one GPU).

The GPU engine is nondeterministic by default only where it accumulates with
fp32 atomics: the split-K weight / bias gradients of the update block and of
the encoder 3x3 convs (csrc/conv_wgrad.hip), the flow-encoder weight gradient
and the on-the-fly correlation backward.  ``set_deterministic(True)`` switches
the first two to per-split partial tiles (plain stores) reduced by a second
kernel in a fixed split order -- the same fp32 sums, one extra read of the
partials -- and makes the third refuse to run (train with the all-pairs
correlation).  It also asks MIOpen for deterministic convolution algorithms
(the encoder's strided / 1x1 convs) via ``torch.backends.cudnn``.

The encoder norm statistics accumulated in the conv epilogues (fp32 atomics)
are also switched off: deterministic mode keeps the two-level reduction.

Everything else on the training path is deterministic by construction:
norm statistics (per-block partials, fp64 finalize), the loss, the convex
upsampling backward (gather), the pyramid lookup backward (row-owned
read-modify-write), the correlation backward GEMMs, and RAFT-small's x8
upsampling adjoint (two matmuls, models/fused_train.py).

The reference has no such mode (its CUDA correlation backward and cuDNN
convolutions are nondeterministic).
"""
from __future__ import annotations

import contextlib

import torch

from ..ops import _ext


def set_deterministic(on: bool = True) -> None:
    on = bool(on)
    torch.backends.cudnn.deterministic = on
    if on:
        torch.backends.cudnn.benchmark = False
    if _ext.load():
        torch.ops.raft_stir.set_deterministic(on)


def is_deterministic() -> bool:
    if _ext.load():
        return bool(torch.ops.raft_stir.is_deterministic())
    return bool(torch.backends.cudnn.deterministic)


@contextlib.contextmanager
def deterministic(on: bool = True):
    prev = (is_deterministic(), torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark)
    set_deterministic(on)
    try:
        yield
    finally:
        if _ext.load():
            torch.ops.raft_stir.set_deterministic(prev[0])
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = prev[1], prev[2]
