"""Model configuration.

The reference configures RAFT through an ``argparse.Namespace`` that the model
mutates in place (reference core/raft.py:29-45: ``corr_levels``/``corr_radius``
are written into ``args``; ``dropout``/``alternate_corr`` default when absent).
We keep that contract (``RAFT(args)`` accepts any Namespace-like object and
fills the same attributes) but resolve it once into an immutable
:class:`RAFTConfig` that the rest of the engine reads.
"""
from __future__ import annotations

import argparse
import os
from dataclasses import dataclass, asdict


@dataclass(frozen=True)
class RAFTConfig:
    small: bool = False
    mixed_precision: bool = False      # bf16 autocast on MI355X (reference: fp16 AMP)
    alternate_corr: bool = False       # on-the-fly correlation (alt_cuda_corr path)
    dropout: float = 0.0
    corr_levels: int = 4
    corr_radius: int = 4
    hidden_dim: int = 128
    context_dim: int = 128
    fnet_dim: int = 256
    # engine knobs (not in the reference): kernel choices for the GPU path
    fused_gru: bool = True             # fused HIP gate kernels in the ConvGRU
    fused_train: bool = True           # whole-loop fused training engine (RAFT / RAFT-small, bf16 or fp32)
    overlap_encoders: bool = True      # context encoder on a second HIP stream (GPU)
    # storage dtype of the all-pairs pyramid: "float32" (reference, core/corr.py:58),
    # "bfloat16" (half the volume bytes; needs bf16 autocast features), or "auto"
    # (bf16 storage exactly when mixed_precision)
    corr_dtype: str = "float32"
    # bitwise-reproducible GPU training steps (runtime/determinism.py)
    deterministic: bool = False

    @property
    def pyr_dtype(self):
        import torch
        bf = self.corr_dtype in ("bfloat16", "bf16") or (self.corr_dtype == "auto" and self.mixed_precision)
        return torch.bfloat16 if bf else torch.float32

    @property
    def corr_planes(self) -> int:
        return self.corr_levels * (2 * self.corr_radius + 1) ** 2

    def to_dict(self):
        return asdict(self)


def _get(args, name, default):
    if args is None:
        return default
    if isinstance(args, dict):
        return args.get(name, default)
    # Namespace supports ``in`` (reference relies on it: core/raft.py:41)
    try:
        if name in args:
            return getattr(args, name)
        return default
    except TypeError:
        return getattr(args, name, default)


def resolve_config(args=None, **overrides) -> RAFTConfig:
    """Build a RAFTConfig from a Namespace/dict and mutate the Namespace the
    way the reference does so downstream reference-style code keeps working."""
    small = bool(overrides.pop("small", _get(args, "small", False)))
    if small:
        dims = dict(hidden_dim=96, context_dim=64, fnet_dim=128, corr_radius=3)
    else:
        dims = dict(hidden_dim=128, context_dim=128, fnet_dim=256, corr_radius=4)
    cfg = dict(
        small=small,
        mixed_precision=bool(_get(args, "mixed_precision", False)),
        alternate_corr=bool(_get(args, "alternate_corr", False)),
        dropout=float(_get(args, "dropout", 0.0) or 0.0),
        corr_levels=4,
        fused_gru=bool(_get(args, "fused_gru", True)),
        fused_train=bool(_get(args, "fused_train", True)),
        overlap_encoders=bool(_get(args, "overlap_encoders", os.environ.get("RS_OVERLAP_ENCODERS", "1") != "0")),
        corr_dtype=str(_get(args, "corr_dtype", os.environ.get("RS_CORR_DTYPE", "float32"))),
        deterministic=bool(_get(args, "deterministic", False)),
        **dims,
    )
    cfg.update(overrides)
    conf = RAFTConfig(**cfg)
    if isinstance(args, argparse.Namespace):
        args.corr_levels = conf.corr_levels
        args.corr_radius = conf.corr_radius
        if "dropout" not in args:
            args.dropout = 0
        if "alternate_corr" not in args:
            args.alternate_corr = False
        if "mixed_precision" not in args:
            args.mixed_precision = False
    return conf


def make_args(**kw) -> argparse.Namespace:
    """Convenience: a reference-style Namespace (small/mixed_precision/...)."""
    base = dict(small=False, mixed_precision=False, alternate_corr=False, dropout=0.0)
    base.update(kw)
    return argparse.Namespace(**base)
