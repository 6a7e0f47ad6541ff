"""Kernel-backed ops. GPU tensors run the in-tree HIP kernels (``_C.so``),
CPU tensors / tracing / export run the ATen references in ``reference.py``."""
from . import _ext, reference
from .corr import AllPairsCorr, OnTheFlyCorr, CorrState, to_nhwc, from_nhwc
from .upsample import convex_upsample, upflow8
from . import gru

__all__ = ["_ext", "reference", "AllPairsCorr", "OnTheFlyCorr", "CorrState", "to_nhwc",
           "from_nhwc", "convex_upsample", "upflow8", "gru"]
