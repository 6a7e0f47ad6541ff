"""Compatibility shim for reference core/utils/utils.py."""
import os as _os, sys as _sys
_ROOT = _os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
if _ROOT not in _sys.path:
    _sys.path.insert(0, _ROOT)

from raft_stir_amd.utils.geometry import (bilinear_sampler, coords_grid,  # noqa: E402,F401
                                          forward_interpolate, upflow8)
from raft_stir_amd.utils.padder import InputPadder  # noqa: E402,F401
