"""Compatibility shim for reference core/update.py."""
import os as _os, sys as _sys
_ROOT = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
if _ROOT not in _sys.path:
    _sys.path.insert(0, _ROOT)

from raft_stir_amd.models.update import (BasicMotionEncoder, BasicUpdateBlock, ConvGRU,  # noqa: E402,F401
                                         FlowHead, SepConvGRU, SmallMotionEncoder,
                                         SmallUpdateBlock)
