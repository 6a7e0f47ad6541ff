"""Compatibility shim: ``core.raft.RAFT`` / ``from raft import RAFT`` (reference core/raft.py)."""
import os as _os, sys as _sys
_ROOT = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
if _ROOT not in _sys.path:
    _sys.path.insert(0, _ROOT)

from raft_stir_amd.models.raft import RAFT  # noqa: E402,F401

__all__ = ["RAFT"]
