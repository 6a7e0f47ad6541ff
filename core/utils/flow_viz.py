"""Compatibility shim for reference core/utils/flow_viz.py."""
import os as _os, sys as _sys
_ROOT = _os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
if _ROOT not in _sys.path:
    _sys.path.insert(0, _ROOT)

from raft_stir_amd.utils.flow_viz import flow_to_image, flow_uv_to_colors, make_colorwheel  # noqa: E402,F401
