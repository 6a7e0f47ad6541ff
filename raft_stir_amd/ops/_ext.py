"""Loader for the in-tree HIP extension (``raft_stir_amd/_C.so``).

The extension registers its kernels as ``torch.ops.raft_stir.*`` through
``TORCH_LIBRARY`` (csrc/ops.cpp); no pybind module is involved. It is built
in-tree by :mod:`raft_stir_amd.build` (``hipcc --offload-arch=gfx950``) so the
``.so`` travels with the repository snapshot to the GPU box.

Policy: CPU tensors use the ATen reference path (ops/reference.py). GPU tensors
REQUIRE the extension: if it is missing we raise instead of silently falling
back, so a GPU run can never pass on an eager fallback unnoticed.
"""
from __future__ import annotations

import os
import threading

import torch

_LOCK = threading.Lock()
_LOADED = None
_ERROR = None

LIB_NAME = "_C.so"
PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def library_path() -> str:
    return os.path.join(PKG_DIR, LIB_NAME)


def load(raise_on_error: bool = False) -> bool:
    global _LOADED, _ERROR
    if _LOADED is not None:
        if raise_on_error and not _LOADED:
            raise RuntimeError(f"raft_stir_amd HIP extension unavailable: {_ERROR}")
        return _LOADED
    with _LOCK:
        if _LOADED is None:
            path = library_path()
            if os.environ.get("RAFT_STIR_NO_EXT") == "1":
                _LOADED, _ERROR = False, "disabled by RAFT_STIR_NO_EXT=1"
            elif not os.path.exists(path):
                _LOADED, _ERROR = False, f"{path} not built (run python -m raft_stir_amd.build)"
            else:
                try:
                    torch.ops.load_library(path)
                    _LOADED = True
                    if os.environ.get("RS_NORM_REDUCE_BLOCKS"):  # in-situ A/B knob (csrc/norm.hip)
                        torch.ops.raft_stir.norm_set_reduce_blocks(int(os.environ["RS_NORM_REDUCE_BLOCKS"]))
                except Exception as e:  # pragma: no cover - depends on box
                    _LOADED, _ERROR = False, repr(e)
    if raise_on_error and not _LOADED:
        raise RuntimeError(f"raft_stir_amd HIP extension unavailable: {_ERROR}")
    return _LOADED


def ops():
    load(raise_on_error=True)
    return torch.ops.raft_stir


def error() -> str | None:
    load()
    return _ERROR


def use_hip(*tensors) -> bool:
    """True when the HIP kernels must be used for these tensors.

    GPU tensors always take the HIP path (raising if the extension is missing);
    tracing/export always takes the ATen path so exported graphs hold only
    standard ops.
    """
    dev = None
    for t in tensors:
        if isinstance(t, torch.Tensor):
            dev = t.device
            break
    if dev is None or dev.type != "cuda" or _exporting():
        return False
    if not _LOADED:
        load(raise_on_error=True)
    return True


try:  # bound once: called for every op dispatch on the hot path
    _onnx_exporting = torch.onnx.is_in_onnx_export
except Exception:  # pragma: no cover - onnx namespace unavailable
    _onnx_exporting = lambda: False  # noqa: E731


def _exporting() -> bool:
    if _FORCE_REFERENCE[0] or torch.jit.is_tracing() or torch.jit.is_scripting():
        return True
    try:
        return bool(_onnx_exporting())
    except Exception:
        return False


_FORCE_REFERENCE = [False]


class reference_mode:
    """Context manager forcing the ATen reference path (export, A/B tests)."""

    def __enter__(self):
        self._prev = _FORCE_REFERENCE[0]
        _FORCE_REFERENCE[0] = True
        return self

    def __exit__(self, *exc):
        _FORCE_REFERENCE[0] = self._prev
        return False
