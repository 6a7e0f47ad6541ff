"""Weight-update generation counter for packed-weight caches.

The HIP convolution kernels read weights in packed bf16 layouts that are
cached per parameter (ops/enc_conv.py, models/fused_update.py, ops/gru.py).
A parameter's ``_version`` counter is NOT bumped by the fused / foreach
optimizer kernels (torch.optim.AdamW(fused=True) updates the storage in place
behind autograd's back), so a cache keyed on ``_version`` alone would keep
serving the weights of step 0.  Every torch optimizer step bumps this
process-wide generation (global optimizer step post-hook); caches key on
(generation, _version, data_ptr) and repack after any update.

hipGraphs: an inference graph replays the packed storage it was captured
with; GraphedInference refreshes the caches in place (``refresh_all``) before
a replay whenever the weights moved.  A captured TRAINING step contains its
own optimizer step, so its capture runs under ``repack_in_graph()``: the
packing kernels are recorded and re-run by every replay.
"""
from __future__ import annotations

import torch
from torch.optim.optimizer import register_optimizer_step_post_hook

_GEN = [0]


def generation() -> int:
    return _GEN[0]


def bump(*_args, **_kw) -> None:
    _GEN[0] += 1


def capturing() -> bool:
    try:
        return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
    except RuntimeError:
        return False


_FORCE = [False]
_REFRESHERS = []


def force_repack() -> bool:
    """True while a training-step hipGraph is being captured."""
    return _FORCE[0]


class repack_in_graph:
    def __enter__(self):
        self._prev = _FORCE[0]
        _FORCE[0] = True

    def __exit__(self, *exc):
        _FORCE[0] = self._prev


def register_refresher(fn) -> None:
    """``fn()`` re-packs a cache's stale entries into their existing storage."""
    _REFRESHERS.append(fn)


def refresh_all(model=None) -> None:
    for fn in _REFRESHERS:
        fn()
    if model is not None:
        eng = model.__dict__.get("_fused")
        if eng is not None:
            eng.refresh()


def weights_key(model) -> tuple:
    return (generation(),) + tuple((p.data_ptr(), p._version) for p in model.parameters())


_HANDLE = register_optimizer_step_post_hook(bump)
