"""Batched packing of the encoder conv weights for the HIP kernels.

The implicit-GEMM kernels read every weight in a packed bf16 layout
([Cout_pad][taps][Ktot], transposed / flipped / phase-split for the input
gradients).  ~50 such layouts exist for the two encoders.  Repacking each
one with its own permute / zero / copy / cast kernels after every optimizer
step is ~250 launches and ~2 ms of host time per training step; instead every
layout is registered once as a static INDEX MAP into the concatenation of
the source parameters (the layout function evaluated on an index tensor),
and all layouts live as views of ONE flat bf16 buffer.  A repack of
everything is then three kernels: cat(parameters) -> index_select -> cast
into the flat buffer.

Staleness: runtime/weights.generation() (bumped by every optimizer step --
fused AdamW does not bump ``_version``) plus the parameters' own version
counters.  Under ``runtime.weights.repack_in_graph()`` (a captured training
step) lookups never repack; the step body calls :func:`repack` itself so the
three kernels are part of every replay.
"""
from __future__ import annotations

import weakref
from typing import Callable, Dict, List, Sequence

import torch

from ..runtime import weights as _wgen


class _Entry:
    __slots__ = ("refs", "layout", "local_map", "shape", "view", "vers")

    def __init__(self, refs, layout, local_map, shape):
        self.refs = refs
        self.layout = layout
        self.local_map = local_map  # long, -1 = zero, else index into cat(weights of this entry)
        self.shape = shape
        self.view = None
        self.vers = None


class _Registry:
    def __init__(self, dev):
        self.dev = dev
        self.entries: Dict[tuple, _Entry] = {}
        self.srcs: List[weakref.ref] = []      # distinct source parameters, registration order
        self.src_ids: Dict[int, int] = {}
        self.flat = None
        self.gmap = None
        self.dirty = True
        self.gen = None
        self._retired = []  # flat buffers of earlier layouts (registration phase only)

    # ---------------------------------------------------------------- layout
    def _src_index(self, w):
        i = self.src_ids.get(id(w))
        if i is not None and self.srcs[i]() is w:
            return i
        self.srcs.append(weakref.ref(w))
        self.src_ids[id(w)] = len(self.srcs) - 1
        self.dirty = True
        return len(self.srcs) - 1

    def _rebuild(self, dev):
        """Flat buffer + global gather map over every live entry."""
        live = {k: e for k, e in self.entries.items() if all(r() is not None for r in e.refs)}
        self.entries = live
        # compact the source list to live parameters
        srcs = []
        ids = {}
        for e in live.values():
            for r in e.refs:
                w = r()
                if id(w) not in ids:
                    ids[id(w)] = len(srcs)
                    srcs.append(r)
        self.srcs, self.src_ids = srcs, ids
        offs, o = [], 0
        for r in srcs:
            offs.append(o)
            o += r().numel()
        zero = o  # the appended zero
        maps, n = [], 0
        for e in live.values():
            # local index space = cat(this entry's weights); translate to the global one
            lo, trans = 0, []
            for r in e.refs:
                w = r()
                trans.append((lo, lo + w.numel(), offs[ids[id(w)]]))
                lo += w.numel()
            lm = e.local_map
            g = torch.full_like(lm, zero)
            for a, b, go in trans:
                sel = (lm >= a) & (lm < b)
                g[sel] = lm[sel] - a + go
            maps.append(g)
            n += g.numel()
        self.gmap = torch.cat(maps).to(dev) if maps else torch.zeros(0, dtype=torch.long, device=dev)
        if self.flat is not None:  # earlier views may still be read by queued kernels on other streams
            self._retired.append(self.flat)
        self.flat = torch.empty(n, dtype=torch.bfloat16, device=dev)
        o = 0
        for e in live.values():
            k = e.local_map.numel()
            e.view = self.flat[o:o + k].view(e.shape)
            o += k
        self.dirty = False

    # ---------------------------------------------------------------- values
    @torch.no_grad()
    def repack(self):
        """Every registered layout from the current parameter values (3 kernels)."""
        STATS["repacks"] += 1
        # strong references for the whole repack: a cyclic GC pass triggered by
        # an allocation below must not free a parameter between the liveness
        # check and its use
        hold, live = [], {}
        for k, e in self.entries.items():
            ws_ = [r() for r in e.refs]
            if all(w is not None for w in ws_):
                live[k] = e
                hold.extend(ws_)
        if len(live) != len(self.entries):
            self.entries, self.dirty = live, True
        if not live:
            return
        dev = self.dev
        if self.dirty or self.flat is None:
            self._rebuild(dev)
        ws = [r() for r in self.srcs]
        src = torch.cat([w.detach().reshape(-1).float() for w in ws] + [torch.zeros(1, device=dev)])
        self.flat.copy_(src.index_select(0, self.gmap))
        gen = _wgen.generation()
        for e in self.entries.values():
            e.vers = tuple((r().data_ptr(), r()._version) for r in e.refs)
        self.gen = gen

    def get(self, key, weights: Sequence[torch.Tensor], layout: Callable) -> torch.Tensor:
        e = self.entries.get(key)
        if e is None or any(r() is not w for r, w in zip(e.refs, weights)) or len(e.refs) != len(weights):
            e = self._register(key, weights, layout)
        if _wgen.force_repack():  # captured training step: the body repacks explicitly
            return e.view
        vers = tuple((w.data_ptr(), w._version) for w in weights)
        if self.dirty or e.view is None or self.gen != _wgen.generation() or e.vers != vers:
            self.repack()
        return e.view

    @torch.no_grad()
    def _register(self, key, weights, layout):
        # index map: the layout evaluated on (local index + 1) so that the
        # layout's zero padding maps to -1
        n, idx = 0, []
        for w in weights:
            idx.append(torch.arange(n + 1, n + 1 + w.numel(), dtype=torch.float64).view(w.shape))
            n += w.numel()
        assert n < (1 << 24), "index map must be exact in fp32"
        lm = layout([t.float() for t in idx]).round().long() - 1
        e = _Entry(tuple(weakref.ref(w) for w in weights), layout, lm.reshape(-1).cpu(), tuple(lm.shape))
        self.entries[key] = e
        for w in weights:
            self._src_index(w)
        self.dirty = True
        return e


_REGS: Dict[torch.device, _Registry] = {}  # one per device
STATS = {"repacks": 0}  # tests / scripts: how often everything was repacked


def packed(key, weights: Sequence[torch.Tensor], layout: Callable) -> torch.Tensor:
    """The bf16 packed tensor ``layout(weights)`` (a view of the flat buffer),
    current with respect to every optimizer step / in-place write."""
    dev = weights[0].device
    reg = _REGS.get(dev)
    if reg is None:
        reg = _REGS[dev] = _Registry(dev)
    return reg.get(key, list(weights), layout)


def repack() -> None:
    for reg in _REGS.values():
        reg.repack()


def _stale(reg) -> bool:
    return reg.dirty or reg.gen != _wgen.generation() or any(
        e.vers != tuple((r().data_ptr(), r()._version) for r in e.refs)
        for e in reg.entries.values() if all(r() is not None for r in e.refs))


def refresh() -> None:
    """Repack if anything moved (start of every RAFT forward; GraphedInference
    before a replay).  Not recorded into an inference graph capture."""
    if _wgen.capturing() and not _wgen.force_repack():
        return
    for reg in _REGS.values():
        if reg.entries and _stale(reg):
            reg.repack()


_wgen.register_refresher(refresh)
