"""Batched packing of the encoder conv weights for the HIP kernels.

The implicit-GEMM kernels read every weight in a packed bf16 layout
([Cout_pad][taps][Ktot], transposed / flipped / phase-split for the input
gradients).  ~50 such layouts exist for the two encoders.  Repacking each
one with its own permute / zero / copy / cast kernels after every optimizer
step is ~250 launches and ~2 ms of host time per training step; instead every
layout is registered once as a static INDEX MAP into the concatenation of
its source parameters (the layout function evaluated on an index tensor).

Layouts registered together live as views of one flat bf16 buffer (a
CHUNK); a repack of a chunk is three kernels: cat(parameters) ->
index_select -> cast into the flat buffer.  A chunk's storage never moves:
layouts registered later (a second model, a deep copy, re-registration of a
key) go into a NEW chunk, so a hipGraph captured against earlier views --
``GraphedInference`` or the repack recorded by ``GraphedTrainStep`` -- keeps
reading live, current storage (``snapshot()`` hands a captured graph strong
references to every chunk it recorded).  A chunk is dropped once every
parameter it was built from is gone.

Staleness: runtime/weights.generation() (bumped by every optimizer step --
fused AdamW does not bump ``_version``) plus the parameters' own version
counters.  Under ``runtime.weights.repack_in_graph()`` (a captured training
step) lookups never repack; the step body calls :func:`repack` itself so the
three kernels per chunk are part of every replay.
"""
from __future__ import annotations

import weakref
from typing import Callable, Dict, List, Sequence

import torch

from ..runtime import weights as _wgen


class _Entry:
    __slots__ = ("refs", "layout", "local_map", "shape", "view", "vers", "chunk")

    def __init__(self, refs, layout, local_map, shape):
        self.refs = refs
        self.layout = layout
        self.local_map = local_map  # long, -1 = zero, else index into cat(weights of this entry)
        self.shape = shape
        self.view = None
        self.vers = None
        self.chunk = None

    def alive(self) -> bool:
        return all(r() is not None for r in self.refs)


class _Chunk:
    """Entries packed together: one flat bf16 buffer, one gather map over
    cat(the chunk's own distinct source parameters) + a trailing zero."""

    def __init__(self, entries: List[_Entry], dev):
        srcs, ids = [], {}
        for e in entries:
            for r in e.refs:
                w = r()
                if id(w) not in ids:
                    ids[id(w)] = len(srcs)
                    srcs.append(r)
        offs, o = {}, 0
        for r in srcs:
            offs[id(r())] = o
            o += r().numel()
        zero = o
        maps, n = [], 0
        for e in entries:
            lo, trans = 0, []
            for r in e.refs:
                w = r()
                trans.append((lo, lo + w.numel(), offs[id(w)]))
                lo += w.numel()
            lm = e.local_map
            g = torch.full_like(lm, zero)
            for a, b, go in trans:
                sel = (lm >= a) & (lm < b)
                g[sel] = lm[sel] - a + go
            maps.append(g)
            n += g.numel()
        self.srcs = srcs
        self.numels = [r().numel() for r in srcs]
        self.entries = list(entries)
        self.gmap = torch.cat(maps).to(dev)
        self.flat = torch.empty(n, dtype=torch.bfloat16, device=dev)
        o = 0
        for e in entries:
            k = e.local_map.numel()
            e.view = self.flat[o:o + k].view(e.shape)
            e.chunk = self
            o += k

    def alive(self) -> bool:
        return any(e.alive() for e in self.entries)

    @torch.no_grad()
    def repack(self):
        dev = self.flat.device
        ws = [r() for r in self.srcs]
        # a source that died (another model of the chunk was freed) packs as zeros:
        # its layouts are unreachable, the live ones keep their offsets
        parts = [w.detach().reshape(-1).float() if w is not None else torch.zeros(n, device=dev)
                 for w, n in zip(ws, self.numels)]
        src = torch.cat(parts + [torch.zeros(1, device=dev)])
        self.flat.copy_(src.index_select(0, self.gmap))
        for e in self.entries:
            if e.alive():
                e.vers = tuple((r().data_ptr(), r()._version) for r in e.refs)


class _Registry:
    def __init__(self, dev):
        self.dev = dev
        self.entries: Dict[tuple, _Entry] = {}   # key -> current entry
        self.chunks: List[_Chunk] = []
        self.pending: List[_Entry] = []          # registered, not yet in a chunk
        self.gen = None

    # ---------------------------------------------------------------- layout
    def _flush(self):
        """Build a chunk for the pending entries; drop chunks whose sources died."""
        hold = []  # strong references across the allocations below (a GC pass must not free a source)
        for e in self.pending:
            hold.extend(r() for r in e.refs)
        live = [e for e in self.pending if e.alive()]
        self.pending = []
        self.chunks = [c for c in self.chunks if c.alive()]
        self.entries = {k: e for k, e in self.entries.items() if e.alive()}
        if live:
            self.chunks.append(_Chunk(live, self.dev))
        del hold

    # ---------------------------------------------------------------- values
    @torch.no_grad()
    def repack(self):
        """Every registered layout from the current parameter values (3 kernels per chunk)."""
        STATS["repacks"] += 1
        if self.pending:
            self._flush()
        for c in self.chunks:
            c.repack()
        self.gen = _wgen.generation()

    def get(self, key, weights: Sequence[torch.Tensor], layout: Callable) -> torch.Tensor:
        e = self.entries.get(key)
        if e is None or len(e.refs) != len(weights) or any(r() is not w for r, w in zip(e.refs, weights)):
            e = self._register(key, weights, layout)
        if _wgen.force_repack() and e.view is not None:  # captured training step: the body repacks explicitly
            return e.view
        vers = tuple((w.data_ptr(), w._version) for w in weights)
        if e.view is None or self.gen != _wgen.generation() or e.vers != vers:
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
        self.pending.append(e)
        return e

    def stale(self) -> bool:
        if self.pending or self.gen != _wgen.generation():
            return True
        return any(e.vers != tuple((r().data_ptr(), r()._version) for r in e.refs)
                   for e in self.entries.values() if e.alive())


_REGS: Dict[torch.device, _Registry] = {}  # one per device
STATS = {"repacks": 0}  # tests / scripts: how often everything was repacked


def packed(key, weights: Sequence[torch.Tensor], layout: Callable) -> torch.Tensor:
    """The bf16 packed tensor ``layout(weights)`` (a view of a chunk's flat
    buffer), current with respect to every optimizer step / in-place write."""
    dev = weights[0].device
    reg = _REGS.get(dev)
    if reg is None:
        reg = _REGS[dev] = _Registry(dev)
    return reg.get(key, list(weights), layout)


def repack() -> None:
    for reg in _REGS.values():
        reg.repack()


def snapshot() -> list:
    """Strong references to every chunk's storage and gather map: a hipGraph
    that recorded ``repack()`` keeps them for its whole life."""
    return [(c.flat, c.gmap, list(c.srcs)) for reg in _REGS.values() for c in reg.chunks]


def refresh() -> None:
    """Repack if anything moved (start of every RAFT forward; GraphedInference
    before a replay).  Not recorded into an inference graph capture."""
    if _wgen.capturing() and not _wgen.force_repack():
        return
    for reg in _REGS.values():
        if (reg.entries or reg.pending) and reg.stale():
            reg.repack()


_wgen.register_refresher(refresh)
