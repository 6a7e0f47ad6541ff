"""Batched packing of the encoder conv weights for the HIP kernels.

The implicit-GEMM kernels read every weight in a packed bf16 layout
([Cout_pad][taps][Ktot], transposed / flipped / phase-split for the input
gradients).  ~50 such layouts exist for the two encoders.  Repacking each
one with its own permute / zero / copy / cast kernels after every optimizer
step is ~250 launches and ~2 ms of host time per training step; instead every
layout is registered once as a static INDEX MAP into the concatenation of
its source parameters (the layout function evaluated on an index tensor).

Layouts registered together live as views of a CHUNK, a contiguous region
of an ARENA: one flat bf16 buffer plus one int32 code per element (source
row << 24 | index into that source).  A repack is ONE gather launch per arena
(csrc/wpack.hip) that reads the parameters in place with their own strides
and casts.  Storage never moves: layouts registered later (a second model, a
deep copy, re-registration of a key) go into a NEW chunk appended to the
arena (or a new arena), so a hipGraph captured against earlier views --
``GraphedInference`` or the repack recorded by ``GraphedTrainStep`` -- keeps
reading live, current storage (``snapshot()`` hands a captured graph strong
references to every chunk it recorded).  A chunk is dropped once every
parameter it was built from is gone.

Staleness: runtime/weights.generation() (bumped by every optimizer step --
fused AdamW does not bump ``_version``) plus the parameters' own version
counters.  Under ``runtime.weights.repack_in_graph()`` (a captured training
step) lookups never repack; the step body calls :func:`repack` itself so the
gather launches are part of every replay.
"""
from __future__ import annotations

import weakref
from typing import Callable, Dict, List, Sequence

import torch

from . import _ext
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


_MAX_SRC = 63           # source rows per arena (code = lo << 30 | src << 24 | index)
_LOF = 1 << 40          # index-map flag: the element is lo = bf16(w - bf16(w)) (split layouts)
_ARENA_MIN = 1 << 23    # packed elements per arena (bf16 flat + int32 codes: 48 MiB)


class _Arena:
    """Consecutive chunks in one flat bf16 buffer with one int32 code per
    element (source row << 24 | logical index into that source, -1 = zero)
    over the arena's source table: a repack of the whole arena is ONE gather
    launch (csrc/wpack.hip) reading the parameters in place -- their own
    strides, channels_last included.  Storage never moves or shrinks."""

    def __init__(self, dev, cap):
        self.dev = dev
        self.cap = cap
        self.flat = torch.zeros(cap, dtype=torch.bfloat16, device=dev)
        self.code = torch.full((cap,), -1, dtype=torch.int32, device=dev)
        self.used = 0
        self.srcs = []      # weakrefs, row order of the source table
        self.numels = []    # element counts of the sources (dead ones pack as zeros)
        self.sid = {}       # id(param) -> row
        self.tab = None     # device int64 [rows][10]
        self.tab_key = None
        self.hip = dev.type == "cuda"
        self.gmap = None    # CPU fallback: index into cat(sources) + zero, int64 [used]

    def fits(self, n, refs) -> bool:
        new = len({id(r()) for r in refs
                   if id(r()) not in self.sid or self.srcs[self.sid[id(r())]]() is not r()})
        return self.used + n <= self.cap and len(self.srcs) + new <= _MAX_SRC

    def add(self, entries) -> int:
        """Append the entries' codes; returns the chunk offset."""
        codes = []
        for e in entries:
            lo, trans = 0, []
            for r in e.refs:
                w = r()
                row = self.sid.get(id(w))
                if row is None or self.srcs[row]() is not w:  # new source (or a dead one's reused id)
                    self.sid[id(w)] = len(self.srcs)
                    self.srcs.append(r)
                    self.numels.append(w.numel())
                trans.append((lo, lo + w.numel(), self.sid[id(w)]))
                lo += w.numel()
            lm = e.local_map
            lo = lm >= _LOF
            base = torch.where(lo, lm - _LOF, lm)
            c = torch.full_like(lm, -1)
            for a, b, row in trans:
                sel = (base >= a) & (base < b)
                c[sel] = (base[sel] - a) | (row << 24) | (lo[sel].long() << 30)
            codes.append(c)
        code = torch.cat(codes).to(torch.int32)
        off = self.used
        self.code[off:off + code.numel()].copy_(code.to(self.dev))
        self.used += code.numel()
        self.gmap = None
        return off

    def _table(self):
        ws = [r() for r in self.srcs]
        key = tuple(None if w is None else (w.data_ptr(), w.dtype, tuple(w.shape), w.stride()) for w in ws)
        if key != self.tab_key:
            rows = []
            for w in ws:
                if w is None or w.dim() > 4 or w.dtype not in (torch.float32, torch.bfloat16):
                    rows.append([0] * 10)
                    continue
                pad = 4 - w.dim()
                rows.append([w.data_ptr(), int(w.dtype == torch.bfloat16)] + [1] * pad + list(w.shape)
                            + [0] * pad + list(w.stride()))
            self.tab = torch.tensor(rows or [[0] * 10], dtype=torch.int64).to(self.dev)
            self.tab_key = key
        return self.tab

    @torch.no_grad()
    def repack(self):
        if self.used == 0:
            return
        if self.hip and _ext.use_hip(self.flat):
            torch.ops.raft_stir.wpack_gather(self.code[:self.used], self._table(), self.flat[:self.used],
                                             [], [], [])
            return
        # reference path (CPU): cat(sources) + zero, gathered by the decoded codes
        ws = [r() for r in self.srcs]
        numels = list(self.numels)
        if self.gmap is None or self.gmap[1] != numels:
            offs, o = [], 0
            for n in numels:
                offs.append(o)
                o += n
            code = self.code[:self.used].long().cpu()
            row, li = (code >> 24) & 63, code & 0xffffff
            g = torch.full_like(code, o)
            ok = code >= 0
            g[ok] = torch.tensor(offs, dtype=torch.long)[row[ok]] + li[ok]
            lo = ok & ((code >> 30) & 1).bool()
            self.gmap = (g.to(self.dev), numels, lo.to(self.dev) if lo.any() else None)
        parts = [w.detach().reshape(-1).float() if w is not None else torch.zeros(n, device=self.dev)
                 for w, n in zip(ws, numels)]
        src = torch.cat(parts + [torch.zeros(1, device=self.dev)])
        v = src.index_select(0, self.gmap[0])
        if self.gmap[2] is not None:
            v = torch.where(self.gmap[2], v - v.to(torch.bfloat16).float(), v)
        self.flat[:self.used].copy_(v)


class _Chunk:
    """Entries registered together: a contiguous region of an arena."""

    def __init__(self, entries: List[_Entry], arena: _Arena):
        self.arena = arena
        self.entries = list(entries)
        n = sum(e.local_map.numel() for e in entries)
        o = arena.add(entries)
        self.flat = arena.flat[o:o + n]
        for e in entries:
            k = e.local_map.numel()
            e.view = arena.flat[o:o + k].view(e.shape)
            e.chunk = self
            o += k

    def alive(self) -> bool:
        return any(e.alive() for e in self.entries)

    def mark_packed(self):
        for e in self.entries:
            if e.alive():
                e.vers = tuple((r().data_ptr(), r()._version) for r in e.refs)


class _Registry:
    def __init__(self, dev):
        self.dev = dev
        self.entries: Dict[tuple, _Entry] = {}   # key -> current entry
        self.chunks: List[_Chunk] = []
        self.arenas: List[_Arena] = []
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
            n = sum(e.local_map.numel() for e in live)
            refs = [r for e in live for r in e.refs]
            arena = self.arenas[-1] if self.arenas else None
            if arena is None or not arena.fits(n, refs):
                arena = _Arena(self.dev, max(n, _ARENA_MIN))
                self.arenas.append(arena)
            self.chunks.append(_Chunk(live, arena))
        live_arenas = {id(c.arena) for c in self.chunks}
        self.arenas = [a for a in self.arenas if id(a) in live_arenas or a is self.arenas[-1]]
        del hold

    # ---------------------------------------------------------------- values
    @torch.no_grad()
    def repack(self):
        """Every registered layout from the current parameter values (one
        gather launch per arena)."""
        STATS["repacks"] += 1
        if self.pending:
            self._flush()
        for a in {id(c.arena): c.arena for c in self.chunks}.values():
            a.repack()
        for c in self.chunks:
            c.mark_packed()
        self.gen = _wgen.generation()

    def get(self, key, weights: Sequence[torch.Tensor], layout: Callable, split: bool = False) -> torch.Tensor:
        e = self.entries.get(key)
        if e is None or len(e.refs) != len(weights) or any(r() is not w for r, w in zip(e.refs, weights)):
            e = self._register(key, weights, layout, split)
        if _wgen.force_repack() and e.view is not None:  # captured training step: the body repacks explicitly
            return e.view
        vers = tuple((w.data_ptr(), w._version) for w in weights)
        if e.view is None or self.gen != _wgen.generation() or e.vers != vers:
            self.repack()
        return e.view

    @torch.no_grad()
    def _register(self, key, weights, layout, split=False):
        # index map: the layout evaluated on (local index + 1) so that the
        # layout's zero padding maps to -1
        n, idx = 0, []
        for w in weights:
            idx.append(torch.arange(n + 1, n + 1 + w.numel(), dtype=torch.float64).view(w.shape))
            n += w.numel()
        assert n < (1 << 24), "index map must be exact in fp32"
        lm = layout([t.float() for t in idx]).round().long() - 1
        if split:  # [.., K] -> [.., 2K]: per 32-wide K chunk [w_hi 32 | w_lo 32] (ops/conv.py split_weight)
            *lead, k = lm.shape
            assert k % 32 == 0
            m = lm.reshape(*lead, k // 32, 1, 32)
            lm = torch.cat([m, torch.where(m >= 0, m + _LOF, m)], -2).reshape(*lead, 2 * k)
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


def packed_split(key, weights: Sequence[torch.Tensor], layout: Callable) -> torch.Tensor:
    """:func:`packed` of an fp32-style layout in the split [wh | wl] form of
    the F32 conv tiles (per 32-wide K chunk, wl = bf16(w - bf16(w)))."""
    dev = weights[0].device
    reg = _REGS.get(dev)
    if reg is None:
        reg = _REGS[dev] = _Registry(dev)
    return reg.get(("split",) + tuple(key), list(weights), layout, True)


def repack() -> None:
    for reg in _REGS.values():
        reg.repack()


def snapshot() -> list:
    """Strong references to every arena's storage, codes and source table: a
    hipGraph that recorded ``repack()`` keeps them for its whole life."""
    out = []
    for reg in _REGS.values():
        for a in {id(c.arena): c.arena for c in reg.chunks}.values():
            out.append((a.flat, a.code, a._table(), list(a.srcs)))
    return out


def refresh() -> None:
    """Repack if anything moved (start of every RAFT forward; GraphedInference
    before a replay).  Not recorded into an inference graph capture."""
    if _wgen.capturing() and not _wgen.force_repack():
        return
    for reg in _REGS.values():
        if (reg.entries or reg.pending) and reg.stale():
            reg.repack()


_wgen.register_refresher(refresh)
