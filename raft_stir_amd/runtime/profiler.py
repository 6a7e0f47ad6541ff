"""Lightweight tracing for the engine (the reference has none).

* :class:`PhaseTimer` -- named phases timed with HIP events on the current
  stream (no host sync until :meth:`summary`), optionally wrapped in roctx
  ranges (``torch.cuda.nvtx`` is roctx on ROCm) so they show up as regions
  in ``rocprofv3 --marker-trace`` / ``--sys-trace`` timelines.
* :func:`trace` -- a ``torch.profiler`` context writing a Chrome trace plus
  an op table, for one-off investigations.

Usage::

    pt = PhaseTimer(enabled=True)
    with pt("encoders"):
        ...
    with pt("refinement"):
        ...
    print(pt.summary())       # {"encoders": ms, "refinement": ms, ...}
"""
from __future__ import annotations

import contextlib
import os
import time
from collections import defaultdict
from typing import Dict, List, Tuple

import torch


class PhaseTimer:
    """Per-phase timer.  On a GPU it records HIP events (asynchronous); on
    CPU-only hosts it falls back to wall-clock ``perf_counter``."""

    def __init__(self, enabled: bool = True, roctx: bool = True):
        self.enabled = enabled
        self.gpu = torch.cuda.is_available()
        self.roctx = roctx and self.gpu
        self._events: Dict[str, List[Tuple[object, object]]] = defaultdict(list)

    @contextlib.contextmanager
    def __call__(self, name: str):
        if not self.enabled:
            yield
            return
        if not self.gpu:
            t0 = time.perf_counter()
            try:
                yield
            finally:
                self._events[name].append((t0, time.perf_counter()))
            return
        if self.roctx:
            torch.cuda.nvtx.range_push(name)
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        try:
            yield
        finally:
            e.record()
            if self.roctx:
                torch.cuda.nvtx.range_pop()
            self._events[name].append((s, e))

    def summary(self, reset: bool = True) -> Dict[str, float]:
        """Mean milliseconds per phase (synchronizes once)."""
        if not self.enabled:
            return {}
        if self.gpu:
            torch.cuda.synchronize()
            dur = lambda s, e: s.elapsed_time(e)  # noqa: E731
        else:
            dur = lambda s, e: (e - s) * 1e3  # noqa: E731
        out = {k: sum(dur(s, e) for s, e in v) / len(v) for k, v in self._events.items() if v}
        if reset:
            self._events.clear()
        return out


@contextlib.contextmanager
def trace(out_dir: str = "gpurun_out/trace", record_shapes: bool = True):
    """torch.profiler over the block; writes trace.json and ops.txt to out_dir."""
    from torch.profiler import ProfilerActivity, profile
    os.makedirs(out_dir, exist_ok=True)
    acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if torch.cuda.is_available() else [])
    with profile(activities=acts, record_shapes=record_shapes) as prof:
        yield prof
    prof.export_chrome_trace(os.path.join(out_dir, "trace.json"))
    key = "cuda_time_total" if torch.cuda.is_available() else "cpu_time_total"
    with open(os.path.join(out_dir, "ops.txt"), "w") as f:
        f.write(prof.key_averages().table(sort_by=key, row_limit=80))
