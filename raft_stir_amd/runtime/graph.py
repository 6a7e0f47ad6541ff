"""hipGraph capture of the whole RAFT inference forward.

At batch 1 the 12-32-iteration refinement loop is ~15 small kernels per
iteration and is launch-bound on the host.  Instead of a tracing compiler we
capture the full forward (encoders + correlation volume + every iteration +
final upsampling) once per input shape into a HIP graph
(``torch.cuda.CUDAGraph`` is hipGraph on ROCm) and replay it: one host call
per image pair.  Inputs are copied into static device buffers; outputs alias
static buffers owned by the graph (clone them if they must outlive the next
call).
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch

from .weights import bump, refresh_all, repack_in_graph, weights_key


class GraphedInference:
    def __init__(self, model, shape, iters=12, warm_start=False, warmup=2, pool=None):
        self.model = model
        self.iters = iters
        self.warm_start = warm_start
        dev = next(model.parameters()).device
        B, C, H, W = shape
        self.i1 = torch.zeros(shape, device=dev).contiguous(memory_format=torch.channels_last)
        self.i2 = torch.zeros_like(self.i1)
        self.flow_init = torch.zeros(B, 2, H // 8, W // 8, device=dev) if warm_start else None
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.no_grad(), torch.cuda.stream(s):
            for _ in range(warmup):
                self._run()
        torch.cuda.current_stream(dev).wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(self.graph, pool=pool):
            self.out = self._run()
        self._wkey = weights_key(model)

    def _run(self):
        return self.model(self.i1, self.i2, iters=self.iters, flow_init=self.flow_init,
                          test_mode=True)

    @torch.no_grad()
    def __call__(self, image1, image2, flow_init=None):
        self.i1.copy_(image1)
        self.i2.copy_(image2)
        if self.warm_start:
            if flow_init is None:
                self.flow_init.zero_()
            else:
                self.flow_init.copy_(flow_init)
        key = weights_key(self.model)
        if key != self._wkey:  # weights moved since capture: re-pack into the captured storage
            refresh_all(self.model)
            self._wkey = key
        self.graph.replay()
        return self.out


class GraphCache:
    """Per-(shape, iters) graph cache for variable-resolution evaluation."""

    def __init__(self, model, max_graphs=8):
        self.model = model
        self.max_graphs = max_graphs
        self.graphs: Dict[Tuple, GraphedInference] = {}
        self.pool = None

    def __call__(self, image1, image2, iters=12, flow_init=None):
        key = (tuple(image1.shape), iters, flow_init is not None)
        g = self.graphs.get(key)
        if g is None:
            if len(self.graphs) >= self.max_graphs:
                self.graphs.pop(next(iter(self.graphs)))
            g = GraphedInference(self.model, image1.shape, iters=iters,
                                 warm_start=flow_init is not None, pool=self.pool)
            self.pool = g.graph.pool()
            self.graphs[key] = g
        return g(image1, image2, flow_init)


class GraphedTrainStep:
    """hipGraph capture of a WHOLE training step (reference train.py:162-183):
    forward (encoders, correlation volume, the 12-iteration fused loop on
    its HIP streams), sequence loss, backward, gradient clipping and the
    AdamW update, replayed with one host call.

    The eager step costs ~12 ms of host time (Python + ~950 kernel launches)
    against ~20 ms of GPU work, so the host -- not the GPU -- bounds the step
    as soon as the kernels get faster (scripts/host_overhead.py).  The
    standard whole-network capture recipe is used: warm up on a side stream,
    capture with the gradients set to None (the captured backward then
    WRITES, not accumulates, the .grad tensors on every replay), static
    input buffers, and an optimizer built with ``capturable=True`` and a
    device learning-rate tensor that the (uncaptured) LR scheduler updates
    in place between replays.

    ``step(batch)`` copies the batch into the static buffers, replays and
    returns the static loss tensor (valid until the next replay).

    Measured on MI355X (RAFT, batch 8, 368x496, bench.py --train-graph):
    round 2, 22.30 ms/step graphed vs 22.47 ms eager; round 4, 22.37 vs
    20.49 ms (357 vs 390 pairs/s, profiles/r4/ab_train_graph_s27.txt) -- the
    eager step is GPU-bound, and the replay (which also repacks every weight
    layout inside the graph) is slower, so the bench keeps the eager step and
    this stays an opt-in.  One GPU only: the data-parallel step stays eager
    under DDP.
    """

    def __init__(self, model, optimizer, loss_fn, sample_batch, clip=1.0, warmup=3, iters=12):
        self.model = model
        self.optimizer = optimizer
        self.loss_fn = loss_fn
        self.clip = clip
        self.iters = iters
        for g in optimizer.param_groups:
            if not isinstance(g["lr"], torch.Tensor) or not g.get("capturable", False):
                raise ValueError("GraphedTrainStep needs an optimizer with capturable=True and a tensor lr")
        self.params = [p for p in model.parameters() if p.requires_grad]
        self.static = [t.clone() for t in sample_batch]
        dev = self.static[0].device
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                optimizer.zero_grad(set_to_none=True)
                self._body()
        torch.cuda.current_stream(dev).wait_stream(s)
        optimizer.zero_grad(set_to_none=True)
        self.graph = torch.cuda.CUDAGraph()
        # the step's own optimizer update moves the weights: record the
        # weight-packing kernels too, so every replay packs the current weights
        with torch.cuda.graph(self.graph), repack_in_graph():
            self.loss = self._body()
        # the recorded repack reads these chunks' gather maps and writes their
        # flat buffers on every replay: hold them for the graph's whole life
        # (later registrations go to new chunks and never move these)
        from ..ops import wpack
        self._packed_storage = wpack.snapshot()

    def _body(self):
        from ..ops import wpack
        wpack.repack()  # recorded: every replay packs the weights its own optimizer step wrote
        i1, i2, flow, valid = self.static
        preds = self.model(i1, i2, iters=self.iters)
        loss = self.loss_fn(preds, flow, valid)
        loss.backward()
        if hasattr(self.optimizer, "clip_and_step"):
            self.optimizer.clip_and_step(self.clip if self.clip and self.clip > 0 else 0.0)
        else:
            if self.clip and self.clip > 0:
                torch.nn.utils.clip_grad_norm_(self.params, self.clip)
            self.optimizer.step()
        return loss.detach()

    def step(self, batch):
        for dst, src in zip(self.static, batch):
            dst.copy_(src, non_blocking=True)
        self.graph.replay()
        # the replayed optimizer step moved the weights without touching
        # _version / data_ptr: invalidate every packed-weight cache
        bump()
        return self.loss
