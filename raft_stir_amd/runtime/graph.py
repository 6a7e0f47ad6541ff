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
