#!/usr/bin/env python
"""The training step's encoder phase alone: fnet (2B images, main stream) and
cnet (B images, side stream) forward + backward, issued exactly as
RAFT.forward issues them (stage by stage, interleaved), timed eager and
replayed from one hipGraph.  Equal times = the phase is GPU-bound; the graph
replay under ``rocprofv3 --kernel-trace`` then shows the phase's real
dependency structure without the profiler's host slowdown.

    python scripts/bench_encoders.py [--batch 8] [--size 368 496] [--reps 20] [--graph-only]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, nargs=2, default=[368, 496])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--graph-only", action="store_true")
    ap.add_argument("--small", action="store_true")
    a = ap.parse_args()
    from raft_stir_amd.config import make_args
    from raft_stir_amd.models import RAFT
    from raft_stir_amd.models.raft import _StreamHandoff
    from raft_stir_amd.ops import wpack
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = RAFT(make_args(mixed_precision=True, small=a.small)).to(dev).to(memory_format=torch.channels_last).train()
    B, (H, W) = a.batch, a.size
    xf = (torch.rand(2 * B, 3, H, W, device=dev) * 2 - 1).contiguous(memory_format=torch.channels_last)
    xc = xf[:B]
    side = RAFT._side_stream(dev)
    params = [p for n, p in m.named_parameters() if n.startswith(("fnet", "cnet"))]
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        of, oc = m.fnet(xf), m.cnet(xc)
    gf = torch.randn(of.shape, device=dev).to(of.dtype).contiguous(memory_format=torch.channels_last)
    gc = torch.randn(oc.shape, device=dev).to(oc.dtype).contiguous(memory_format=torch.channels_last)

    from raft_stir_amd.models.fused_encoder import FusedEncoders
    with torch.autocast("cuda", dtype=torch.bfloat16):
        fused = FusedEncoders.eligible(m, xf)
    print(f"encoder path: {'fused engine (models/fused_encoder.py)' if fused else 'per-module autograd'}")

    def step():
        wpack.refresh()
        main = torch.cuda.current_stream(dev)
        side.wait_stream(main)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            if fused:
                f, c = m._encoder_engine().run(xf, xc, side)
                main.wait_stream(side)
                c = _StreamHandoff.apply(c, side)
                loss = (f.float() * gf.float()).sum() + (c.float() * gc.float()).sum()
                loss.backward()
                return
            f, c = xf, xc
            ff, fc = m.fnet.stage_fns(), m.cnet.stage_fns()
            for k in range(max(len(ff), len(fc))):
                if k < len(ff):
                    f = ff[k](f)
                if k < len(fc):
                    with torch.cuda.stream(side):
                        c = fc[k](c)
            main.wait_stream(side)
            c = _StreamHandoff.apply(c, side)
        loss = (f.float() * gf.float()).sum() + (c.float() * gc.float()).sum()
        loss.backward()

    def zero():
        for p in params:
            p.grad = None

    for _ in range(3):
        zero()
        step()
    torch.cuda.synchronize()
    res = {}
    if not a.graph_only:
        ts = []
        for _ in range(5):  # host enqueue of one step (GPU idle at the start)
            zero()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            step()
            ts.append(time.perf_counter() - t0)
            torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            zero()
            step()
        e1.record()
        torch.cuda.synchronize()
        res["eager_ms"] = e0.elapsed_time(e1) / a.reps
        res["host_enqueue_ms"] = 1e3 * min(ts)
    # whole phase in one graph (weights do not change: no repack needed inside)
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for _ in range(2):
            zero()
            step()
    torch.cuda.current_stream(dev).wait_stream(s)
    zero()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    res["graph_ms"] = e0.elapsed_time(e1) / a.reps
    gflop = (74.4 if not a.small else 17.0) * 3 * B * (H * W) / (368 * 496)
    res["tflops_graph"] = round(gflop / res["graph_ms"], 1)
    print({k: round(v, 3) if isinstance(v, float) else v for k, v in res.items()}, flush=True)


if __name__ == "__main__":
    main()
