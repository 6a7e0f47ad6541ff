#!/usr/bin/env python
"""Microbenchmark of the all-pairs volume + pyramid kernel (csrc/corr_volume.hip)
at a given 1/8-resolution shape: graph-timed us, effective write TB/s.

    python scripts/bench_corr.py [--hw 55 136] [--batch 1] [--C 256] [--reps 20]
"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hw", type=int, nargs=2, default=[55, 136])
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--C", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from raft_stir_amd.ops import _ext
    _ext.load(raise_on_error=True)
    dev = torch.device("cuda", 0)
    B, (H, W), C = a.batch, a.hw, a.C
    f1 = torch.randn(B, H * W, C, device=dev).bfloat16()
    f2 = torch.randn(B, H, W, C, device=dev).bfloat16()
    for dt, ob in (("bf16 in / fp32 pyramid", False), ("bf16 in / bf16 pyramid", True),
                   ("fp32 in / fp32 pyramid", None)):
        x1, x2 = (f1.float(), f2.float()) if ob is None else (f1, f2)
        fn = lambda: torch.ops.raft_stir.corr_volume(x1, x2, 4, 1.0 / math.sqrt(C), bool(ob))
        out = fn()
        nbytes = sum(p.numel() * p.element_size() for p in out)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st), torch.cuda.graph(g, stream=st):
            for _ in range(a.reps):
                fn()
        torch.cuda.current_stream().wait_stream(st)
        g.replay()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 1000 / a.reps
        print(f"{dt:24s} B={B} {H}x{W} C={C}: {us:8.1f} us  {nbytes / us / 1e6:6.2f} TB/s written", flush=True)


if __name__ == "__main__":
    main()
