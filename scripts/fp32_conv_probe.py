#!/usr/bin/env python
"""Probe: MIOpen fp32 conv timing, NCHW vs NHWC, for the RAFT-small update-block
shapes at the STIR size (1 x 64 x 80 at 1/8 of 512x640)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raft_stir_amd  # noqa: F401,E402  (find-db path)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def t(fn, reps=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / reps


dev = torch.device("cuda")
for (cin, cout, k, H, W) in [(242, 192, 3, 64, 80), (242, 96, 3, 64, 80), (196, 96, 1, 64, 80), (128, 80, 3, 64, 80),
                             (96, 128, 3, 64, 80), (64, 32, 3, 64, 80)]:
    x = torch.randn(1, cin, H, W, device=dev)
    w = torch.randn(cout, cin, k, k, device=dev)
    b = torch.randn(cout, device=dev)
    line = f"{cin:4d}->{cout:4d} k{k}:"
    for name, fmt in (("nchw", torch.contiguous_format), ("nhwc", torch.channels_last)):
        xx = x.contiguous(memory_format=fmt)
        ww = w.contiguous(memory_format=fmt)
        us = t(lambda: F.conv2d(xx, ww, b, padding=k // 2))
        line += f" {name} {us:7.1f}us"
    for name, fmt in (("bf16nhwc", torch.channels_last),):
        xx = x.to(torch.bfloat16).contiguous(memory_format=fmt)
        ww = w.to(torch.bfloat16).contiguous(memory_format=fmt)
        us = t(lambda: F.conv2d(xx, ww, b.bfloat16(), padding=k // 2))
        line += f" {name} {us:7.1f}us"
    print(line, flush=True)
