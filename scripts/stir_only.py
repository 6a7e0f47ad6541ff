#!/usr/bin/env python
"""Profiling driver for the STIR point tracker (reference rafttoonnx.py:137-169:
RAFT-small, 12 iterations, 1x3x512x640, 32 query points) served from one
hipGraph (export/pointtrack.py PointTrackServer); random-init weights.

    python scripts/stir_only.py [--bf16] [--reps 20]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--bf16", action="store_true")
    a = ap.parse_args()
    from raft_stir_amd.config import make_args
    from raft_stir_amd.export.pointtrack import PointTrackServer
    from raft_stir_amd.models import RAFT
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = RAFT(make_args(small=True, mixed_precision=a.bf16)).to(dev).eval()
    i1 = torch.rand(1, 3, 512, 640, device=dev) * 255
    i2 = torch.rand(1, 3, 512, 640, device=dev) * 255
    pts = torch.rand(1, 32, 2, device=dev) * 500
    srv = PointTrackServer(m, iters=12)
    for _ in range(3):
        srv(pts, i1, i2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        srv(pts, i1, i2)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.reps
    print(f"stir {'bf16' if a.bf16 else 'fp32'}: {1000 * dt:.3f} ms/pair")


if __name__ == "__main__":
    main()
