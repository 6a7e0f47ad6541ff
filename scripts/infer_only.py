#!/usr/bin/env python
"""Inference-only driver for profiling: RAFT full, bf16, 12 iterations,
1088x436 (padded to 1088x440), batch 1, random-init weights, synthetic pair;
the pyramid dtype follows bench.py (--corr-dtype auto: bf16 under bf16).

    python scripts/infer_only.py [--reps 10] [--graph] [--small] [--size H W] [--alt]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--size", type=int, nargs=2, default=[436, 1088])
    ap.add_argument("--graph", action="store_true")
    ap.add_argument("--small", action="store_true")
    ap.add_argument("--alt", action="store_true", help="on-the-fly correlation")
    ap.add_argument("--fp32", action="store_true")
    ap.add_argument("--corr-dtype", default="auto", choices=["auto", "float32", "bfloat16"],
                    help="pyramid storage, as bench.py (auto = bf16 under bf16 autocast)")
    a = ap.parse_args()
    from raft_stir_amd.config import make_args
    from raft_stir_amd.models import RAFT
    from raft_stir_amd.utils.padder import InputPadder
    from raft_stir_amd.runtime.graph import GraphedInference

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = RAFT(make_args(small=a.small, mixed_precision=not a.fp32, alternate_corr=a.alt,
                            corr_dtype=a.corr_dtype))
    model = model.to(dev).to(memory_format=torch.channels_last).eval()
    h, w = a.size
    i1 = torch.rand(1, 3, h, w, device=dev) * 255
    i2 = torch.rand(1, 3, h, w, device=dev) * 255
    i1, i2 = InputPadder(i1.shape).pad(i1, i2)
    if a.graph:
        g = GraphedInference(model, i1.shape, iters=a.iters)
        run = lambda: g(i1, i2)
    else:
        def run():
            with torch.no_grad():
                return model(i1, i2, iters=a.iters, test_mode=True)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.reps
    print(f"infer {'graph' if a.graph else 'eager'} {h}x{w} iters={a.iters}: "
          f"{1000 * dt:.3f} ms/pair, {1 / dt:.2f} FPS")


if __name__ == "__main__":
    main()
