#!/usr/bin/env python
"""Microbenchmark: the persistent halo-tile 3x3 conv (csrc/enc_halo.hip) vs the
implicit-GEMM tiles of csrc/conv.hip at the encoder training shapes (Chairs
crop 368x496, batch 8: fnet on 16 images, cnet on 8), numerics vs tile 17.

    python scripts/bench_enc_halo.py [--reps 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from raft_stir_amd.ops import _ext
    from raft_stir_amd.ops.conv import EPI_BIAS, conv_fused, pack_weight, pad_to
    _ext.load(raise_on_error=True)
    dev = torch.device("cuda", 0)
    shapes = [("fnet.l1", 16, 184, 248, 64), ("cnet.l1", 8, 184, 248, 64),
              ("fnet.l2", 16, 92, 124, 96), ("cnet.l2", 8, 92, 124, 96)]
    for name, n, h, w, c in shapes:
        x = (torch.randn(n, h, w, c, device=dev) * 0.5).to(torch.bfloat16)
        wt = torch.randn(c, c, 3, 3, device=dev) * 0.05
        wp = pack_weight(wt, [(c, [(0, c, 0)])], pad_to(c, 128))
        y0 = torch.empty(n, h, w, c, device=dev, dtype=torch.bfloat16)
        y1 = torch.empty_like(y0)
        flop = 2.0 * n * h * w * c * c * 9
        line = f"{name:8s} P={n * h * w:7d} {c}->{c} GF={flop / 1e9:5.1f} |"
        tiles = [17, 21, 3, 4] if c % 64 == 0 else [3, 4]
        ref = None
        for tile in tiles:
            fn = lambda: conv_fused([(x, 0, c)], wp, None, 3, 3, c, EPI_BIAS, y0, 0, tile=tile)
            us = timeit(fn, a.reps)
            if ref is None:
                fn()
                ref = y0.float().clone()
            line += f" tile{tile} {us:6.1f}"
        hfn = lambda: torch.ops.raft_stir.conv3x3_halo(x, wp, y1, c, c)
        us = timeit(hfn, a.reps)
        hfn()
        rel = ((y1.float() - ref).norm() / ref.norm()).item()
        line += f" | halo {us:6.1f} us ({flop / us / 1e6:6.1f} TF/s, rel {rel:.1e})"
        print(line, flush=True)


if __name__ == "__main__":
    main()
