#!/usr/bin/env python
"""Isolated timing of the fused NHWC norm kernels (csrc/norm.hip) at the
encoders' training shapes, with the HBM bytes each pass must move:

  stats  (reduce<0> + finalize)   reads x
  apply  (apply_fwd)              reads x (+ residual), writes y
  bwd    (reduce<1> + finalize + apply_bwd)  reads x, dy (+ residual) twice, writes dx (+ dres)

    python scripts/bench_norm.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from raft_stir_amd.ops import _ext  # noqa: E402

SHAPES = [  # (B, H, W, C, per_sample, residual)
    (16, 184, 248, 64, True, False), (16, 184, 248, 64, True, True),
    (16, 92, 124, 96, True, False), (16, 46, 62, 128, True, False),
    (8, 184, 248, 64, False, False), (8, 92, 124, 96, False, True),
    (2, 218, 544, 64, True, False), (2, 109, 272, 96, True, False),
]


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    _ext.load(raise_on_error=True)
    ops = torch.ops.raft_stir
    dev = torch.device("cuda")
    for B, H, W, C, ps, use_res in SHAPES:
        x = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
        dy = torch.randn_like(x)
        res = torch.randn_like(x) if use_res else None
        g = None if ps else torch.ones(C, device=dev)
        bta = None if ps else torch.zeros(C, device=dev)
        nb = x.numel() * 2
        mean, rstd = ops.norm_stats(x, ps, 1e-5)
        t_s = timeit(lambda: ops.norm_stats(x, ps, 1e-5))
        t_a = timeit(lambda: ops.norm_act(x, mean, rstd, g, bta, res, True))
        t_b = timeit(lambda: ops.norm_act_backward(dy, x, mean, rstd, g, bta, res, True, True))
        r = 1 if use_res else 0
        print(f"B={B:2d} {H}x{W}x{C} {'IN' if ps else 'BN'}{' +res' if use_res else ''}: "
              f"stats {t_s:6.1f} us ({nb / t_s / 1e6:4.2f} TB/s)  "
              f"apply {t_a:6.1f} us ({nb * (2 + r) / t_a / 1e6:4.2f} TB/s)  "
              f"bwd {t_b:6.1f} us ({nb * (2 * (2 + r) + 1 + r) / t_b / 1e6:4.2f} TB/s)", flush=True)


if __name__ == "__main__":
    main()
