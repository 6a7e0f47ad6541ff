"""Microbenchmark of the correlation-volume backward (csrc/corr_bwd.hip: fold
into a padded bf16 G + both feature-gradient GEMMs in one MFMA launch)
against the library path (fold + two hipBLASLt bf16 bmm) at the RAFT training
shape (B=8, 46x62 1/8-res grid, 256 channels) and RAFT-small's (128 ch)."""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_stir_amd.ops import _ext  # noqa: E402


def gtime(fn, reps):
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
    args = ap.parse_args()
    _ext.load(raise_on_error=True)
    dev = torch.device("cuda")
    for B, H, W, C in ((8, 46, 62, 256), (8, 46, 62, 128), (2, 46, 124, 256)):
        N = H * W
        shapes = [(H >> l, W >> l) for l in range(4)]
        gpyr = [torch.randn(B, N, h, w, device=dev) for h, w in shapes]
        f1 = torch.randn(B, N, C, device=dev).to(torch.bfloat16)
        f2 = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
        scale = 1.0 / math.sqrt(C)

        def ours():
            return torch.ops.raft_stir.corr_volume_backward(gpyr, f1, f2, scale)

        G = torch.empty(B, N, N, device=dev, dtype=torch.bfloat16)

        def lib():
            torch.ops.raft_stir.pyr_grad_fold_bf16(gpyr, scale, G)
            return torch.bmm(G, f2.view(B, N, C)), torch.bmm(G.transpose(1, 2), f1)

        def fold_only():
            torch.ops.raft_stir.pyr_grad_fold_bf16(gpyr, scale, G)

        d1, d2 = ours()
        r1, r2 = lib()
        err = max(((d1.float() - r1.float()).norm() / r1.float().norm()).item(),
                  ((d2.float().view(B, N, C) - r2.float()).norm() / r2.float().norm()).item())
        t_ours, t_lib, t_fold = gtime(ours, args.reps), gtime(lib, args.reps), gtime(fold_only, args.reps)
        gf = 2 * 2 * B * N * N * C / 1e9
        print(f"B={B} {H}x{W} C={C}: GEMM GF={gf:.1f} | ours {t_ours:7.1f}us | library {t_lib:7.1f}us "
              f"(fold {t_fold:6.1f}us, GEMMs {t_lib - t_fold:6.1f}us = {gf / (t_lib - t_fold) * 1e3:5.0f}TF) | "
              f"ours GEMM ~{t_ours - t_fold:6.1f}us = {gf / max(t_ours - t_fold, 1e-3) * 1e3:5.0f}TF | rel err {err:.1e}",
              flush=True)


if __name__ == "__main__":
    main()
