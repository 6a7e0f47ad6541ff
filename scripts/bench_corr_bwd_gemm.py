#!/usr/bin/env python
"""Micro-benchmark of the correlation-volume backward GEMMs (bf16, fp32 acc):
df1 = G @ f2 and df2 = G^T @ f1 with G (B, N, N), N = 46*62, C = 256 -- the
two bmm calls of ops/corr.py::_CorrVolume.backward.  Compares BLAS backends and
operand layouts.  Writes one line per variant to stdout.
"""
import torch


def timeit(fn, reps=20):
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
    dev = torch.device("cuda", 0)
    B, N, C = 8, 46 * 62, 256
    G = torch.randn(B, N, N, device=dev, dtype=torch.bfloat16)
    f1 = torch.randn(B, N, C, device=dev, dtype=torch.bfloat16)
    f2 = torch.randn(B, N, C, device=dev, dtype=torch.bfloat16)
    ref1 = torch.bmm(G.float(), f2.float())
    ref2 = torch.bmm(G.float().transpose(1, 2), f1.float())
    flops = 2 * B * N * N * C
    variants = {
        "df1 G@f2": lambda: torch.bmm(G, f2),
        "df2 G^T@f1": lambda: torch.bmm(G.transpose(1, 2), f1),
        "df2 (f1^T@G)^T": lambda: torch.bmm(f1.transpose(1, 2), G).transpose(1, 2),
        "df1 (f2^T@G^T)^T": lambda: torch.bmm(f2.transpose(1, 2), G.transpose(1, 2)).transpose(1, 2),
        "both cat [f2|f1]": None,
    }
    for lib in ("default", "cublas", "cublaslt"):
        if lib != "default":
            try:
                torch.backends.cuda.preferred_blas_library(lib)
            except Exception as ex:  # noqa: BLE001
                print(f"{lib}: unavailable ({ex})")
                continue
        for name, fn in variants.items():
            if fn is None:
                continue
            us = timeit(fn)
            out = fn().float()
            ref = ref1 if name.startswith("df1") else ref2
            err = ((out - ref).abs().max() / ref.abs().max()).item()
            print(f"{lib:9s} {name:20s} {us:8.1f} us  {flops / us / 1e6:7.1f} TFLOP/s  relerr {err:.2e}",
                  flush=True)


if __name__ == "__main__":
    main()
