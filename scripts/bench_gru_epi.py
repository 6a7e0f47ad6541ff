#!/usr/bin/env python
"""Microbenchmark: the SepConvGRU z|r and q convolutions as the fused training
engine runs them (three input segments h | inp | motion, GRU epilogues) vs the
same GEMM with one 384-channel segment and a plain ReLU epilogue, at the
training shape (batch 8, 46x62 at 1/8 of 368x496).  Separates the cost of the
segmented K walk from the cost of the gate epilogues (csrc/conv.hip)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def timeit(fn, reps=50):
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
    from raft_stir_amd.ops import _ext
    from raft_stir_amd.ops.conv import EPI_GRU_Q, EPI_GRU_ZR, EPI_RELU, conv_fused, pack_bias, pack_weight, pad_to
    _ext.load(raise_on_error=True)
    dev = torch.device("cuda", 0)
    B, H, W, HD = 8, 46, 62, 128
    e = lambda c: (torch.randn(B, H, W, c, device=dev) * 0.5).to(torch.bfloat16)
    hx, inp, h1 = e(256), e(128), e(HD)
    x384 = e(384)
    z, r, rh, q, hn = e(HD), e(HD), e(HD), e(HD), e(HD)
    segs3 = [(HD, [(0, HD, 0)]), (128, [(HD, 128, 0)]), (128, [(HD + 128, 128, 0)])]
    for kh, kw in ((1, 5), (5, 1)):
        wzr = torch.randn(2 * HD, 384, kh, kw, device=dev) * 0.02
        wq = torch.randn(HD, 384, kh, kw, device=dev) * 0.02
        b2, b1 = pack_bias(torch.randn(2 * HD, device=dev)), pack_bias(torch.randn(HD, device=dev))
        pzr3, pq3 = pack_weight(wzr, segs3, 256), pack_weight(wq, segs3, 128)
        pzr1, pq1 = pack_weight(wzr, [(384, [(0, 384, 0)])], 256), pack_weight(wq, [(384, [(0, 384, 0)])], 128)
        out = torch.empty(B, H, W, 2 * HD, device=dev, dtype=torch.bfloat16)
        res = {
            "zr 1seg relu": timeit(lambda: conv_fused([(x384, 0, 384)], pzr1, b2, kh, kw, 2 * HD, EPI_RELU, out)),
            "zr 3seg relu": timeit(lambda: conv_fused([(hx, 0, HD), (inp, 0, 128), (hx, HD, 128)], pzr3, b2, kh, kw,
                                                      2 * HD, EPI_RELU, out)),
            "zr 3seg gru": timeit(lambda: conv_fused([(hx, 0, HD), (inp, 0, 128), (hx, HD, 128)], pzr3, b2, kh, kw,
                                                     2 * HD, EPI_GRU_ZR, z, 0, hd=HD, out2=rh, out3=r, aux1=hx,
                                                     a1off=0)),
            "q 1seg relu": timeit(lambda: conv_fused([(x384, 0, 384)], pq1, b1, kh, kw, HD, EPI_RELU, out)),
            "q 3seg gru": timeit(lambda: conv_fused([(rh, 0, HD), (inp, 0, 128), (hx, HD, 128)], pq3, b1, kh, kw, HD,
                                                    EPI_GRU_Q, hn, 0, out2=q, aux1=hx, a1off=0, aux2=z)),
        }
        print(f"{kh}x{kw}: " + " | ".join(f"{k} {v:6.1f}us" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
