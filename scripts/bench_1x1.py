#!/usr/bin/env python
"""The update block's 1x1 convs at the training shape (8 x 46 x 62 pixels):
conv_fused tiles (70: conv_gemm1.hip, 31: the 8-wave buffer-DMA tile) vs
the same GEMM on hipBLASLt through torch (addmm / matmul), graph-timed.

    python scripts/bench_1x1.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def timeit(fn, reps=50):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return 1e3 * e0.elapsed_time(e1) / reps


def scan():
    """Time vs K and Cout for tiles 70 / 71 (fixed cost vs per-K-step cost)."""
    from raft_stir_amd.ops.conv import EPI_BIAS, EPI_RELU, conv_fused, pack_weight, pad_to
    dev = torch.device("cuda")
    B, H, W = 8, 46, 62
    for cin, cout, epi in [(64, 256, EPI_RELU), (128, 256, EPI_RELU), (256, 256, EPI_RELU), (384, 256, EPI_RELU),
                           (768, 256, EPI_RELU), (256, 128, EPI_RELU), (256, 512, EPI_RELU), (384, 256, EPI_BIAS)]:
        x = torch.randn(B, H, W, cin, device=dev).to(torch.bfloat16)
        w = torch.randn(cout, cin, 1, 1, device=dev) * 0.05
        b = torch.randn(cout, device=dev) if epi == EPI_RELU else None
        wp = pack_weight(w, [(cin, [(0, cin, 0)])], pad_to(cout, 256))
        out = torch.empty(B, H, W, cout, device=dev, dtype=torch.bfloat16)
        r = {t: timeit(lambda: conv_fused([(x, 0, cin)], wp, b, 1, 1, cout, epi, out, 0, tile=t)) for t in (70, 31)}
        print(f"scan cin {cin:4d} cout {cout:4d} epi {epi}: " + "  ".join(f"{k}: {v:6.1f} us" for k, v in r.items()),
              flush=True)


def main():
    from raft_stir_amd.ops.conv import EPI_BIAS, EPI_RELU, EPI_RELU_BWD, EPI_SCALE, conv_fused, pack_weight, pad_to
    from raft_stir_amd.ops import _ext
    _ext.load(raise_on_error=True)
    dev = torch.device("cuda")
    B, H, W = 8, 46, 62
    P = B * H * W
    cases = [("c1 fwd 384->256 relu", 384, 256, EPI_RELU), ("mask fwd 256->576 scale", 256, 576, EPI_SCALE),
             ("mask dgrad 576->256 relu_bwd", 576, 256, EPI_RELU_BWD), ("c1 dgrad 256->384", 256, 384, EPI_BIAS)]
    for name, cin, cout, epi in cases:
        x = torch.randn(B, H, W, cin, device=dev).to(torch.bfloat16)
        w = torch.randn(cout, cin, 1, 1, device=dev) * 0.05
        b = torch.randn(cout, device=dev)
        wp = pack_weight(w, [(cin, [(0, cin, 0)])], pad_to(cout, 256))
        out = torch.empty(B, H, W, cout, device=dev, dtype=torch.bfloat16)
        aux = torch.randn(B, H, W, cout, device=dev).to(torch.bfloat16)
        res = {}
        for tile in (70, 31, 16):
            kw = dict(scale=0.25, tile=tile)
            if epi == EPI_RELU_BWD:
                kw["aux1"] = aux
            try:
                res[tile] = timeit(lambda: conv_fused([(x, 0, cin)], wp, b if epi != EPI_RELU_BWD else None, 1, 1,
                                                      cout, epi, out, 0, **kw))
            except Exception as e:  # tile not valid for the shape
                print(f"  tile {tile}: {str(e).splitlines()[0][:160]}")
                res[tile] = None
        X = x.view(P, cin)
        Wt = w.view(cout, cin).to(torch.bfloat16)
        bb = b.to(torch.bfloat16)
        if epi == EPI_RELU:
            f = lambda: torch._addmm_activation(bb, X, Wt.t(), use_gelu=False)
        elif epi == EPI_SCALE:
            f = lambda: torch.addmm(bb, X, Wt.t())
        elif epi == EPI_RELU_BWD:
            A = aux.view(P, cout)
            f = lambda: torch.matmul(X, Wt.t()) * (A > 0)
        else:
            f = lambda: torch.matmul(X, Wt.t())
        res["hipblaslt"] = timeit(f)
        gf = 2 * P * cin * cout / 1e9
        o2 = torch.empty_like(out)
        res["copy_out"] = timeit(lambda: o2.copy_(out))
        res["fill_out"] = timeit(lambda: o2.fill_(1.0))
        print(f"{name:32s} {gf:5.2f} GF  " + "  ".join(f"{k}: {v:6.1f} us" if v else f"{k}: -" for k, v in res.items()),
              flush=True)


if __name__ == "__main__":
    from raft_stir_amd.ops import _ext
    _ext.load(raise_on_error=True)
    scan() if "--scan" in sys.argv else main()
