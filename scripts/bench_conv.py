#!/usr/bin/env python
"""Microbenchmark of the fused update-block convolution (csrc/conv.hip) on
every conv shape of the RAFT update block, vs MIOpen (F.conv2d, bf16,
channels_last) on the same shape.  Prints one line per (shape, variant).

    python scripts/bench_conv.py [--hw 55 136] [--batch 1] [--reps 50] [--tiles 0 1]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

# name, cin, cout, kh, kw
SHAPES = [
    ("convc1", 352, 256, 1, 1),
    ("convc1p", 384, 256, 1, 1),
    ("convc2", 256, 192, 3, 3),
    ("convf2", 128, 64, 3, 3),
    ("conv", 256, 126, 3, 3),
    ("gru_zr", 384, 256, 1, 5),
    ("gru_q", 384, 128, 1, 5),
    ("head", 128, 512, 3, 3),
    ("flow", 256, 2, 3, 3),
    ("mask2", 256, 576, 1, 1),
    # input gradients of the training step (Cout = the forward's Cin)
    ("zr_dg", 256, 384, 1, 5),
    ("q_dg", 128, 384, 1, 5),
    ("head_dg", 512, 128, 3, 3),
    ("c2_dg", 192, 256, 3, 3),
    ("cv_dg", 128, 256, 3, 3),
    ("f2_dg", 64, 128, 3, 3),
    ("c1_dg", 256, 384, 1, 1),
    ("m2_dg", 576, 256, 1, 1),
]


GRAPH = True  # --no-graph: time eager launches (includes host dispatch)


def timeit(fn, reps):
    """GPU time per call.  The reps are captured in one hipGraph so the host
    dispatch of the op (~10 us of Python + TORCH_CHECKs per call) does not
    hide the kernel time at small shapes."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if GRAPH:
        g = torch.cuda.CUDAGraph()
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            with torch.cuda.graph(g, stream=st):
                for _ in range(reps):
                    fn()
        torch.cuda.current_stream().wait_stream(st)
        g.replay()
        torch.cuda.synchronize()
        s.record()
        g.replay()
        e.record()
    else:
        s.record()
        for _ in range(reps):
            fn()
        e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hw", type=int, nargs=2, default=[55, 136])
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--wgrad", type=int, default=0, help="also bench wgrad with this many iterations batched")
    ap.add_argument("--tiles", type=int, nargs="*", default=[5, 6, 7, 8])
    ap.add_argument("--only", nargs="+", default=None, help="shape names to run")
    ap.add_argument("--gemm", action="store_true", help="also time the plain GEMM of the same M/N/K (hipBLASLt)")
    ap.add_argument("--no-miopen", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="time eager launches instead of one hipGraph")
    ap.add_argument("--v3wgrad", action="store_true", help="also time csrc/wgrad_v3.hip (64 / 128 rows per block)")
    ap.add_argument("--ksweep", type=int, nargs="*", default=None,
                    help="instead of SHAPES: a 1x5 conv to 256 channels for each of these input widths")
    ap.add_argument("--wvars", type=int, nargs="+", default=[0, 1, 2, 3, 4, 5],
                    help="wgrad tile variants (csrc/conv_wgrad.hip wgrad_launch)")
    a = ap.parse_args()
    global GRAPH
    GRAPH = not a.no_graph
    from raft_stir_amd.ops import _ext
    from raft_stir_amd.ops.conv import EPI_RELU, V3_TILES, conv_fused, frag_weight, pack_bias, pack_weight, pad_to
    _ext.load(raise_on_error=True)
    dev = torch.device("cuda", 0)
    B, (H, W) = a.batch, a.hw
    P = B * H * W
    tot = {}
    shapes = SHAPES if a.ksweep is None else [(f"k{c}", c, 256, 1, 5) for c in a.ksweep]
    for name, cin, cout, kh, kw in shapes:
        if (a.only and name not in a.only) or not a.tiles:
            continue
        x = torch.randn(B, H, W, cin, device=dev).to(torch.bfloat16)
        w = torch.randn(cout, cin, kh, kw, device=dev) * 0.05
        b = torch.randn(cout, device=dev)
        out = torch.empty(B, H, W, pad_to(cout, 8), device=dev, dtype=torch.bfloat16)
        wp = pack_weight(w, [(cin, [(0, cin, 0)])], pad_to(cout, 256))
        wf = frag_weight(wp) if cin % 64 == 0 else None
        bp = pack_bias(b)
        flop = 2.0 * P * cout * cin * kh * kw
        line = f"{name:8s} P={P:6d} K={cin * kh * kw:5d} N={cout:4d} GF={flop / 1e9:6.2f} |"
        ref_out = None
        for t in a.tiles:
            if (t == 5) != (cout <= 16) or (t >= 6 and t not in (12, 13, 14) and cin % 64):
                continue
            if t in V3_TILES and kh * kw not in (5, 9):
                continue
            try:
                us = timeit(lambda: conv_fused([(x, 0, cin)], wp, bp, kh, kw, cout, EPI_RELU, out, 0, tile=t, wf=wf),
                            a.reps)
            except RuntimeError as e:  # tile constraint (e.g. kernel too large for a halo tile)
                line += f" tile{t} n/a |"
                continue
            if ref_out is None:
                ref_out = out[..., :cout].float().clone()
            err = (out[..., :cout].float() - ref_out).abs().max().item()
            line += f" tile{t} {us:7.1f}us {flop / us / 1e6:6.1f}TF err={err:.2g} |"
            tot.setdefault(f"tile{t}", 0.0)
            tot[f"tile{t}"] += us
        if a.gemm:
            ga = torch.randn(P, cin * kh * kw, device=dev).to(torch.bfloat16)
            gb = torch.randn(cin * kh * kw, cout, device=dev).to(torch.bfloat16)
            us = timeit(lambda: torch.mm(ga, gb), a.reps)
            line += f" gemm {us:7.1f}us {flop / us / 1e6:6.1f}TF |"
            del ga, gb
        if not a.no_miopen:
            xc = x.permute(0, 3, 1, 2)
            wb = w.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            us = timeit(lambda: F.relu(F.conv2d(xc, wb, b.to(torch.bfloat16), padding=(kh // 2, kw // 2))), a.reps)
            line += f" miopen {us:7.1f}us {flop / us / 1e6:6.1f}TF"
            tot["miopen"] = tot.get("miopen", 0.0) + us
        print(line, flush=True)
    print("sum per iteration-set:", {k: round(v, 1) for k, v in tot.items()})
    if a.wgrad:
        # batched weight-gradient GEMMs over iters*B*H*W pixels
        n = a.wgrad * B
        for name, cin, cout, kh, kw in SHAPES:
            if cin % 64 or cout <= 2 or (a.only and name not in a.only):
                continue
            x = torch.randn(n, H, W, cin, device=dev).to(torch.bfloat16)
            dy = torch.randn(n, H, W, pad_to(cout, 128), device=dev).to(torch.bfloat16)
            dw = torch.zeros(pad_to(cout, 128), kh * kw, cin, device=dev)
            db = torch.zeros(cout, device=dev)
            flop = 2.0 * n * H * W * cout * cin * kh * kw
            line = f"wgrad {name:8s} K(px)={n * H * W:7d} M={cout:4d} N={cin * kh * kw:5d} |"
            ref = None
            if a.v3wgrad and kh * kw in (5, 9):
                for bm in (64, 128):
                    dw.zero_(); db.zero_()
                    torch.ops.raft_stir.wgrad_v3(dy, 0, cout, [x], [0], [cin], [n * H * W], kh, kw, dw, db, bm)
                    got = torch.cat([dw[:cout].flatten(), db[:cout]])
                    us = timeit(lambda: torch.ops.raft_stir.wgrad_v3(dy, 0, cout, [x], [0], [cin], [n * H * W], kh,
                                                                      kw, dw, db, bm), max(5, a.reps // 5))
                    line += f" v3/{bm} {us:8.1f}us {flop / us / 1e6:6.1f}TF |"
                    ref = got.clone() if ref is None else ref
            for v in a.wvars:
                def run():
                    dw.zero_(); db.zero_()
                    torch.ops.raft_stir.conv_wgrad(dy, 0, cout, [x], [0], [cin], [n * H * W], kh, kw, dw, db, v)
                run()
                got = torch.cat([dw[:cout].flatten(), db[:cout]])
                if ref is None:
                    ref = got.clone()
                err = ((got - ref).abs().max() / ref.abs().max().clamp_min(1e-6)).item()
                us = timeit(lambda: torch.ops.raft_stir.conv_wgrad(dy, 0, cout, [x], [0], [cin], [n * H * W], kh, kw,
                                                                     dw, db, v), max(5, a.reps // 5))
                line += f" v{v} {us:8.1f}us {flop / us / 1e6:6.1f}TF rel={err:.1g} |"
            print(line, flush=True)


if __name__ == "__main__":
    main()
