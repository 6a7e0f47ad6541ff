#!/usr/bin/env python
"""Microbenchmark: the encoders' stride-1 3x3 convs (reference
core/extractor.py:6-56) forward and input gradient at the training shape on
the current kernels (csrc/enc_halo.hip for 64 / 96 channels, the conv.hip
tiles for 128) against the weight-streaming tiles of csrc/conv_v3.h (96
channels read as two overlapping 64-channel segments with zero weights on
the duplicated half).

    python scripts/bench_enc_v3.py [--batch 8] [--tiles 61 63 65]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def timeit(fn, reps):
    for _ in range(2):
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
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, nargs=2, default=[368, 496])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tiles", type=int, nargs="+", default=[60, 61, 63, 65])
    ap.add_argument("--wgrad", action="store_true", help="also time the weight gradients (enc_wgrad vs wgrad_v3)")
    a = ap.parse_args()
    from raft_stir_amd.ops import _ext
    from raft_stir_amd.ops.conv import EPI_BIAS, conv_fused, frag_weight, pack_weight, pad_to
    from raft_stir_amd.ops.enc_conv import _conv3x3_into
    _ext.load(raise_on_error=True)
    dev = torch.device("cuda", 0)
    H, W = a.size
    shapes = []
    for net, n in (("fnet", 2 * a.batch), ("cnet", a.batch)):
        shapes += [(f"{net}.l1", n, 2, 64, 64), (f"{net}.l2", n, 4, 96, 96), (f"{net}.l3", n, 8, 128, 128)]
    tot = {}
    for name, n, div, cin, cout in shapes:
        h, w = H // div, W // div
        P = n * h * w
        flop = 2.0 * P * cout * cin * 9
        x = (torch.randn(n, h, w, cin, device=dev) * 0.5).to(torch.bfloat16)
        wt = torch.randn(cout, cin, 3, 3, device=dev) * 0.05
        ref = F.conv2d(x.permute(0, 3, 1, 2).float(), wt.to(torch.bfloat16).float(), None, padding=1).permute(0, 2, 3, 1)
        out = torch.empty(n, h, w, cout, device=dev, dtype=torch.bfloat16)
        line = f"{name:8s} P={P:8d} {cin}->{cout} GF={flop / 1e9:6.1f} |"
        wp = pack_weight(wt, [(cin, [(0, cin, 0)])], pad_to(cout, 128))
        t0 = timeit(lambda: _conv3x3_into(x, wp, cin, cout, out, P), a.reps)
        e0 = ((out.float() - ref).abs().max() / ref.abs().max()).item()
        line += f" cur {t0:7.1f}us {flop / t0 / 1e6:5.0f}TF ({e0:.0e}) |"
        tot["cur"] = tot.get("cur", 0.0) + t0
        if cin % 64 == 0:
            segs, wsegs = [(x, 0, cin)], [(cin, [(0, cin, 0)])]
        else:  # 96 = [0, 64) + [32, 96) with zero weights on channels 32..63 of the second window
            segs, wsegs = [(x, 0, 64), (x, cin - 64, 64)], [(64, [(0, 64, 0)]), (64, [(64, cin - 64, 128 - cin)])]
        wv = pack_weight(wt, wsegs, pad_to(cout, 128))
        wf = frag_weight(wv)
        best = None
        for t in a.tiles:
            tt = timeit(lambda: conv_fused(segs, wv, None, 3, 3, cout, EPI_BIAS, out, 0, tile=t, wf=wf), a.reps)
            e = ((out.float() - ref).abs().max() / ref.abs().max()).item()
            line += f" t{t} {tt:7.1f}us {flop / tt / 1e6:5.0f}TF ({e:.0e}) |"
            best = tt if best is None else min(best, tt)
        tot["v3best"] = tot.get("v3best", 0.0) + best
        if a.wgrad:
            dy = (torch.randn(n, h, w, cout, device=dev) * 0.5).to(torch.bfloat16)
            t_e = timeit(lambda: torch.ops.raft_stir.enc_wgrad(dy, x), a.reps)
            line += f" enc_wgrad {t_e:7.1f}us |"
            tot["enc_wgrad"] = tot.get("enc_wgrad", 0.0) + t_e
            if cin % 64 == 0:
                dw = torch.zeros(cout, 9, cin, device=dev)
                for bm in (64, 128):
                    t3 = timeit(lambda: torch.ops.raft_stir.wgrad_v3(dy, 0, cout, [x], [0], [cin], [P], 3, 3, dw, None, bm),
                                a.reps)
                    line += f" wg3/{bm} {t3:7.1f}us |"
        print(line, flush=True)
    print("sum (us):", {k: round(v, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main()
