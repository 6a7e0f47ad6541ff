#!/usr/bin/env python
"""Microbenchmark: the stride-1 3x3 encoder convolutions (reference
core/extractor.py:6-56 ResidualBlock convs) at the training shape, MIOpen
(F.conv2d / aten.convolution_backward, bf16, channels_last) vs the
hand-written implicit-GEMM kernels (csrc/conv.hip forward + dgrad with
flipped weights, csrc/conv_wgrad.hip weight gradient).

    python scripts/bench_encoder_conv.py [--batch 8] [--size 368 496] [--reps 20] [--tiles 16 17 20 21 3 4]
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
    ap.add_argument("--tiles", type=int, nargs="+", default=[16, 17, 20, 21, 3, 4])
    a = ap.parse_args()
    from raft_stir_amd.ops import _ext
    from raft_stir_amd.ops.conv import EPI_BIAS, conv_fused, pack_weight, pad_to
    _ext.load(raise_on_error=True)
    dev = torch.device("cuda", 0)
    H, W = a.size
    # (name, images, spatial divisor, cin, cout): fnet runs on 2B images, cnet on B
    shapes = []
    for net, n in (("fnet", 2 * a.batch), ("cnet", a.batch)):
        shapes += [(f"{net}.l1", n, 2, 64, 64), (f"{net}.l2", n, 4, 96, 96), (f"{net}.l3", n, 8, 128, 128)]
    tot = {}
    for name, n, div, cin, cout in shapes:
        h, w = H // div, W // div
        P = n * h * w
        flop = 2.0 * P * cout * cin * 9
        x = (torch.randn(n, h, w, cin, device=dev) * 0.5).to(torch.bfloat16)
        dy = (torch.randn(n, h, w, pad_to(cout, 128), device=dev) * 0.5).to(torch.bfloat16)
        wt = torch.randn(cout, cin, 3, 3, device=dev) * 0.05
        xc = x.permute(0, 3, 1, 2)
        dyc = dy[..., :cout].contiguous().permute(0, 3, 1, 2)
        wb = wt.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        line = f"{name:8s} P={P:8d} {cin}->{cout} GF={flop / 1e9:6.1f} |"
        # MIOpen
        t_f = timeit(lambda: F.conv2d(xc, wb, None, padding=1), a.reps)
        t_d = timeit(lambda: torch.ops.aten.convolution_backward(dyc, xc, wb, None, [1, 1], [1, 1], [1, 1], False,
                                                                   [0, 0], 1, [True, False, False]), a.reps)
        t_w = timeit(lambda: torch.ops.aten.convolution_backward(dyc, xc, wb, None, [1, 1], [1, 1], [1, 1], False,
                                                                   [0, 0], 1, [False, True, False]), a.reps)
        line += f" miopen f {t_f:7.1f} d {t_d:7.1f} w {t_w:7.1f} = {t_f + t_d + t_w:7.1f}us |"
        tot["miopen"] = tot.get("miopen", 0.0) + t_f + t_d + t_w
        ref = F.conv2d(xc.float(), wb.float(), None, padding=1).permute(0, 2, 3, 1)
        ref_dx = torch.ops.aten.convolution_backward(dyc.float(), xc.float(), wb.float(), None, [1, 1], [1, 1],
                                                     [1, 1], False, [0, 0], 1, [True, True, False])
        ref_dw = ref_dx[1]
        ref_dx = ref_dx[0].permute(0, 2, 3, 1)
        wp = pack_weight(wt, [(cin, [(0, cin, 0)])], pad_to(cout, 128))
        wd = pack_weight(wt.transpose(0, 1).flip(2, 3), [(cout, [(0, cout, 0)])], pad_to(cin, 128))
        out = torch.empty(n, h, w, cout, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(n, h, w, cin, device=dev, dtype=torch.bfloat16)
        best_f = best_d = None
        for t in a.tiles:
            if t >= 16 and (cin % 64 or cout % 64):
                continue
            try:
                tf = timeit(lambda: conv_fused([(x, 0, cin)], wp, None, 3, 3, cout, EPI_BIAS, out, 0, tile=t), a.reps)
                td = timeit(lambda: conv_fused([(dy, 0, cout)], wd, None, 3, 3, cin, EPI_BIAS, dx, 0, tile=t), a.reps)
            except RuntimeError as e:  # tile constraint
                line += f" tile{t} n/a ({str(e).splitlines()[0][:40]}) |"
                continue
            ef = ((out.float() - ref).abs().max() / ref.abs().max()).item()
            ed = ((dx.float() - ref_dx).abs().max() / ref_dx.abs().max()).item()
            line += f" tile{t} f {tf:7.1f} d {td:7.1f} (rel {ef:.1e}/{ed:.1e}) |"
            best_f = tf if best_f is None else min(best_f, tf)
            best_d = td if best_d is None else min(best_d, td)
        t_ww = None
        if cin % 32 == 0 and cin >= 64:
            # 64-wide input-channel segments; 96 = two overlapping segments (ops/enc_conv.py)
            segs = [(0, cin)] if cin % 64 == 0 else [(0, cin - 32), (cin - 64, 64)]
            kt = sum(c for _, c in segs)
            dw = torch.zeros(pad_to(cout, 128), 9, kt, device=dev)

            def wg(v):
                torch.ops.raft_stir.conv_wgrad(dy, 0, cout, [x] * len(segs), [o for o, _ in segs],
                                               [c for _, c in segs], [P] * len(segs), 3, 3, dw, None, v)
            for v in (0, 1, 2, 4):
                t = timeit(lambda: (dw.zero_(), wg(v)), a.reps)
                line += f" wg v{v} {t:7.1f} |"
                t_ww = t if t_ww is None else min(t_ww, t)
            dw.zero_()
            wg(0)
            acc = dw[:cout]
            if len(segs) > 1:
                acc = torch.cat([acc[..., :cin - 32], acc[..., cin:cin + 32]], -1)
            got = acc.reshape(cout, 3, 3, cin).permute(0, 3, 1, 2)
            ew = ((got - ref_dw).abs().max() / ref_dw.abs().max()).item()
            line += f" wgrad {t_ww:7.1f} (rel {ew:.1e}) |"
        if best_f is not None:
            ours = best_f + best_d + (t_ww if t_ww is not None else t_w)
            line += f" ours {ours:7.1f}us"
            tot["ours"] = tot.get("ours", 0.0) + ours
        print(line, flush=True)
    print("total fwd+dgrad+wgrad over the shapes (us):", {k: round(v, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main()
