#!/usr/bin/env python
"""fp32 update-block convs at the training / Sintel inference shapes: the F32
register tiles (6-8, 38-40) vs the fp32 weight-streaming tiles 81-83
(csrc/conv_v3f.hip), graph-timed.

    python scripts/bench_v3f.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench_1x1 import timeit  # noqa: E402


def main():
    from raft_stir_amd.ops import _ext
    _ext.load(raise_on_error=True)
    from raft_stir_amd.ops.conv import (EPI_BIAS, EPI_RELU, conv_fused, frag_weight_split, pack_bias,
                                        pack_weight_split, pad_to)
    dev = torch.device("cuda")
    for (B, H, W) in [(8, 46, 62), (1, 55, 136)]:
        for (kh, kw, cin, cout) in [(1, 5, 384, 256), (1, 5, 384, 128), (3, 3, 256, 192), (3, 3, 128, 512),
                                    (5, 1, 384, 256)]:
            x = torch.randn(B, H, W, cin, device=dev)
            w = torch.randn(cout, cin, kh, kw, device=dev) * 0.05
            ws = pack_weight_split(w, [(cin, [(0, cin, 0)])], pad_to(cout, 128))
            ws._rs_frag32 = frag_weight_split(ws)
            b = pack_bias(torch.randn(cout, device=dev))
            out = torch.empty(B, H, W, cout, device=dev)
            res = {}
            for t in (6, 7, 8, 38, 40, 81, 82, 83):
                try:
                    res[t] = timeit(lambda: conv_fused([(x, 0, cin)], ws, b, kh, kw, cout, EPI_RELU, out, 0, tile=t), 20)
                except Exception as e:  # noqa: BLE001
                    res[t] = None
            gf = 2 * B * H * W * cin * cout * kh * kw / 1e9
            print(f"{B}x{H}x{W} {kh}x{kw} {cin}->{cout} {gf:6.2f} GF  " +
                  "  ".join(f"t{t}: {v:7.1f}" for t, v in res.items() if v), flush=True)


if __name__ == "__main__":
    main()
