"""7x7 / stride-2 stem (3 -> 64) at the training shapes: csrc/stem.hip forward
and weight gradient vs MIOpen (torch conv2d / convolution_backward on
channels_last bf16), fnet (16 images) and cnet (8 images) at 368x496."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_stir_amd.ops import _ext  # noqa: E402
from raft_stir_amd.ops.enc_conv import _stem_layout  # noqa: E402

CL = torch.channels_last


def gtime(fn, reps=20):
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
    _ext.load(raise_on_error=True)
    dev = torch.device("cuda")
    for N in (16, 8):
        H, W, cout = 368, 496, 64
        x = torch.randn(N, 3, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
        w = torch.randn(cout, 3, 7, 7, device=dev) * 0.1
        wb = w.to(torch.bfloat16).contiguous(memory_format=CL)
        Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        out = torch.empty(N, Ho, Wo, cout, device=dev, dtype=torch.bfloat16)
        wp = _stem_layout([w]).to(torch.bfloat16).contiguous()
        xn = x.permute(0, 2, 3, 1)
        dy = torch.randn(N, cout, Ho, Wo, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
        dyn = dy.permute(0, 2, 3, 1)
        g = torch.empty(w.shape, device=dev, dtype=torch.float32)

        def ours_f():
            torch.ops.raft_stir.stem_conv(xn, wp, None, out, cout, 0)

        def ours_w():
            torch.ops.raft_stir.stem_wgrad(xn, dyn, cout, g)

        def mi_f():
            return F.conv2d(x, wb, None, 2, 3)

        def mi_w():
            return torch.ops.aten.convolution_backward(dy, x, wb, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1,
                                                       [False, True, False])[1]

        ours_f()
        ref = mi_f()
        err_f = ((out.float().permute(0, 3, 1, 2) - ref.float()).norm() / ref.float().norm()).item()
        ours_w()
        rw = mi_w().float()
        err_w = ((g - rw).norm() / rw.norm()).item()
        gf = 2 * N * Ho * Wo * cout * 147 / 1e9
        tf, tw, mf, mw = gtime(ours_f), gtime(ours_w), gtime(mi_f), gtime(mi_w)
        print(f"N={N}: GF={gf:.1f} | fwd ours {tf:6.1f}us ({gf / tf * 1e3:4.0f}TF) miopen {mf:6.1f}us | "
              f"wgrad ours {tw:6.1f}us ({gf / tw * 1e3:4.0f}TF) miopen {mw:6.1f}us | err fwd {err_f:.1e} wgrad {err_w:.1e}",
              flush=True)


if __name__ == "__main__":
    main()
