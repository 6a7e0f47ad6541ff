#!/usr/bin/env python
"""Time the on-the-fly correlation backward (csrc/corr_onthefly.hip
otf_tile_bwd_kernel) at the RAFT-small and RAFT training shapes, with a
realistic smooth flow.  A zero upstream gradient makes every df2 atomic a
no-op (the kernel skips cells whose gradient is all zero), so the difference
between the two rows is the cost of the df2 atomics.

    python scripts/bench_otf_bwd.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from raft_stir_amd.ops import _ext  # noqa: E402


def run(name, B, C, H, W, r, levels=4, reps=20):
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    f1 = torch.randn(B, C, H, W, generator=g).to(dev, torch.bfloat16)
    f2 = torch.randn(B, C, H, W, generator=g).to(dev, torch.bfloat16)
    lv = [f2]
    for _ in range(levels - 1):
        lv.append(F.avg_pool2d(lv[-1], 2, stride=2))
    f1n = f1.permute(0, 2, 3, 1).contiguous()
    f2n = [t.permute(0, 2, 3, 1).contiguous() for t in lv]
    yy, xx = torch.meshgrid(torch.arange(H, device=dev, dtype=torch.float32),
                            torch.arange(W, device=dev, dtype=torch.float32), indexing="ij")
    flow = F.interpolate(torch.randn(B, 2, 4, 5, generator=g).to(dev) * 6, size=(H, W), mode="bilinear",
                         align_corners=True)
    coords = (torch.stack([xx, yy])[None] + flow).contiguous()
    scale = C ** -0.5
    out = torch.ops.raft_stir.corr_otf(f1n, f2n, coords, r, scale, True)
    for label, dout in (("random dout", torch.randn_like(out.float()).to(out.dtype)),
                        ("zero dout (no df2 atomics)", torch.zeros_like(out))):
        for _ in range(3):
            torch.ops.raft_stir.corr_otf_backward(f1n, f2n, coords, r, scale, dout)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            torch.ops.raft_stir.corr_otf_backward(f1n, f2n, coords, r, scale, dout)
        e1.record()
        torch.cuda.synchronize()
        print(f"{name:>10} B={B} C={C} {H}x{W} r={r}: {label:>28}: {e0.elapsed_time(e1) / reps * 1e3:8.1f} us/call "
              "(incl. df2 zero-fill / casts)", flush=True)


def main():
    _ext.load(raise_on_error=True)
    run("raft-small", 8, 128, 46, 62, 3)
    run("raft", 8, 256, 46, 62, 4)


if __name__ == "__main__":
    main()
