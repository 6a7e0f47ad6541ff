#!/usr/bin/env python
"""Microbenchmark of the small (non-GEMM) training-loop kernels at the
training shape (batch 8, 368x496 -> 46x62, 12 iterations): flow encoder
(7x7 2->128 conv + ReLU, csrc/conv.hip flow_enc_kernel), batched convex
upsampling forward / backward (csrc/convex_upsample.hip), with fp32 PyTorch
references for correctness."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def timeit(fn, reps=20):
    """GPU time per call: the calls are captured in a hipGraph and replayed, so
    host-side op dispatch (10-15 us per torch.ops call) is not measured."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / (5 * reps)


def main():
    from raft_stir_amd.ops import _ext
    from raft_stir_amd.ops import reference as ref
    _ext.load(raise_on_error=True)
    R = torch.ops.raft_stir
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    B, H, W, IT = 8, 46, 62, 12
    # flow encoder
    c0 = ref.coords_grid(B, H, W, device=dev)
    coords = (c0 + torch.randn(B, 2, H, W, device=dev) * 4).contiguous()
    w = torch.randn(128, 2, 7, 7, device=dev) * 0.05
    bsc = torch.randn(128, device=dev) * 0.1
    wk = w.permute(2, 3, 1, 0).contiguous()  # [7][7][2][128]
    out = torch.empty(B, H, W, 128, device=dev, dtype=torch.bfloat16)
    hx = torch.zeros(B, H, W, 256, device=dev, dtype=torch.bfloat16)
    us = timeit(lambda: R.flow_encode(coords, wk, bsc, out, 0, hx, 254))
    r = F.relu(F.conv2d(coords - c0, w, bsc, padding=3)).permute(0, 2, 3, 1)
    err = ((out.float() - r).abs().max() / r.abs().max()).item()
    ferr = (hx[..., 254:].float() - (coords - c0).permute(0, 2, 3, 1)).abs().max().item()
    print(f"flow_encode 7x7 2->128  {us:7.1f} us  rel err {err:.2e}  flow slot err {ferr:.2e}", flush=True)
    # flow-head output conv (3x3 256->2 + coords epilogue) and its dgrad
    head = torch.relu(torch.randn(B, H, W, 512, device=dev)).to(torch.bfloat16)
    w2k = (torch.randn(2, 256, 3, 3, device=dev) * 0.05).permute(0, 2, 3, 1).contiguous()
    b2 = torch.randn(2, device=dev)
    crd = torch.empty_like(coords)
    us = timeit(lambda: R.flow_head(head, 0, 256, w2k, b2, crd, coords))
    dfl = torch.randn(B, 2, H, W, device=dev)
    dh = torch.empty(B, H, W, 512, device=dev, dtype=torch.bfloat16)
    us2 = timeit(lambda: R.flow_head_dgrad(dfl, w2k, 256, head, 0, dh, 0))
    print(f"flow_head 3x3 256->2     {us:7.1f} us   dgrad {us2:7.1f} us", flush=True)
    # convex upsampling, all iterations batched
    n = IT * B
    flow = torch.randn(n, 2, H, W, device=dev) * 3
    mask = torch.randn(n, H, W, 576, device=dev).to(torch.bfloat16)
    us = timeit(lambda: R.convex_upsample(flow, mask))
    up = R.convex_upsample(flow, mask)
    r = ref.convex_upsample(flow[:8], mask[:8].float().permute(0, 3, 1, 2))
    err = (up[:8] - r).abs().max().item()
    mb = (up.numel() * 4 + mask.numel() * 2) / 1e6
    print(f"convex_up fwd x{n}       {us:7.1f} us  {mb / us:.2f} TB/s  max err {err:.2e}", flush=True)
    g = torch.randn_like(up)
    us = timeit(lambda: R.convex_upsample_backward(flow, mask, g))
    dflow, dmask = R.convex_upsample_backward(flow, mask, g)
    fr = flow[:8].clone().requires_grad_(True)
    mr = mask[:8].float().permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    ref.convex_upsample(fr, mr).backward(g[:8])
    e1 = (dflow[:8] - fr.grad).abs().max().item() / fr.grad.abs().max().item()
    e2 = (dmask[:8].float().permute(0, 3, 1, 2) - mr.grad).abs().max().item() / mr.grad.abs().max().item()
    mb = (g.numel() * 4 + 2 * mask.numel() * 2) / 1e6
    print(f"convex_up bwd x{n}       {us:7.1f} us  {mb / us:.2f} TB/s  rel err dflow {e1:.2e} dmask {e2:.2e}",
          flush=True)


if __name__ == "__main__":
    main()
