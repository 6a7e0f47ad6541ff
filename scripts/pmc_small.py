#!/usr/bin/env python
"""Drive one small kernel a few times for rocprofv3 --pmc counter runs.
    python scripts/pmc_small.py {wgrad|fwd|dgrad|enc}"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from raft_stir_amd.ops import _ext
    _ext.load(raise_on_error=True)
    R = torch.ops.raft_stir
    dev = torch.device("cuda", 0)
    which = sys.argv[1]
    B, H, W, IT = 8, 46, 62, 12
    if which == "wgrad":  # convf1 weight gradient over all iterations (csrc/conv_wgrad.hip flow_wgrad_kernel)
        crd = torch.randn(IT * B, 2, H, W, device=dev) * 4
        dfs = torch.randn(IT * B, H, W, 128, device=dev).to(torch.bfloat16)
        dw = torch.zeros(49, 2, 128, device=dev)
        db = torch.zeros(128, device=dev)
        fn = lambda: R.flow_wgrad(crd, dfs, dw, db)
    elif which in ("fwd", "dgrad"):
        head = torch.relu(torch.randn(B, H, W, 512, device=dev)).to(torch.bfloat16)
        w2 = torch.randn(2, 3, 3, 256, device=dev)
        crd = torch.randn(B, 2, H, W, device=dev)
        src = torch.randn(B, 2, H, W, device=dev)
        dh = torch.empty(B, H, W, 512, device=dev, dtype=torch.bfloat16)
        b2 = torch.randn(2, device=dev)
        if which == "fwd":
            fn = lambda: R.flow_head(head, 0, 256, w2, b2, crd, src)
        else:
            fn = lambda: R.flow_head_dgrad(src, w2, 256, head, 0, dh, 0)
    else:
        coords = torch.randn(B, 2, H, W, device=dev)
        wk = torch.randn(7, 7, 2, 128, device=dev)
        bk = torch.randn(128, device=dev)
        out = torch.empty(B, H, W, 128, device=dev, dtype=torch.bfloat16)
        fn = lambda: R.flow_encode(coords, wk, bk, out, 0, None, 0)
    for _ in range(5):
        fn()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
