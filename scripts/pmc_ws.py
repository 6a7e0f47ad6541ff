#!/usr/bin/env python
"""One update-block conv launched N times (for rocprofv3 --pmc runs):
weight-stationary kernel with a given configuration, or a tile kernel.

    python scripts/pmc_ws.py --shape 8 46 62 --k 1 5 --cin 384 --cout 256 --epi 3 --cfg 6 1 4 2 24
    python scripts/pmc_ws.py ... --tile 31
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", type=int, nargs=3, default=[8, 46, 62])
    ap.add_argument("--k", type=int, nargs=2, default=[1, 5])
    ap.add_argument("--cin", type=int, default=384)
    ap.add_argument("--cout", type=int, default=256)
    ap.add_argument("--epi", type=int, default=1)
    ap.add_argument("--cfg", type=int, nargs=5, default=None)
    ap.add_argument("--tile", type=int, default=None)
    ap.add_argument("--n", type=int, default=10)
    ap.add_argument("--stamps", default=None, help="RS_WS_STAMPS build: write per-wave stamps of the last launch (.npy)")
    args = ap.parse_args()
    from raft_stir_amd.ops import _ext
    from raft_stir_amd.ops import conv as C
    _ext.load(raise_on_error=True)
    dev = torch.device("cuda", 0)
    B, H, W = args.shape
    kh, kw = args.k
    x = torch.randn(B, H, W, args.cin, device=dev).to(torch.bfloat16)
    w = torch.randn(args.cout, args.cin, kh, kw, device=dev) * 0.02
    wp = C.pack_weight(w, [(args.cin, [(0, args.cin, 0)])], C.pad_to(args.cout, 128))
    wf = C.frag_layout(wp)
    b = torch.randn(args.cout, device=dev)
    hd = args.cout // 2
    kw_ = {}
    if args.epi == C.EPI_GRU_ZR:
        out = torch.empty(B, H, W, hd, device=dev, dtype=torch.bfloat16)
        kw_ = dict(hd=hd, out2=torch.empty_like(out), aux1=x, a1off=0)
    else:
        out = torch.empty(B, H, W, args.cout, device=dev, dtype=torch.bfloat16)
    cfg = args.cfg
    st = None
    if args.stamps:
        st = torch.zeros(8192 * 8 * 66, dtype=torch.int64, device=dev)
        cfg = list(cfg) + [st.data_ptr()]
    for _ in range(args.n):
        if args.tile is not None:
            C.conv_fused([(x, 0, args.cin)], wp, b, kh, kw, args.cout, args.epi, out, 0, tile=args.tile, **kw_)
        else:
            C.conv_fused([(x, 0, args.cin)], None, b, kh, kw, args.cout, args.epi, out, 0, tile=C.WS_TILE, wf=wf,
                         ws_cfg=cfg, **kw_)
    torch.cuda.synchronize()
    if st is not None:
        import numpy as np
        a = st.view(-1, 66).cpu().numpy()
        np.save(args.stamps, a[a[:, 0] > 0])
    print("ok")


if __name__ == "__main__":
    main()
