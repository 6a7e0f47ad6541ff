#!/usr/bin/env python
"""Weight-stationary conv kernel (csrc/conv_ws.hip) vs the tuned tile kernels
on every distinct update-block conv call of one training step and one
inference forward at the bench shapes (calls recorded as in tune_conv.py).

For each call: graph-timed latency of the current tile choice, of the
weight-stationary kernel with the cost-model configuration and (--sweep)
with every feasible configuration; the outputs are cross-checked.  With
--write the fastest weight-stationary configuration per call shape is
stored in the "ws" section of raft_stir_amd/conv_tuning.json.

    python scripts/bench_conv_ws.py [--sweep] [--write] [--reps 20]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import torch  # noqa: E402


def candidates(C, B, H, W, cout, ktot, kh, kw, cout_pad, epi):
    """rows-per-chunk variants of the one configuration (grid ~1x / 2x the CUs)"""
    base = C.ws_config(B, H, W, cout, ktot, kh, kw, cout_pad, epi)
    if base is None:
        return []
    out = []
    for target in (128, 256, 512):
        cfg = base[:4] + [C.ws_rows_per_chunk(B, H, W, cout, target)]
        if cfg not in out:
            out.append(cfg)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--write", action="store_true")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, nargs=2, default=[368, 496])
    ap.add_argument("--infer-size", type=int, nargs=2, default=[436, 1088])
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--small", action="store_true")
    ap.add_argument("--out", default=os.path.join(ROOT, "raft_stir_amd", "conv_tuning.json"))
    args = ap.parse_args()
    os.environ["RS_CONV_WS"] = "0"  # record on the tile kernels
    from raft_stir_amd.ops import _ext
    from raft_stir_amd.ops import conv as C
    from tune_conv import gtime, record_calls
    _ext.load(raise_on_error=True)
    t0 = time.time()
    calls = record_calls(args)
    print(f"{len(calls)} distinct conv calls recorded in {time.time() - t0:.1f}s", flush=True)
    best_ws, tot = {}, [0.0, 0.0, 0.0]
    for key, (tag, c) in sorted(calls.items()):
        kw = {k: v for k, v in c.items() if k not in ("tile", "wf", "ws_cfg")}
        for k in ("out", "out2", "out3"):
            if kw[k] is not None:
                kw[k] = kw[k].clone()
        t_in = kw["segs"][0][0]
        B, H, W = t_in.shape[:3]
        ktot = sum(s[2] for s in kw["segs"])
        wf = C.frag_layout(kw["w"])
        auto = C.ws_config(B, H, W, kw["cout"], ktot, kw["kh"], kw["kw"], wf.shape[0], kw["epi"])
        t_tile = gtime(lambda: C.conv_fused(**kw), args.reps)
        outs = {}
        ref_out = kw["out"].clone()
        if auto is None:
            print(f"{tag:5s} {key:44s} tile {t_tile:7.1f}us  ws: no configuration", flush=True)
            tot[0] += t_tile
            tot[1] += t_tile
            tot[2] += t_tile
            continue
        res = {}
        cands = candidates(C, B, H, W, kw["cout"], ktot, kw["kh"], kw["kw"], wf.shape[0], kw["epi"]) if args.sweep else []
        if auto not in cands:
            cands = [auto] + cands
        for cfg in cands:
            try:
                res[tuple(cfg)] = gtime(lambda: C.conv_fused(**kw, wf=wf, ws_cfg=cfg, tile=C.WS_TILE), args.reps)
            except RuntimeError as e:
                print("  skip", cfg, str(e).splitlines()[0])
        # numerics: one clean run of each path from the same initial output
        init = {k: (kw[k].clone() if kw[k] is not None else None) for k in ("out", "out2", "out3")}
        C.conv_fused(**kw)
        a = kw["out"].float().clone()
        for k in ("out", "out2", "out3"):
            if init[k] is not None:
                kw[k].copy_(init[k])
        C.conv_fused(**kw, wf=wf, ws_cfg=auto, tile=C.WS_TILE)
        b = kw["out"].float()
        err = float((a - b).abs().max()) / max(float(a.abs().max()), 1e-6)
        best = min(res, key=res.get)
        best_ws[f"{B}x{H}x{W}|{kw['cout']}|{ktot}|{kw['kh']}x{kw['kw']}"] = list(best)
        tot[0] += t_tile
        tot[1] += res[tuple(auto)]
        tot[2] += min(res[best], t_tile)
        print(f"{tag:5s} {key:44s} tile {t_tile:7.1f}us  ws-auto {res[tuple(auto)]:7.1f}us {auto}  "
              f"ws-best {res[best]:7.1f}us {list(best)}  relerr {err:.2e}", flush=True)
    print(f"sum over distinct calls: tiles {tot[0]:.1f}us  ws-auto {tot[1]:.1f}us  best-of {tot[2]:.1f}us")
    if args.write:
        old = {}
        if os.path.exists(args.out):
            with open(args.out) as f:
                old = json.load(f)
        old["ws"] = {**old.get("ws", {}), **best_ws}
        with open(args.out, "w") as f:
            json.dump(old, f, indent=1)
        print("wrote", args.out)


if __name__ == "__main__":
    main()
