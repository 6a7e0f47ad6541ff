#!/usr/bin/env python
"""Per-call kernel-variant tuning of the fused update-block convolutions.

Records every ``conv_fused`` call of one fused training step (RAFT full,
bf16, the bench shape: batch 8 at 368x496, 12 iterations) and of one
inference forward (1088x436 -> 440x1088, batch 1), then times every
applicable tile of csrc/conv*.hip on each distinct call (same operands, one
hipGraph of back-to-back launches, so host dispatch is excluded) and writes
the fastest per call signature into raft_stir_amd/conv_tuning.json, which
ops/conv.py consults before its heuristic.

    python scripts/tune_conv.py [--out raft_stir_amd/conv_tuning.json] [--reps 20]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

F32_CANDIDATES = [6, 7, 8, 38, 39, 40, 81, 82, 83, 84, 85]
CANDIDATES = [3, 4, 6, 7, 16, 17, 19, 20, 21, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 42, 43,
              44, 45, 46, 48, 49, 50, 51, 52, 53, 54, 56, 57, 61, 65, 66, 68, 70]  # 56-68: calls that carry a wf weight; 70: 1x1


def record_calls(args):
    from raft_stir_amd.config import make_args
    from raft_stir_amd.data.synthetic import make_batch
    from raft_stir_amd.models import RAFT
    from raft_stir_amd.ops import conv as C
    from raft_stir_amd.train.loss import sequence_loss
    from raft_stir_amd.utils.padder import InputPadder
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = RAFT(make_args(mixed_precision=not args.f32, small=args.small)).to(dev).to(memory_format=torch.channels_last)
    calls = {}

    def grab(tag, fn):
        C._RECORD = []
        fn()
        torch.cuda.synchronize()
        for c in C._RECORD:
            t0 = c["segs"][0][0]
            key = C.tune_key(t0.shape[0], t0.shape[1], t0.shape[2], c["cout"], [s[2] for s in c["segs"]],
                             c["kh"], c["kw"], c["epi"])
            if c["tile"] is None and key not in calls:
                calls[key] = (tag, c)
        C._RECORD = None

    if not args.f32 and not args.infer_only:
        model.train()
        i1, i2, flow, valid = make_batch(args.batch, *args.size, seed=0, device=dev)

        def train_step():
            preds = model(i1, i2, iters=args.iters)
            loss, _ = sequence_loss(preds, flow, valid, 0.8, sync_metrics=False)
            loss.backward()
        train_step()  # warm (engine buffers)
        grab("train", train_step)
    model.eval()
    h, w = args.infer_size
    j1 = torch.rand(1, 3, h, w, device=dev) * 255
    j2 = torch.rand(1, 3, h, w, device=dev) * 255
    j1, j2 = InputPadder(j1.shape).pad(j1, j2)

    def infer():
        with torch.no_grad():
            model(j1, j2, iters=args.iters, test_mode=True)
    infer()
    grab("infer", infer)
    return calls


def gtime(fn, reps):
    fn()
    torch.cuda.synchronize()
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
    best = float("inf")
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) * 1000.0 / reps)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "raft_stir_amd", "conv_tuning.json"))
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, nargs=2, default=[368, 496])
    ap.add_argument("--infer-size", type=int, nargs=2, default=[436, 1088])
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--small", action="store_true", help="tune RAFT-small's calls")
    ap.add_argument("--merge", action="store_true", help="update the existing table instead of replacing it")
    ap.add_argument("--show", default="", help="print every candidate's time (and error) for keys containing this")
    ap.add_argument("--infer-only", action="store_true", help="record only the inference forward's calls")
    ap.add_argument("--f32", action="store_true",
                    help="fp32 inference calls on the split-bf16 F32 tiles -> the 'tiles_f32' table")
    args = ap.parse_args()
    os.environ["RS_CONV_TUNED"] = "0"  # record with the heuristic, compare against it
    from raft_stir_amd.ops import _ext
    from raft_stir_amd.ops import conv as C
    _ext.load(raise_on_error=True)
    t0 = time.time()
    calls = record_calls(args)
    print(f"{len(calls)} distinct conv calls recorded in {time.time() - t0:.1f}s", flush=True)
    table, report = {}, []
    for key, (tag, c) in sorted(calls.items()):
        kw = {k: v for k, v in c.items() if k != "tile"}
        # private copies of everything the kernel writes: timing must not disturb the engine buffers
        for k in ("out", "out2", "out3"):
            if kw[k] is not None:
                kw[k] = kw[k].clone()
        t_in = kw["segs"][0][0]
        if args.f32:
            heur = C.choose_tile_f32(t_in.shape[0] * t_in.shape[1] * t_in.shape[2], kw["cout"],
                                     v3f=getattr(kw["w"], "_rs_frag32", None) is not None)
            cands = F32_CANDIDATES
        else:
            heur = C.choose_tile(t_in.shape[0] * t_in.shape[1] * t_in.shape[2], kw["cout"],
                                 [s[2] for s in kw["segs"]], kw["kh"] * kw["kw"])
            cands = CANDIDATES
        res = {}
        if kw.get("wf") is None and getattr(kw["w"], "_rs_frag", None) is None:
            cands = [t for t in cands if t not in C.V3_TILES]
        for t in sorted(set(cands + [heur])):
            try:
                res[t] = gtime(lambda: C.conv_fused(**kw, tile=t), args.reps)
            except (RuntimeError, ValueError) as e:
                if t == heur:
                    print("  heuristic tile failed:", str(e).splitlines()[0], flush=True)
                if args.show and args.show in key:
                    print(f"  {key} t{t}: {str(e).splitlines()[0][:120]}", flush=True)
                continue
        if args.show and args.show in key:
            print("  " + key + " " + " ".join(f"t{t}={v:.1f}" for t, v in sorted(res.items())), flush=True)
        if not res:
            print(f"{tag:5s} {key:42s} no applicable tile, skipped", flush=True)
            continue
        best = min(res, key=res.get)
        table[key] = best
        report.append(dict(key=key, phase=tag, heuristic=heur, us_heuristic=round(res.get(heur, res[best]), 2), best=best,
                           us_best=round(res[best], 2)))
        print(f"{tag:5s} {key:42s} heur t{heur} {res.get(heur, float('nan')):7.1f}us  best t{best} {res[best]:7.1f}us", flush=True)
    section, rsection = ("tiles_f32", "report_f32") if args.f32 else ("tiles", "report")
    old = {}
    if os.path.exists(args.out):
        with open(args.out) as f:
            old = json.load(f)
    if args.merge:
        keys = set(table)
        table = {**old.get(section, {}), **table}
        report = [r for r in old.get(rsection, []) if r["key"] not in keys] + report
    old.update({"device": torch.cuda.get_device_name(0), "note": "scripts/tune_conv.py", section: table,
                rsection: report})
    with open(args.out, "w") as f:
        json.dump(old, f, indent=1)
    tot_h = sum(r["us_heuristic"] for r in report)
    tot_b = sum(r["us_best"] for r in report)
    print(f"sum over distinct calls: heuristic {tot_h:.1f}us -> tuned {tot_b:.1f}us; wrote {args.out}")


if __name__ == "__main__":
    main()
