#!/usr/bin/env python
"""Measure every BASELINE.json config (one JSON line each; synthetic inputs,
random-init weights).  Config 3 (training) is bench.py's headline and is not
repeated here.

  1  RAFT-small 4-iter forward on two demo-frame-sized images, CPU (plumbing)
  2  RAFT full 12-iter inference 1088x436, 1 MI355X, bf16 (hipGraph replay)
  4  KITTI 1242x375, on-the-fly correlation (alt_cuda_corr path), bf16
  5  STIR point tracker (RAFT-small, 12 iters, 1x3x512x640, 32 query points):
     graphed serving latency, plus TorchScript export + parity check
  6  config 2 in fp32 (the reference's default eval / export precision)
  7  config 5's served latency in bf16 (mixed precision)

    python scripts/bench_configs.py [--only 2 4] [--out profiles/bench_configs.jsonl]
"""
import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from raft_stir_amd.config import make_args  # noqa: E402
from raft_stir_amd.models import RAFT  # noqa: E402
from raft_stir_amd.utils.padder import InputPadder  # noqa: E402


def _time(fn, reps, sync):
    for _ in range(3):
        fn()
    sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    sync()
    return (time.perf_counter() - t0) / reps


def cfg1():
    torch.manual_seed(0)
    m = RAFT(make_args(small=True)).eval()
    i1 = torch.rand(1, 3, 436, 1024) * 255
    i2 = torch.rand(1, 3, 436, 1024) * 255
    i1, i2 = InputPadder(i1.shape).pad(i1, i2)
    with torch.no_grad():
        dt = _time(lambda: m(i1, i2, iters=4, test_mode=True), 3, lambda: None)
    return {"config": "raft-small 4-iter forward, 436x1024 pair, CPU", "ms": round(dt * 1e3, 1),
            "threads": torch.get_num_threads()}


def _infer(size, alt, iters, reps, bf16=True):
    from raft_stir_amd.runtime.graph import GraphedInference
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = RAFT(make_args(mixed_precision=bf16, alternate_corr=alt)).to(dev)
    m = m.to(memory_format=torch.channels_last).eval()
    h, w = size
    i1 = torch.rand(1, 3, h, w, device=dev) * 255
    i2 = torch.rand(1, 3, h, w, device=dev) * 255
    i1, i2 = InputPadder(i1.shape).pad(i1, i2)
    torch.cuda.reset_peak_memory_stats()
    g = GraphedInference(m, i1.shape, iters=iters)
    dt = _time(lambda: g(i1, i2), reps, torch.cuda.synchronize)
    return dt, torch.cuda.max_memory_allocated() / 2 ** 20, tuple(i1.shape[2:])


def cfg2():
    dt, mem, padded = _infer((436, 1088), False, 12, 30)
    return {"config": "raft full 12-iter inference 1088x436, bf16, hipGraph", "fps": round(1 / dt, 2),
            "ms_per_pair": round(dt * 1e3, 3), "padded": padded, "peak_mem_mib": round(mem)}


def cfg4():
    out = {"config": "KITTI 1242x375 12-iter inference, bf16, hipGraph"}
    for alt in (True, False):
        dt, mem, padded = _infer((375, 1242), alt, 12, 30)
        out["on_the_fly" if alt else "all_pairs"] = {"fps": round(1 / dt, 2), "ms_per_pair": round(dt * 1e3, 3),
                                                     "peak_mem_mib": round(mem), "padded": padded}
    return out


def cfg6():
    dt, mem, padded = _infer((436, 1088), False, 12, 30, bf16=False)
    return {"config": "raft full 12-iter inference 1088x436, fp32, hipGraph", "fps": round(1 / dt, 2),
            "ms_per_pair": round(dt * 1e3, 3), "padded": padded, "peak_mem_mib": round(mem)}


def cfg7():
    from raft_stir_amd.export.pointtrack import PointTrackServer
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = RAFT(make_args(small=True, mixed_precision=True)).to(dev).eval()
    i1 = torch.rand(1, 3, 512, 640, device=dev) * 255
    i2 = torch.rand(1, 3, 512, 640, device=dev) * 255
    pts = torch.rand(1, 32, 2, device=dev) * 500
    srv = PointTrackServer(m, iters=12)
    dt = _time(lambda: srv(pts, i1, i2), 50, torch.cuda.synchronize)
    return {"config": "STIR point tracker raft-small 12 iters 1x3x512x640, 32 points, bf16",
            "served_ms": round(dt * 1e3, 3), "served_fps": round(1 / dt, 1)}


def cfg5():
    from raft_stir_amd.export.pointtrack import PointTrackServer, RaftPointTrack, export_torchscript
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = RAFT(make_args(small=True)).to(dev).eval()
    H, W = 512, 640
    i1 = torch.rand(1, 3, H, W, device=dev) * 255
    i2 = torch.rand(1, 3, H, W, device=dev) * 255
    pts = torch.rand(1, 32, 2, device=dev) * 500
    srv = PointTrackServer(m, iters=12)
    dt = _time(lambda: srv(pts, i1, i2), 50, torch.cuda.synchronize)
    with torch.no_grad():
        ref = RaftPointTrack(m, 12)(pts, i1, i2)
    err = (srv(pts, i1, i2) - ref).abs().max().item()
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "raft_pointtrackSTIR.pt")
        export_torchscript(RaftPointTrack(m, 12).eval(), (pts, i1, i2), p)
        ts = torch.jit.load(p, map_location=dev)
        with torch.no_grad():
            ts_err = (ts(pts, i1, i2) - ref).abs().max().item()
            dts = _time(lambda: ts(pts, i1, i2), 10, torch.cuda.synchronize)
    return {"config": "STIR point tracker raft-small 12 iters 1x3x512x640, 32 points",
            "served_ms": round(dt * 1e3, 3), "served_fps": round(1 / dt, 1), "served_vs_eager_max_err": err,
            "torchscript_ms": round(dts * 1e3, 3), "torchscript_vs_eager_max_err": ts_err}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", type=int, nargs="+", default=[1, 2, 4, 5, 6, 7])
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    fns = {1: cfg1, 2: cfg2, 4: cfg4, 5: cfg5, 6: cfg6, 7: cfg7}
    lines = []
    for k in a.only:
        r = {"id": k, **fns[k]()}
        print(json.dumps(r), flush=True)
        lines.append(r)
    if a.out:
        with open(a.out, "a") as f:
            for r in lines:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
