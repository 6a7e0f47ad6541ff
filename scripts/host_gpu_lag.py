#!/usr/bin/env python
"""How far ahead of the GPU does the host run in the eager training step?

For each bench step: the host wall clock when the step's enqueue starts and
ends, and the GPU clock (events, mapped onto the host clock by one
synchronised reference point) when the step's first / last kernels finish.
A step whose enqueue starts AFTER the previous step's GPU work finished
leaves the GPU idle (host-bound); the lead column says by how much the host
was ahead.

    python scripts/host_gpu_lag.py [--steps 20]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=8)
    a = ap.parse_args()
    import argparse as ap_
    from raft_stir_amd.config import make_args
    from raft_stir_amd.data.synthetic import DevicePool
    from raft_stir_amd.models import RAFT
    from raft_stir_amd.train.loss import sequence_loss
    from raft_stir_amd.train.optim import fetch_optimizer
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = RAFT(make_args(mixed_precision=True)).to(dev).to(memory_format=torch.channels_last).train()
    opt, sched = fetch_optimizer(ap_.Namespace(lr=4e-4, wdecay=1e-4, epsilon=1e-8, num_steps=1000), model)
    pool = DevicePool(4, a.batch, 368, 496, dev, seed=0)
    marks = {}

    def step(i):
        ev = lambda k: marks.setdefault(k, []).append((time.perf_counter(), torch.cuda.Event(enable_timing=True)))
        i1, i2, flow, valid = pool.next()
        opt.zero_grad(set_to_none=True)
        ev("start"); marks["start"][-1][1].record()
        preds = model(i1, i2, iters=12)
        ev("fwd"); marks["fwd"][-1][1].record()
        loss, _ = sequence_loss(preds, flow, valid, gamma=0.8, sync_metrics=False)
        loss.backward()
        ev("bwd"); marks["bwd"][-1][1].record()
        opt.clip_and_step(1.0)
        sched.step()
        ev("end"); marks["end"][-1][1].record()

    for i in range(5):
        step(i)
    torch.cuda.synchronize()
    marks.clear()
    ref = torch.cuda.Event(enable_timing=True)
    ref.record()
    torch.cuda.synchronize()
    t_ref = time.perf_counter()
    for i in range(a.steps):
        step(i)
    torch.cuda.synchronize()
    g = lambda e: t_ref + ref.elapsed_time(e) / 1000.0  # GPU completion time on the host clock
    print("step  host_start  gpu_fwd_done  gpu_bwd_done  gpu_end   (ms, relative to the first step's host start)"
          "   host_lead_at_start(ms)")
    t0 = marks["start"][0][0]
    prev_end = None
    for i in range(a.steps):
        hs = marks["start"][i][0]
        ge = g(marks["end"][i][1])
        lead = (prev_end - hs) * 1e3 if prev_end is not None else float("nan")
        print(f"{i:4d} {1e3 * (hs - t0):10.2f} {1e3 * (g(marks['fwd'][i][1]) - t0):12.2f} "
              f"{1e3 * (g(marks['bwd'][i][1]) - t0):12.2f} {1e3 * (ge - t0):9.2f} {lead:10.2f}")
        prev_end = ge
    n = a.steps
    host_ms = [(marks["end"][i][0] - marks["start"][i][0]) * 1e3 for i in range(n)]
    gpu_ms = [marks["start"][i][1].elapsed_time(marks["end"][i][1]) for i in range(n)]
    gf = [marks["start"][i][1].elapsed_time(marks["fwd"][i][1]) for i in range(n)]
    gb = [marks["fwd"][i][1].elapsed_time(marks["bwd"][i][1]) for i in range(n)]
    print(f"host enqueue per step {sum(host_ms) / n:.2f} ms; GPU per step {sum(gpu_ms) / n:.2f} ms "
          f"(forward {sum(gf) / n:.2f}, loss+backward {sum(gb) / n:.2f})")


if __name__ == "__main__":
    main()
