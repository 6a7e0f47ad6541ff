#!/usr/bin/env python
"""Host-side cost of a training step, per op and per thread: torch.profiler
(CPU activity only, so the GPU timeline is not perturbed by tracing) over 3
steps of the bench's eager step.  The autograd engine runs the backward on
its own device thread, which cProfile (scripts/host_profile.py) cannot see;
the profiler records both threads.  Prints the top ops by self CPU time and
the host time of each phase (forward / backward / optimizer) per step.

    python scripts/host_ops_profile.py [--top 40]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--fp32", action="store_true")
    a = ap.parse_args()
    from raft_stir_amd.config import make_args
    from raft_stir_amd.data.synthetic import DevicePool
    from raft_stir_amd.models import RAFT
    from raft_stir_amd.train.loss import sequence_loss
    from raft_stir_amd.train.optim import fetch_optimizer
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = RAFT(make_args(mixed_precision=not a.fp32)).to(dev).to(memory_format=torch.channels_last).train()
    opt, sched = fetch_optimizer(argparse.Namespace(lr=4e-4, wdecay=1e-4, epsilon=1e-8, num_steps=1000), model)
    pool = DevicePool(4, 8, 368, 496, dev, seed=0)
    phase = {}

    def step(rec=False):
        t0 = time.perf_counter()
        i1, i2, flow, valid = pool.next()
        opt.zero_grad(set_to_none=True)
        preds = model(i1, i2, iters=12)
        loss, _ = sequence_loss(preds, flow, valid, gamma=0.8, sync_metrics=False)
        t1 = time.perf_counter()
        loss.backward()
        t2 = time.perf_counter()
        if hasattr(opt, "clip_and_step"):
            opt.clip_and_step(1.0)
        else:
            torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
            opt.step()
        sched.step()
        t3 = time.perf_counter()
        if rec:
            for k, v in (("forward", t1 - t0), ("backward", t2 - t1), ("optimizer", t3 - t2)):
                phase.setdefault(k, []).append(v * 1e3)

    for _ in range(4):
        step()
    torch.cuda.synchronize()
    # host enqueue time per phase, GPU kept busy (no sync inside the step)
    for _ in range(5):
        step(True)
    torch.cuda.synchronize()
    print("host enqueue ms per step (no sync):", {k: round(sum(v) / len(v), 2) for k, v in phase.items()})
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU], record_shapes=False) as prof:
        for _ in range(3):
            step()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=a.top, max_name_column_width=60))


if __name__ == "__main__":
    main()
