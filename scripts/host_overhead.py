#!/usr/bin/env python
"""Is the training step host-bound?  Times the host side of each bench step
(enqueue only, no synchronisation) against the GPU time per step.

    python scripts/host_overhead.py [--steps 20]
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
    from raft_stir_amd.config import make_args
    from raft_stir_amd.data.synthetic import DevicePool
    from raft_stir_amd.models import RAFT
    from raft_stir_amd.train.loss import sequence_loss
    from raft_stir_amd.train.optim import fetch_optimizer
    import argparse as ap_
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = RAFT(make_args(mixed_precision=True, corr_dtype="auto")).to(dev).to(memory_format=torch.channels_last).train()
    opt, sched = fetch_optimizer(ap_.Namespace(lr=4e-4, wdecay=1e-4, epsilon=1e-8, num_steps=1000), model)
    pool = DevicePool(4, a.batch, 368, 496, dev, seed=0)

    def step():
        i1, i2, flow, valid = pool.next()
        opt.zero_grad(set_to_none=True)
        preds = model(i1, i2, iters=12)
        loss, _ = sequence_loss(preds, flow, valid, gamma=0.8, sync_metrics=False)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        sched.step()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    m0 = torch.cuda.memory_stats()
    host = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        h0 = time.perf_counter()
        step()
        host.append(time.perf_counter() - h0)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.steps
    m1 = torch.cuda.memory_stats()
    keys = ("num_alloc_retries", "num_device_alloc", "num_device_free", "num_sync_all_streams")
    print("allocator over the timed steps:", {k: m1.get(k, 0) - m0.get(k, 0) for k in keys})
    # host time of a step when the GPU is idle at its start (sync before each)
    iso = []
    for _ in range(5):
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        step()
        iso.append(time.perf_counter() - h0)
    torch.cuda.synchronize()
    print(f"wall {1e3 * wall:.2f} ms/step; host enqueue in the stream {1e3 * sum(host) / len(host):.2f} ms/step "
          f"(max {1e3 * max(host):.2f}); host enqueue from idle {1e3 * min(iso):.2f} ms")


if __name__ == "__main__":
    main()
