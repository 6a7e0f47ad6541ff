#!/usr/bin/env python
"""Where does the host time of a training step go?  cProfile of 5 steps
(synchronising after each) -> top functions by cumulative / internal time.

    python scripts/host_profile.py [--small]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--small", action="store_true")
    ap.add_argument("--top", type=int, default=45)
    a = ap.parse_args()
    from raft_stir_amd.config import make_args
    from raft_stir_amd.data.synthetic import DevicePool
    from raft_stir_amd.models import RAFT
    from raft_stir_amd.train.loss import sequence_loss
    from raft_stir_amd.train.optim import fetch_optimizer
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = RAFT(make_args(mixed_precision=True, small=a.small, corr_dtype="auto")).to(dev)
    model = model.to(memory_format=torch.channels_last).train()
    opt, sched = fetch_optimizer(argparse.Namespace(lr=4e-4, wdecay=1e-4, epsilon=1e-8, num_steps=1000), model)
    pool = DevicePool(4, 8, 368, 496, dev, seed=0)

    def step():
        i1, i2, flow, valid = pool.next()
        opt.zero_grad(set_to_none=True)
        preds = model(i1, i2, iters=12)
        loss, _ = sequence_loss(preds, flow, valid, gamma=0.8, sync_metrics=False)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        sched.step()
    for _ in range(4):
        step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    for _ in range(5):
        torch.cuda.synchronize()
        pr.enable()
        step()
        pr.disable()
    torch.cuda.synchronize()
    for key in ("tottime", "cumulative"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(a.top)
        print(f"==== by {key} (5 steps)")
        print(s.getvalue())


if __name__ == "__main__":
    main()
