#!/usr/bin/env python
"""Whole-step hipGraph training (runtime/graph.py GraphedTrainStep) vs the
eager step: ms/step and the loss trajectory from the same initialisation.

    python scripts/graph_train_probe.py [--steps 20] [--batch 8]
"""
import argparse
import copy
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
    from raft_stir_amd.runtime.graph import GraphedTrainStep
    from raft_stir_amd.train.loss import sequence_loss
    from raft_stir_amd.train.optim import fetch_optimizer
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m_e = RAFT(make_args(mixed_precision=True, corr_dtype="auto")).to(dev).to(memory_format=torch.channels_last).train()
    m_g = copy.deepcopy(m_e)
    targs = argparse.Namespace(lr=4e-4, wdecay=1e-4, epsilon=1e-8, num_steps=1000)
    loss_fn = lambda p, f, v: sequence_loss(p, f, v, gamma=0.8, sync_metrics=False)[0]
    pool = DevicePool(4, a.batch, 368, 496, dev, seed=0)
    batches = [pool.next() for _ in range(4)]

    # eager
    opt_e, sch_e = fetch_optimizer(targs, m_e)
    def estep(b):
        opt_e.zero_grad(set_to_none=True)
        loss = loss_fn(m_e(b[0], b[1], iters=12), b[2], b[3])
        loss.backward()
        torch.nn.utils.clip_grad_norm_(m_e.parameters(), 1.0)
        opt_e.step()
        sch_e.step()
        return loss.detach()
    # graphed (warmup steps inside the constructor advance the weights: mirror them eagerly)
    opt_g, sch_g = fetch_optimizer(targs, m_g, capturable=True)
    t0 = time.perf_counter()
    gs = GraphedTrainStep(m_g, opt_g, loss_fn, batches[0], clip=1.0, warmup=3)
    print(f"capture {time.perf_counter() - t0:.1f}s", flush=True)
    for _ in range(3 + 1):  # warmup + the captured step itself both ran one update each... capture does not execute
        pass
    torch.cuda.synchronize()
    le, lg = [], []
    for i in range(a.steps):
        b = batches[i % 4]
        le.append(estep(b))
        lg.append(gs.step(b).clone())
        sch_g.step()
    torch.cuda.synchronize()
    print("eager losses ", [round(float(x), 3) for x in le[:6]])
    print("graph losses ", [round(float(x), 3) for x in lg[:6]])
    for name, fn in (("eager", lambda b: estep(b)), ("graph", lambda b: (gs.step(b), sch_g.step()))):
        for i in range(3):
            fn(batches[i % 4])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            fn(batches[i % 4])
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        print(f"{name}: {1e3 * dt:.2f} ms/step, {a.batch / dt:.1f} pairs/s", flush=True)


if __name__ == "__main__":
    main()
