#!/usr/bin/env python
"""Host (CPU) time of the training step's phases, without device syncs
inside the step: wraps the engine's backward pieces with perf_counter and
reports the mean per step (where the host, not the GPU, sets the pace of the
step's issue -- the main-queue gaps of scripts/trace_streams.py).

    python scripts/host_profile.py [--steps 20] [--small]
"""
import argparse
import collections
import functools
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

T = collections.defaultdict(float)


def wrap(owner, name, label, static=False):
    fn = getattr(owner, name)
    raw = fn.__func__ if isinstance(fn, (staticmethod, classmethod)) else fn

    @functools.wraps(raw)
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return raw(*a, **k)
        finally:
            T[label] += time.perf_counter() - t0
    setattr(owner, name, staticmethod(w) if static else w)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--small", action="store_true")
    a = ap.parse_args()
    from raft_stir_amd.config import make_args
    from raft_stir_amd.models import RAFT
    from raft_stir_amd.models import fused_train as FT
    from raft_stir_amd.models import fused_encoder as FE
    from raft_stir_amd.ops import corr as OC
    from raft_stir_amd.train.loss import sequence_loss
    from raft_stir_amd.train.optim import fetch_optimizer
    from raft_stir_amd.data.synthetic import DevicePool
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = RAFT(make_args(small=a.small, mixed_precision=True)).to(dev).to(memory_format=torch.channels_last).train()
    opt, sched = fetch_optimizer(argparse.Namespace(lr=4e-4, wdecay=1e-4, epsilon=1e-8, num_steps=100000), model)
    pool = DevicePool(4, 8, 368, 496, dev, seed=0)
    wrap(FT.FusedTrainLoop, "_param_grads", "update: _param_grads (all)", static=True)
    wrap(FT.FusedTrainLoop, "_wgrads", "update: _wgrads issue", static=True)
    wrap(FT, "_small_wgrads", "update: _small_wgrads issue")
    wrap(FT.FusedTrainEngine, "unpack_grads", "update: unpack_grads")
    wrap(FT.FusedTrainEngine, "grad_buffers", "update: grad_buffers")
    wrap(FT.FusedTrainLoop, "backward", "update: FusedTrainLoop.backward", static=True)
    wrap(FT.FusedTrainLoop, "forward", "update: FusedTrainLoop.forward", static=True)
    wrap(OC._CorrVolume, "backward", "corr: volume backward", static=True)
    wrap(FE._StageFn, "backward", "encoders: stage backward", static=True)
    wrap(FE._StageFn, "forward", "encoders: stage forward", static=True)

    def step():
        i1, i2, flow, valid = pool.next()
        t0 = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        preds = model(i1, i2, iters=12)
        t1 = time.perf_counter()
        loss, _ = sequence_loss(preds, flow, valid, gamma=0.8, sync_metrics=False)
        t2 = time.perf_counter()
        loss.backward()
        t3 = time.perf_counter()
        opt.clip_and_step(1.0) if hasattr(opt, "clip_and_step") else opt.step()
        sched.step()
        t4 = time.perf_counter()
        T["step: forward"] += t1 - t0
        T["step: loss"] += t2 - t1
        T["step: backward"] += t3 - t2
        T["step: optimizer"] += t4 - t3
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    T.clear()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(a.steps):
        step()
    t_host = time.perf_counter() - t0
    e1.record()
    torch.cuda.synchronize()
    print(f"host issue {1e3 * t_host / a.steps:.3f} ms/step, GPU {e0.elapsed_time(e1) / a.steps:.3f} ms/step")
    for k in sorted(T):
        print(f"  {k:40s} {1e3 * T[k] / a.steps:8.3f} ms")


if __name__ == "__main__":
    main()
