#!/usr/bin/env python
"""200-step training fidelity probe (tests/test_train_fidelity_gpu.py setup):
deterministic fp32 through the fused HIP engine, deterministic bf16, and a
second fp32 run from weights perturbed by 1e-6 relative (the trajectory's own
chaos: how far two fp32 runs that differ only in round-off end up apart).
Prints the first / last 50-step mean loss of each run.

    python scripts/fidelity_probe.py [--steps 200]
"""
import argparse
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    from raft_stir_amd.config import make_args
    from raft_stir_amd.data.synthetic import make_batch
    from raft_stir_amd.models import RAFT
    from raft_stir_amd.runtime.determinism import deterministic
    from raft_stir_amd.train.loss import sequence_loss
    from raft_stir_amd.train.optim import fetch_optimizer
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    base = RAFT(make_args()).to(dev).to(memory_format=torch.channels_last).train()

    def run(model, steps):
        opt, sched = fetch_optimizer(make_args(lr=4e-4, wdecay=1e-5, epsilon=1e-8, num_steps=steps), model)
        out = []
        for s in range(steps):
            i1, i2, flow, valid = make_batch(2, 128, 192, seed=1000 + s, device=dev, max_disp=16.0)
            opt.zero_grad(set_to_none=True)
            preds = model(i1, i2, iters=6)
            loss, _ = sequence_loss(preds, flow, valid, 0.8, sync_metrics=False)
            loss.backward()
            opt.clip_and_step(1.0) if hasattr(opt, "clip_and_step") else None
            sched.step()
            out.append(loss.detach())
        return torch.stack(out).float().cpu()

    variants = {}
    m32 = copy.deepcopy(base)
    mbf = copy.deepcopy(base)
    mbf.cfg = mbf.cfg.__class__(**{**mbf.cfg.to_dict(), "mixed_precision": True})
    mpt = copy.deepcopy(base)
    with torch.no_grad():
        g = torch.Generator(device="cpu").manual_seed(7)
        for p in mpt.parameters():
            p.mul_(1 + 1e-6 * torch.randn(p.shape, generator=g).to(dev))
    with deterministic(True):
        for name, m in (("fp32", m32), ("bf16", mbf), ("fp32_perturbed", mpt)):
            l = run(m, a.steps)
            variants[name] = l
            w = min(50, a.steps // 4)
            print(f"{name:15s} first {l[:w].mean():.3f} last {l[-w:].mean():.3f}", flush=True)
    with deterministic(True):
        again = run(copy.deepcopy(base), 20)
    print("fp32 deterministic repeat (20 steps) bitwise equal:", torch.equal(again, variants["fp32"][:20]))


if __name__ == "__main__":
    main()
