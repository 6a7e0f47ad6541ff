#!/usr/bin/env python
"""Small-ensemble version of the 200-step training-fidelity check
(tests/test_train_fidelity_gpu.py setup): for each weight-init seed, fp32
(fused HIP engine, deterministic mode), bf16 default, bf16 deterministic
mode and fp32 on stock PyTorch ops.  Prints each run's first / last 50-step mean loss and the per-arm
ensemble means, to separate bf16 / determinism effects from the trajectory
chaos of a single run.

    python scripts/fidelity_ensemble.py [--seeds 3] [--steps 200]
"""
import argparse
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    from raft_stir_amd.config import make_args
    from raft_stir_amd.data.synthetic import make_batch
    from raft_stir_amd.models import RAFT
    from raft_stir_amd.runtime.determinism import deterministic
    from raft_stir_amd.train.loss import sequence_loss
    from raft_stir_amd.train.optim import fetch_optimizer
    dev = torch.device("cuda", 0)

    def run(model, steps):
        opt, sched = fetch_optimizer(make_args(lr=4e-4, wdecay=1e-5, epsilon=1e-8, num_steps=steps), model)
        out = []
        for s in range(steps):
            i1, i2, flow, valid = make_batch(2, 128, 192, seed=1000 + s, device=dev, max_disp=16.0)
            opt.zero_grad(set_to_none=True)
            preds = model(i1, i2, iters=6)
            loss, _ = sequence_loss(preds, flow, valid, 0.8, sync_metrics=False)
            loss.backward()
            opt.clip_and_step(1.0)
            sched.step()
            out.append(loss.detach())
        return torch.stack(out).float().cpu()

    w = 50
    arms = {"fp32_det": [], "bf16": [], "bf16_det": [], "fp32_stock": []}
    for seed in range(a.seeds):
        torch.manual_seed(seed)
        base = RAFT(make_args()).to(dev).to(memory_format=torch.channels_last).train()
        for arm in arms:
            m = copy.deepcopy(base)
            if arm.startswith("bf16"):
                m.cfg = m.cfg.__class__(**{**m.cfg.to_dict(), "mixed_precision": True})
            if arm.endswith("det"):
                with deterministic(True):
                    l = run(m, a.steps)
            elif arm == "fp32_stock":  # the model on stock PyTorch ops (reference semantics), same optimizer
                from raft_stir_amd.ops import _ext
                with _ext.reference_mode():
                    l = run(m, a.steps)
            else:
                l = run(m, a.steps)
            first, last = l[:w].mean().item(), l[-w:].mean().item()
            arms[arm].append((first, last))
            print(f"seed {seed} {arm:9s} first {first:.3f} last {last:.3f}", flush=True)
    for arm, v in arms.items():
        f = sum(x[0] for x in v) / len(v)
        l = sum(x[1] for x in v) / len(v)
        print(f"mean {arm:9s} first {f:.3f} last {l:.3f}  (lasts: {', '.join(f'{x[1]:.2f}' for x in v)})")


if __name__ == "__main__":
    main()
