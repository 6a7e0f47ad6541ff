#!/usr/bin/env python
"""fp32 training parity: CPU fp32 oracle vs the GPU fused fp32 engine vs the
GPU fp32 module graph (PyTorch convs), same weights / batch.  Prints the loss
and the relative gradient error of each GPU path against the CPU oracle
(whole vector and the five worst parameters).

    python scripts/fp32_train_parity.py [--small] [--iters 3]
"""
import argparse
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--small", action="store_true")
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--size", type=int, nargs=2, default=[128, 192])
    a = ap.parse_args()
    from raft_stir_amd.config import make_args
    from raft_stir_amd.models import RAFT
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    cpu = RAFT(make_args(small=a.small)).train()
    fused = copy.deepcopy(cpu).to(dev).to(memory_format=torch.channels_last).train()
    mod = copy.deepcopy(cpu).to(dev).to(memory_format=torch.channels_last).train()
    mod.cfg = mod.cfg.__class__(**{**mod.cfg.to_dict(), "fused_train": False})
    g = torch.Generator().manual_seed(2)
    H, W = a.size
    i1 = torch.rand(2, 3, H, W, generator=g) * 255
    i2 = torch.rand(2, 3, H, W, generator=g) * 255
    gt = torch.randn(2, 2, H, W, generator=g) * 4
    out = {}
    for name, net, d in (("cpu", cpu, "cpu"), ("fused", fused, dev), ("module", mod, dev)):
        preds = net(i1.to(d), i2.to(d), iters=a.iters)
        loss = sum((p - gt.to(d)).abs().mean() for p in preds)
        loss.backward()
        out[name] = (loss.item(), {n: p.grad.detach().float().cpu() for n, p in net.named_parameters()
                                   if p.grad is not None})
    lc, gc = out["cpu"]
    flat = lambda gd: torch.cat([gd[k].flatten() for k in sorted(gc)])
    for name in ("fused", "module"):
        lg, gg = out[name]
        rel = ((flat(gg) - flat(gc)).norm() / flat(gc).norm()).item()
        normed = lambda k: k.split(".")[0] in ("fnet", "cnet") and k.endswith(".bias") and not k.endswith("conv2.bias")
        worst = sorted((((gg[k] - gc[k]).norm() / gc[k].norm().clamp_min(1e-12)).item(), k) for k in gc
                       if gc[k].norm() > 1e-8 and not normed(k))[::-1][:5]
        print(f"{name:7s} loss {lg:.6f} (cpu {lc:.6f}) grad rel {rel:.2e} worst "
              + ", ".join(f"{k} {r:.1e}" for r, k in worst), flush=True)


if __name__ == "__main__":
    main()
