"""Optimizer + LR schedule (reference train.py:79-86).

AdamW(lr, weight_decay=wdecay, eps=epsilon) and a linear OneCycle schedule over
num_steps + 100 with pct_start 0.05 and no momentum cycling.  On GPU the
AdamW update runs as PyTorch's fused multi-tensor kernel (one launch for all
5.3 M parameters instead of one per tensor).
"""
from __future__ import annotations

import torch
import torch.optim as optim


def fetch_optimizer(args, model, fused=None, capturable=False):
    """``capturable``: the learning rate lives in a device tensor (updated in
    place by the scheduler) and the update reads no host state, so the whole
    step can be replayed from a hipGraph (runtime/graph.py GraphedTrainStep)."""
    params = [p for p in model.parameters() if p.requires_grad]
    if fused is None:
        fused = bool(params) and params[0].is_cuda
    kw = dict(lr=args.lr, weight_decay=args.wdecay, eps=args.epsilon)
    if capturable:
        kw.update(lr=torch.tensor(float(args.lr), device=params[0].device), capturable=True)
    try:
        optimizer = optim.AdamW(params, fused=fused, **kw)
    except (RuntimeError, TypeError):
        optimizer = optim.AdamW(params, foreach=fused, **kw)
    scheduler = optim.lr_scheduler.OneCycleLR(
        optimizer, args.lr, args.num_steps + 100, pct_start=0.05, cycle_momentum=False,
        anneal_strategy="linear")
    return optimizer, scheduler


def count_parameters(model):
    return sum(p.numel() for p in model.parameters() if p.requires_grad)
