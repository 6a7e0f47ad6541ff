"""Probe: batched weight repacks per training step (expect 1)."""
import argparse

import torch

from raft_stir_amd.config import make_args
from raft_stir_amd.data.synthetic import make_batch
from raft_stir_amd.models import RAFT
from raft_stir_amd.ops import wpack
from raft_stir_amd.train.loss import sequence_loss
from raft_stir_amd.train.optim import fetch_optimizer

dev = torch.device("cuda")
m = RAFT(make_args(mixed_precision=True)).to(dev).to(memory_format=torch.channels_last).train()
opt, sched = fetch_optimizer(argparse.Namespace(lr=4e-4, wdecay=1e-4, epsilon=1e-8, num_steps=1000), m)
i1, i2, flow, valid = make_batch(8, 368, 496, seed=1, device=dev)
orig_repack = wpack._Registry.repack
def traced(self):
    import traceback
    st = traceback.extract_stack(limit=6)
    print("   repack from", " <- ".join(f"{f.name}:{f.lineno}" for f in st[-5:-1]))
    return orig_repack(self)
for step in range(4):
    if step == 2:
        wpack._Registry.repack = traced
    r0 = wpack.STATS["repacks"]
    opt.zero_grad(set_to_none=True)
    preds = m(i1, i2, iters=12)
    loss, _ = sequence_loss(preds, flow, valid, 0.8, sync_metrics=False)
    loss.backward()
    torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)
    opt.step()
    sched.step()
    torch.cuda.synchronize()
    print("step", step, "repacks", wpack.STATS["repacks"] - r0, flush=True)
