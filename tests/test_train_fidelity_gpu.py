"""Fidelity of the fused bf16 TRAINING engine (the path bench.py measures)
against fp32 references (reference train.py:47-72 loss, :162-183 step).

* one step: fused-bf16 gradients vs the fp32 CPU oracle on identical weights
  and data, as ONE aggregate relative error over all parameters, bounded by
  the drift of stock PyTorch bf16 autocast (the reference's own AMP mode) on
  the same step;
* 200 steps: fused-bf16 training vs fp32 (ATen-only) training from the same
  initialisation on the same synthetic stream, AdamW + OneCycle as the
  reference: both loss curves must fall and agree.

Measured on MI355X (round 2): one step, gradient relative error vs the fp32
oracle 1.46 % for the fused engine and 1.65 % for stock bf16 autocast; loss
32.388 vs 32.380.  200 steps (batch 2, 128x192, 6 iterations), means of the
first / last 25 steps: fp32 23.12 -> 13.49, fused bf16 23.18 -> 13.77 in one
process; fp32 23.13 -> 17.70, fused 23.10 -> 18.74 in another (nondeterminism).
"""
import copy

import pytest
import torch

from raft_stir_amd.config import make_args
from raft_stir_amd.models import RAFT

pytestmark = pytest.mark.gpu


def _flat_grads(model):
    """All parameter gradients as one fp32 vector (CPU), skipping biases of
    encoder convs that feed a train-mode norm: their true gradient is exactly
    zero and both paths only carry round-off there."""
    out = []
    for n, p in model.named_parameters():
        normed = n.split(".")[0] in ("fnet", "cnet") and n.endswith(".bias") and n not in (
            "fnet.conv2.bias", "cnet.conv2.bias")
        if p.grad is None or normed:
            continue
        out.append(p.grad.detach().float().flatten().cpu())
    return torch.cat(out)


def _step_grads(model, batch, iters):
    from raft_stir_amd.train.loss import sequence_loss
    i1, i2, flow, valid = batch
    model.zero_grad(set_to_none=True)
    preds = model(i1, i2, iters=iters)
    loss, _ = sequence_loss(preds, flow, valid, 0.8, sync_metrics=False)
    loss.backward()
    return loss.item(), _flat_grads(model)


def test_fused_bf16_step_vs_fp32_oracle(cuda):
    from raft_stir_amd.data.synthetic import make_batch
    from raft_stir_amd.models.fused_train import FusedTrainEngine
    from raft_stir_amd.ops import _ext
    torch.manual_seed(0)
    cpu = RAFT(make_args()).train()                                   # fp32 oracle (ATen, CPU)
    fused = copy.deepcopy(cpu).to(cuda).to(memory_format=torch.channels_last).train()
    fused.cfg = fused.cfg.__class__(**{**fused.cfg.to_dict(), "mixed_precision": True})
    aten = copy.deepcopy(fused)                                       # stock bf16 autocast on the GPU
    batch = make_batch(2, 192, 256, seed=5)
    gbatch = tuple(t.to(cuda) for t in batch)
    iters = 6
    l32, g32 = _step_grads(cpu, batch, iters)
    calls = []
    orig = FusedTrainEngine.eligible
    FusedTrainEngine.eligible = staticmethod(lambda *a: calls.append(orig(*a)) or calls[-1])
    try:
        lf, gf = _step_grads(fused, gbatch, iters)
    finally:
        FusedTrainEngine.eligible = staticmethod(orig)
    assert calls and all(calls), "the fused training engine did not run"
    with _ext.reference_mode():
        la, ga = _step_grads(aten, gbatch, iters)
    rel_f = ((gf - g32).norm() / g32.norm()).item()
    rel_a = ((ga - g32).norm() / g32.norm()).item()
    print(f"loss fp32 {l32:.5f} fused {lf:.5f} aten-bf16 {la:.5f}; grad rel err fused {rel_f:.4f} aten-bf16 {rel_a:.4f}")
    assert abs(lf - l32) <= 0.02 * abs(l32) + 1e-3, (lf, l32)
    assert rel_f <= max(1.5 * rel_a, 0.02), (rel_f, rel_a)
    assert rel_f < 0.1, rel_f


def _train(model, steps, batches, lr):
    from raft_stir_amd.train.loss import sequence_loss
    from raft_stir_amd.train.optim import fetch_optimizer
    args = make_args(lr=lr, wdecay=1e-5, epsilon=1e-8, num_steps=steps)
    opt, sched = fetch_optimizer(args, model)
    losses = []
    for s in range(steps):
        i1, i2, flow, valid = batches(s)
        opt.zero_grad(set_to_none=True)
        preds = model(i1, i2, iters=6)
        loss, _ = sequence_loss(preds, flow, valid, 0.8, sync_metrics=False)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        sched.step()
        losses.append(loss.detach())
    return torch.stack(losses).float().cpu()


@pytest.mark.timeout(300)
def test_fused_bf16_training_curve_tracks_fp32(cuda):
    from raft_stir_amd.data.synthetic import make_batch
    from raft_stir_amd.ops import _ext
    torch.manual_seed(0)
    m32 = RAFT(make_args()).to(cuda).to(memory_format=torch.channels_last).train()
    mbf = copy.deepcopy(m32)
    mbf.cfg = mbf.cfg.__class__(**{**mbf.cfg.to_dict(), "mixed_precision": True})
    steps = 200

    def batches(s):
        return make_batch(2, 128, 192, seed=1000 + s, device=cuda, max_disp=16.0)

    from raft_stir_amd.runtime.determinism import deterministic
    # 200 steps of a chaotic recurrent model.  The fused bf16 run is in
    # deterministic mode (bitwise reproducible: 22.41 -> 20.23 on every run);
    # the fp32 reference (stock ops) is not -- its own 50-step mean at step 200
    # spans 10.8 .. 20.4 across processes on one box (profiles/r3/
    # fidelity_spread.txt), so single end points differ by up to ~2x without
    # any numerical fault.  The bounds: the two curves agree tightly BEFORE the
    # trajectories decorrelate (first 50 steps, <= 3 %), both learn, and the
    # end points stay within that measured ensemble spread.
    with deterministic(True):
        lbf = _train(mbf, steps, batches, 4e-4)
    with _ext.reference_mode():
        l32 = _train(m32, steps, batches, 4e-4)
    w = 50
    first_bf, last_bf = lbf[:w].mean().item(), lbf[-w:].mean().item()
    first_32, last_32 = l32[:w].mean().item(), l32[-w:].mean().item()
    print(f"fp32 {first_32:.3f} -> {last_32:.3f}; fused bf16 {first_bf:.3f} -> {last_bf:.3f}")
    assert torch.isfinite(lbf).all() and torch.isfinite(l32).all()
    assert abs(first_bf - first_32) <= 0.03 * first_32, (first_bf, first_32)  # before decorrelation
    assert last_32 < 0.95 * first_32, (first_32, last_32)   # the fp32 run learns
    assert last_bf < 0.95 * first_bf, (first_bf, last_bf)   # the fused run learns
    assert 0.5 * last_32 <= last_bf <= 2.0 * last_32, (last_bf, last_32)  # within the fp32 ensemble spread
