"""Fidelity of the fused bf16 TRAINING engine (the path bench.py measures)
against fp32 references (reference train.py:47-72 loss, :162-183 step).

* one step: fused-bf16 gradients vs the fp32 CPU oracle on identical weights
  and data, as ONE aggregate relative error over all parameters, bounded by
  the drift of stock PyTorch bf16 autocast (the reference's own AMP mode) on
  the same step;
* 200 steps, three weight-init seeds: the fused bf16 engine vs the fused
  fp32 engine (split-bf16 F32 kernels), both deterministic, AdamW + OneCycle
  as the reference: the first windows agree per seed, every run learns, and
  the ensemble end points agree (see the test's docstring for the numbers);
  for seed 0 the fused fp32 engine's first window also tracks an independent
  stock-op arm (ATen module graph + torch.optim.AdamW).

Measured on MI355X (round 2): one step, gradient relative error vs the fp32
oracle 1.46 % for the fused engine and 1.65 % for stock bf16 autocast; loss
32.388 vs 32.380.
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


def _train(model, steps, batches, lr, num_steps=None, stock=False):
    from raft_stir_amd.train.loss import sequence_loss
    from raft_stir_amd.train.optim import fetch_optimizer
    args = make_args(lr=lr, wdecay=1e-5, epsilon=1e-8, num_steps=num_steps or steps)
    opt, sched = fetch_optimizer(args, model, fused=False if stock else None)
    losses = []
    for s in range(steps):
        i1, i2, flow, valid = batches(s)
        opt.zero_grad(set_to_none=True)
        preds = model(i1, i2, iters=6)
        loss, _ = sequence_loss(preds, flow, valid, 0.8, sync_metrics=False)
        loss.backward()
        if hasattr(opt, "clip_and_step"):  # the trainer's path (train/trainer.py)
            opt.clip_and_step(1.0)
        else:
            torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
            opt.step()
        sched.step()
        losses.append(loss.detach())
    return torch.stack(losses).float().cpu()


@pytest.mark.timeout(300)
def test_fused_bf16_training_curve_tracks_fp32(cuda):
    """200 steps of the fused bf16 engine vs the fused fp32 engine (the
    reference's default training precision, on the split-bf16 F32 kernels),
    both in deterministic mode (bitwise reproducible), over three weight-init
    seeds.  Measured (profiles/r4/fidelity_ensemble_s24.txt, same setup):

        first 50 steps   fp32 22.33 / 21.91 / 22.10   bf16 22.33 / 21.90 / 22.23
        last 50 steps    fp32 19.01 / 10.97 / 12.35   bf16 19.16 / 13.55 /  6.55
        (stock-op fp32, nondeterministic: 20.39 / 15.69 / 13.51)

    The trajectories of this chaotic recurrent model decorrelate after the
    first ~50 steps (single end points of one seed differ by up to ~2x between
    precisions, and between two processes of the stock fp32 run), so the
    bounds are: the first window agrees tightly per seed (<= 2 %); every run
    learns; and the ensemble means of the last window agree within 30 %."""
    from raft_stir_amd.data.synthetic import make_batch
    from raft_stir_amd.runtime.determinism import deterministic

    def batches(s):
        return make_batch(2, 128, 192, seed=1000 + s, device=cuda, max_disp=16.0)

    steps, w = 200, 50
    ends = {"fp32": [], "bf16": []}
    for seed in range(3):
        torch.manual_seed(seed)
        base = RAFT(make_args()).to(cuda).to(memory_format=torch.channels_last).train()
        curves = {}
        for arm in ("fp32", "bf16"):
            m = copy.deepcopy(base)
            if arm == "bf16":
                m.cfg = m.cfg.__class__(**{**m.cfg.to_dict(), "mixed_precision": True})
            with deterministic(True):
                curves[arm] = _train(m, steps, batches, 4e-4)
            assert torch.isfinite(curves[arm]).all()
        for arm, l in curves.items():
            first, last = l[:w].mean().item(), l[-w:].mean().item()
            print(f"seed {seed} {arm}: {first:.3f} -> {last:.3f}")
            assert last < 0.95 * first, (seed, arm, first, last)  # every run learns
            ends[arm].append((first, last))
        f32, fbf = ends["fp32"][-1][0], ends["bf16"][-1][0]
        assert abs(fbf - f32) <= 0.02 * f32, (seed, fbf, f32)  # before the trajectories decorrelate
        if seed == 0:
            # independent arm: the stock-op module graph (ATen convs, grid_sample,
            # matmul volume) with torch.optim.AdamW, no fused kernel or optimizer
            # in common with the two engines; the fused fp32 engine must track it
            # over the first window (same schedule: OneCycle over 200 steps)
            from raft_stir_amd.ops import _ext
            m = copy.deepcopy(base)
            with _ext.reference_mode():
                stock = _train(m, w, batches, 4e-4, num_steps=steps, stock=True)
            s_first, f_first = stock.mean().item(), curves["fp32"][:w].mean().item()
            print(f"seed 0 stock-op fp32 first {w}: {s_first:.3f} (fused fp32 {f_first:.3f})")
            assert abs(f_first - s_first) <= 0.03 * s_first, (f_first, s_first)
    mean = {arm: (sum(a for a, _ in v) / 3, sum(b for _, b in v) / 3) for arm, v in ends.items()}
    print("means", mean)
    for arm, (first, last) in mean.items():
        assert last < 0.8 * first, (arm, first, last)  # the ensemble learns
    assert abs(mean["bf16"][1] - mean["fp32"][1]) <= 0.3 * mean["fp32"][1], mean
