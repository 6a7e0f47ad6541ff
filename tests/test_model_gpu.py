"""End-to-end model on the GPU (HIP path) vs the CPU ATen oracle."""
import copy
import os

import pytest
import torch

from raft_stir_amd.config import make_args
from raft_stir_amd.models import RAFT

pytestmark = pytest.mark.gpu


def _imgs(B, H, W, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(B, 3, H, W, generator=g) * 255, torch.rand(B, 3, H, W, generator=g) * 255


@pytest.mark.parametrize("small", [False, True])
@pytest.mark.parametrize("alt", [False, True])
def test_inference_fp32_matches_cpu(cuda, small, alt):
    torch.manual_seed(0)
    cpu = RAFT(make_args(small=small, alternate_corr=alt)).eval()
    gpu = copy.deepcopy(cpu).to(cuda).to(memory_format=torch.channels_last).eval()
    i1, i2 = _imgs(1, 128, 192)
    with torch.no_grad():
        lo_c, up_c = cpu(i1, i2, iters=6, test_mode=True)
        lo_g, up_g = gpu(i1.to(cuda), i2.to(cuda), iters=6, test_mode=True)
    # MIOpen conv algorithms differ from CPU in summation order; the recurrent
    # loop amplifies fp32 noise a little.
    torch.testing.assert_close(lo_g.cpu(), lo_c, atol=2e-2, rtol=1e-3)
    torch.testing.assert_close(up_g.cpu(), up_c, atol=5e-2, rtol=1e-3)


def test_bf16_inference_close_to_fp32(cuda):
    """bf16 engine drift vs fp32 must be no worse than the ATen composite
    path's own bf16-autocast drift (same weights, smooth synthetic pair)."""
    from raft_stir_amd.data.synthetic import make_batch
    from raft_stir_amd.ops import _ext
    torch.manual_seed(0)
    m32 = RAFT(make_args()).to(cuda).to(memory_format=torch.channels_last).eval()
    mbf = copy.deepcopy(m32)
    mbf.cfg = mbf.cfg.__class__(**{**mbf.cfg.to_dict(), "mixed_precision": True})
    i1, i2, _, _ = make_batch(1, 192, 256, seed=1, device=cuda)
    with torch.no_grad():
        _, a = m32(i1, i2, iters=12, test_mode=True)
        _, b = mbf(i1, i2, iters=12, test_mode=True)
        with _ext.reference_mode():
            _, c = mbf(i1, i2, iters=12, test_mode=True)
    err = (a - b).norm(dim=1).mean().item()
    err_ref = (a - c).norm(dim=1).mean().item()
    assert err < 2.0 * err_ref + 1e-2, (err, err_ref)


def test_bf16_pyramid_epe_drift(cuda):
    """EPE-drift gate for bf16 pyramid storage (RAFTConfig.corr_dtype,
    SURVEY 7.3-1): at 12 iterations the bf16-pyramid engine must stay as close
    to the fp32 model as the fp32-pyramid bf16 engine does (+ a small margin)."""
    from raft_stir_amd.data.synthetic import make_batch
    torch.manual_seed(0)
    m32 = RAFT(make_args()).to(cuda).to(memory_format=torch.channels_last).eval()
    mix = copy.deepcopy(m32)
    mix.cfg = mix.cfg.__class__(**{**mix.cfg.to_dict(), "mixed_precision": True})
    mbp = copy.deepcopy(mix)
    mbp.cfg = mbp.cfg.__class__(**{**mbp.cfg.to_dict(), "corr_dtype": "bfloat16"})
    i1, i2, _, _ = make_batch(1, 192, 256, seed=11, device=cuda)
    with torch.no_grad():
        _, a = m32(i1, i2, iters=12, test_mode=True)
        _, b = mix(i1, i2, iters=12, test_mode=True)
        _, c = mbp(i1, i2, iters=12, test_mode=True)
    e_mix = (a - b).norm(dim=1).mean().item()
    e_bp = (a - c).norm(dim=1).mean().item()
    print(f"EPE vs fp32: bf16 engine {e_mix:.4f}, + bf16 pyramid {e_bp:.4f}")
    assert e_bp <= 1.25 * e_mix + 0.02, (e_bp, e_mix)


SINTEL = os.path.join(os.path.dirname(__file__), "data", "sintel_demo")


def test_bf16_drift_real_frames_trained_model(cuda):
    """EPE-drift gate on the reference's real Sintel demo pair (frame_0016 /
    frame_0017, 1024x436, copied from reference demo-frames/) with a model
    first trained for 200 synthetic steps, so its flows are non-trivial: the
    bf16 engine (fp32 pyramid) and the bf16 engine + bf16 pyramid (the bench
    configuration) vs the fp32 model (the reference's default precision,
    evaluate.py:174)."""
    import numpy as np
    from PIL import Image
    from raft_stir_amd.data.synthetic import make_batch
    from raft_stir_amd.train.loss import sequence_loss
    from raft_stir_amd.utils.padder import InputPadder
    torch.manual_seed(0)
    m = RAFT(make_args(mixed_precision=True)).to(cuda).to(memory_format=torch.channels_last).train()
    opt = torch.optim.AdamW(m.parameters(), lr=4e-4, weight_decay=1e-4, eps=1e-8)
    for step in range(200):
        i1, i2, fl, v = make_batch(4, 192, 256, seed=1000 + step, device=cuda)
        opt.zero_grad(set_to_none=True)
        loss, _ = sequence_loss(m(i1, i2, iters=6), fl, v, 0.8, sync_metrics=False)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)
        opt.step()
    m.eval()

    def load(name):
        a = np.asarray(Image.open(os.path.join(SINTEL, name)).convert("RGB"), dtype=np.float32)
        return torch.from_numpy(a).permute(2, 0, 1)[None].to(cuda)
    i1, i2 = load("frame_0016.png"), load("frame_0017.png")
    i1, i2 = InputPadder(i1.shape).pad(i1, i2)
    m32 = copy.deepcopy(m)
    m32.cfg = m32.cfg.__class__(**{**m32.cfg.to_dict(), "mixed_precision": False})
    mbp = copy.deepcopy(m)
    mbp.cfg = mbp.cfg.__class__(**{**mbp.cfg.to_dict(), "corr_dtype": "bfloat16"})
    with torch.no_grad():
        _, a = m32(i1, i2, iters=12, test_mode=True)
        _, b = m(i1, i2, iters=12, test_mode=True)
        _, c = mbp(i1, i2, iters=12, test_mode=True)
    mag = a.norm(dim=1).mean().item()
    e_mix = (a - b).norm(dim=1).mean().item()
    e_bp = (a - c).norm(dim=1).mean().item()
    print(f"trained model on Sintel demo: mean |flow| {mag:.3f} px, EPE vs fp32: bf16 engine {e_mix:.4f}, "
          f"+ bf16 pyramid {e_bp:.4f}")
    assert mag > 0.5, mag  # the gate is only meaningful on non-trivial flows
    assert e_mix <= 0.05 * mag + 0.05, (e_mix, mag)
    assert e_bp <= 1.25 * e_mix + 0.02, (e_bp, e_mix)


@pytest.mark.parametrize("small", [False, True])
def test_training_grads_match_cpu(cuda, small):
    torch.manual_seed(0)
    cpu = RAFT(make_args(small=small)).train()
    gpu = copy.deepcopy(cpu).to(cuda).to(memory_format=torch.channels_last).train()
    i1, i2 = _imgs(2, 128, 192, seed=2)
    gt = torch.randn(2, 2, 128, 192) * 4
    preds = cpu(i1, i2, iters=3)
    loss_c = sum((p - gt).abs().mean() for p in preds)
    loss_c.backward()
    preds_g = gpu(i1.to(cuda), i2.to(cuda), iters=3)
    loss_g = sum((p - gt.to(cuda)).abs().mean() for p in preds_g)
    loss_g.backward()
    torch.testing.assert_close(loss_g.cpu(), loss_c.detach(), rtol=1e-3, atol=1e-3)
    gc = torch.cat([p.grad.flatten() for p in cpu.parameters()])
    gg = torch.cat([p.grad.flatten().cpu() for p in gpu.parameters()])
    cos = torch.nn.functional.cosine_similarity(gc, gg, dim=0).item()
    assert cos > 0.999, cos
    # fp32 training on the GPU runs the fused engine (split-bf16 conv tiles,
    # relative error ~2^-17 per product) and the encoders' fp32 convs
    rel = ((gc - gg).norm() / gc.norm()).item()
    names = [n for n, _ in cpu.named_parameters()]
    worst = sorted(((((p.grad - q.grad.cpu()).norm() / p.grad.norm().clamp_min(1e-12)).item(), n)
                    for n, p, q in zip(names, cpu.parameters(), gpu.parameters())), reverse=True)[:5]
    assert rel < 1e-3, (rel, worst)


# whole-gradient relative errors of the bf16 engines vs the fp32 CPU oracle,
# measured 0.030 (RAFT) / 0.010 (RAFT-small), update block 0.018 / 0.007
# (profiles/r6/README.md); the bounds are ~2-3x the measurement
_BF16_GRAD_REL = {False: 0.06, True: 0.03}


@pytest.mark.parametrize("small", [False, True])
def test_bf16_training_grads_match_cpu_fp32(cuda, small):
    """The bf16 training step (fused update-block engine, HIP encoders, bf16
    pyramid) against the fp32 CPU oracle of the same weights and inputs:
    the relative error of the WHOLE gradient vector and of the loss, not only
    per-parameter cosines against another HIP path (the fused-train tests)."""
    torch.manual_seed(0)
    cpu = RAFT(make_args(small=small, mixed_precision=True)).train()  # autocast is CUDA-only: fp32 on CPU
    gpu = copy.deepcopy(cpu).to(cuda).to(memory_format=torch.channels_last).train()
    i1, i2 = _imgs(2, 128, 192, seed=2)
    gt = torch.randn(2, 2, 128, 192) * 4
    preds = cpu(i1, i2, iters=3)
    loss_c = sum((p - gt).abs().mean() for p in preds)
    loss_c.backward()
    preds_g = gpu(i1.to(cuda), i2.to(cuda), iters=3)
    eng = gpu.__dict__.get("_fused_train")
    assert eng is not None, "the bf16 step did not run the fused training engine"
    loss_g = sum((p.float() - gt.to(cuda)).abs().mean() for p in preds_g)
    loss_g.backward()
    torch.testing.assert_close(loss_g.cpu(), loss_c.detach(), rtol=1e-2, atol=1e-2)
    gc = torch.cat([p.grad.flatten() for p in cpu.parameters()])
    gg = torch.cat([p.grad.float().flatten().cpu() for p in gpu.parameters()])
    rel = ((gc - gg).norm() / gc.norm()).item()
    names = [n for n, _ in cpu.named_parameters()]
    worst = sorted(((((p.grad - q.grad.float().cpu()).norm() / p.grad.norm().clamp_min(1e-12)).item(), n)
                    for n, p, q in zip(names, cpu.parameters(), gpu.parameters())), reverse=True)[:5]
    ub = torch.cat([p.grad.flatten() for n, p in cpu.named_parameters() if n.startswith("update_block")])
    ug = torch.cat([q.grad.float().flatten().cpu() for n, q in gpu.named_parameters() if n.startswith("update_block")])
    rel_u = ((ub - ug).norm() / ub.norm()).item()
    print(f"bf16 vs fp32 CPU oracle ({'small' if small else 'raft'}): whole-gradient rel {rel:.4f}, "
          f"update block {rel_u:.4f}, worst {worst[:3]}")
    assert rel < _BF16_GRAD_REL[small], (rel, worst)
    assert rel_u < _BF16_GRAD_REL[small], (rel_u, worst)


@pytest.mark.parametrize("mixed,tol", [(False, 2e-3), (True, 3e-2)])
def test_graphed_inference_matches_eager(cuda, mixed, tol):
    from raft_stir_amd.runtime.graph import GraphedInference
    torch.manual_seed(0)
    m = RAFT(make_args(mixed_precision=mixed)).to(cuda).to(memory_format=torch.channels_last).eval()
    i1, i2 = _imgs(1, 128, 256, seed=3)
    i1, i2 = i1.to(cuda), i2.to(cuda)
    with torch.no_grad():
        lo, up = m(i1, i2, iters=8, test_mode=True)
    g = GraphedInference(m, i1.shape, iters=8)
    lo2, up2 = g(i1, i2)
    torch.testing.assert_close(up2, up, atol=tol, rtol=tol)
    lo3, up3 = g(i2, i1)  # replay with new inputs
    with torch.no_grad():
        _, upe = m(i2, i1, iters=8, test_mode=True)
    torch.testing.assert_close(up3, upe, atol=tol, rtol=tol)
