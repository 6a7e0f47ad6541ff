"""Fused clip + AdamW (csrc/optim.hip, train/optim.py FusedClipAdamW) vs
torch.nn.utils.clip_grad_norm_ + torch.optim.AdamW (single-tensor reference
path, fp32) on the same parameters and gradients."""
import pytest
import torch

from raft_stir_amd.train.optim import FusedClipAdamW

pytestmark = pytest.mark.gpu


def _params(dev, n=130, seed=0):
    """> 96 tensors (two launch groups), channels_last 4-D weights, 1-D
    biases, odd sizes, a few tensors larger than one 8192-element block."""
    g = torch.Generator().manual_seed(seed)
    ps = []
    for i in range(n):
        k = i % 5
        if k == 0:
            t = torch.randn(24, 17, 3, 3, generator=g).to(dev).contiguous(memory_format=torch.channels_last)
        elif k == 1:
            t = torch.randn(37, generator=g).to(dev)
        elif k == 2:
            t = torch.randn(129, 70, generator=g).to(dev)
        elif k == 3:
            t = torch.randn(3, generator=g).to(dev)
        else:
            t = torch.randn(8, 5, 1, 7, generator=g).to(dev)
        ps.append(t.requires_grad_())
    return ps


def _grads(ps, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return [(torch.randn(p.shape, generator=g) * scale).to(p.device).contiguous(
        memory_format=torch.channels_last if p.dim() == 4 else torch.contiguous_format) for p in ps]


@pytest.mark.parametrize("max_norm", [1.0, 0.0, 1e6])
@pytest.mark.parametrize("lr_tensor", [False, True])
def test_fused_clip_adamw_matches_torch(cuda, max_norm, lr_tensor):
    a = _params(cuda)
    b = [p.detach().clone().requires_grad_() for p in a]
    lr = torch.tensor(3e-3, device=cuda) if lr_tensor else 3e-3
    fo = FusedClipAdamW(a, lr=lr, weight_decay=1e-2, eps=1e-8, capturable=lr_tensor)
    ro = torch.optim.AdamW(b, lr=3e-3, weight_decay=1e-2, eps=1e-8, foreach=False)
    for step in range(4):
        gs = _grads(a, 10 + step, scale=0.3 + step)
        for p, q, g in zip(a, b, gs):
            p.grad = g.clone()
            q.grad = g.clone()
        norm = fo.clip_and_step(max_norm)
        if max_norm > 0:
            want = torch.nn.utils.clip_grad_norm_(b, max_norm)
            torch.testing.assert_close(norm, want, rtol=1e-5, atol=1e-6)
        ro.step()
        for p, q in zip(a, b):
            torch.testing.assert_close(p.detach(), q.detach(), rtol=2e-5, atol=2e-6)
    # moments as torch AdamW's per-parameter state, steps counted
    sd = fo.state_dict()
    for i, q in enumerate(b):
        st = ro.state[q]
        torch.testing.assert_close(sd["state"][i]["exp_avg"], st["exp_avg"], rtol=2e-5, atol=1e-7)
        torch.testing.assert_close(sd["state"][i]["exp_avg_sq"], st["exp_avg_sq"], rtol=2e-5, atol=1e-9)
        assert float(sd["state"][i]["step"]) == 4.0


def test_fused_clip_adamw_skips_nonfinite_and_resumes(cuda):
    a = _params(cuda, n=20, seed=3)
    b = [p.detach().clone().requires_grad_() for p in a]
    fo = FusedClipAdamW(a, lr=1e-3, weight_decay=1e-4)
    ro = torch.optim.AdamW(b, lr=1e-3, weight_decay=1e-4, foreach=False)
    seq = [1, 2, "inf", 3]
    for s in seq:
        gs = _grads(a, 50 + (0 if s == "inf" else s))
        if s == "inf":
            gs[6][3] = float("inf")
        before = [p.detach().clone() for p in a]
        for p, g in zip(a, gs):
            p.grad = g
        norm = fo.clip_and_step(1.0)
        if s == "inf":
            assert not torch.isfinite(norm)
            for p, q in zip(a, before):
                assert torch.equal(p.detach(), q)  # skipped on the device
            continue
        for q, g in zip(b, gs):
            q.grad = g.clone()
        torch.nn.utils.clip_grad_norm_(b, 1.0)
        ro.step()
    for p, q in zip(a, b):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=2e-5, atol=2e-6)
    sd = fo.state_dict()
    assert float(sd["state"][0]["step"]) == 3.0  # the skipped step is not counted
    # resume into a fresh optimizer: identical continuation
    c = [p.detach().clone().requires_grad_() for p in a]
    fo2 = FusedClipAdamW(c, lr=1e-3, weight_decay=1e-4)
    fo2.load_state_dict(sd)
    gs = _grads(a, 99)
    for p, q, g in zip(a, c, gs):
        p.grad = g.clone()
        q.grad = g.clone()
    fo.clip_and_step(1.0)
    fo2.clip_and_step(1.0)
    for p, q in zip(a, c):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=0, atol=0)


def test_fetch_optimizer_uses_fused_clip_adamw(cuda):
    import argparse

    from raft_stir_amd.train.optim import fetch_optimizer
    m = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.Conv2d(8, 4, 1)).to(cuda)
    m = m.to(memory_format=torch.channels_last)
    opt, sched = fetch_optimizer(argparse.Namespace(lr=4e-4, wdecay=1e-4, epsilon=1e-8, num_steps=100), m)
    assert isinstance(opt, FusedClipAdamW)
    x = torch.randn(2, 3, 9, 9, device=cuda).contiguous(memory_format=torch.channels_last)
    m(x).square().mean().backward()
    w0 = m[0].weight.detach().clone()
    opt.clip_and_step(1.0)
    sched.step()
    assert not torch.equal(w0, m[0].weight.detach())
    assert opt.param_groups[0]["lr"] != 4e-4 / 25  # OneCycle moved the lr


def test_clip_and_step_refreshes_packed_weights(cuda):
    """clip_and_step bypasses the wrapped Optimizer.step (whose global post-hook
    advances runtime/weights.generation) and its custom op bumps no _version:
    it must advance the generation itself, or the HIP kernels keep reading the
    packed weights of the previous step.  After one large-lr step the HIP
    forward must agree with the stock-op forward on the UPDATED weights."""
    from raft_stir_amd.config import make_args
    from raft_stir_amd.data.synthetic import make_batch
    from raft_stir_amd.models import RAFT
    from raft_stir_amd.ops import _ext
    from raft_stir_amd.runtime import weights

    torch.manual_seed(0)
    model = RAFT(make_args(mixed_precision=True)).to(cuda).to(memory_format=torch.channels_last).train()
    opt = FusedClipAdamW([p for p in model.parameters() if p.requires_grad], lr=2e-2, weight_decay=0.0)
    i1, i2, flow, valid = make_batch(1, 96, 128, seed=3, device=cuda)

    def infer():
        model.eval()
        with torch.no_grad():
            out = model(i1, i2, iters=3, test_mode=True)[1].float()
        model.train()
        return out

    infer()  # pack every weight cache at the initial weights
    model(i1, i2, iters=3)[-1].float().sub(flow).abs().mean().backward()
    gen = weights.generation()
    opt.clip_and_step(1.0)
    assert weights.generation() > gen
    hip = infer()
    with _ext.reference_mode():
        ref = infer()
    rel = ((hip - ref).norm() / ref.norm()).item()
    assert rel < 5e-2, rel  # stale packed weights give O(1) differences after this step
