"""Fused sequence loss (csrc/loss.hip) vs the composite fp32 PyTorch loss."""
import pytest
import torch

from raft_stir_amd.train.loss import _stacked, sequence_loss

pytestmark = pytest.mark.gpu


def _composite(preds, gt, valid, gamma, max_flow):
    n = len(preds)
    mag = torch.sum(gt ** 2, dim=1).sqrt()
    vf = ((valid >= 0.5) & (mag < max_flow))[:, None].float()
    return sum(gamma ** (n - i - 1) * (vf * (p - gt).abs()).mean() for i, p in enumerate(preds))


def test_seq_loss_matches_composite(cuda):
    torch.manual_seed(0)
    N, B, H, W = 5, 3, 40, 56
    base = torch.randn(N * B, 2, H, W, device=cuda) * 20
    base.requires_grad_(True)
    preds = list(base.view(N, B, 2, H, W).unbind(0))
    assert _stacked(preds) is not None
    gt = torch.randn(B, 2, H, W, device=cuda) * 20
    gt[0, :, :4] = 500.0                        # |gt| >= max_flow -> masked
    with torch.no_grad():  # the last prediction within a few px of gt: nontrivial px accuracies
        base[(N - 1) * B:] = gt + torch.randn_like(gt) * 3
    valid = (torch.rand(B, H, W, device=cuda) > 0.3).float()
    loss, metrics = sequence_loss(preds, gt, valid, 0.8, sync_metrics=False)
    base2 = base.detach().clone().requires_grad_(True)
    ref = _composite(list(base2.view(N, B, 2, H, W).unbind(0)), gt, valid, 0.8, 400)
    torch.testing.assert_close(loss, ref, atol=1e-4, rtol=1e-5)
    (loss * 3).backward()
    (ref * 3).backward()
    torch.testing.assert_close(base.grad, base2.grad, atol=1e-9, rtol=1e-6)
    assert set(metrics) == {"epe", "1px", "3px", "5px"}
    # the kernel's metrics vs flow_metrics over the same valid mask (last prediction)
    from raft_stir_amd.train.loss import flow_metrics
    mag = torch.sum(gt ** 2, dim=1).sqrt()
    want = flow_metrics(preds[-1].detach(), gt, (valid >= 0.5) & (mag < 400))
    for k in want:
        torch.testing.assert_close(metrics[k], want[k], atol=1e-5, rtol=1e-5)


def test_separate_preds_use_composite(cuda):
    preds = [torch.randn(2, 2, 16, 16, device=cuda) for _ in range(3)]
    assert _stacked(preds) is None
    gt = torch.randn(2, 2, 16, 16, device=cuda)
    loss, _ = sequence_loss(preds, gt, torch.ones(2, 16, 16, device=cuda), 0.8, sync_metrics=False)
    torch.testing.assert_close(loss, _composite(preds, gt, torch.ones(2, 16, 16, device=cuda), 0.8, 400))
