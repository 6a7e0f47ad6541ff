"""ops/fp32conv.py: layout-tuned fp32 convolutions == F.conv2d (either layout), channels_last out;
the backward follows the forward's choice."""
import pytest
import torch
import torch.nn.functional as F

from raft_stir_amd.ops import fp32conv

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cin,cout,k,stride", [(242, 192, 3, 1), (384, 256, (1, 5), 1), (64, 96, 3, 2)])
def test_tuned_conv_matches(cuda, cin, cout, k, stride):
    torch.manual_seed(0)
    kk = k if isinstance(k, tuple) else (k, k)
    pad = (kk[0] // 2, kk[1] // 2)
    x = torch.randn(2, cin, 24, 40, device=cuda).contiguous(memory_format=torch.channels_last)
    w = torch.randn(cout, cin, *kk, device=cuda) * 0.05
    b = torch.randn(cout, device=cuda)
    ref = F.conv2d(x.contiguous(), w, b, stride, pad)
    y = fp32conv.conv2d(x, w, b, stride, pad)
    assert y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y, ref, atol=1e-3, rtol=1e-3)
    key = next(k_ for k_ in fp32conv._CHOICE if k_[0] == tuple(x.shape) and k_[1] == tuple(w.shape))
    for forced in (True, False):  # both layouts are numerically the same conv
        fp32conv._CHOICE[key] = forced
        torch.testing.assert_close(fp32conv.conv2d(x, w, b, stride, pad), ref, atol=1e-3, rtol=1e-3)
        dy = torch.randn_like(ref)
        dx, dw, db = fp32conv.conv_backward(dy, x, w, (stride, stride), pad)
        xr, wr = x.detach().clone().requires_grad_(True), w.detach().clone().requires_grad_(True)
        F.conv2d(xr, wr, b, stride, pad).backward(dy)
        torch.testing.assert_close(dx, xr.grad, atol=2e-3, rtol=2e-3)
        torch.testing.assert_close(dw, wr.grad, atol=5e-2, rtol=2e-3)


def test_bf16_passthrough(cuda):
    x = torch.randn(1, 32, 8, 8, device=cuda, dtype=torch.bfloat16)
    w = torch.randn(16, 32, 3, 3, device=cuda, dtype=torch.bfloat16)
    assert not fp32conv.active(x)
    torch.testing.assert_close(fp32conv.conv2d(x, w, None, 1, 1), F.conv2d(x, w, None, 1, 1))
