"""Narrow-channel encoder convs in training (RAFT-small, reference
core/extractor.py:60-116, :195-267): forward and input gradient on
csrc/sconv.hip (stride 2 through a zero-interleaved dY), weight gradient on
csrc/sconv_train.hip, vs an fp32 PyTorch conv2d of the same operands."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from raft_stir_amd.ops import enc_conv

pytestmark = pytest.mark.gpu
CL = torch.channels_last


@pytest.mark.parametrize("cin,cout,k,s", [(8, 8, 3, 1), (16, 16, 3, 2), (24, 24, 3, 2), (32, 16, 1, 1),
                                          (32, 64, 1, 2), (96, 160, 1, 1), (64, 24, 1, 1)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_sconv_train_fwd_bwd(cuda, cin, cout, k, s, dtype, monkeypatch):
    monkeypatch.setattr(enc_conv, "_WIDE_GEO", 0)  # the wide shapes too (RS_WIDE_GEO=0)
    torch.manual_seed(cin + cout + k + s)
    N, H, W = 3, 23, 37
    conv = nn.Conv2d(cin, cout, k, stride=s, padding=k // 2).to(cuda)
    x = (torch.randn(N, cin, H, W, device=cuda) * 0.5).to(dtype).contiguous(memory_format=CL).requires_grad_(True)
    with enc_conv.geo_scope(False), torch.autocast("cuda", dtype=torch.bfloat16, enabled=dtype == torch.bfloat16):
        assert enc_conv.sconv_train_eligible(conv, x)
        y = enc_conv.sconv_train(conv, x)
    assert y.dtype == dtype
    g = torch.randn_like(y.float()).to(dtype)
    y.backward(g)
    cast = (lambda t: t.to(torch.bfloat16).float()) if dtype == torch.bfloat16 else (lambda t: t)
    xr = x.detach().float().requires_grad_(True)
    wr = cast(conv.weight.detach()).requires_grad_(True)
    br = conv.bias.detach().clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, br, stride=s, padding=k // 2)
    yr.backward(g.float())

    def rel(a, b):
        return ((a.double() - b.double()).norm() / b.double().norm()).item()
    tol = 1e-2 if dtype == torch.bfloat16 else 1e-5
    assert rel(y.float(), yr) < tol
    assert rel(x.grad.float(), xr.grad) < tol
    assert rel(conv.weight.grad, wr.grad) < (1e-4 if dtype == torch.bfloat16 else 1e-5)
    assert rel(conv.bias.grad, br.grad) < 1e-4
    # deterministic weight gradient
    w1 = conv.weight.grad.clone()
    conv.weight.grad = None
    with enc_conv.geo_scope(False), torch.autocast("cuda", dtype=torch.bfloat16, enabled=dtype == torch.bfloat16):
        enc_conv.sconv_train(conv, x).backward(g)
    assert torch.equal(conv.weight.grad, w1)


@pytest.mark.parametrize("cin,cout,k,s", [(96, 160, 1, 1), (96, 128, 1, 1), (64, 96, 1, 2)])
def test_wide_convs_leave_the_narrow_kernels(cuda, cin, cout, k, s):
    """RAFT-small's projection and layer-3 shortcut (>= 64 channels in and out)
    take the MFMA geometry path inside the narrow-kernel scope in bf16 (fp32
    keeps sconv)."""
    conv = nn.Conv2d(cin, cout, k, stride=s, padding=k // 2).to(cuda)
    x = torch.randn(2, cin, 16, 24, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL).requires_grad_(True)
    with enc_conv.geo_scope(False), torch.autocast("cuda", dtype=torch.bfloat16):
        assert enc_conv.eligible_geo(conv, x)
        assert not enc_conv.sconv_train_eligible(conv, x) and not enc_conv.sconv_eligible(conv, x)
    xf = x.detach().float().contiguous(memory_format=CL).requires_grad_(True)
    with enc_conv.geo_scope(False):
        assert enc_conv.sconv_train_eligible(conv, xf) and not enc_conv.eligible_geo(conv, xf)
