"""7x7 / stride-2 encoder stem on csrc/stem.hip (reference
core/extractor.py:135, :212): forward in bf16 (what autocast feeds the
reference conv) and split-bf16 fp32, the statistics and eval-BN epilogues,
and the deterministic MFMA weight gradient, vs plain PyTorch on the same
operands."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from raft_stir_amd.ops import enc_conv
from raft_stir_amd.ops.conv import EPI_NORM

pytestmark = pytest.mark.gpu
CL = torch.channels_last


def _bf(t):
    return t.to(torch.bfloat16).float()


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


def _img(B, H, W, cuda, seed):
    g = torch.Generator(device=cuda).manual_seed(seed)
    return (torch.rand(B, 3, H, W, device=cuda, generator=g) * 2 - 1).contiguous(memory_format=CL)


@pytest.mark.parametrize("shape", [(1, 37, 53), (3, 96, 130)])
@pytest.mark.parametrize("cout", [64, 32])
def test_stem_forward_bf16(cuda, shape, cout):
    B, H, W = shape
    torch.manual_seed(cout)
    conv = nn.Conv2d(3, cout, 7, stride=2, padding=3).to(cuda)
    x = _img(B, H, W, cuda, 1)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = enc_conv.stem(conv, x)
    assert y.dtype == torch.bfloat16
    ref = F.conv2d(_bf(x), _bf(conv.weight), stride=2, padding=3)
    assert y.shape == ref.shape
    torch.testing.assert_close(y.float(), ref, atol=2e-2, rtol=1e-2)


@pytest.mark.parametrize("cout", [64, 32])
def test_stem_forward_f32(cuda, cout):
    torch.manual_seed(2)
    conv = nn.Conv2d(3, cout, 7, stride=2, padding=3).to(cuda)
    x = _img(2, 61, 90, cuda, 2)
    with torch.no_grad():
        y = enc_conv.stem(conv, x)
    assert y.dtype == torch.float32
    ref = F.conv2d(x.double(), conv.weight.double(), stride=2, padding=3)
    assert _rel(y, ref) < 2e-5, _rel(y, ref)


@pytest.mark.parametrize("f32", [False, True])
def test_stem_eval_bn(cuda, f32):
    torch.manual_seed(4)
    conv = nn.Conv2d(3, 64, 7, stride=2, padding=3).to(cuda)
    sc = torch.rand(64, device=cuda) + 0.5
    sh = torch.randn(64, device=cuda) * 0.1
    x = _img(2, 44, 66, cuda, 4)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16, enabled=not f32):
        y = enc_conv.stem_norm(conv, x, sc, sh, True)
    if f32:
        ref = F.conv2d(x.double(), conv.weight.double(), stride=2, padding=3)
        ref = (ref * sc.double().view(1, -1, 1, 1) + sh.double().view(1, -1, 1, 1)).relu()
        assert _rel(y, ref) < 2e-5
    else:
        ref = F.conv2d(_bf(x), _bf(conv.weight), stride=2, padding=3)
        ref = (ref * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1)).relu()
        torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=1e-2)


@pytest.mark.parametrize("cout", [64, 32])
@pytest.mark.parametrize("shape", [(2, 75, 99), (4, 184, 300)])
def test_stem_wgrad(cuda, cout, shape):
    """64-pixel row chunks: one partial chunk per row (Wo = 50) and three
    per row with a partial last one (Wo = 150); blocks span row boundaries."""
    torch.manual_seed(5)
    conv = nn.Conv2d(3, cout, 7, stride=2, padding=3).to(cuda)
    x = _img(*shape, cuda, 5)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = enc_conv.stem(conv, x)
    g = torch.randn_like(y.float()).to(torch.bfloat16)
    y.backward(g)
    wr = _bf(conv.weight).detach().requires_grad_()
    F.conv2d(_bf(x), wr, stride=2, padding=3).backward(g.float())
    assert _rel(conv.weight.grad, wr.grad) < 1e-5, _rel(conv.weight.grad, wr.grad)
    # deterministic: the same gradient again, bitwise
    g1 = conv.weight.grad.clone()
    conv.weight.grad = None
    with torch.autocast("cuda", dtype=torch.bfloat16):
        enc_conv.stem(conv, x).backward(g)
    assert torch.equal(conv.weight.grad, g1)


def test_stem_fp32_training(cuda):
    """fp32 training (the reference's default precision) through the HIP stem:
    split-bf16 forward and the three-product split weight gradient, vs fp64."""
    torch.manual_seed(7)
    conv = nn.Conv2d(3, 64, 7, stride=2, padding=3).to(cuda)
    x = _img(2, 75, 99, cuda, 7)
    assert enc_conv.stem_eligible(conv, x)
    y = enc_conv.stem(conv, x)
    assert y.dtype == torch.float32
    g = torch.randn_like(y)
    y.backward(g)
    wr = conv.weight.detach().double().requires_grad_()
    yr = F.conv2d(x.double(), wr, stride=2, padding=3)
    yr.backward(g.double())
    assert _rel(y, yr) < 2e-5, _rel(y, yr)
    assert _rel(conv.weight.grad, wr.grad) < 5e-5, _rel(conv.weight.grad, wr.grad)
