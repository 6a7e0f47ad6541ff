"""ops/enc_conv.py (stride-1 3x3 encoder convs on csrc/conv.hip + csrc/conv_wgrad.hip)
vs an fp32 PyTorch conv2d of the same bf16 operands: forward, input and weight gradients."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from raft_stir_amd.ops import enc_conv

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cin,cout", [(64, 64), (96, 96), (128, 128), (64, 96), (96, 128)])
@pytest.mark.parametrize("shape", [(2, 23, 31), (3, 46, 62)])
def test_conv3x3_fwd_bwd(cuda, cin, cout, shape):
    torch.manual_seed(0)
    N, H, W = shape
    conv = nn.Conv2d(cin, cout, 3, padding=1).to(cuda)
    x = (torch.randn(N, cin, H, W, device=cuda) * 0.5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    assert enc_conv.eligible(conv, x)
    x.requires_grad_(True)
    y = enc_conv.conv3x3(conv, x)
    g = torch.randn_like(y.float()).to(torch.bfloat16)
    y.backward(g)

    xr = x.detach().float().requires_grad_(True)
    wr = conv.weight.detach().to(torch.bfloat16).float().requires_grad_(True)
    yr = F.conv2d(xr, wr, None, padding=1)
    yr.backward(g.float())

    def rel(a, b):
        return ((a.float() - b).abs().max() / b.abs().max()).item()

    assert y.shape == yr.shape and y.dtype == torch.bfloat16
    assert rel(y, yr) < 1e-2
    assert rel(x.grad, xr.grad) < 1e-2
    # weight gradient: fp32 accumulation over bf16 operands
    assert rel(conv.weight.grad, wr.grad) < 1e-2


def test_packed_weight_cache_tracks_updates(cuda):
    torch.manual_seed(1)
    conv = nn.Conv2d(64, 64, 3, padding=1).to(cuda)
    x = torch.randn(1, 64, 9, 17, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        y0 = enc_conv.conv3x3(conv, x).float()
        conv.weight.mul_(2.0)  # in-place update (optimizer step): the packed copy must follow
        y1 = enc_conv.conv3x3(conv, x).float()
    torch.testing.assert_close(y1, 2 * y0, atol=2e-2, rtol=2e-2)


def test_ineligible_shapes(cuda):
    x = torch.randn(1, 64, 8, 8, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    assert not enc_conv.eligible(nn.Conv2d(64, 64, 3, padding=1, stride=2).to(cuda), x)
    assert not enc_conv.eligible(nn.Conv2d(64, 64, 1).to(cuda), x)
    assert not enc_conv.eligible(nn.Conv2d(64, 64, 3, padding=1).to(cuda), x.float())
    assert not enc_conv.eligible(nn.Conv2d(64, 24, 3, padding=1).to(cuda), x)


@pytest.mark.parametrize("cin,cout", [(64, 64), (96, 96), (64, 128), (96, 32)])
@pytest.mark.parametrize("shape", [(2, 37, 45), (1, 8, 32), (3, 13, 70)])
def test_conv3x3_halo_kernel(cuda, cin, cout, shape):
    """csrc/enc_halo.hip (persistent halo-tile 3x3 conv) vs the fp32 PyTorch conv:
    partial tiles in both directions, zero padding at every border, channel
    strides wider than the conv (x with 32 extra channels, y with 8)."""
    from raft_stir_amd.ops.conv import pack_weight, pad_to
    B, H, W = shape
    g = torch.Generator(device="cpu").manual_seed(7)
    x = (torch.randn(B, H, W, cin + 32, generator=g) * 0.5).to(cuda, torch.bfloat16)
    w = (torch.randn(cout, cin, 3, 3, generator=g) * 0.05).to(cuda)
    wp = pack_weight(w, [(cin, [(0, cin, 0)])], pad_to(cout, 128))
    y = torch.full((B, H, W, cout + 8), 7.0, device=cuda, dtype=torch.bfloat16)
    torch.ops.raft_stir.conv3x3_halo(x, wp, y, cin, cout)
    want = F.conv2d(x[..., :cin].permute(0, 3, 1, 2).float(), w.to(torch.bfloat16).float(), padding=1)
    got = y[..., :cout].permute(0, 3, 1, 2).float()
    rel = ((got - want).norm() / want.norm()).item()
    assert rel < 1e-2, rel
    assert (y[..., cout:] == 7.0).all()  # channels past cout untouched


@pytest.mark.parametrize("cin,cout,shape", [(64, 64, (14, 184, 248)), (64, 64, (2, 23, 31)), (96, 96, (2, 23, 31))])
def test_grad_sink_adds_skip_gradient(cuda, cin, cout, shape):
    """GradSink: a first conv whose input gradient runs on the halo kernel
    (1/2-res 64 -> 64 of fnet's size) arms the sink and adds the residual skip
    gradient in that kernel's epilogue; convs on the v3 tiles leave it unarmed
    (the norm then returns the skip gradient to autograd)."""
    torch.manual_seed(2)
    N, H, W = shape
    conv = nn.Conv2d(cin, cout, 3, padding=1).to(cuda)
    x = (torch.randn(N, cin, H, W, device=cuda) * 0.5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    sink = enc_conv.GradSink()
    y = enc_conv.conv3x3(conv, x, sink)
    halo = enc_conv._halo_ok(cout, cin) and enc_conv._v3_tile(N * H * W, cout, cin) is None
    assert sink.armed == halo
    skip = torch.randn(N, H, W, cin, device=cuda).to(torch.bfloat16)   # NHWC, as norm_act_backward makes it
    if halo:
        sink.dres = skip.clone()
    g = torch.randn_like(y.float()).to(torch.bfloat16)
    y.backward(g)
    assert sink.dres is None
    xr = x.detach().float().requires_grad_(True)
    F.conv2d(xr, conv.weight.detach().to(torch.bfloat16).float(), None, padding=1).backward(g.float())
    ref = xr.grad + (skip.float().permute(0, 3, 1, 2) if halo else 0)
    assert ((x.grad.float() - ref).abs().max() / ref.abs().max()).item() < 1e-2
