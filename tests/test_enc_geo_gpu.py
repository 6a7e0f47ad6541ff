"""Strided / 1x1 encoder convolutions on the HIP kernels (ops/enc_conv.py
conv_geo / conv_pair; csrc/conv.hip conv_lds_kernel<GEO>, csrc/conv_wgrad.hip
strided DMA weight gradient) vs plain fp32 PyTorch of the same op."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from raft_stir_amd.ops import enc_conv

pytestmark = pytest.mark.gpu
CL = torch.channels_last


def _ref(conv, x, dy):
    """fp32 forward / input / weight / bias gradients of conv at the bf16 input."""
    xr = x.detach().float().requires_grad_()
    w = conv.weight.detach().float().requires_grad_()
    b = None if conv.bias is None else conv.bias.detach().float().requires_grad_()
    y = F.conv2d(xr, w, b, conv.stride, conv.padding)
    y.backward(dy.float())
    return y.detach(), xr.grad, w.grad, (None if b is None else b.grad)


def _close(a, b, tol, name):
    err = (a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)
    assert err < tol, (name, err.item())


@pytest.mark.parametrize("k,s,cin,cout,hw,bias", [
    (3, 2, 64, 96, (40, 56), False),
    (3, 2, 96, 128, (37, 51), False),    # odd input: unequal phase grids
    (1, 2, 64, 96, (40, 56), False),     # 1x1/s2 shortcut alone: three empty phases
    (1, 2, 96, 128, (23, 31), False),
    (1, 1, 128, 256, (24, 32), True),    # projection head, with bias
])
def test_conv_geo_matches_fp32(cuda, k, s, cin, cout, hw, bias):
    torch.manual_seed(0)
    conv = nn.Conv2d(cin, cout, k, stride=s, padding=k // 2, bias=bias).to(cuda)
    x = torch.randn(2, cin, *hw, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    assert enc_conv.eligible_geo(conv, x)
    xg = x.clone().requires_grad_()
    y = enc_conv.conv_geo(conv, xg)
    dy = torch.randn(y.shape, device=cuda).to(torch.bfloat16)
    y.backward(dy)
    yr, dxr, dwr, dbr = _ref(conv, x, dy)
    assert y.shape == yr.shape and y.is_contiguous(memory_format=CL)
    _close(y, yr, 1e-2, "y")
    _close(xg.grad, dxr, 1e-2, "dx")
    _close(conv.weight.grad, dwr, 1e-2, "dw")
    if bias:
        _close(conv.bias.grad, dbr, 1e-2, "db")


@pytest.mark.parametrize("cin,cout,hw", [(64, 96, (40, 56)), (96, 128, (35, 49))])
def test_conv_pair_matches_fp32(cuda, cin, cout, hw):
    """Residual block's stride-2 3x3 + stride-2 1x1 shortcut: one input
    gradient with the shortcut fused into the (0, 0) phase."""
    torch.manual_seed(1)
    c1 = nn.Conv2d(cin, cout, 3, stride=2, padding=1).to(cuda)
    cd = nn.Conv2d(cin, cout, 1, stride=2).to(cuda)
    x = torch.randn(2, cin, *hw, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    assert enc_conv.pair_eligible(c1, cd, x)
    xg = x.clone().requires_grad_()
    y1, yd = enc_conv.conv_pair(c1, cd, xg)
    g1 = torch.randn(y1.shape, device=cuda).to(torch.bfloat16)
    gd = torch.randn(yd.shape, device=cuda).to(torch.bfloat16)
    (y1.float() * g1.float()).sum().add((yd.float() * gd.float()).sum()).backward()
    r1, dx1, dw1, _ = _ref(_nobias(c1), x, g1)
    rd, dxd, dwd, _ = _ref(_nobias(cd), x, gd)
    _close(y1, r1, 1e-2, "y1")
    _close(yd, rd, 1e-2, "yd")
    _close(xg.grad, dx1 + dxd, 1e-2, "dx")
    _close(c1.weight.grad, dw1, 1e-2, "dw1")
    _close(cd.weight.grad, dwd, 1e-2, "dwd")
    assert c1.bias.grad is None and cd.bias.grad is None  # folded into the norms by the caller


def _nobias(conv):
    c = nn.Conv2d(conv.in_channels, conv.out_channels, conv.kernel_size, stride=conv.stride, padding=conv.padding,
                  bias=False).to(conv.weight.device)
    with torch.no_grad():
        c.weight.copy_(conv.weight)
    return c


def test_encoder_uses_geo_path(cuda):
    """BasicEncoder on the GPU bf16 path with its strided / 1x1 convs on the HIP
    kernels is as close to the fp32 encoder as the MIOpen bf16 path is."""
    from raft_stir_amd.models.extractor import BasicEncoder
    torch.manual_seed(2)
    enc = BasicEncoder(output_dim=256, norm_fn="instance").to(cuda).to(memory_format=CL)
    x = (torch.rand(2, 3, 96, 128, device=cuda) * 2 - 1).contiguous(memory_format=CL)
    res = {}
    for mode in ("geo", "miopen", "fp32"):
        enc_conv._GEO = mode == "geo"
        enc.zero_grad(set_to_none=True)
        try:
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=mode != "fp32"):
                y = enc(x)
            y.float().square().mean().backward()
        finally:
            enc_conv._GEO = True
        res[mode] = (y.detach().float(), {n: p.grad.detach().clone() for n, p in enc.named_parameters()
                                          if p.grad is not None})
    rel = lambda a, b: ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()
    yr, gr = res["fp32"]
    assert rel(res["geo"][0], yr) < 2e-2
    for n in gr:
        if n.endswith(".bias") and "conv2" not in n:  # folded into instance norm: ~0 exact gradient
            continue
        eg, em = rel(res["geo"][1][n], gr[n]), rel(res["miopen"][1][n], gr[n])
        assert eg < 1.5 * em + 2e-2, (n, eg, em)


def test_packed_weights_follow_fused_adamw(cuda):
    """torch.optim.AdamW(fused=True) does not bump parameter versions: the
    packed-weight caches must still see every step (runtime/weights.py)."""
    from raft_stir_amd.models.extractor import BasicEncoder
    torch.manual_seed(3)
    enc = BasicEncoder(output_dim=256, norm_fn="instance").to(cuda).to(memory_format=CL)
    x = (torch.rand(2, 3, 96, 128, device=cuda) * 2 - 1).contiguous(memory_format=CL)
    opt = torch.optim.AdamW(enc.parameters(), lr=1e-2, fused=True)
    for _ in range(2):
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = enc(x)
        y.float().square().mean().backward()
        opt.step()
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            ya = enc(x).float()
            enc_conv._GEO, enc_conv._ENABLED = False, False
            try:
                yb = enc(x).float()
            finally:
                enc_conv._GEO, enc_conv._ENABLED = True, True
        _close(ya, yb, 2e-2, "fmap after a fused AdamW step")


@pytest.mark.parametrize("small", [False, True])
def test_graphed_inference_sees_weight_updates(cuda, small):
    """A captured inference graph re-packs its cached weights (in place)
    when an optimizer step moved them (RAFT-small: the permuted sconv
    encoder weights, ops/enc_conv.py _refresh_sconv)."""
    from raft_stir_amd.config import make_args
    from raft_stir_amd.models import RAFT
    from raft_stir_amd.runtime.graph import GraphedInference
    torch.manual_seed(4)
    m = RAFT(make_args(mixed_precision=True, small=small)).to(cuda).to(memory_format=CL).eval()
    i1 = torch.rand(1, 3, 128, 192, device=cuda) * 255
    i2 = torch.rand(1, 3, 128, 192, device=cuda) * 255
    gi = GraphedInference(m, i1.shape, iters=4)
    before = gi(i1, i2)[1].clone()
    opt = torch.optim.AdamW(m.parameters(), lr=5e-3, fused=True)
    for p in m.parameters():
        p.grad = torch.randn_like(p)
    opt.step()
    got = gi(i1, i2)[1].clone()
    with torch.no_grad():
        want = m(i1, i2, iters=4, test_mode=True)[1]
    # stale weights would leave the replay at ~the pre-update flow; graph and
    # eager run the same kernels (no atomics at inference)
    moved = ((before - want).norm() / want.norm()).item()
    assert moved > 1e-2, moved
    _close(got, want, min(1e-3, 0.1 * moved), "graphed flow after the update")
