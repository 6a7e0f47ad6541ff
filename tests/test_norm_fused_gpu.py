"""Normalisation folded into the encoder convolutions (ops/norm.py,
csrc/conv_common.h stats_pix / EPI_NORM, csrc/enc_halo.hip epilogue):

  * statistics epilogue: each conv kernel family (halo 3x3, tile 3x3, strided
    geometry) adds the per-channel (sum, sum of squares) of its bf16 output
    -- checked against fp32 sums of that output, per sample and per batch,
    including tiles whose pixels span two images;
  * norm_finalize -> mean / rstd and a re-zeroed buffer;
  * EPI_NORM: eval-mode BatchNorm scale / shift, ReLU, residual add + ReLU
    in the epilogue vs plain PyTorch fp32 on the same bf16 operands;
  * the encoders (reference core/extractor.py:118-192) with the fused paths
    vs the unfused HIP path: instance norm fwd/bwd, train-mode batch norm
    (outputs, gradients, running statistics) and eval-mode batch norm."""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from raft_stir_amd.ops import enc_conv
from raft_stir_amd.ops import norm as N
from raft_stir_amd.ops.conv import EPI_BIAS, EPI_NORM, conv_fused, pack_weight, pad_to

pytestmark = pytest.mark.gpu
CL = torch.channels_last


def _bf(x):
    return x.to(torch.bfloat16).float()


def _ref_sums(y, per_sample):
    """fp32 (sum, sum of squares) per channel of an NHWC bf16 tensor -> [G][C][2]"""
    y = y.float()
    if per_sample:
        s1, s2 = y.sum((1, 2)), (y * y).sum((1, 2))
    else:
        s1, s2 = y.sum((0, 1, 2))[None], (y * y).sum((0, 1, 2))[None]
    return torch.stack([s1, s2], -1)


def _check_sums(got, y, per_sample):
    want = _ref_sums(y, per_sample)
    scale = want.abs().amax().clamp_min(1.0)
    assert ((got - want).abs().amax() / scale).item() < 2e-5, (got - want).abs().amax().item()


@pytest.mark.parametrize("cin,cout,path", [(64, 64, "halo"), (96, 96, "halo"), (128, 128, "tile"),
                                           (64, 128, "halo")])
@pytest.mark.parametrize("per_sample", [True, False])
@pytest.mark.parametrize("hw", [(24, 40), (13, 21)])  # (13, 21): tiles cross image boundaries
def test_conv3x3_stats(cuda, cin, cout, path, per_sample, hw):
    torch.manual_seed(cin + cout + hw[0])
    B, (H, W) = 3, hw
    x = torch.randn(B, H, W, cin, device=cuda).to(torch.bfloat16)
    w = torch.randn(cout, cin, 3, 3, device=cuda) * 0.05
    wp = pack_weight(w, [(cin, [(0, cin, 0)])], pad_to(cout, 128))
    G = B if per_sample else 1
    st = torch.zeros(G, cout, 2, device=cuda)
    out = torch.empty(B, H, W, cout, device=cuda, dtype=torch.bfloat16)
    if path == "halo":
        assert enc_conv._halo_ok(cin, cout)
        torch.ops.raft_stir.conv3x3_halo(x, wp, out, cin, cout, st, per_sample)
    else:
        conv_fused([(x, 0, cin)], wp, None, 3, 3, cout, EPI_BIAS, out, 0,
                   tile=enc_conv.choose_enc_tile(B * H * W, cin, cout), stats=st, stats_per_sample=per_sample)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), _bf(w), padding=1).permute(0, 2, 3, 1)
    torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=2e-2)
    _check_sums(st, out, per_sample)
    mean, rstd = torch.ops.raft_stir.norm_finalize(st, B * H * W // G, 1e-5)
    assert (st == 0).all(), "norm_finalize must re-zero the sums"
    o = out.float().reshape(G, -1, cout)
    torch.testing.assert_close(mean, o.mean(1), atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(rstd, torch.rsqrt(o.var(1, unbiased=False) + 1e-5), atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("k,s,cin,cout", [(3, 2, 64, 96), (1, 2, 64, 96), (3, 2, 96, 128), (1, 1, 128, 256)])
@pytest.mark.parametrize("per_sample", [True, False])
def test_conv_geo_stats(cuda, k, s, cin, cout, per_sample):
    torch.manual_seed(k * 10 + cin)
    B, H, W = 2, 21, 30
    x = torch.randn(B, cin, H, W, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    conv = nn.Conv2d(cin, cout, k, stride=s, padding=k // 2).to(cuda)
    G = B if per_sample else 1
    st = torch.zeros(G, cout, 2, device=cuda)
    y = enc_conv._conv_geo_fwd(x, conv.weight, None, conv.stride, conv.padding, (st, per_sample))
    ref = F.conv2d(x.float(), _bf(conv.weight), stride=s, padding=k // 2).permute(0, 2, 3, 1)
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=2e-2)
    _check_sums(st, y, per_sample)


def _bn_eval(cout, cuda):
    bn = nn.BatchNorm2d(cout).to(cuda).eval()
    with torch.no_grad():
        bn.running_mean.normal_(0, 0.3)
        bn.running_var.uniform_(0.5, 2.0)
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.normal_(0, 0.2)
    return bn


@pytest.mark.parametrize("cin,cout", [(64, 64), (96, 96), (128, 128)])
@pytest.mark.parametrize("relu,residual", [(True, False), (False, False), (True, True)])
def test_conv3x3_eval_bn_epilogue(cuda, cin, cout, relu, residual):
    torch.manual_seed(cin + relu + 2 * residual)
    conv = nn.Conv2d(cin, cout, 3, padding=1).to(cuda)
    bn = _bn_eval(cout, cuda)
    x = torch.randn(2, cin, 17, 45, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    res = (torch.randn(2, cout, 17, 45, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
           if residual else None)
    sc, sh = N._eval_affine(bn, conv.bias)
    with torch.no_grad():
        y = enc_conv.conv_norm(conv, x, sc, sh, relu, res)
        ref = bn(F.conv2d(x.float(), _bf(conv.weight), conv.bias, padding=1))
        if relu:
            ref = ref.relu()
        if residual:
            ref = (ref + res.float()).relu()
    torch.testing.assert_close(y.float(), ref, atol=4e-2, rtol=2e-2)


@pytest.mark.parametrize("k,cin,cout,relu", [(3, 64, 96, True), (1, 64, 96, False), (3, 96, 128, True)])
def test_conv_geo_eval_bn_epilogue(cuda, k, cin, cout, relu):
    torch.manual_seed(k + cin)
    conv = nn.Conv2d(cin, cout, k, stride=2, padding=k // 2).to(cuda)
    bn = _bn_eval(cout, cuda)
    x = torch.randn(2, cin, 33, 50, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    sc, sh = N._eval_affine(bn, conv.bias)
    with torch.no_grad():
        y = enc_conv.conv_norm(conv, x, sc, sh, relu)
        ref = bn(F.conv2d(x.float(), _bf(conv.weight), conv.bias, stride=2, padding=k // 2))
        if relu:
            ref = ref.relu()
    torch.testing.assert_close(y.float(), ref, atol=4e-2, rtol=2e-2)


def _encoder(norm_fn, cuda, seed=7):
    from raft_stir_amd.models.extractor import BasicEncoder
    torch.manual_seed(seed)
    return BasicEncoder(output_dim=128, norm_fn=norm_fn).to(cuda).to(memory_format=CL)


def _run(enc, x, fused, train, bf16=True):
    prev, N._FUSED_STATS = N._FUSED_STATS, fused
    try:
        enc.zero_grad(set_to_none=True)
        enc.train(train)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
            y = enc(x)
        y.float().square().mean().backward()
    finally:
        N._FUSED_STATS = prev
    return y.detach().float(), {n: p.grad.detach().clone() for n, p in enc.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("norm_fn", ["instance", "batch"])
def test_encoder_fused_stats_match_unfused(cuda, norm_fn):
    """Encoder forward + backward with the conv-epilogue statistics vs the
    separate reduction pass, both against the fp32 encoder: the fused path
    must be as close to fp32 as the unfused bf16 path is (bf16 rounding flips
    dominate any fp32 summation-order difference), with the same (batch norm)
    running statistics."""
    enc = _encoder(norm_fn, cuda)
    x = (torch.rand(3, 3, 88, 120, device=cuda) * 2 - 1).contiguous(memory_format=CL)
    ea, eb, ec = enc, copy.deepcopy(enc), copy.deepcopy(enc)
    ya, ga = _run(ea, x, True, True)
    yb, gb = _run(eb, x, False, True)
    yc, gc = _run(ec, x, False, True, bf16=False)
    rel = lambda a, b: ((a - b).norm() / b.norm().clamp_min(1e-12)).item()
    assert rel(ya, yc) <= 1.25 * rel(yb, yc) + 2e-3, (rel(ya, yc), rel(yb, yc))
    for n in gc:
        if n.endswith(".bias") and "conv2" not in n and "layer" in n:
            continue  # folded into the norm: exactly-zero gradient either way
        assert rel(ga[n], gc[n]) <= 1.25 * rel(gb[n], gc[n]) + 5e-3, (n, rel(ga[n], gc[n]), rel(gb[n], gc[n]))
    if norm_fn == "batch":
        for (n, a), (_, b) in zip(ea.named_buffers(), eb.named_buffers()):
            if a.dtype.is_floating_point:
                torch.testing.assert_close(a, b, atol=2e-3, rtol=2e-2, msg=n)
    # every fused-statistics buffer is handed back zeroed
    for m in ea.modules():
        buf = m.__dict__.get("_rs_sums")
        if buf is not None:
            assert (buf == 0).all()


def test_encoder_eval_bn_fused(cuda):
    """Eval-mode batch-norm encoder under no_grad (everything in the conv
    epilogues) vs the same model with autograd on (norm passes)."""
    enc = _encoder("batch", cuda, seed=9)
    with torch.no_grad():
        for m in enc.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.running_mean.normal_(0, 0.2)
                m.running_var.uniform_(0.5, 2.0)
                m.weight.uniform_(0.5, 1.5)
                m.bias.normal_(0, 0.1)
    enc.eval()
    x = (torch.rand(2, 3, 96, 136, device=cuda) * 2 - 1).contiguous(memory_format=CL)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        with torch.no_grad():
            ya = enc(x).float()
        yb = enc(x.requires_grad_()).float().detach()
    rel = ((ya - yb).norm() / yb.norm()).item()
    assert rel < 1e-2, rel
    # the scale / shift caches follow a weight change (in place)
    with torch.no_grad():
        for m in enc.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.weight.mul_(1.5)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        with torch.no_grad():
            yc = enc(x).float()
        yd = enc(x).float().detach()
    assert ((yc - yd).norm() / yd.norm()).item() < 1e-2
    assert ((yc - ya).norm() / ya.norm()).item() > 1e-2
