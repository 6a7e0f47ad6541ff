"""Eval-mode BatchNorm folded into the encoder convolutions (ops/norm.py,
csrc/conv_common.h / csrc/enc_halo.hip EPI_NORM epilogue; reference
core/extractor.py:118-192):

  * EPI_NORM: eval-mode BatchNorm scale / shift, ReLU, residual add + ReLU
    in the epilogue vs plain PyTorch fp32 on the same bf16 operands;
  * the eval-mode batch-norm encoder under no_grad (everything in the conv
    epilogues) vs the same model with its norm passes, and its scale / shift
    caches following a weight change."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from raft_stir_amd.ops import enc_conv
from raft_stir_amd.ops import norm as N

pytestmark = pytest.mark.gpu
CL = torch.channels_last


def _bf(x):
    return x.to(torch.bfloat16).float()


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
