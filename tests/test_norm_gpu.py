"""csrc/norm.hip (fused NHWC norm + ReLU [+ residual + ReLU]) vs the fp32 PyTorch composite."""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from raft_stir_amd.ops.norm import norm_act

pytestmark = pytest.mark.gpu


def _ref(norm, x, relu, res):
    y = norm(x)
    if relu:
        y = F.relu(y)
    if res is not None:
        y = F.relu(res + y)
    return y


@pytest.mark.parametrize("kind", ["instance", "batch_train", "batch_eval"])
@pytest.mark.parametrize("C", [32, 64, 96])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("relu,use_res", [(True, False), (False, False), (True, True)])
def test_norm_act_fwd_bwd(cuda, kind, C, dtype, relu, use_res):
    torch.manual_seed(0)
    B, H, W = 3, 13, 21
    if kind == "instance":
        norm = nn.InstanceNorm2d(C)
    else:
        norm = nn.BatchNorm2d(C)
        with torch.no_grad():
            norm.weight.uniform_(0.5, 1.5)
            norm.bias.uniform_(-0.3, 0.3)
            norm.running_mean.uniform_(-0.2, 0.2)
            norm.running_var.uniform_(0.5, 2.0)
        norm.train(kind == "batch_train")
    norm = norm.to(cuda)
    ref_norm = copy.deepcopy(norm)
    x0 = (torch.randn(B, C, H, W, device=cuda) * 2 + 0.5)
    x = x0.to(dtype).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    res = None
    if use_res:
        res = torch.randn(B, C, H, W, device=cuda).to(dtype).contiguous(memory_format=torch.channels_last)
        res.requires_grad_(True)
    y = norm_act(norm, x, relu=relu, residual=res)
    xr = x.detach().float().requires_grad_(True)
    rr = res.detach().float().requires_grad_(True) if use_res else None
    yr = _ref(ref_norm, xr, relu, rr)
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    torch.testing.assert_close(y.float(), yr, atol=tol, rtol=tol)
    g = torch.randn_like(yr)
    y.backward(g.to(dtype).contiguous(memory_format=torch.channels_last))
    yr.backward(g.to(dtype).float())
    gtol = 2e-4 if dtype == torch.float32 else 6e-2
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=gtol, rtol=gtol)
    if use_res:
        torch.testing.assert_close(res.grad.float(), rr.grad, atol=gtol, rtol=gtol)
    if kind != "instance":
        torch.testing.assert_close(norm.weight.grad, ref_norm.weight.grad, atol=gtol * 10, rtol=gtol)
        torch.testing.assert_close(norm.bias.grad, ref_norm.bias.grad, atol=gtol * 10, rtol=gtol)
        torch.testing.assert_close(norm.running_mean, ref_norm.running_mean, atol=1e-4, rtol=1e-3)
        torch.testing.assert_close(norm.running_var, ref_norm.running_var, atol=1e-3, rtol=1e-3)
        assert int(norm.num_batches_tracked) == int(ref_norm.num_batches_tracked)


def test_norm_act_large_spatial(cuda):
    """Encoder-stem sized map (many split blocks, fp64 finalize)."""
    torch.manual_seed(1)
    x = (torch.randn(4, 64, 92, 124, device=cuda) * 3 + 1).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    norm = nn.InstanceNorm2d(64)
    y = norm_act(norm, x)
    yr = F.relu(norm(x.float()))
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("kind", ["instance", "batch_train", "batch_eval"])
def test_conv_norm_act_folds_bias(cuda, kind):
    """conv_norm_act (bias folded into the norm) vs relu(norm(conv(x) + b)) in fp32."""
    from raft_stir_amd.ops.norm import conv_norm_act
    torch.manual_seed(2)
    C = 64
    conv = nn.Conv2d(32, C, 3, padding=1)
    with torch.no_grad():
        conv.bias.uniform_(-1, 1)
    if kind == "instance":
        norm = nn.InstanceNorm2d(C)
    else:
        norm = nn.BatchNorm2d(C)
        with torch.no_grad():
            norm.weight.uniform_(0.5, 1.5)
            norm.running_mean.uniform_(-0.2, 0.2)
            norm.running_var.uniform_(0.5, 2.0)
        norm.train(kind == "batch_train")
    conv, norm = conv.to(cuda), norm.to(cuda)
    rconv, rnorm = copy.deepcopy(conv), copy.deepcopy(norm)
    x = torch.randn(2, 32, 24, 40, device=cuda).contiguous(memory_format=torch.channels_last)
    y = conv_norm_act(conv, norm, x)
    yr = F.relu(rnorm(rconv(x)))
    torch.testing.assert_close(y, yr, atol=1e-4, rtol=1e-4)
    g = torch.randn_like(yr)
    y.backward(g.contiguous(memory_format=torch.channels_last))
    yr.backward(g)
    torch.testing.assert_close(conv.weight.grad, rconv.weight.grad, atol=1e-3, rtol=1e-3)
    if kind == "batch_eval":
        torch.testing.assert_close(conv.bias.grad, rconv.bias.grad, atol=1e-3, rtol=1e-3)
    else:  # exactly zero (the reference carries round-off only)
        assert conv.bias.grad.abs().max() == 0 and rconv.bias.grad.abs().max() < 1e-3
        if kind == "batch_train":
            torch.testing.assert_close(norm.running_mean, rnorm.running_mean, atol=1e-5, rtol=1e-5)


def test_bn_recalibration_then_eval(cuda):
    """Train-mode forwards under no_grad (BN recalibration) update the running
    buffers inside the statistics launch (norm_stats running_mean / running_var /
    nbt, csrc/norm.hip finalize_kernel); a following eval()
    forward must see the new buffers, not the eval-affine cache of the old ones
    (ops/norm.py bumps the version counters the cache is keyed on)."""
    from raft_stir_amd.ops.norm import conv_norm_act
    torch.manual_seed(5)
    C = 64
    conv = nn.Conv2d(32, C, 3, padding=1).to(cuda)
    norm = nn.BatchNorm2d(C).to(cuda)
    rconv, rnorm = copy.deepcopy(conv), copy.deepcopy(norm)
    x = torch.randn(2, 32, 24, 40, device=cuda).contiguous(memory_format=torch.channels_last)
    x2 = (torch.randn(2, 32, 24, 40, device=cuda) * 3 + 1).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        norm.eval()
        rnorm.eval()
        conv_norm_act(conv, norm, x)  # populate the eval-mode cache
        norm.train()
        rnorm.train()
        for _ in range(3):
            conv_norm_act(conv, norm, x2)
            F.relu(rnorm(rconv(x2)))
        norm.eval()
        rnorm.eval()
        torch.testing.assert_close(norm.running_mean, rnorm.running_mean, atol=1e-4, rtol=1e-4)
        torch.testing.assert_close(norm.running_var, rnorm.running_var, atol=1e-4, rtol=1e-4)
        assert norm.num_batches_tracked.item() == rnorm.num_batches_tracked.item() == 3
        y = conv_norm_act(conv, norm, x)
        yr = F.relu(rnorm(rconv(x)))
    torch.testing.assert_close(y, yr, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("kind", ["instance", "batch"])
def test_norm_affine_residual_and_second_grad(cuda, kind):
    """csrc/norm.hip extensions used by models/fused_encoder.py: the output
    pass relu(relu(n2(a)) + n3(d)) with the shortcut's norm n3 applied on the
    fly to the RAW d, its backward (gradient of a AND of raw d, both norms'
    parameter sums) and a second upstream gradient added inside the kernels,
    against fp32 autograd on the module composite."""
    torch.manual_seed(0)
    B, C, H, W = 3, 96, 12, 20
    mk = (lambda: nn.InstanceNorm2d(C)) if kind == "instance" else (lambda: nn.BatchNorm2d(C))
    n2, n3 = mk().to(cuda), mk().to(cuda)
    if kind == "batch":
        with torch.no_grad():
            for n in (n2, n3):
                n.weight.uniform_(0.5, 1.5)
                n.bias.uniform_(-0.3, 0.3)
    a = (torch.randn(B, C, H, W, device=cuda) * 2 + 0.5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    d = (torch.randn(B, C, H, W, device=cuda) - 0.3).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g1 = torch.randn(B, C, H, W, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g2 = torch.randn(B, C, H, W, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    # reference (fp32 autograd)
    af, df = a.float().requires_grad_(), d.float().requires_grad_()
    ref = torch.relu(torch.relu(n2(af)) + n3(df))
    (ref * (g1.float() + g2.float())).sum().backward()
    nh = lambda t: t.permute(0, 2, 3, 1).contiguous()
    R = torch.ops.raft_stir
    inst = kind == "instance"
    st2 = R.norm_stats(nh(a), inst, n2.eps)
    st3 = R.norm_stats(nh(d), inst, n3.eps)
    gm = lambda n: None if inst else n.weight.detach()
    bt = lambda n: None if inst else n.bias.detach()
    y = R.norm_act(nh(a), st2[0], st2[1], gm(n2), bt(n2), nh(d), True, st3[0], st3[1], gm(n3), bt(n3))
    torch.testing.assert_close(y.float(), nh(ref.detach()), atol=3e-2, rtol=2e-2)
    out = R.norm_act_backward(nh(g1), nh(a), st2[0], st2[1], gm(n2), bt(n2), nh(d), True, True, nh(g2),
                              st3[0], st3[1], gm(n3), bt(n3))
    da, dd, r12 = out[0], out[1], out[5]
    scale = lambda t: t.abs().max().item()
    assert (da.float() - nh(af.grad)).abs().max().item() < 3e-2 * scale(af.grad)
    assert (dd.float() - nh(df.grad)).abs().max().item() < 3e-2 * scale(df.grad)
    if not inst:
        dgamma3, dbeta3 = r12[1].sum(0), r12[0].sum(0)
        torch.testing.assert_close(dbeta3, n3.bias.grad, atol=2e-2 * scale(n3.bias.grad), rtol=2e-2)
        torch.testing.assert_close(dgamma3, n3.weight.grad, atol=2e-2 * scale(n3.weight.grad), rtol=2e-2)
        s12 = out[4]
        torch.testing.assert_close(s12[0].sum(0), n2.bias.grad, atol=2e-2 * scale(n2.bias.grad), rtol=2e-2)
