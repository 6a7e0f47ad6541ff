"""Halo-tile weight gradient of the encoders' stride-1 3x3 convolutions
(csrc/enc_wgrad.hip; reference core/extractor.py:6-56 ResidualBlock convs,
backward of reference train.py:173-181) vs the fp32 PyTorch weight gradient
of the same bf16 operands."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from raft_stir_amd.ops import _ext
    _ext.load(raise_on_error=True)
    return torch.device("cuda", 0)


def _ref(dy, x):
    """fp32 dW [Cout, Cin, 3, 3] from NHWC bf16 operands."""
    xf = x.float().permute(0, 3, 1, 2)
    df = dy.float().permute(0, 3, 1, 2)
    return torch.nn.grad.conv2d_weight(xf, (df.shape[1], xf.shape[1], 3, 3), df, padding=1)


@pytest.mark.parametrize("shape", [(2, 19, 45, 64, 64), (3, 13, 70, 128, 64), (1, 8, 32, 64, 128),
                                   (2, 46, 62, 128, 128), (1, 5, 7, 64, 64), (2, 23, 31, 96, 96),
                                   (1, 17, 40, 96, 64), (1, 9, 33, 64, 160)])
def test_enc_wgrad_vs_fp32(cuda, shape):
    B, H, W, cin, cout = shape
    torch.manual_seed(0)
    x = torch.randn(B, H, W, cin, device=cuda).to(torch.bfloat16)
    dy = torch.randn(B, H, W, cout, device=cuda).to(torch.bfloat16)
    got = torch.ops.raft_stir.enc_wgrad(dy, x)
    ref = _ref(dy, x)
    assert got.shape == (cout, cin, 3, 3) and got.dtype == torch.float32
    scale = ref.abs().max().item()
    torch.testing.assert_close(got, ref, atol=2e-4 * scale + 1e-3, rtol=1e-3)


def test_enc_wgrad_channel_strided_views_and_determinism(cuda):
    """Operands as channel windows of wider NHWC buffers (pixel stride > C)."""
    torch.manual_seed(1)
    B, H, W = 2, 24, 40
    xb = torch.randn(B, H, W, 96, device=cuda).to(torch.bfloat16)
    yb = torch.randn(B, H, W, 128, device=cuda).to(torch.bfloat16)
    x, dy = xb[..., 32:96], yb[..., 64:128]
    got = torch.ops.raft_stir.enc_wgrad(dy, x)
    torch.testing.assert_close(got, _ref(dy, x), atol=2e-4 * _ref(dy, x).abs().max().item() + 1e-3, rtol=1e-3)
    again = torch.ops.raft_stir.enc_wgrad(dy, x)
    assert torch.equal(got, again)  # fixed-order partial reduction


def test_encoder_conv_uses_enc_wgrad(cuda, monkeypatch):
    """The 64 / 128-channel stride-1 encoder convs take their weight gradient
    from enc_wgrad (bf16 training path), matching the module's fp32 gradient."""
    from raft_stir_amd.ops import enc_conv
    calls = []
    orig = torch.ops.raft_stir.enc_wgrad
    monkeypatch.setattr(enc_conv, "_enc_wgrad_op", lambda dy, x: calls.append(1) or orig(dy, x))
    torch.manual_seed(2)
    conv = torch.nn.Conv2d(64, 64, 3, padding=1).to(cuda)
    x = torch.randn(2, 64, 30, 44, device=cuda).to(memory_format=torch.channels_last)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = enc_conv.conv3x3(conv, x.to(torch.bfloat16))
    g = torch.randn_like(y.float())
    y.float().backward(g)
    assert calls, "enc_wgrad not used"
    xb = x.to(torch.bfloat16).float()
    ref = torch.nn.grad.conv2d_weight(xb, conv.weight.shape, g.to(torch.bfloat16).float(), padding=1)
    torch.testing.assert_close(conv.weight.grad, ref, atol=2e-4 * ref.abs().max().item() + 1e-3, rtol=1e-3)
