"""Narrow-channel encoder convs of RAFT-small on csrc/sconv.hip (reference
core/extractor.py:60-116 BottleneckBlock, :195-267 SmallEncoder) vs fp64
PyTorch, and the RAFT-small encoders / STIR tracker with and without them."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CL = torch.channels_last


@pytest.fixture(scope="module")
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from raft_stir_amd.ops import _ext
    _ext.load(raise_on_error=True)
    return torch.device("cuda", 0)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("k,s,cin,cout", [(1, 1, 32, 8), (3, 1, 8, 8), (1, 1, 8, 32), (1, 2, 32, 64), (3, 2, 16, 16),
                                          (3, 2, 24, 24), (1, 1, 96, 160), (3, 1, 24, 24), (1, 1, 64, 24)])
@pytest.mark.parametrize("epi", ["bias", "relu", "res"])
def test_sconv_vs_conv2d(cuda, dtype, k, s, cin, cout, epi):
    torch.manual_seed(k * 100 + s * 10 + cin + cout)
    B, H, W = 2, 21, 35
    x = torch.randn(B, H, W, cin, device=cuda).to(dtype)
    w = torch.randn(cout, cin, k, k, device=cuda) / (cin * k * k) ** 0.5
    b = torch.randn(cout, device=cuda)
    p = k // 2
    ref = F.conv2d(x.double().permute(0, 3, 1, 2), w.double(), b.double(), stride=s, padding=p)
    Ho, Wo = ref.shape[2:]
    res = None
    if epi in ("relu", "res"):
        ref = ref.relu()
    if epi == "res":
        res = torch.randn(B, Ho, Wo, cout, device=cuda).to(dtype)
        ref = (ref + res.double().permute(0, 3, 1, 2)).relu()
    out = torch.full((B, Ho, Wo, cout + 16), 7.0, device=cuda, dtype=dtype)
    torch.ops.raft_stir.sconv(x, w.permute(0, 2, 3, 1).contiguous(), b, s, p, epi != "bias", out, 8, res)
    got = out[..., 8:8 + cout].double().permute(0, 3, 1, 2)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    assert ((got - ref).norm() / ref.norm()).item() < tol
    assert (out[..., :8] == 7).all() and (out[..., 8 + cout:] == 7).all()


@pytest.mark.parametrize("norm_fn", ["instance", "none"])
@pytest.mark.parametrize("bf16", [True, False])
def test_small_encoder_sconv_matches_miopen(cuda, norm_fn, bf16):
    """Encoder output with the narrow convs on sconv vs on MIOpen, both
    against the fp32 MIOpen encoder: in fp32 they agree to ~1e-6; under bf16
    autocast sconv keeps fp32 weights (MIOpen gets bf16-cast ones), so it must
    be at least as close to fp32 as the MIOpen bf16 run."""
    from raft_stir_amd.models.extractor import SmallEncoder
    from raft_stir_amd.ops import enc_conv
    torch.manual_seed(5)
    enc = SmallEncoder(output_dim=128 if norm_fn == "instance" else 160, norm_fn=norm_fn).to(cuda)
    enc = enc.to(memory_format=CL).eval()
    x = (torch.rand(2, 3, 128, 160, device=cuda) * 2 - 1).contiguous(memory_format=CL)

    def run(on, amp):
        prev = enc_conv._SCONV
        enc_conv._SCONV = on
        try:
            with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
                return enc(x).float()
        finally:
            enc_conv._SCONV = prev
    ref = run(False, False)
    rel = lambda a: ((a - ref).norm() / ref.norm()).item()
    if bf16:
        e_s, e_m = rel(run(True, True)), rel(run(False, True))
        assert e_s <= 1.25 * e_m + 1e-3, (e_s, e_m)
    else:
        assert rel(run(True, False)) < 1e-4


def test_stir_tracker_uses_sconv(cuda, monkeypatch):
    from raft_stir_amd.config import make_args
    from raft_stir_amd.models import RAFT
    from raft_stir_amd.ops import enc_conv
    torch.manual_seed(0)
    m = RAFT(make_args(small=True, mixed_precision=True)).to(cuda).to(memory_format=CL).eval()
    n = []
    orig = enc_conv.sconv
    monkeypatch.setattr(enc_conv, "sconv", lambda *a, **k: n.append(1) or orig(*a, **k))
    i1 = torch.rand(1, 3, 128, 160, device=cuda) * 255
    i2 = torch.rand(1, 3, 128, 160, device=cuda) * 255
    with torch.no_grad():
        lo, up = m(i1, i2, iters=3, test_mode=True)
    # 2 encoders x 21 convs, less the projection and layer-3 shortcut of each
    # (>= 64 channels in and out: MFMA geometry path, ops/enc_conv.py _wide)
    assert len(n) >= 38 and torch.isfinite(up).all(), len(n)
