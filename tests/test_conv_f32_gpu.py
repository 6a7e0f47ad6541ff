"""fp32 convolutions on the bf16 MFMAs by operand splitting (csrc/conv.hip
conv_lds_kernel<..., F32>, split [wh | wl] weights from ops/conv.py
split_weight): every forward epilogue, multi-segment inputs with channel
offsets, the three tile shapes and the strided geometry, vs float64 PyTorch
(the reference's default inference precision is fp32: evaluate.py:174).
Reference ops: /root/reference/core/update.py:6-136, core/extractor.py:6-56."""
import pytest
import torch
import torch.nn.functional as F

from raft_stir_amd.ops.conv import (EPI_BIAS, EPI_GRU_Q, EPI_GRU_ZR, EPI_NORM, EPI_RELU, EPI_SCALE, conv_fused,
                                    pack_bias, pack_weight_split, pad_to)

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("tile", [6, 7, 8, 38, 39, 40])
@pytest.mark.parametrize("k", [(3, 3), (1, 5), (5, 1), (1, 1)])
@pytest.mark.parametrize("epi", [EPI_BIAS, EPI_RELU, EPI_SCALE])
def test_conv_f32_plain(cuda, tile, k, epi):
    torch.manual_seed(tile * 10 + k[0] + epi)
    kh, kw = k
    B, H, W = 2, 13, 27
    a = torch.randn(B, H, W, 96, device=cuda)       # segment 1: channels [32:96) of a 96-wide buffer
    b = torch.randn(B, H, W, 64, device=cuda)       # segment 2
    x = torch.cat([a[..., 32:96], b], -1)
    cout = 72
    w = torch.randn(cout, 128, kh, kw, device=cuda) * (1.0 / (128 * kh * kw) ** 0.5)
    bias = torch.randn(cout, device=cuda)
    wp = pack_weight_split(w, [(64, [(0, 64, 0)]), (64, [(64, 64, 0)])], pad_to(cout, 128))
    out = torch.full((B, H, W, 80), 7.0, device=cuda)
    conv_fused([(a, 32, 64), (b, 0, 64)], wp, pack_bias(bias), kh, kw, cout, epi, out, 4, scale=0.25, tile=tile)
    ref = F.conv2d(x.double().permute(0, 3, 1, 2), w.double(), bias.double(), padding=(kh // 2, kw // 2))
    if epi == EPI_RELU:
        ref = ref.relu()
    if epi == EPI_SCALE:
        ref = ref * 0.25
    got = out[..., 4:4 + cout].permute(0, 3, 1, 2)
    assert _rel(got, ref) < 2e-5, _rel(got, ref)
    assert (out[..., :4] == 7).all() and (out[..., 4 + cout:] == 7).all()


@pytest.mark.parametrize("k", [(1, 5), (3, 3)])
def test_conv_f32_gru(cuda, k):
    """z|r and q convs of one (Sep)ConvGRU pass in fp32 with the gate / update epilogues."""
    torch.manual_seed(3)
    kh, kw = k
    pad = (kh // 2, kw // 2)
    B, H, W, hd = 2, 11, 23, 128
    hx = torch.randn(B, H, W, 3 * hd, device=cuda) * 0.5
    wz, wr, wq = (torch.randn(hd, 3 * hd, kh, kw, device=cuda) * 0.03 for _ in range(3))
    bz, br, bq = (torch.randn(hd, device=cuda) * 0.1 for _ in range(3))
    wzr = pack_weight_split(torch.cat([wz, wr]), [(3 * hd, [(0, 3 * hd, 0)])], 256)
    z = torch.empty(B, H, W, hd, device=cuda)
    rh = torch.empty_like(z)
    conv_fused([(hx, 0, 3 * hd)], wzr, pack_bias(torch.cat([bz, br])), kh, kw, 2 * hd, EPI_GRU_ZR, z, 0,
               hd=hd, out2=rh, aux1=hx, a1off=0, tile=7)
    xin = hx.double().permute(0, 3, 1, 2)
    h = xin[:, :hd]
    z_ = torch.sigmoid(F.conv2d(xin, wz.double(), bz.double(), padding=pad))
    r_ = torch.sigmoid(F.conv2d(xin, wr.double(), br.double(), padding=pad))
    assert _rel(z.permute(0, 3, 1, 2), z_) < 2e-5
    assert _rel(rh.permute(0, 3, 1, 2), r_ * h) < 2e-5
    wqp = pack_weight_split(wq, [(hd, [(0, hd, 0)]), (2 * hd, [(hd, 2 * hd, 0)])], 128)
    hx2 = hx.clone()
    conv_fused([(rh, 0, hd), (hx2, hd, 2 * hd)], wqp, pack_bias(bq), kh, kw, hd, EPI_GRU_Q, hx2, 0,
               aux1=hx2, a1off=0, aux2=z, a2off=0, tile=6)
    qin = torch.cat([rh.double().permute(0, 3, 1, 2), xin[:, hd:]], 1)
    q = torch.tanh(F.conv2d(qin, wq.double(), bq.double(), padding=pad))
    zz = z.double().permute(0, 3, 1, 2)
    hn = (1 - zz) * h + zz * q
    assert _rel(hx2[..., :hd].permute(0, 3, 1, 2), hn) < 2e-5
    assert torch.equal(hx2[..., hd:], hx[..., hd:])


@pytest.mark.parametrize("residual", [False, True])
def test_conv_f32_norm_epilogue(cuda, residual):
    torch.manual_seed(4)
    B, H, W, cin, cout = 2, 17, 30, 128, 128
    x = torch.randn(B, H, W, cin, device=cuda)
    w = torch.randn(cout, cin, 3, 3, device=cuda) * 0.03
    sc = torch.rand(cout, device=cuda) + 0.5
    sh = torch.randn(cout, device=cuda) * 0.2
    res = torch.randn(B, H, W, cout, device=cuda) if residual else None
    out = torch.empty(B, H, W, cout, device=cuda)
    conv_fused([(x, 0, cin)], pack_weight_split(w, [(cin, [(0, cin, 0)])], 128), sh, 3, 3, cout, EPI_NORM, out, 0,
               hd=1, aux1=res, tile=7, nscale=sc)
    ref = F.conv2d(x.double().permute(0, 3, 1, 2), w.double(), padding=1)
    ref = (ref * sc.double().view(1, -1, 1, 1) + sh.double().view(1, -1, 1, 1)).relu()
    if residual:
        ref = (ref + res.double().permute(0, 3, 1, 2)).relu()
    assert _rel(out.permute(0, 3, 1, 2), ref) < 2e-5


@pytest.mark.parametrize("k,s", [(3, 2), (1, 2), (1, 1)])
def test_conv_geo_f32(cuda, k, s):
    torch.manual_seed(k + s)
    B, H, W, cin, cout = 2, 25, 38, 64, 96
    x = torch.randn(B, H, W, cin, device=cuda)
    w = torch.randn(cout, cin, k, k, device=cuda) * 0.05
    bias = torch.randn(cout, device=cuda)
    p = k // 2
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    out = torch.empty(B, Ho, Wo, cout, device=cuda)
    wp = pack_weight_split(w, [(cin, [(0, cin, 0)])], 128)
    torch.ops.raft_stir.conv_geo([x], [0], [cin], wp, bias, k, k, p, p, s, s, Ho, Wo, cout, out, 0, 1, 1, 0, 0, 7)
    ref = F.conv2d(x.double().permute(0, 3, 1, 2), w.double(), bias.double(), stride=s, padding=p)
    assert _rel(out.permute(0, 3, 1, 2), ref) < 2e-5
