"""Weight-stationary update-block convolution (csrc/conv_ws.hip) vs plain
fp32 PyTorch on the same bf16 operands: every instantiated (taps, G), channel
slices and co-blocks per block, multi-segment inputs with channel offsets,
ragged strips (W % 16 != 0) and row chunks, the forward epilogues (bias /
ReLU / scale / GRU gates / GRU update) and the dgrad epilogues (fp32
accumulation, through-ReLU), and the auto-selected configuration.
Reference ops: /root/reference/core/update.py:6-136."""
import pytest
import torch
import torch.nn.functional as F

from raft_stir_amd.ops.conv import (EPI_ACC_F32, EPI_BIAS, EPI_GRU_Q, EPI_GRU_ZR, EPI_RELU, EPI_RELU_BWD,
                                    EPI_SCALE, WS_INST, WS_TILE, conv_fused, frag_layout, pack_bias, pack_weight,
                                    pad_to, ws_config, ws_geometry)

pytestmark = pytest.mark.gpu


def _bf(x):
    return x.to(torch.bfloat16).float()


def _cases():
    out = []
    for (kh, kw), gs in WS_INST["acc"].items():
        for G in gs:
            if ws_geometry(kh, kw, G) is not None:
                out.append((kh, kw, G, 4, 1))
    return out


CASES = _cases()


@pytest.mark.parametrize("kh,kw,G,ncs,ncb", CASES)
def test_conv_ws_vs_conv2d(cuda, kh, kw, G, ncs, ncb):
    torch.manual_seed(kh * 100 + kw * 10 + G + ncs * 7 + ncb)
    B, H, W = 2, 11, 19
    ktot = 16 * G * ncs
    # input = cat[a[..., 8:40] (32 ch of a 48-wide buffer), b (ktot - 32 ch)]
    a_buf = torch.randn(B, H, W, 48, device=cuda).to(torch.bfloat16)
    segs = [(a_buf, 8, 32)]
    xs = [a_buf[..., 8:40]]
    if ktot > 32:
        b_buf = torch.randn(B, H, W, ktot - 32, device=cuda).to(torch.bfloat16)
        segs.append((b_buf, 0, ktot - 32))
        xs.append(b_buf)
    x = torch.cat(xs, -1).float().permute(0, 3, 1, 2)
    plain = (kh, kw) in WS_INST["plain"]  # 1x5 / 5x1: the fp32-accumulating (dgrad) epilogue
    cout = 70 if plain else 72
    w = torch.randn(cout, ktot, kh, kw, device=cuda) * (0.5 / (ktot * kh * kw) ** 0.5)
    b = torch.randn(cout, device=cuda)
    wp = pack_weight(w, [(ktot, [(0, ktot, 0)])], pad_to(cout, 128))
    ref = F.conv2d(x, _bf(w), b[:cout] if plain else None, padding=(kh // 2, kw // 2))
    if plain:
        ref = ref.relu()
    for rpc in (4, 6, 64):
        if plain:
            out = torch.full((B, H, W, 80), 7.0, device=cuda, dtype=torch.bfloat16)
            conv_fused(segs, None, pack_bias(b), kh, kw, cout, EPI_RELU, out, 4, tile=WS_TILE, wf=frag_layout(wp),
                       ws_cfg=[G, 1, ncs, ncb, rpc])
        else:
            out = torch.full((B, H, W, 80), 7.0, device=cuda)
            conv_fused(segs, None, None, kh, kw, cout, EPI_ACC_F32, out, 4, tile=WS_TILE, wf=frag_layout(wp),
                       ws_cfg=[G, 1, ncs, ncb, rpc])
            out = out.clone()
            out[..., 4:4 + cout] -= 7.0
        got = out[..., 4:4 + cout].float().permute(0, 3, 1, 2)
        torch.testing.assert_close(got, ref, atol=3e-2, rtol=2e-2)
        assert (out[..., :4] == 7).all() and (out[..., 4 + cout:] == 7).all()


@pytest.mark.parametrize("epi", [EPI_BIAS, EPI_SCALE, EPI_ACC_F32, EPI_RELU_BWD])
@pytest.mark.parametrize("shape", [(1, 55, 136), (3, 46, 62)])
def test_conv_ws_epilogues_auto_config(cuda, epi, shape):
    """The auto-selected configuration at the bench shapes (3x3, 256 -> 192)."""
    torch.manual_seed(5)
    B, H, W = shape
    cin, cout = 256, 192
    x = torch.randn(B, H, W, cin, device=cuda).to(torch.bfloat16)
    w = torch.randn(cout, cin, 3, 3, device=cuda) * 0.03
    b = torch.randn(cout, device=cuda) if epi in (EPI_BIAS, EPI_SCALE) else None
    wp = pack_weight(w, [(cin, [(0, cin, 0)])], 256)
    assert ws_config(B, H, W, cout, cin, 3, 3, 256, epi) is not None
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), _bf(w), b, padding=1)
    aux = None
    if epi == EPI_ACC_F32:
        out = torch.randn(B, H, W, cout, device=cuda)
        ref = ref + out.permute(0, 3, 1, 2)
    else:
        out = torch.zeros(B, H, W, cout, device=cuda, dtype=torch.bfloat16)
    if epi == EPI_SCALE:
        ref = ref * 0.25
    if epi == EPI_RELU_BWD:
        aux = torch.randn(B, H, W, cout, device=cuda).to(torch.bfloat16)
        ref = ref * (aux.float().permute(0, 3, 1, 2) > 0)
    conv_fused([(x, 0, cin)], None, pack_bias(b) if b is not None else None, 3, 3, cout, epi, out, 0, scale=0.25,
               aux1=aux, tile=WS_TILE, wf=frag_layout(wp))
    torch.testing.assert_close(out.float().permute(0, 3, 1, 2), ref, atol=4e-2, rtol=2e-2)


@pytest.mark.parametrize("k", [(1, 5), (5, 1)])
def test_conv_ws_gru(cuda, k):
    """SepConvGRU pass at the real widths: z|r (384 -> 256, gate epilogue) and q
    (cat[r*h, x] -> 128, GRU update epilogue) on the weight-stationary kernel."""
    torch.manual_seed(1)
    B, H, W, hd = 2, 13, 21, 128
    kh, kw = k
    pad = (kh // 2, kw // 2)
    hx = (torch.randn(B, H, W, 3 * hd, device=cuda) * 0.5).to(torch.bfloat16)
    wz, wr, wq = (torch.randn(hd, 3 * hd, kh, kw, device=cuda) * 0.03 for _ in range(3))
    bz, br, bq = (torch.randn(hd, device=cuda) * 0.1 for _ in range(3))
    wzr = pack_weight(torch.cat([wz, wr]), [(3 * hd, [(0, 3 * hd, 0)])], 256)
    z = torch.empty(B, H, W, hd, device=cuda, dtype=torch.bfloat16)
    rh = torch.empty_like(z)
    conv_fused([(hx, 0, 3 * hd)], None, pack_bias(torch.cat([bz, br])), kh, kw, 2 * hd, EPI_GRU_ZR, z, 0,
               hd=hd, out2=rh, aux1=hx, a1off=0, tile=WS_TILE, wf=frag_layout(wzr))
    xin = hx.float().permute(0, 3, 1, 2)
    h = xin[:, :hd]
    z_ = torch.sigmoid(F.conv2d(xin, _bf(wz), bz, padding=pad))
    r_ = torch.sigmoid(F.conv2d(xin, _bf(wr), br, padding=pad))
    torch.testing.assert_close(z.float().permute(0, 3, 1, 2), z_, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(rh.float().permute(0, 3, 1, 2), r_ * h, atol=3e-2, rtol=3e-2)
    wqp = pack_weight(wq, [(hd, [(0, hd, 0)]), (2 * hd, [(hd, 2 * hd, 0)])], 128)
    hx2 = hx.clone()
    conv_fused([(rh, 0, hd), (hx2, hd, 2 * hd)], None, pack_bias(bq), kh, kw, hd, EPI_GRU_Q, hx2, 0,
               aux1=hx2, a1off=0, aux2=z, a2off=0, tile=WS_TILE, wf=frag_layout(wqp))
    qin = torch.cat([rh.float().permute(0, 3, 1, 2), xin[:, hd:]], 1)
    q = torch.tanh(F.conv2d(qin, _bf(wq), bq, padding=pad))
    zz = z.float().permute(0, 3, 1, 2)
    hn = (1 - zz) * h + zz * q
    torch.testing.assert_close(hx2[..., :hd].float().permute(0, 3, 1, 2), hn, atol=3e-2, rtol=3e-2)
    assert torch.equal(hx2[..., hd:], hx[..., hd:])
