"""csrc/conv_v3f.hip (tiles 81-83): the fp32 weight-streaming convs of the
fp32 engines (reference core/update.py:6-136 at fp32) -- split-bf16 products
(xh.wh + xl.wh + xh.wl) with fp32 activations split in registers -- against
the F32 register tile 7 (the same product, another accumulation order) for
every epilogue kind the fp32 engines run, and against an fp64 conv2d."""
import pytest
import torch
import torch.nn.functional as F

from raft_stir_amd.ops.conv import (EPI_ACC_F32, EPI_BIAS, EPI_GRU_Q, EPI_GRU_QBWD, EPI_GRU_ZR, EPI_RELU,
                                    EPI_RELU_BWD, EPI_SCALE, V3F_TILES, conv_fused, frag_weight_split,
                                    pack_bias, pack_weight_split, pad_to)

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("k", [(3, 3), (1, 5), (5, 1)])
@pytest.mark.parametrize("tile", [t for t in V3F_TILES if t != 85])  # (85: Ktot = 64 only, below)
@pytest.mark.parametrize("shape", [(2, 13, 37), (1, 9, 70)])
@pytest.mark.parametrize("cout", [160, 64])
def test_v3f_matches_fp64_conv(cuda, k, tile, shape, cout):
    torch.manual_seed(k[0] * 10 + tile)
    B, H, W = shape
    x0 = torch.randn(B, H, W, 128, device=cuda)
    x1 = torch.randn(B, H, W, 64, device=cuda)
    w = torch.randn(cout, 192, *k, device=cuda) * 0.05
    b = torch.randn(cout, device=cuda)
    ws = pack_weight_split(w, [(128, [(0, 128, 0)]), (64, [(128, 64, 0)])], pad_to(cout, 128))
    ws._rs_frag32 = frag_weight_split(ws)
    out = torch.full((B, H, W, cout + 8), 7.0, device=cuda)
    conv_fused([(x0, 0, 128), (x1, 0, 64)], ws, pack_bias(b), k[0], k[1], cout, EPI_BIAS, out, 4, tile=tile)
    xr = torch.cat([x0, x1], -1).permute(0, 3, 1, 2).double()
    ref = F.conv2d(xr, w.double(), b.double(), padding=(k[0] // 2, k[1] // 2)).permute(0, 2, 3, 1)
    got = out[..., 4:4 + cout].double()
    rel = ((got - ref).norm() / ref.norm()).item()
    assert rel < 2e-5, rel
    assert torch.equal(out[..., :4], torch.full_like(out[..., :4], 7.0))
    assert torch.equal(out[..., 4 + cout:], torch.full_like(out[..., 4 + cout:], 7.0))


@pytest.mark.parametrize("epi", [EPI_RELU, EPI_SCALE, EPI_GRU_ZR, EPI_GRU_Q, EPI_RELU_BWD, EPI_ACC_F32,
                                 EPI_GRU_QBWD])
def test_v3f_epilogues_match_f32_tile(cuda, epi):
    torch.manual_seed(6)
    B, H, W, hd = 2, 13, 37, 64
    segs = [torch.randn(B, H, W, 128, device=cuda) for _ in range(2)]
    cout = 2 * hd if epi == EPI_GRU_ZR else (hd if epi == EPI_GRU_Q else 192)
    w = torch.randn(cout, 256, 1, 5, device=cuda) * 0.05
    b = torch.randn(cout, device=cuda) * 0.1
    ws = pack_weight_split(w, [(128, [(0, 128, 0)]), (128, [(128, 128, 0)])], pad_to(cout, 128))
    ws._rs_frag32 = frag_weight_split(ws)
    aux1 = torch.rand(B, H, W, 256, device=cuda) - 0.3
    aux2 = torch.rand(B, H, W, 256, device=cuda)
    outs = []
    for tile in (7, 81):
        torch.manual_seed(7)
        out = torch.randn(B, H, W, 256, device=cuda)
        out2 = torch.zeros(B, H, W, 256, device=cuda)
        out3 = torch.zeros_like(out2)
        kw_ = dict(scale=0.25, tile=tile)
        if epi == EPI_GRU_ZR:
            kw_.update(hd=hd, out2=out2, out3=out3, aux1=aux1, a1off=8)
        elif epi == EPI_GRU_Q:
            kw_.update(out2=out2, aux1=aux1, a1off=0, aux2=aux2, a2off=64)
        elif epi == EPI_RELU_BWD:
            kw_.update(aux1=aux1, a1off=16)
        elif epi == EPI_GRU_QBWD:
            kw_.update(hd=hd, out2=out2, aux1=aux1, aux2=aux2)
        bias = None if epi in (EPI_RELU_BWD, EPI_ACC_F32, EPI_GRU_QBWD) else pack_bias(b)
        conv_fused([(s, 0, 128) for s in segs], ws, bias, 1, 5, cout, epi, out, 0, **kw_)
        outs.append((out, out2, out3))
    for x, y in zip(*outs):
        torch.testing.assert_close(y, x, atol=2e-5, rtol=1e-4)


@pytest.mark.parametrize("relu,use_res", [(False, False), (True, False), (True, True)])
def test_v3f_eval_bn_epilogue_matches_f32_tile(cuda, relu, use_res):
    """EPI_NORM (eval BatchNorm folded: acc * scale + shift, ReLU, + residual):
    the fp32 inference encoders' stride-1 3x3 convs."""
    from raft_stir_amd.ops.conv import EPI_NORM
    torch.manual_seed(3)
    B, H, W, cin, cout = 2, 21, 45, 64, 96
    x = torch.randn(B, H, W, cin, device=cuda)
    w = torch.randn(cout, cin, 3, 3, device=cuda) * 0.05
    ws = pack_weight_split(w, [(cin, [(0, cin, 0)])], pad_to(cout, 128))
    ws._rs_frag32 = frag_weight_split(ws)
    scale = torch.rand(cout, device=cuda) + 0.5
    shift = torch.randn(cout, device=cuda) * 0.1
    res = torch.randn(B, H, W, cout, device=cuda) if use_res else None
    outs = []
    for tile in (7, 81):
        out = torch.empty(B, H, W, cout, device=cuda)
        conv_fused([(x, 0, cin)], ws, shift, 3, 3, cout, EPI_NORM, out, 0, hd=int(relu), aux1=res, tile=tile,
                   nscale=scale)
        outs.append(out)
    torch.testing.assert_close(outs[1], outs[0], atol=2e-5, rtol=1e-4)


@pytest.mark.parametrize("k", [(3, 3), (1, 5), (5, 1)])
def test_v3f_single_buffer_tile(cuda, k):
    """Tile 85 (one halo buffer, Ktot = 64) against tile 84 and an fp64 conv."""
    torch.manual_seed(11)
    B, H, W, cin, cout = 2, 29, 70, 64, 64
    x = torch.randn(B, H, W, cin, device=cuda)
    w = torch.randn(cout, cin, *k, device=cuda) * 0.05
    ws = pack_weight_split(w, [(cin, [(0, cin, 0)])], pad_to(cout, 128))
    ws._rs_frag32 = frag_weight_split(ws)
    outs = []
    for tile in (84, 85):
        out = torch.empty(B, H, W, cout, device=cuda)
        conv_fused([(x, 0, cin)], ws, None, k[0], k[1], cout, EPI_BIAS, out, 0, tile=tile)
        outs.append(out)
    torch.testing.assert_close(outs[1], outs[0], atol=0, rtol=0)
    ref = F.conv2d(x.permute(0, 3, 1, 2).double(), w.double(), padding=(k[0] // 2, k[1] // 2)).permute(0, 2, 3, 1)
    assert ((outs[1].double() - ref).norm() / ref.norm()).item() < 2e-5
