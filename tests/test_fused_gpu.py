"""Fused update-block convolution (csrc/conv.hip) and the fused inference
engine (models/fused_update.py) vs plain fp32 PyTorch."""
import copy

import pytest
import torch
import torch.nn.functional as F

from raft_stir_amd.config import make_args
from raft_stir_amd.models import RAFT
from raft_stir_amd.ops.conv import (EPI_ACC_F32, EPI_BIAS, EPI_FLOW, EPI_GRU_Q, EPI_GRU_QBWD, EPI_GRU_ZR,
                                    EPI_RELU, EPI_RELU_BWD, EPI_SCALE, GEMM1_TILE, V3_TILES, conv_fused, frag_weight,
                                    pack_bias, pack_weight, pad_to)

pytestmark = pytest.mark.gpu


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def _bf(x):
    return x.to(torch.bfloat16).float()


@pytest.mark.parametrize("k", [(1, 1), (3, 3), (1, 5), (5, 1)])
@pytest.mark.parametrize("tile", [0, 1, 2, 3, 4, 6, 7, 11, 15, 16, 17, 18, 19, 20, 21, 23, 24, 25, 26,
                                  27, 28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 41])
@pytest.mark.parametrize("epi", [EPI_BIAS, EPI_RELU, EPI_SCALE])
def test_conv_segments_vs_conv2d(cuda, k, tile, epi):
    torch.manual_seed(0)
    B, H, W = 2, 11, 19
    kh, kw = k
    # input = cat[a (40 ch, stored in a 64-wide buffer at offset 8), b (32 ch)]
    cb = 64 if tile >= 6 else 32   # 64-deep K tiles need 64-channel segments
    a_buf = torch.randn(B, H, W, 64, device=cuda).to(torch.bfloat16)
    b_buf = torch.randn(B, H, W, cb, device=cuda).to(torch.bfloat16)
    x = torch.cat([a_buf[..., 8:48], b_buf], -1).float().permute(0, 3, 1, 2)
    cout = 70
    w = torch.randn(cout, 40 + cb, kh, kw, device=cuda) * 0.1
    b = torch.randn(cout, device=cuda)
    # segment 0 reads 64 channels from a_buf at offset 0: weights for [8,48) only
    wp = pack_weight(w, [(64, [(0, 40, 8)]), (cb, [(40, cb, 0)])], pad_to(cout, 256))
    out = torch.full((B, H, W, 80), 7.0, device=cuda, dtype=torch.bfloat16)
    conv_fused([(a_buf, 0, 64), (b_buf, 0, cb)], wp, pack_bias(b), kh, kw, cout, epi, out, 4,
               scale=0.25, tile=tile)
    ref = F.conv2d(x, _bf(w), b, padding=(kh // 2, kw // 2))
    if epi == EPI_RELU:
        ref = ref.relu()
    if epi == EPI_SCALE:
        ref = ref * 0.25
    got = out[..., 4:4 + cout].float().permute(0, 3, 1, 2)
    torch.testing.assert_close(got, ref, atol=3e-2, rtol=2e-2)
    assert (out[..., :4] == 7).all() and (out[..., 4 + cout:] == 7).all()  # no writes outside the window


@pytest.mark.parametrize("k", [(3, 3), (1, 5), (5, 1)])
@pytest.mark.parametrize("tile", list(range(42, 55)))
@pytest.mark.parametrize("shape", [(2, 11, 19), (1, 9, 70)])
def test_conv_v2_tiles_vs_conv2d(cuda, k, tile, shape):
    """csrc/conv_v2.hip (unrolled taps, 32x32x16 MFMAs, halo per 64-channel
    chunk): every tile 42-54 -- 4-, 6- and 8-wave blocks, one or two A fragments
    per wave, 2- to 6-slot weight rings -- on partial patches in both
    directions, three input segments (two 64-channel, one 128), Cout not a
    multiple of the block's."""
    torch.manual_seed(3)
    B, H, W = shape
    kh, kw = k
    segs = [torch.randn(B, H, W, c, device=cuda).to(torch.bfloat16) for c in (64, 64, 128)]
    cin = 64 + 64 + 128
    cout = 200
    w = torch.randn(cout, cin, kh, kw, device=cuda) * 0.05
    b = torch.randn(cout, device=cuda)
    wp = pack_weight(w, [(64, [(0, 64, 0)]), (64, [(64, 64, 0)]), (128, [(128, 128, 0)])],
                     pad_to(cout, 192 if tile == 54 else 256))
    out = torch.full((B, H, W, cout + 8), 7.0, device=cuda, dtype=torch.bfloat16)
    conv_fused([(s, 0, s.shape[-1]) for s in segs], wp, pack_bias(b), kh, kw, cout, EPI_RELU, out, 0, tile=tile)
    x = torch.cat(segs, -1).float().permute(0, 3, 1, 2)
    ref = F.conv2d(x, _bf(w), b, padding=(kh // 2, kw // 2)).relu()
    got = out[..., :cout].float().permute(0, 3, 1, 2)
    torch.testing.assert_close(got, ref, atol=3e-2, rtol=2e-2)
    assert (out[..., cout:] == 7).all()


@pytest.mark.parametrize("k", [(3, 3), (1, 5), (5, 1)])
@pytest.mark.parametrize("tile", list(V3_TILES))
@pytest.mark.parametrize("shape", [(2, 11, 19), (1, 9, 70), (1, 14, 33)])
def test_conv_v3_tiles_vs_conv2d(cuda, k, tile, shape):
    """csrc/conv_v3.h (weight-streaming tiles: per-wave A fragments global ->
    VGPR from the fragment-major layout, halo per 64-channel chunk in LDS, one
    barrier per chunk): every tile on partial patches in both
    directions, three input segments (4 chunks: the halo double buffer flips
    an even and an odd number of times), Cout not a multiple of the block's
    (the row blocks past the packed weight read as zeros)."""
    torch.manual_seed(5)
    B, H, W = shape
    kh, kw = k
    chans = (64, 64, 128) if H != 14 else (64, 128, 128)  # 4 / 5 chunks
    segs = [torch.randn(B, H, W, c, device=cuda).to(torch.bfloat16) for c in chans]
    cin = sum(chans)
    cout = 200
    w = torch.randn(cout, cin, kh, kw, device=cuda) * 0.05
    b = torch.randn(cout, device=cuda)
    pieces, o = [], 0
    for c in chans:
        pieces.append((c, [(o, c, 0)]))
        o += c
    wp = pack_weight(w, pieces, pad_to(cout, 32))
    out = torch.full((B, H, W, cout + 8), 7.0, device=cuda, dtype=torch.bfloat16)
    conv_fused([(s, 0, s.shape[-1]) for s in segs], wp, pack_bias(b), kh, kw, cout, EPI_RELU, out, 0, tile=tile,
               wf=frag_weight(wp))
    x = torch.cat(segs, -1).float().permute(0, 3, 1, 2)
    ref = F.conv2d(x, _bf(w), b, padding=(kh // 2, kw // 2)).relu()
    got = out[..., :cout].float().permute(0, 3, 1, 2)
    torch.testing.assert_close(got, ref, atol=3e-2, rtol=2e-2)
    assert (out[..., cout:] == 7).all()


@pytest.mark.parametrize("tile", list(V3_TILES))
def test_conv_v3_tiles_segment_offsets(cuda, tile):
    """The v3 tiles on segment windows that start inside their tensors, the
    layout of RAFT-small's padded GRU-q conv (models/fused_update.py: r*h in
    a 128-channel buffer, x read as hx[64:256] of a 256-channel buffer with
    zero weights on the pad): nonzero offsets and strides wider than the
    window, vs F.conv2d on the same windows."""
    torch.manual_seed(6)
    B, H, W = 1, 13, 45
    rh = torch.randn(B, H, W, 128, device=cuda).to(torch.bfloat16)
    hx = torch.randn(B, H, W, 256, device=cuda).to(torch.bfloat16)
    segs = [(rh, 0, 128), (hx, 64, 192)]
    cin, cout = 128 + 192, 96
    for kh, kw in ((1, 5), (5, 1), (3, 3)):
        w = torch.randn(cout, cin, kh, kw, device=cuda) * 0.05
        w[:, 96:128] = 0  # the zero-weight pad channels of the small engine's r*h buffer
        b = torch.randn(cout, device=cuda)
        wp = pack_weight(w, [(128, [(0, 128, 0)]), (192, [(128, 192, 0)])], pad_to(cout, 32))
        out = torch.zeros(B, H, W, cout, device=cuda, dtype=torch.bfloat16)
        conv_fused(segs, wp, pack_bias(b), kh, kw, cout, EPI_SCALE, out, 0, scale=0.5, tile=tile, wf=frag_weight(wp))
        x = torch.cat([rh, hx[..., 64:]], -1).float().permute(0, 3, 1, 2)
        ref = F.conv2d(x, _bf(w), b, padding=(kh // 2, kw // 2)) * 0.5
        torch.testing.assert_close(out.float().permute(0, 3, 1, 2), ref, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("cout", [256, 576, 70])
@pytest.mark.parametrize("epi", [EPI_BIAS, EPI_RELU, EPI_SCALE, EPI_RELU_BWD, EPI_ACC_F32])
@pytest.mark.parametrize("shape", [(2, 11, 19), (1, 9, 70), (8, 46, 62)])
@pytest.mark.parametrize("ooff", [0, 8])
def test_conv1x1_gemm_vs_conv2d(cuda, cout, epi, shape, ooff):
    """csrc/conv_gemm1.hip (tile 70): two input segments read from windows of
    wider buffers, pixel counts that are not a multiple of the 128-pixel tile,
    Cout a multiple of 32 (batched epilogue) or not (element-wise epilogue),
    the epilogue kinds the update block's 1x1 convs use (bias / ReLU / scale /
    ReLU backward through the LDS-staged row stores when the output rows are
    16-B aligned); channels outside the output window untouched."""
    torch.manual_seed(9)
    B, H, W = shape
    a_buf = torch.randn(B, H, W, 192, device=cuda).to(torch.bfloat16)
    b_buf = torch.randn(B, H, W, 256, device=cuda).to(torch.bfloat16)
    x = torch.cat([a_buf[..., 64:192], b_buf], -1).float().permute(0, 3, 1, 2)
    w = torch.randn(cout, 384, 1, 1, device=cuda) * 0.05
    b = torch.randn(cout, device=cuda)
    wp = pack_weight(w, [(128, [(0, 128, 0)]), (256, [(128, 256, 0)])], pad_to(cout, 128))
    f32out = epi == EPI_ACC_F32
    out0 = torch.randn(B, H, W, cout + 16, device=cuda)
    out0 = out0 if f32out else out0.to(torch.bfloat16)
    out = out0.clone()
    aux = torch.randn(B, H, W, cout, device=cuda).to(torch.bfloat16)
    kw_ = dict(scale=0.25, tile=GEMM1_TILE)
    if epi == EPI_RELU_BWD:
        kw_.update(aux1=aux, a1off=0)
    bias = None if epi in (EPI_RELU_BWD, EPI_ACC_F32) else pack_bias(b)
    conv_fused([(a_buf, 64, 128), (b_buf, 0, 256)], wp, bias, 1, 1, cout, epi, out, ooff, **kw_)
    ref = F.conv2d(x, _bf(w), None if bias is None else b)
    if epi == EPI_RELU:
        ref = ref.relu()
    elif epi == EPI_SCALE:
        ref = ref * 0.25
    elif epi == EPI_RELU_BWD:
        ref = ref * (aux.float().permute(0, 3, 1, 2) > 0)
    elif epi == EPI_ACC_F32:
        ref = ref + out0[..., ooff:ooff + cout].permute(0, 3, 1, 2)
    got = out[..., ooff:ooff + cout].float().permute(0, 3, 1, 2)
    torch.testing.assert_close(got, ref, atol=3e-2, rtol=2e-2)
    assert torch.equal(out[..., :ooff], out0[..., :ooff])
    assert torch.equal(out[..., ooff + cout:], out0[..., ooff + cout:])


@pytest.mark.parametrize("epi", [EPI_GRU_ZR, EPI_GRU_Q, EPI_RELU_BWD, EPI_ACC_F32, EPI_GRU_QBWD, EPI_SCALE])
def test_conv_v3_epilogues_match_v2(cuda, epi):
    """Every epilogue kind the training step runs on the update-block convs:
    tile 61 (fragment-major weights) against tile 52 (conv_v2, the standard
    layout) on the same inputs -- same fused epilogue code, different K
    accumulation order."""
    torch.manual_seed(6)
    B, H, W, hd = 2, 13, 37, 64
    segs = [torch.randn(B, H, W, 128, device=cuda).to(torch.bfloat16) for _ in range(2)]
    cout = 2 * hd if epi == EPI_GRU_ZR else (hd if epi == EPI_GRU_Q else 192)
    w = torch.randn(cout, 256, 1, 5, device=cuda) * 0.05
    b = torch.randn(cout, device=cuda) * 0.1
    wp = pack_weight(w, [(128, [(0, 128, 0)]), (128, [(128, 128, 0)])], pad_to(cout, 256))
    wf = frag_weight(wp)
    aux1 = torch.rand(B, H, W, 256, device=cuda).to(torch.bfloat16) - 0.3
    aux2 = torch.rand(B, H, W, 256, device=cuda).to(torch.bfloat16)
    f32out = epi in (EPI_ACC_F32, EPI_GRU_QBWD)
    outs = []
    for tile in (52, 61):
        torch.manual_seed(7)
        out = torch.randn(B, H, W, 256, device=cuda)
        out = out if f32out else out.to(torch.bfloat16)
        out2 = torch.zeros(B, H, W, 256, device=cuda, dtype=torch.bfloat16)
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
        conv_fused([(s, 0, 128) for s in segs], wp, bias, 1, 5, cout, epi, out, 0, wf=wf, **kw_)
        outs.append((out.float(), out2.float(), out3.float()))
    for x, y in zip(*outs):
        torch.testing.assert_close(y, x, atol=2e-2, rtol=2e-2)


def test_gru_epilogues(cuda):
    torch.manual_seed(1)
    B, H, W, hd = 1, 9, 13, 64
    hx = torch.randn(B, H, W, 3 * hd, device=cuda).to(torch.bfloat16)   # [h | x(2hd)]
    wz = torch.randn(hd, 3 * hd, 1, 5, device=cuda) * 0.05
    wr = torch.randn(hd, 3 * hd, 1, 5, device=cuda) * 0.05
    wq = torch.randn(hd, 3 * hd, 1, 5, device=cuda) * 0.05
    bz, br, bq = (torch.randn(hd, device=cuda) * 0.1 for _ in range(3))
    wzr = pack_weight(torch.cat([wz, wr]), [(3 * hd, [(0, 3 * hd, 0)])], 128)
    z = torch.empty(B, H, W, hd, device=cuda, dtype=torch.bfloat16)
    rh = torch.empty_like(z)
    rs = torch.empty_like(z)
    conv_fused([(hx, 0, 3 * hd)], wzr, pack_bias(torch.cat([bz, br])), 1, 5, 2 * hd, EPI_GRU_ZR, z, 0,
               hd=hd, out2=rh, out3=rs, aux1=hx, a1off=0)
    xin = hx.float().permute(0, 3, 1, 2)
    h = xin[:, :hd]
    zr_ = torch.sigmoid(F.conv2d(xin, _bf(wz), bz, padding=(0, 2)))
    r_ = torch.sigmoid(F.conv2d(xin, _bf(wr), br, padding=(0, 2)))
    torch.testing.assert_close(z.float().permute(0, 3, 1, 2), zr_, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(rs.float().permute(0, 3, 1, 2), r_, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(rh.float().permute(0, 3, 1, 2), r_ * h, atol=3e-2, rtol=3e-2)
    wqp = pack_weight(wq, [(hd, [(0, hd, 0)]), (2 * hd, [(hd, 2 * hd, 0)])], 128)
    hx2 = hx.clone()
    conv_fused([(rh, 0, hd), (hx2, hd, 2 * hd)], wqp, pack_bias(bq), 1, 5, hd, EPI_GRU_Q, hx2, 0,
               aux1=hx2, a1off=0, aux2=z, a2off=0)
    qin = torch.cat([rh.float().permute(0, 3, 1, 2), xin[:, hd:]], 1)
    q = torch.tanh(F.conv2d(qin, _bf(wq), bq, padding=(0, 2)))
    zz = z.float().permute(0, 3, 1, 2)
    hn = (1 - zz) * h + zz * q
    torch.testing.assert_close(hx2[..., :hd].float().permute(0, 3, 1, 2), hn, atol=3e-2, rtol=3e-2)
    assert torch.equal(hx2[..., hd:], hx[..., hd:])


def test_flow_epilogue_and_flow_encode(cuda):
    torch.manual_seed(2)
    B, H, W = 2, 10, 12
    feat = torch.randn(B, H, W, 64, device=cuda).to(torch.bfloat16)
    w = torch.randn(2, 64, 3, 3, device=cuda) * 0.1
    b = torch.randn(2, device=cuda)
    coords = torch.randn(B, 2, H, W, device=cuda) * 3
    c0 = coords.clone()
    c1 = coords.clone()
    conv_fused([(feat, 0, 64)], pack_weight(w, [(64, [(0, 64, 0)])], 128), pack_bias(b), 3, 3, 2, EPI_FLOW,
               coords)
    conv_fused([(feat, 0, 64)], pack_weight(w, [(64, [(0, 64, 0)])], 128), pack_bias(b), 3, 3, 2, EPI_FLOW,
               c1, tile=5)  # split-K small-N kernel
    torch.testing.assert_close(c1, coords, atol=1e-3, rtol=1e-3)
    delta = F.conv2d(feat.float().permute(0, 3, 1, 2), _bf(w), b, padding=1)
    torch.testing.assert_close(coords, c0 + delta, atol=2e-2, rtol=2e-2)
    # flow encoder: relu(conv7x7(coords - grid)) and the flow itself into a slot
    from raft_stir_amd.ops.reference import coords_grid
    grid = coords_grid(B, H, W, device=cuda)
    crd = grid + torch.randn(B, 2, H, W, device=cuda) * 4
    wf = torch.randn(128, 2, 7, 7, device=cuda) * 0.1
    bf = torch.randn(128, device=cuda)
    out = torch.zeros(B, H, W, 128, device=cuda, dtype=torch.bfloat16)
    slot = torch.zeros(B, H, W, 8, device=cuda, dtype=torch.bfloat16)
    torch.ops.raft_stir.flow_encode(crd, wf.permute(2, 3, 1, 0).contiguous(), bf, out, 0, slot, 6)
    ref = F.conv2d(crd - grid, wf, bf, padding=3).relu()
    torch.testing.assert_close(out.float().permute(0, 3, 1, 2), ref, atol=5e-2, rtol=2e-2)
    torch.testing.assert_close(slot[..., 6:8].float().permute(0, 3, 1, 2), crd - grid, atol=5e-2, rtol=1e-2)


@pytest.mark.parametrize("small,alt", [(False, False), (True, False), (False, True)])
def test_fused_inference_matches_unfused(cuda, small, alt):
    """Fused engine vs the module graph (same bf16 autocast), and vs fp32."""
    from raft_stir_amd.data.synthetic import make_batch
    torch.manual_seed(0)
    m = RAFT(make_args(small=small, mixed_precision=True, alternate_corr=alt)).to(cuda)
    m = m.to(memory_format=torch.channels_last).eval()
    unf = copy.deepcopy(m)
    unf.set_fused_gru(False)
    unf.cfg = unf.cfg.__class__(**{**unf.cfg.to_dict(), "fused_gru": False})
    f32 = copy.deepcopy(m)
    f32.cfg = f32.cfg.__class__(**{**f32.cfg.to_dict(), "mixed_precision": False})
    i1, i2, _, _ = make_batch(1, 256, 320, seed=1, device=cuda)
    with torch.no_grad():
        lo_f, up_f = m(i1, i2, iters=12, test_mode=True)
        lo_u, up_u = unf(i1, i2, iters=12, test_mode=True)
        lo_r, up_r = f32(i1, i2, iters=12, test_mode=True)
        preds = m(i1, i2, iters=3, test_mode=False)
    assert len(preds) == 3 and preds[-1].shape == up_f.shape
    err_fused = (up_f - up_r).norm(dim=1).mean().item()
    err_unfused = (up_u - up_r).norm(dim=1).mean().item()
    # the fused engine must be as close to fp32 as the bf16 module graph is
    assert err_fused < 1.5 * err_unfused + 2e-2, (err_fused, err_unfused)
    assert torch.isfinite(up_f).all()


def test_fused_graph_replay(cuda):
    from raft_stir_amd.runtime.graph import GraphedInference
    torch.manual_seed(0)
    m = RAFT(make_args(mixed_precision=True)).to(cuda).to(memory_format=torch.channels_last).eval()
    g = torch.Generator().manual_seed(3)
    i1 = (torch.rand(1, 3, 128, 256, generator=g) * 255).to(cuda)
    i2 = (torch.rand(1, 3, 128, 256, generator=g) * 255).to(cuda)
    with torch.no_grad():
        _, up = m(i1, i2, iters=8, test_mode=True)
    gi = GraphedInference(m, i1.shape, iters=8)
    _, up2 = gi(i1, i2)
    torch.testing.assert_close(up2, up, atol=3e-2, rtol=3e-2)  # MIOpen may pick other algos under capture
    _, up3 = gi(i2, i1)
    with torch.no_grad():
        _, upe = m(i2, i1, iters=8, test_mode=True)
    torch.testing.assert_close(up3, upe, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("cin", [128, 256])
def test_flow_head_fwd_dgrad(cuda, cin):
    """csrc/flowhead.hip: 3x3 Cin->2 conv with the coords epilogue, and its input
    gradient through the hidden ReLU, vs fp32 PyTorch on the same bf16 operands."""
    torch.manual_seed(0)
    B, H, W = 2, 13, 21  # W not a multiple of the 8-pixel wave strip
    act = torch.relu(torch.randn(B, H, W, cin + 64, device=cuda)).to(torch.bfloat16)
    w = torch.randn(2, cin, 3, 3, device=cuda) * 0.05
    b = torch.randn(2, device=cuda)
    w32 = w.permute(0, 2, 3, 1).contiguous()
    src = torch.randn(B, 2, H, W, device=cuda) * 10
    crd = torch.empty_like(src)
    torch.ops.raft_stir.flow_head(act, 64, cin, w32, b, crd, src)
    x = act[..., 64:].float().permute(0, 3, 1, 2)
    ref = src + torch.nn.functional.conv2d(x, w, b, padding=1)
    torch.testing.assert_close(crd, ref, atol=2e-3, rtol=1e-4)
    crd2 = src.clone()  # in place (src aliases crd)
    torch.ops.raft_stir.flow_head(act, 64, cin, w32, b, crd2, None)
    torch.testing.assert_close(crd2, ref, atol=2e-3, rtol=1e-4)
    # dgrad through the ReLU of the hidden state
    dflow = torch.randn(B, 2, H, W, device=cuda)
    out = torch.zeros(B, H, W, cin + 32, device=cuda, dtype=torch.bfloat16)
    torch.ops.raft_stir.flow_head_dgrad(dflow, w32, cin, act, 64, out, 32)
    xr = x.clone().requires_grad_(True)
    torch.nn.functional.conv2d(xr, w, b, padding=1).backward(dflow)
    dref = (xr.grad * (x > 0)).permute(0, 2, 3, 1)
    torch.testing.assert_close(out[..., 32:].float(), dref, atol=2e-2, rtol=1e-2)
    assert out[..., :32].abs().max().item() == 0
