"""HIP kernel numerics vs the plain-PyTorch fp32 references (ops/reference.py).

Odd sizes on purpose (h % 4, w % 8 != 0; pooled levels with floor sizes), both
radii (3: RAFT-small, 4: RAFT), both channel counts (128, 256), B > 1.
"""
import math

import pytest
import torch
import torch.nn.functional as F

from raft_stir_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _fmaps(B, C, H, W, dev, dtype=torch.float32, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    f1 = torch.randn(B, C, H, W, generator=g)
    f2 = torch.randn(B, C, H, W, generator=g)
    return f1.to(dev, dtype), f2.to(dev, dtype)


def _coords(B, H, W, dev, spread=6.0, seed=1):
    g = torch.Generator(device="cpu").manual_seed(seed)
    base = ref.coords_grid(B, H, W)
    return (base + spread * torch.randn(B, 2, H, W, generator=g)).to(dev)


@pytest.mark.parametrize("C", [128, 256])
@pytest.mark.parametrize("HW", [(11, 37), (46, 62), (8, 8)])
@pytest.mark.parametrize("bf16", [False, True])
def test_corr_volume_pyramid(cuda, C, HW, bf16):
    H, W = HW
    B = 2
    dt = torch.bfloat16 if bf16 else torch.float32
    f1, f2 = _fmaps(B, C, H, W, cuda, dt)
    levels = 4 if min(H, W) >= 8 else 3
    pyr = torch.ops.raft_stir.corr_volume(
        f1.permute(0, 2, 3, 1).reshape(B, H * W, C).contiguous(),
        f2.permute(0, 2, 3, 1).contiguous(), levels, 1.0 / math.sqrt(C))
    want = ref.corr_pyramid(f1.float(), f2.float(), levels)
    for l in range(levels):
        got = pyr[l].reshape(want[l].shape)
        # bf16: levels >= 1 are f1 . avgpool^l(f2) with the pooled f2 rounded to bf16
        # once (flat path), ~2^-9 of a pooled feature per channel
        tol = (2e-3 if l == 0 else 6e-3) if bf16 else 1e-4
        torch.testing.assert_close(got, want[l], atol=tol, rtol=tol)


@pytest.mark.parametrize("HW", [(11, 37), (46, 62), (55, 136)])
@pytest.mark.parametrize("out_bf16", [False, True])
def test_corr_volume_flat_storage_and_pitch(cuda, HW, out_bf16):
    """bf16 feature maps take the flat grouped-GEMM path (pooled f2, 128-B
    aligned padded rows); the pyramid is stored in fp32 or bf16."""
    H, W = HW
    B, C = 2, 256
    f1, f2 = _fmaps(B, C, H, W, cuda, torch.bfloat16, seed=4)
    pyr = torch.ops.raft_stir.corr_volume(
        f1.permute(0, 2, 3, 1).reshape(B, H * W, C).contiguous(),
        f2.permute(0, 2, 3, 1).contiguous(), 4, 1.0 / math.sqrt(C), out_bf16)
    want = ref.corr_pyramid(f1.float(), f2.float(), 4)
    for l in range(4):
        hl, wl = H >> l, W >> l
        assert pyr[l].shape == (B, H * W, hl, wl)
        assert pyr[l].dtype == (torch.bfloat16 if out_bf16 else torch.float32)
        assert pyr[l].stride(1) % 64 == 0 and pyr[l].stride(1) >= hl * wl
        got = pyr[l].float().reshape(want[l].shape)
        # level >= 1: one extra bf16 rounding of the pooled f2; bf16 storage: 2^-9 relative
        tol = 1.5e-2 if out_bf16 else (2e-3 if l == 0 else 6e-3)
        torch.testing.assert_close(got, want[l], atol=tol, rtol=tol)


@pytest.mark.parametrize("r", [3, 4])
def test_corr_lookup_bf16_pyramid(cuda, r):
    B, C, H, W = 2, 128, 23, 29
    f1, f2 = _fmaps(B, C, H, W, cuda, torch.bfloat16, seed=6)
    pyr = torch.ops.raft_stir.corr_volume(
        f1.permute(0, 2, 3, 1).reshape(B, H * W, C).contiguous(),
        f2.permute(0, 2, 3, 1).contiguous(), 4, 1.0 / math.sqrt(C), True)
    coords = _coords(B, H, W, "cpu")
    want = ref.corr_lookup(ref.corr_pyramid(f1.float().cpu(), f2.float().cpu(), 4), coords, r)
    got = torch.ops.raft_stir.corr_lookup(list(pyr), coords.to(cuda), r, False)
    torch.testing.assert_close(got.permute(0, 3, 1, 2).cpu(), want, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("r", [3, 4])
@pytest.mark.parametrize("out_bf16", [False, True])
def test_corr_lookup_forward(cuda, r, out_bf16):
    B, C, H, W = 2, 64, 23, 29
    f1, f2 = _fmaps(B, C, H, W, "cpu")
    pyr = ref.corr_pyramid(f1, f2, 4)
    coords = _coords(B, H, W, "cpu")
    want = ref.corr_lookup(pyr, coords, r)
    gp = [p.reshape(B, H * W, p.shape[-2], p.shape[-1]).contiguous().to(cuda) for p in pyr]
    got = torch.ops.raft_stir.corr_lookup(gp, coords.to(cuda), r, out_bf16)
    got = got.permute(0, 3, 1, 2).float().cpu()
    tol = 2e-2 if out_bf16 else 1e-5
    torch.testing.assert_close(got, want, atol=tol, rtol=tol)


@pytest.mark.parametrize("small", [False, True])
def test_allpairs_corr_autograd(cuda, small):
    """Full chain (volume -> 3 lookups -> loss) gradient vs ATen autograd."""
    from raft_stir_amd.ops.corr import AllPairsCorr
    B, C, H, W = 2, (128 if small else 256), 17, 21
    r = 3 if small else 4
    f1, f2 = _fmaps(B, C, H, W, "cpu", seed=3)
    coords = [_coords(B, H, W, "cpu", seed=s) for s in range(3)]
    g = torch.Generator().manual_seed(7)
    wts = [torch.randn(B, 4 * (2 * r + 1) ** 2, H, W, generator=g) for _ in coords]

    a1, a2 = f1.clone().requires_grad_(), f2.clone().requires_grad_()
    pyr = ref.corr_pyramid(a1, a2, 4)
    loss_ref = sum((ref.corr_lookup(pyr, c, r) * w).sum() for c, w in zip(coords, wts))
    loss_ref.backward()

    b1 = f1.to(cuda).contiguous(memory_format=torch.channels_last).requires_grad_()
    b2 = f2.to(cuda).contiguous(memory_format=torch.channels_last).requires_grad_()
    blk = AllPairsCorr(b1, b2, 4, r)
    loss = sum((blk(c.to(cuda)) * w.to(cuda)).sum() for c, w in zip(coords, wts))
    loss.backward()
    torch.testing.assert_close(loss.cpu(), loss_ref.detach(), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(b1.grad.cpu(), a1.grad, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(b2.grad.cpu(), a2.grad, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("C", [128, 256])
@pytest.mark.parametrize("bf16", [False, True])
def test_onthefly_corr_fwd_bwd(cuda, C, bf16):
    from raft_stir_amd.ops.corr import OnTheFlyCorr
    B, H, W, r = 2, 17, 27, 4
    f1, f2 = _fmaps(B, C, H, W, "cpu", seed=5)
    if bf16:
        f1, f2 = f1.bfloat16().float(), f2.bfloat16().float()
    coords = _coords(B, H, W, "cpu", seed=9)
    a1, a2 = f1.clone().requires_grad_(), f2.clone().requires_grad_()
    want = ref.corr_onthefly(a1, a2, coords, r)
    g = torch.randn_like(want)
    (want * g).sum().backward()

    dt = torch.bfloat16 if bf16 else torch.float32
    b1 = f1.to(cuda, dt).contiguous(memory_format=torch.channels_last).requires_grad_()
    b2 = f2.to(cuda, dt).contiguous(memory_format=torch.channels_last).requires_grad_()
    blk = OnTheFlyCorr(b1, b2, 4, r)
    got = blk(coords.to(cuda))
    # bf16: the pooled f2 levels are stored in bf16 (rounding ~2^-9 relative)
    ftol = 1e-2 if bf16 else 1e-4
    torch.testing.assert_close(got.float().cpu(), want.detach(), rtol=ftol, atol=ftol)
    (got * g.to(cuda)).sum().backward()
    tol = 2e-2 if bf16 else 1e-3
    torch.testing.assert_close(b1.grad.float().cpu(), a1.grad, rtol=tol, atol=tol)
    torch.testing.assert_close(b2.grad.float().cpu(), a2.grad, rtol=tol, atol=tol)


@pytest.mark.parametrize("C,r", [(256, 4), (128, 3), (96, 4)])
@pytest.mark.parametrize("out_bf16", [False, True])
def test_onthefly_tiled_forward(cuda, C, r, out_bf16):
    """csrc/corr_onthefly.hip otf_tile_kernel (4 x 4 query tiles, bounding-box
    cell GEMM on MFMA) vs the fp32 reference: smooth affine flow (every level
    on the MFMA path), a band of random flow (per-query fallback tiles next to
    MFMA tiles), partial tiles on both edges, flow pointing out of the image."""
    B, H, W = 2, 23, 38
    f1, f2 = _fmaps(B, C, H, W, "cpu", seed=21)
    f1, f2 = f1.bfloat16().float(), f2.bfloat16().float()
    g = torch.Generator().manual_seed(4)
    base = ref.coords_grid(B, H, W)
    ys, xs = base[:, 1:2], base[:, 0:1]
    flow = torch.cat([3.0 + 0.08 * xs - 0.05 * ys, -2.0 + 0.04 * ys], 1) + 0.3 * torch.randn(B, 2, H, W, generator=g)
    flow[:, :, 8:13] = 9.0 * torch.randn(B, 2, 5, W, generator=g)  # incoherent band
    flow[1, 0, :, -6:] += 30.0  # off the right edge
    coords = base + flow
    want = ref.corr_onthefly(f1, f2, coords, r)  # (B, L*K2, H, W)
    b1 = f1.to(cuda, torch.bfloat16).permute(0, 2, 3, 1).contiguous()
    f2l = [f2]
    for _ in range(3):
        f2l.append(F.avg_pool2d(f2l[-1], 2, stride=2))
    # levels pooled in fp32, stored in bf16 (as OnTheFlyCorr does)
    b2 = [t.to(cuda, torch.bfloat16).permute(0, 2, 3, 1).contiguous() for t in f2l]
    got = torch.ops.raft_stir.corr_otf(b1, b2, coords.to(cuda), r, 1.0 / math.sqrt(C), out_bf16)
    got = got.float().permute(0, 3, 1, 2).cpu()
    ftol = 2e-2 if out_bf16 else 1e-2
    torch.testing.assert_close(got, want.detach(), rtol=ftol, atol=ftol)


@pytest.mark.parametrize("C,r", [(256, 4), (128, 3), (96, 4)])
@pytest.mark.parametrize("det", [False, True])
def test_onthefly_tiled_backward(cuda, C, r, det):
    """csrc/corr_onthefly.hip tiled backward -- otf_tile_bwd_mma_kernel for
    C % 64 == 0 (both contractions on MFMA, split-bf16 cell gradients),
    otf_tile_bwd_kernel for C = 96 (4 x 4 query tiles: cell gradients gathered
    over the tile's bounding box, one df2 atomic per (cell, channel) per tile,
    per-window fallback for incoherent tiles) -- vs
    fp32 autograd through a per-level bilinear oracle (ops/reference.py
    corr_onthefly with the pooled levels as leaves).  Deterministic mode
    (32.32 fixed-point atomics) is bitwise repeatable."""
    B, H, W = 2, 23, 38
    f1, f2 = _fmaps(B, C, H, W, "cpu", seed=31)
    f1, f2 = f1.bfloat16().float(), f2.bfloat16().float()
    g = torch.Generator().manual_seed(6)
    base = ref.coords_grid(B, H, W)
    ys, xs = base[:, 1:2], base[:, 0:1]
    flow = torch.cat([3.0 + 0.08 * xs - 0.05 * ys, -2.0 + 0.04 * ys], 1) + 0.3 * torch.randn(B, 2, H, W, generator=g)
    flow[:, :, 8:13] = 9.0 * torch.randn(B, 2, 5, W, generator=g)  # incoherent band: fallback tiles
    flow[1, 0, :, -6:] += 30.0  # off the right edge
    coords = base + flow
    f2l = [f2]
    for _ in range(3):
        f2l.append(F.avg_pool2d(f2l[-1], 2, stride=2))
    f2l = [t.bfloat16().float() for t in f2l]  # the op stores the pooled levels in bf16
    a1 = f1.clone().requires_grad_()
    a2 = [t.clone().requires_grad_() for t in f2l]
    delta = ref._window_delta(r, coords.device, coords.dtype).reshape(-1, 2)
    pos0 = coords.permute(0, 2, 3, 1)
    outs = []
    for lvl, t in enumerate(a2):
        outs += [(ref.bilinear_sampler(t, pos0 / 2 ** lvl + delta[k]) * a1).sum(1) for k in range(delta.shape[0])]
    want = torch.stack(outs, -1) / math.sqrt(C)  # (B, H, W, L*K2)
    dout = torch.randn(want.shape, generator=g)
    (want * dout).sum().backward()

    b1 = f1.to(cuda, torch.bfloat16).permute(0, 2, 3, 1).contiguous()
    b2 = [t.to(cuda, torch.bfloat16).permute(0, 2, 3, 1).contiguous() for t in f2l]
    args = (b1, b2, coords.to(cuda), r, 1.0 / math.sqrt(C), dout.to(cuda))
    torch.ops.raft_stir.set_deterministic(det)
    try:
        got = torch.ops.raft_stir.corr_otf_backward(*args)
        if det:
            again = torch.ops.raft_stir.corr_otf_backward(*args)
            assert all(torch.equal(x, y) for x, y in zip(got, again))
    finally:
        torch.ops.raft_stir.set_deterministic(False)
    torch.testing.assert_close(got[0].cpu(), a1.grad.permute(0, 2, 3, 1), rtol=1e-4, atol=1e-4)
    for lvl in range(4):
        torch.testing.assert_close(got[1 + lvl].cpu(), a2[lvl].grad.permute(0, 2, 3, 1), rtol=1e-4, atol=1e-4)


def test_onthefly_matches_allpairs(cuda):
    """pyramid[l] == corr(f1, avgpool^l f2): both paths agree."""
    from raft_stir_amd.ops.corr import OnTheFlyCorr, AllPairsCorr
    B, C, H, W = 1, 256, 24, 32
    f1, f2 = _fmaps(B, C, H, W, cuda, seed=11)
    coords = _coords(B, H, W, cuda, seed=12)
    a = AllPairsCorr(f1, f2, 4, 4)(coords)
    b = OnTheFlyCorr(f1, f2, 4, 4)(coords)
    torch.testing.assert_close(a.float(), b.float(), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("mask_bf16", [False, True])
def test_convex_upsample(cuda, mask_bf16):
    from raft_stir_amd.ops.upsample import convex_upsample
    N, H, W = 2, 7, 11
    g = torch.Generator().manual_seed(0)
    flow = torch.randn(N, 2, H, W, generator=g) * 3
    mask = torch.randn(N, 576, H, W, generator=g)
    if mask_bf16:
        mask = mask.bfloat16().float()
    fa, ma = flow.clone().requires_grad_(), mask.clone().requires_grad_()
    want = ref.convex_upsample(fa, ma)
    gout = torch.randn_like(want)
    (want * gout).sum().backward()

    dt = torch.bfloat16 if mask_bf16 else torch.float32
    fb = flow.to(cuda).requires_grad_()
    mb = mask.to(cuda, dt).contiguous(memory_format=torch.channels_last).requires_grad_()
    got = convex_upsample(fb, mb)
    torch.testing.assert_close(got.cpu(), want.detach(), rtol=1e-4, atol=1e-4)
    (got * gout.to(cuda)).sum().backward()
    torch.testing.assert_close(fb.grad.cpu(), fa.grad, rtol=1e-4, atol=1e-3)
    tol = 3e-2 if mask_bf16 else 1e-4
    torch.testing.assert_close(mb.grad.float().cpu(), ma.grad, rtol=tol, atol=tol)
    # dmask_out: written in place into a padded (N, H, W, 640) buffer, pad channels untouched
    mn = mb.detach().permute(0, 2, 3, 1).contiguous()
    pad = torch.full((N, H, W, 640), 7.0, device=cuda, dtype=dt)
    df, dm = torch.ops.raft_stir.convex_upsample_backward(fb.detach(), mn, gout.to(cuda), pad)
    assert dm.data_ptr() == pad.data_ptr()
    assert torch.equal(pad[..., :576], mb.grad.permute(0, 2, 3, 1))
    assert bool((pad[..., 576:] == 7.0).all())
    torch.testing.assert_close(df, fb.grad)


@pytest.mark.parametrize("sep", [True, False])
def test_fused_gru_pass(cuda, sep):
    from raft_stir_amd.models.update import ConvGRU, SepConvGRU, _gru_step_reference
    torch.manual_seed(0)
    hd, cin = (128, 256) if sep else (96, 146)
    mod = (SepConvGRU if sep else ConvGRU)(hidden_dim=hd, input_dim=cin)
    B, H, W = 2, 9, 13
    h = torch.tanh(torch.randn(B, hd, H, W))
    x = torch.randn(B, cin, H, W)

    ha, xa = h.clone().requires_grad_(), x.clone().requires_grad_()
    mod.fused = False
    out_ref = mod(ha, xa)
    gout = torch.randn_like(out_ref)
    (out_ref * gout).sum().backward()
    ref_grads = {n: p.grad.clone() for n, p in mod.named_parameters()}
    mod.zero_grad()

    m2 = mod.to(cuda).to(memory_format=torch.channels_last)
    m2.fused = True
    hb = h.to(cuda).contiguous(memory_format=torch.channels_last).requires_grad_()
    xb = x.to(cuda).contiguous(memory_format=torch.channels_last).requires_grad_()
    out = m2(hb, xb)
    torch.testing.assert_close(out.cpu(), out_ref.detach(), rtol=1e-4, atol=1e-4)
    (out * gout.to(cuda)).sum().backward()
    torch.testing.assert_close(hb.grad.cpu(), ha.grad, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(xb.grad.cpu(), xa.grad, rtol=1e-3, atol=1e-3)
    for n, p in m2.named_parameters():
        torch.testing.assert_close(p.grad.cpu(), ref_grads[n], rtol=1e-3, atol=2e-3)


def test_allpairs_corr_autograd_bf16(cuda):
    """bf16 feature maps: the folded pyramid gradient goes through bf16 GEMMs."""
    from raft_stir_amd.ops.corr import AllPairsCorr
    B, C, H, W, r = 2, 256, 17, 21, 4
    f1, f2 = _fmaps(B, C, H, W, "cpu", seed=5)
    f1, f2 = f1.bfloat16().float(), f2.bfloat16().float()
    coords = [_coords(B, H, W, "cpu", seed=s) for s in range(2)]
    g = torch.Generator().manual_seed(9)
    wts = [torch.randn(B, 4 * (2 * r + 1) ** 2, H, W, generator=g) for _ in coords]
    a1, a2 = f1.clone().requires_grad_(), f2.clone().requires_grad_()
    pyr = ref.corr_pyramid(a1, a2, 4)
    sum((ref.corr_lookup(pyr, c, r) * w).sum() for c, w in zip(coords, wts)).backward()
    b1 = f1.to(cuda).bfloat16().contiguous(memory_format=torch.channels_last).requires_grad_()
    b2 = f2.to(cuda).bfloat16().contiguous(memory_format=torch.channels_last).requires_grad_()
    blk = AllPairsCorr(b1, b2, 4, r)
    sum((blk(c.to(cuda)).float() * w.to(cuda)).sum() for c, w in zip(coords, wts)).backward()
    for got, want in ((b1.grad, a1.grad), (b2.grad, a2.grad)):
        got = got.float().cpu()
        rel = (got - want).norm() / want.norm()
        assert rel < 2e-2, rel


def test_allpairs_corr_autograd_bf16_pyramid(cuda):
    """bf16 features + bf16 pyramid storage: forward and fmap gradients vs
    ATen fp32 autograd on the same (bf16-rounded) feature values."""
    from raft_stir_amd.ops.corr import AllPairsCorr
    B, C, H, W, r = 2, 256, 17, 21, 4
    f1, f2 = _fmaps(B, C, H, W, "cpu", seed=3)
    f1, f2 = f1.bfloat16().float(), f2.bfloat16().float()
    coords = [_coords(B, H, W, "cpu", seed=s) for s in range(3)]
    g = torch.Generator().manual_seed(7)
    wts = [torch.randn(B, 4 * (2 * r + 1) ** 2, H, W, generator=g) for _ in coords]
    a1, a2 = f1.clone().requires_grad_(), f2.clone().requires_grad_()
    pyr = ref.corr_pyramid(a1, a2, 4)
    loss_ref = sum((ref.corr_lookup(pyr, c, r) * w).sum() for c, w in zip(coords, wts))
    loss_ref.backward()
    b1 = f1.to(cuda, torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_()
    b2 = f2.to(cuda, torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_()
    blk = AllPairsCorr(b1, b2, 4, r, pyr_dtype=torch.bfloat16)
    assert blk.state.pyr is not None and blk.state.pyr[0].dtype == torch.bfloat16
    loss = sum((blk(c.to(cuda)) * w.to(cuda)).sum() for c, w in zip(coords, wts))
    loss.backward()
    torch.testing.assert_close(loss.cpu(), loss_ref.detach(), rtol=2e-3, atol=5.0)
    for got, want in ((b1.grad, a1.grad), (b2.grad, a2.grad)):
        rel = ((got.float().cpu() - want).norm() / want.norm()).item()
        assert rel < 2e-2, rel


@pytest.mark.parametrize("HW", [(46, 62), (11, 37), (12, 20)])
@pytest.mark.parametrize("out_bf16", [False, True])
def test_pyr_grad_fold(cuda, HW, out_bf16):
    """Pyramid-gradient fold (avg-pool adjoint of every level onto level 0, times
    the 1/sqrt(C) scale) vs a PyTorch fp32 gather; (46, 62) and (12, 20) take the
    4-wide kernel (H*W % 4 == 0), (11, 37) the per-element one."""
    H, W = HW
    B, N1, levels, scale = 2, 24, 4, 0.0625
    g = torch.Generator(device="cpu").manual_seed(3)
    shapes = [(H >> l, W >> l) for l in range(levels)]
    gpyr = [torch.randn(B, N1, h, w, generator=g).to(cuda) for h, w in shapes]
    want = gpyr[0].clone()
    for l in range(1, levels):
        h, w = shapes[l]
        ys, xs = torch.arange(H, device=cuda) >> l, torch.arange(W, device=cuda) >> l
        m = (ys[:, None] < h) & (xs[None, :] < w)
        up = gpyr[l][:, :, ys.clamp(max=h - 1)][:, :, :, xs.clamp(max=w - 1)]
        want += 0.25 ** l * up * m
    want *= scale
    if out_bf16:
        out = torch.empty(B, N1, H, W, device=cuda, dtype=torch.bfloat16)
        torch.ops.raft_stir.pyr_grad_fold_bf16(gpyr, scale, out)
        torch.testing.assert_close(out.float(), want, rtol=1e-2, atol=1e-2)
    else:
        torch.ops.raft_stir.pyr_grad_fold(gpyr, scale)
        torch.testing.assert_close(gpyr[0], want, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("HW,C", [((46, 62), 256), ((11, 37), 256), ((12, 20), 128), ((23, 31), 128)])
@pytest.mark.parametrize("det", [False, True])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_corr_volume_backward_fused(cuda, HW, C, det, dtype):
    """csrc/corr_bwd.hip: df1 = G f2 and df2 = G^T f1 with G the folded
    pyramid gradient (avg-pool adjoint of every level onto level 0, times
    1/sqrt(C), bf16 rows zero-padded to a multiple of 64), both GEMMs in one
    MFMA launch, vs fp32 PyTorch (fold by gather, then two bmm).  (11, 37):
    N = 407, ragged M and K tiles; deterministic in both modes (bitwise
    repeat)."""
    H, W = HW
    N = H * W
    B, levels, scale = 2, 4, 1.0 / math.sqrt(C)
    g = torch.Generator(device="cpu").manual_seed(4)
    shapes = [(H >> l, W >> l) for l in range(levels)]
    gpyr = [torch.randn(B, N, h, w, generator=g).to(cuda) for h, w in shapes]
    f1 = torch.randn(B, N, C, generator=g).to(cuda).to(dtype)
    f2 = torch.randn(B, H, W, C, generator=g).to(cuda).to(dtype)
    G = gpyr[0].clone()
    for l in range(1, levels):
        h, w = shapes[l]
        ys, xs = torch.arange(H, device=cuda) >> l, torch.arange(W, device=cuda) >> l
        m = (ys[:, None] < h) & (xs[None, :] < w)
        G += 0.25 ** l * gpyr[l][:, :, ys.clamp(max=h - 1)][:, :, :, xs.clamp(max=w - 1)] * m
    G = (G * scale).view(B, N, N)
    want1 = torch.bmm(G, f2.float().view(B, N, C))
    want2 = torch.bmm(G.transpose(1, 2), f1.float()).view(B, H, W, C)
    torch.ops.raft_stir.set_deterministic(det)
    try:
        df1, df2 = torch.ops.raft_stir.corr_volume_backward(gpyr, f1, f2, scale)
        r1, r2 = torch.ops.raft_stir.corr_volume_backward(gpyr, f1, f2, scale)
        assert torch.equal(df1, r1) and torch.equal(df2, r2)
    finally:
        torch.ops.raft_stir.set_deterministic(False)
    assert df1.dtype == dtype and df1.shape == f1.shape and df2.shape == f2.shape
    for got, want in ((df1, want1), (df2, want2)):
        rel = ((got.float() - want).norm() / want.norm()).item()
        # bf16: bf16 G and outputs; fp32: split-bf16 operands (three K passes), fp32 outputs
        assert rel < (1e-2 if dtype == torch.bfloat16 else 1e-4), rel


@pytest.mark.parametrize("n", [1, 7, 4096, 1000003])
def test_split_bf16_matches_aten(cuda, n):
    """csrc/split.hip: hi = bf16(x), lo = bf16(x - hi), bitwise equal to the
    ATen casts (round-to-nearest-even), tails of n % 4 elements included."""
    g = torch.Generator().manual_seed(n)
    x = (torch.randn(n, generator=g) * torch.logspace(-8, 8, n)).to(cuda)
    hi, lo = torch.ops.raft_stir.split_bf16(x)
    want_hi = x.to(torch.bfloat16)
    want_lo = (x - want_hi.float()).to(torch.bfloat16)
    assert torch.equal(hi, want_hi) and torch.equal(lo, want_lo)


@pytest.mark.parametrize("HW", [(46, 62), (11, 37), (1, 5), (7, 1)])
def test_upflow8_backward_matches_autograd(cuda, HW):
    """csrc/convex_upsample.hip upflow8_{cols,rows}_kernel: the adjoint of
    RAFT-small's x8 bilinear upsampling (align_corners=True), two deterministic
    gather passes, vs
    the autograd of F.interpolate (fp32, the training forward's arithmetic)."""
    from raft_stir_amd.models.fused_train import _interp_matrix
    H, W = HW
    g = torch.randn(3, 2, 8 * H, 8 * W, device=cuda)
    got = torch.ops.raft_stir.upflow8_backward(g, _interp_matrix(H, 8 * H, cuda), _interp_matrix(W, 8 * W, cuda))
    f = torch.zeros(3, 2, H, W, device=cuda, requires_grad=True)
    (8 * F.interpolate(f, size=(8 * H, 8 * W), mode="bilinear", align_corners=True)).backward(g)
    torch.testing.assert_close(got, f.grad, atol=1e-3, rtol=1e-4)
    assert torch.equal(got, torch.ops.raft_stir.upflow8_backward(g, _interp_matrix(H, 8 * H, cuda),
                                                                 _interp_matrix(W, 8 * W, cuda)))
