"""ATen oracle ops (ops/reference.py) vs first-principles math, on CPU.

These oracles are what every HIP kernel is tested against on the GPU, so they
are pinned here independently: the window lookup against an explicit
bilinear formula with x-major channel order, the on-the-fly correlation
against the all-pairs pyramid (linearity), the convex upsampler against a
loop implementation, plus fp64 gradchecks.
"""
import math

import pytest
import torch
import torch.nn.functional as F

from raft_stir_amd.ops import reference as ref


def _bilinear_zero(img, x, y):
    """img (H,W), align_corners pixel coords, zero outside."""
    H, W = img.shape
    x0, y0 = math.floor(x), math.floor(y)
    out = 0.0
    for dy in (0, 1):
        for dx in (0, 1):
            xi, yi = x0 + dx, y0 + dy
            w = (1 - abs(x - xi)) * (1 - abs(y - yi))
            if 0 <= xi < W and 0 <= yi < H:
                out += w * float(img[yi, xi])
    return out


def test_corr_volume_matches_einsum():
    g = torch.Generator().manual_seed(0)
    f1 = torch.randn(2, 16, 5, 7, generator=g)
    f2 = torch.randn(2, 16, 5, 7, generator=g)
    v = ref.corr_volume(f1, f2)
    want = torch.einsum("bchw,bcyx->bhwyx", f1, f2).reshape(2, 35, 5, 7) / 4.0
    torch.testing.assert_close(v, want)


@pytest.mark.parametrize("r", [1, 3])
def test_lookup_explicit_bilinear_xmajor(r):
    g = torch.Generator().manual_seed(1)
    B, C, H, W = 1, 8, 6, 9
    f1, f2 = torch.randn(B, C, H, W, generator=g), torch.randn(B, C, H, W, generator=g)
    pyr = ref.corr_pyramid(f1, f2, 2)
    coords = ref.coords_grid(B, H, W) + 2.5 * torch.randn(B, 2, H, W, generator=g)
    out = ref.corr_lookup(pyr, coords, r)
    K = (2 * r + 1) ** 2
    assert out.shape == (B, 2 * K, H, W)
    for (h, w) in [(0, 0), (3, 4), (5, 8)]:
        x, y = float(coords[0, 0, h, w]), float(coords[0, 1, h, w])
        for lvl in range(2):
            vol = pyr[lvl][h * W + w, 0]
            for k in (0, K // 2, K - 1, 2 * r + 3):
                i, j = divmod(k, 2 * r + 1)  # x-offset-major
                want = _bilinear_zero(vol, x / 2 ** lvl + (i - r), y / 2 ** lvl + (j - r))
                got = float(out[0, lvl * K + k, h, w])
                assert abs(got - want) < 1e-4, (h, w, lvl, k, got, want)


def test_pyramid_is_corr_of_pooled_fmap2():
    """pyramid[l] == corr(f1, avgpool^l(f2)) -- the identity the on-the-fly path relies on."""
    g = torch.Generator().manual_seed(2)
    f1, f2 = torch.randn(1, 32, 8, 12, generator=g), torch.randn(1, 32, 8, 12, generator=g)
    pyr = ref.corr_pyramid(f1, f2, 4)
    p = f2
    for lvl in range(4):
        want = ref.corr_volume(f1, p).reshape(pyr[lvl].shape)
        torch.testing.assert_close(pyr[lvl], want, atol=1e-5, rtol=1e-5)
        if lvl < 3:
            p = F.avg_pool2d(p, 2, 2)


@pytest.mark.parametrize("r", [3, 4])
def test_onthefly_equals_allpairs(r):
    g = torch.Generator().manual_seed(3)
    f1, f2 = torch.randn(2, 16, 17, 21, generator=g), torch.randn(2, 16, 17, 21, generator=g)
    coords = ref.coords_grid(2, 17, 21) + 3 * torch.randn(2, 2, 17, 21, generator=g)
    a = ref.corr_lookup(ref.corr_pyramid(f1, f2, 4), coords, r)
    b = ref.corr_onthefly(f1, f2, coords, r, 4)
    torch.testing.assert_close(a, b, atol=1e-4, rtol=1e-4)


def test_convex_upsample_loop():
    g = torch.Generator().manual_seed(4)
    N, H, W = 1, 3, 4
    flow = torch.randn(N, 2, H, W, generator=g)
    mask = torch.randn(N, 576, H, W, generator=g)
    up = ref.convex_upsample(flow, mask)
    m = torch.softmax(mask.view(N, 9, 8, 8, H, W), dim=1)
    fp = F.pad(8 * flow, (1, 1, 1, 1))
    for (y, x, sy, sx) in [(0, 0, 0, 0), (1, 2, 3, 5), (2, 3, 7, 7)]:
        for c in range(2):
            acc = 0.0
            for t in range(9):
                ky, kx = divmod(t, 3)
                acc += float(m[0, t, sy, sx, y, x] * fp[0, c, y + ky, x + kx])
            assert abs(float(up[0, c, 8 * y + sy, 8 * x + sx]) - acc) < 1e-4


def test_gradcheck_lookup_and_upsample():
    g = torch.Generator().manual_seed(5)
    f1 = torch.randn(1, 4, 4, 5, generator=g, dtype=torch.float64, requires_grad=True)
    f2 = torch.randn(1, 4, 4, 5, generator=g, dtype=torch.float64, requires_grad=True)
    coords = (ref.coords_grid(1, 4, 5, dtype=torch.float64)
              + 0.37 * torch.randn(1, 2, 4, 5, generator=g, dtype=torch.float64))

    def fn(a, b):
        return ref.corr_lookup(ref.corr_pyramid(a, b, 2), coords, 1).double()

    # corr_pyramid casts to fp32 internally; check in fp64 via the volume math
    def fn64(a, b):
        B, C, H, W = a.shape
        vol = torch.matmul(a.reshape(B, C, -1).transpose(1, 2), b.reshape(B, C, -1)) / math.sqrt(C)
        lvl = vol.reshape(B * H * W, 1, H, W)
        pyr = [lvl, F.avg_pool2d(lvl, 2, 2)]
        return ref.corr_lookup(pyr, coords, 1)

    assert torch.autograd.gradcheck(fn64, (f1, f2), eps=1e-6, atol=1e-5)
    flow = torch.randn(1, 2, 3, 3, generator=g, dtype=torch.float64, requires_grad=True)
    mask = torch.randn(1, 576, 3, 3, generator=g, dtype=torch.float64, requires_grad=True)
    assert torch.autograd.gradcheck(ref.convex_upsample, (flow, mask), eps=1e-6, atol=1e-5)


def test_sequence_loss_formula():
    from raft_stir_amd.train.loss import sequence_loss
    g = torch.Generator().manual_seed(6)
    gt = torch.randn(2, 2, 8, 8, generator=g) * 3
    gt[0, :, 0, 0] = 500.0  # |gt| >= MAX_FLOW -> invalid
    valid = (torch.rand(2, 8, 8, generator=g) > 0.3).float()
    preds = [torch.randn(2, 2, 8, 8, generator=g) for _ in range(4)]
    loss, metrics = sequence_loss(preds, gt, valid, gamma=0.8)
    mag = gt.pow(2).sum(1).sqrt()
    v = ((valid >= 0.5) & (mag < 400)).float()[:, None]
    want = sum(0.8 ** (3 - i) * (v * (p - gt).abs()).mean() for i, p in enumerate(preds))
    torch.testing.assert_close(loss, want)
    epe = (preds[-1] - gt).pow(2).sum(1).sqrt()[v[:, 0] > 0]
    assert abs(metrics["epe"] - epe.mean().item()) < 1e-5
    assert abs(metrics["1px"] - (epe < 1).float().mean().item()) < 1e-6


def test_frag_weight_layout():
    """ops/conv.py frag_weight: element (rb, c, t, ks, lane, j) of the
    fragment-major layout (csrc/conv_v3.h) is weight[rb*32 + lane%32][t][c*64 +
    16 ks + 8 (lane // 32) + j]."""
    from raft_stir_amd.ops.conv import frag_weight
    cp, taps, k = 64, 5, 128
    w = torch.arange(cp * taps * k, dtype=torch.float32).view(cp, taps, k)
    f = frag_weight(w).reshape(cp // 32, k // 64, taps, 4, 64, 8)
    for rb, c, t, ks, lane, j in [(0, 0, 0, 0, 0, 0), (1, 1, 4, 3, 63, 7), (0, 1, 2, 1, 37, 5), (1, 0, 3, 2, 12, 1)]:
        assert f[rb, c, t, ks, lane, j] == w[rb * 32 + lane % 32, t, c * 64 + 16 * ks + 8 * (lane // 32) + j]
