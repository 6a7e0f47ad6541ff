"""Host side of the fused update-block convolution (csrc/conv.hip).

* :func:`pack_weight` turns a PyTorch conv weight (Cout, Cin, KH, KW) into the
  kernel's [Cout_pad][taps][Ktot] bf16 layout for a given channel-SEGMENT
  layout of its input: each segment is a (padded channel count, pieces) pair
  where a piece maps weight input channels [w0, w0+n) to segment channels
  [s0, s0+n).  Unmapped (padding) channels get zero weights, so the kernel's
  K loop runs over 32-channel chunks with no bounds checks.
* :func:`conv_fused` is a thin, checked wrapper over torch.ops.raft_stir.conv_fused.
"""
from __future__ import annotations

import os
from typing import List, Sequence, Tuple

import torch

(EPI_BIAS, EPI_RELU, EPI_SCALE, EPI_GRU_ZR, EPI_GRU_Q, EPI_FLOW,
 EPI_RELU_BWD, EPI_ACC_F32, EPI_GRU_QBWD, EPI_NORM) = range(10)

Piece = Tuple[int, int, int]          # (weight in-channel start, length, segment channel offset)
SegSpec = Tuple[int, Sequence[Piece]]  # (segment channels read (multiple of 32), pieces)


def pad_to(n: int, m: int) -> int:
    return (n + m - 1) // m * m


@torch.no_grad()
def pack_weight(weight: torch.Tensor, segs: Sequence[SegSpec], cout_pad: int,
                dtype: torch.dtype = torch.bfloat16) -> torch.Tensor:
    cout, cin, kh, kw = weight.shape
    taps = kh * kw
    wt = weight.detach().float().permute(0, 2, 3, 1).reshape(cout, taps, cin)
    ktot = sum(c for c, _ in segs)
    out = torch.zeros(cout_pad, taps, ktot, device=weight.device, dtype=torch.float32)
    kb = 0
    for c, pieces in segs:
        assert c % 32 == 0
        for w0, n, s0 in pieces:
            assert s0 + n <= c and w0 + n <= cin
            out[:cout, :, kb + s0:kb + s0 + n] = wt[:, :, w0:w0 + n]
        kb += c
    return out.to(dtype).contiguous()


@torch.no_grad()
def split_weight(packed: torch.Tensor) -> torch.Tensor:
    """A packed fp32 weight [Cout_pad][taps][Ktot] -> the F32 tiles' split
    layout [Cout_pad][taps][2 * Ktot] bf16: per 32-channel K chunk [wh 32 | wl 32]
    with wh = bf16(w), wl = bf16(w - wh) (csrc/conv.hip conv_lds_kernel<..., F32>)."""
    cp, taps, k = packed.shape
    assert k % 32 == 0
    w = packed.float().view(cp, taps, k // 32, 1, 32)
    hi = w.to(torch.bfloat16)
    lo = (w - hi.float()).to(torch.bfloat16)
    return torch.cat([hi, lo], 3).reshape(cp, taps, 2 * k).contiguous()


@torch.no_grad()
def pack_weight_split(weight: torch.Tensor, segs: Sequence[SegSpec], cout_pad: int) -> torch.Tensor:
    """:func:`pack_weight` in the F32 tiles' split [wh | wl] layout."""
    return split_weight(pack_weight(weight, segs, cout_pad, torch.float32))


# (60, 62-64 and 67 were measured and dropped in round 6: no table entry or
# encoder path selected them, profiles/r5/tune_*.log)
V3_TILES = (56, 57, 61, 65, 66, 68)


@torch.no_grad()
def frag_weight(w: torch.Tensor) -> torch.Tensor:
    """A packed weight [Cout_pad][taps][Ktot] in the fragment-major layout of
    the weight-streaming tiles 56-68 (csrc/conv_v3.h): per 32-row block, per
    64-channel K chunk, per tap, per 16-channel slice, the 1 KB A fragment of a
    32x32x16 MFMA (lane h*32 + r holds row r, channels 16 ks + 8 h .. + 8), so
    each wave's weight stream is one contiguous run of 1 KB loads.  Same shape
    and element count as the input (a permutation of it)."""
    cp, taps, k = w.shape
    assert cp % 32 == 0 and k % 64 == 0, (cp, k)
    v = w.view(cp // 32, 32, taps, k // 64, 4, 2, 8)  # rb, r, t, c, ks, h, j
    return v.permute(0, 3, 2, 4, 5, 1, 6).contiguous().view(cp, taps, k)


F32_TILES = (6, 7, 8)
# csrc/conv_v3f.hip: the fp32 weight-streaming tiles (81 = 3 patch rows,
# 82 = 1 row for batch-1 grids, 83 = 2 rows, 84 = 64 Cout x 4 rows, 85 = 84
# with one halo buffer for Ktot = 64), fed by frag_weight_split
V3F_TILES = (81, 82, 83, 84, 85)


@torch.no_grad()
def frag_weight_split(w_split: torch.Tensor) -> torch.Tensor:
    """The F32 tiles' split weight [Cout_pad][taps][2 Ktot] (per 32-channel
    chunk [wh 32 | wl 32], :func:`split_weight`) -> [frag(wh) ; frag(wl)]
    [2 Cout_pad][taps][Ktot]: the hi and lo fragment streams of the fp32
    weight-streaming tiles 81-83, lo blocks after all hi blocks."""
    cp, taps, k2 = w_split.shape
    v = w_split.view(cp, taps, k2 // 64, 2, 32)
    hi = v[:, :, :, 0].reshape(cp, taps, k2 // 2)
    lo = v[:, :, :, 1].reshape(cp, taps, k2 // 2)
    return torch.cat([frag_weight(hi), frag_weight(lo)], 0)


def frag32_eligible(w_split: torch.Tensor, kh: int, kw: int) -> bool:
    """Can the fp32 weight-streaming tiles 81-83 serve this split weight?"""
    return kh * kw in (5, 9) and w_split.dim() == 3 and w_split.shape[0] % 32 == 0 and w_split.shape[2] % 128 == 0


_V3F = os.environ.get("RS_V3F", "1") != "0"  # RS_V3F=0: the fp32 engines stay on the register tiles


def choose_tile_f32(P: int, cout: int, geo: bool = False, v3f: bool = False, taps: int = 9, ktot: int = 0) -> int:
    """Split-bf16 fp32 tile: 64x64 for narrow outputs / small grids, else
    128x64 (128x128 at large pixel counts).  Batch-1 grids (<= 768 64x64
    tiles: STIR 1x64x80, Sintel 1x55x136) take the intra-block split-K
    variants, 4 K groups (38) when the grid has at most one tile per CU, else
    2 (40): their register-staged K loop is load-latency bound there."""
    if v3f and _V3F and not geo:  # split fragment-major weight available: the weight-streaming tiles
        # (training shape, scripts/bench_v3f.py: 3x3 on 2 patch rows 78-91 us, 1x5 / 5x1 on 3 rows 71-91 us)
        if P >= 16384:
            if cout <= 64:
                return 85 if ktot == 64 else 84
            return 83 if taps == 9 else 81
        return 82
    nb64 = -(-P // 64) * -(-cout // 64)
    if nb64 <= 256 and not geo:  # (conv_geo's strided tiles have no split-K variant)
        return 38
    if nb64 <= 768 and not geo:
        return 40
    if cout <= 64:
        return 6
    return 8 if (P >= 16384 and cout >= 256) else 7


@torch.no_grad()
def pack_bias(bias: torch.Tensor, n: int | None = None) -> torch.Tensor:
    b = bias.detach().float()
    if n is not None and n > b.numel():
        b = torch.cat([b, b.new_zeros(n - b.numel())])
    return b.contiguous()


# bitmask A/B switch for the 8-wave tiles; in-situ training bench (30 steps x2):
# bit 4 (192-wide conv on the 192x96 tile) +0.4 %, bit 1 (Cout <= 128 on 128x96)
# -1.4 %, bit 2 (Cout > 192) neutral -- default 4.
_WIDE = 4


# csrc/conv_gemm1.hip: the update block's 1x1 convs (convc1, the mask head's
# second conv; forward and input gradient) as plain MFMA GEMMs over
# K-contiguous weight and activation rows (bf16, every segment % 64 channels,
# packed weights with >= round_up(Cout, 128) rows, no EPI_NORM).  A tuning
# candidate: it beats the implicit-GEMM tiles on the training shape's convc1 /
# mask-head forward and the mask-head dgrad, not at batch 1
# (profiles/r5/bench_conv_1x1_s22.log)
GEMM1_TILE = 70


def gemm1_ok(w: torch.Tensor, cout: int, chans, nscale=None) -> bool:
    return (w.dtype == torch.bfloat16 and nscale is None and all(int(c) % 64 == 0 for c in chans)
            and w.shape[0] >= pad_to(cout, 128))


def choose_tile(P: int, cout: int, seg_chans, taps: int = 9) -> int:
    """Kernel variant for a conv (measured on MI355X, scripts/bench_conv.py;
    profiles/conv_tiles_r1.md):
    5 = split-K small-N (Cout <= 16); 16 / 17 = 128x64 / 64x64 tiles fed by
    buffer_load...lds DMA with a scalar K walk (every segment % 64 == 0, at
    most 32 taps); 31 / 29 = the same kernel with 8 waves and 128x96 /
    192x96 tiles (training shape: GRU 1x5 zr 34.7 -> 32.8 us, 3x3 256->192
    40.2 -> 33.0 us); 3/4 = 64x64 / 128x64 register-staged tiles with 32-deep
    K steps otherwise."""
    if cout <= 16:
        return 5
    if all(c % 64 == 0 for c in seg_chans) and taps <= 32:
        k = taps * sum(seg_chans)
        if P >= 16384:  # training shape: 8-wave 128x96 / 192x96 tiles where they measured faster
            if 64 < cout <= 128 and _WIDE & 1:
                return 31
            if cout > 192 and k >= 1024 and _WIDE & 2:
                return 31
            if 128 < cout <= 192 and k >= 1024 and _WIDE & 4:
                return 29
        return 16 if (P >= 16384 and cout >= 192 and k >= 384) else 17
    if -(-P // 64) * -(-cout // 64) <= 256:
        return 41  # tile 3 with 4-way intra-block split-K: batch-1 grids (RAFT-small / STIR ConvGRU)
    big = cout >= 192 or (cout >= 126 and P >= 16384)
    return 4 if big else 3


# Measured per-call tile table (scripts/tune_conv.py on MI355X): the kernel
# variant with the lowest graph-timed latency for every conv_fused call of the
# training step and of inference at the benchmark shapes, keyed by
# tune_key().  Calls not in the table use the choose_tile heuristic.
# RS_CONV_TUNING_FILE: another tile table (A/B of a retune against the shipped one)
_TUNED_PATH = os.environ.get("RS_CONV_TUNING_FILE") or os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "conv_tuning.json")
_TUNED: dict | None = None
_RECORD: list | None = None  # scripts/tune_conv.py: conv_fused calls are appended here


def tune_key(B: int, H: int, W: int, cout: int, chans, kh: int, kw: int, epi: int) -> str:
    return f"{B}x{H}x{W}|{cout}|{','.join(str(int(c)) for c in chans)}|{kh}x{kw}|{epi}"


def tuned_tiles() -> dict:
    global _TUNED
    if _TUNED is None:
        _TUNED = {}
        if os.environ.get("RS_CONV_TUNED", "1") != "0" and os.path.exists(_TUNED_PATH):
            import json
            with open(_TUNED_PATH) as f:
                _TUNED = {k: int(v) for k, v in json.load(f).get("tiles", {}).items()}
    return _TUNED


_TUNED_F32: dict | None = None


def tuned_tiles_f32() -> dict:
    """Measured F32-tile table (scripts/tune_conv.py --f32), keyed by tune_key."""
    global _TUNED_F32
    if _TUNED_F32 is None:
        _TUNED_F32 = {}
        if os.environ.get("RS_CONV_TUNED", "1") != "0" and os.path.exists(_TUNED_PATH):
            import json
            with open(_TUNED_PATH) as f:
                _TUNED_F32 = {k: int(v) for k, v in json.load(f).get("tiles_f32", {}).items()}
    return _TUNED_F32


def frag_eligible(w: torch.Tensor, kh: int, kw: int) -> bool:
    """Can the weight-streaming tiles 56-68 serve this packed weight?"""
    return kh * kw in (5, 9) and w.dim() == 3 and w.shape[0] % 32 == 0 and w.shape[2] % 64 == 0


def conv_fused(segs: List[Tuple[torch.Tensor, int, int]], w, bias, kh, kw, cout, epi, out, ooff=0,
               scale=1.0, hd=0, out2=None, o2off=0, out3=None, o3off=0, aux1=None, a1off=0,
               aux2=None, a2off=0, tile=None, nscale=None, wf=None):
    """segs: list of (NHWC bf16 buffer, channel offset, channels read).
    ``nscale`` with ``epi=EPI_NORM``: out = [relu if hd](acc * nscale + bias)
    [then relu(. + aux1)].  ``wf``: the same weight in the fragment-major
    layout (:func:`frag_weight`), which the weight-streaming tiles 56-68 read;
    without it those tiles are not chosen."""
    if wf is None:  # the training engine tags its packed weights with their fragment-major copy
        wf = getattr(w, "_rs_frag", None)
    tensors = [s[0] for s in segs]
    offs = [int(s[1]) for s in segs]
    chans = [int(s[2]) for s in segs]
    if _RECORD is not None:
        _RECORD.append(dict(segs=segs, w=w, bias=bias, kh=kh, kw=kw, cout=cout, epi=epi, out=out, ooff=ooff,
                            scale=scale, hd=hd, out2=out2, o2off=o2off, out3=out3, o3off=o3off, aux1=aux1,
                            a1off=a1off, aux2=aux2, a2off=a2off, tile=tile, nscale=nscale, wf=wf))
    if tile is None:
        t0 = tensors[0]
        key = tune_key(t0.shape[0], t0.shape[1], t0.shape[2], cout, chans, kh, kw, epi)
        P = t0.shape[0] * t0.shape[1] * t0.shape[2]
        if t0.dtype == torch.float32:  # split-bf16 F32 tiles: measured table, else the heuristic
            tile = tuned_tiles_f32().get(key)
            has32 = getattr(w, "_rs_frag32", None) is not None and all(c % 64 == 0 for c in chans)
            if tile is None or (tile in V3F_TILES and not (has32 and _V3F)):
                tile = choose_tile_f32(P, cout, v3f=has32, taps=kh * kw, ktot=sum(chans))
        else:
            tile = tuned_tiles().get(key)
            if tile is None or (tile in V3_TILES and wf is None) or (tile == GEMM1_TILE and not gemm1_ok(
                    w, cout, chans, nscale)):
                tile = choose_tile(P, cout, chans, kh * kw)
    if tile in V3_TILES:
        if wf is None:
            raise ValueError("conv_fused: tiles 56-68 read the fragment-major weight: pass wf=frag_weight(w)")
        w = wf
    elif tile in V3F_TILES:
        wf32 = getattr(w, "_rs_frag32", None)
        if wf32 is None:
            raise ValueError("conv_fused: tiles 81-83 read the split fragment-major weight: tag the split "
                             "weight with _rs_frag32 = frag_weight_split(w)")
        w = wf32
    if nscale is None:
        torch.ops.raft_stir.conv_fused(tensors, offs, chans, w, bias, kh, kw, cout, epi, float(scale), hd,
                                       out, ooff, out2, o2off, out3, o3off, aux1, a1off, aux2, a2off, tile)
    else:
        torch.ops.raft_stir.conv_fused(tensors, offs, chans, w, bias, kh, kw, cout, epi, float(scale), hd,
                                       out, ooff, out2, o2off, out3, o3off, aux1, a1off, aux2, a2off, tile,
                                       nscale)
