// Fused implicit-GEMM convolution for the RAFT update block (bf16 MFMA, NHWC).
//
// The reference update operator (core/update.py:6-136) is ~13 small
// convolutions per refinement iteration glued together by cat / sigmoid /
// tanh / relu / mul / add kernels.  Here every one of them is ONE launch of
// this kernel:
//
//   out[p, co] = epilogue( bias[co] + sum_{tap, ci} X[p + tap, ci] * W[co, tap, ci] )
//
// * GEMM orientation: M = output channels (A = packed weights), N = pixels
//   (B = implicit im2col of the NHWC input), K = taps x input channels.
//   mfma_f32_16x16x32_bf16 fragments are 16-byte K-runs for both operands:
//   A: W[co][tap][k0 + 8*(lane>>4) .. +7], B: X[pixel'][k0 + 8*(lane>>4) .. +7]
//   -- channels-last rows, so no im2col buffer and no LDS transpose.
// * The input is up to 3 channel SEGMENTS, each a (base, channel count,
//   row stride) view, so concatenations (cat[h, x], cat[r*h, x],
//   cat[inp, motion, flow]) are never materialised: the producer kernels
//   write straight into slices of shared NHWC buffers.
// * Zero padding ("same" convolutions, stride 1) by predicated loads.
// * Epilogues fuse what the reference does in separate kernels:
//   bias, ReLU, scale (mask x0.25), the ConvGRU gates (z, r*h) and the GRU
//   update h' = (1-z) h + z tanh(q), and the coords update coords += delta.
// * Register double-buffered fragment loads (step k+1 issued before the
//   MFMAs of step k); weights are tiny and L1/L2-resident.
//
// Weights are packed on the host (ops/conv.py) into [Cout_pad][taps][Ktot]
// bf16, Ktot = sum of the segment channel counts (each a multiple of 32),
// with zeros for padding channels, so the K loop needs no bounds checks.
#include "conv_common.h"

namespace rs {
namespace conv {

// ------------------------------------------------------------------ LDS-staged variant
// Block tile BM output channels x BN pixels, 256 threads (WAVES_M x WAVES_N
// waves).  Per 32-deep K step the block stages the A (weights) and B (pixel
// rows) tiles once in LDS -- XOR-swizzled 64-B rows so the 16 rows a
// ds_read_b128 lane group reads land on 16 distinct bank slots -- and every
// wave reads its fragments from there: each global byte is fetched once per
// block instead of once per wave.  Global loads for step k+1 are in flight
// while the MFMAs of step k run (register prefetch, LDS double buffer, one
// barrier per step).
// rows of CPR 16-byte chunks; XOR so the 16 rows of a ds_read_b128 lane group
// hit 16 distinct 16-B bank slots (256-B bank rows hold 4 (BK=32) / 2 (BK=64) rows)
template <int CPR>
__device__ __forceinline__ int swz(int r, int c) {
  return CPR == 4 ? r * 4 + (c ^ ((r >> 2) & 3)) : r * 8 + (c ^ ((r >> 1) & 7));
}

// GEO: strided input / remapped output pixels (Args geometry fields): the
// encoder's stride-2 convolutions and the phase-split dgrads of them.
// F32: fp32 activations in and out (the reference's default inference
// precision) on the bf16 MFMAs by operand splitting: x = xh + xl and
// w = wh + wl (hi = bf16(x), lo = bf16(x - hi)), x.w ~= xh.wh + xl.wh + xh.wl
// (relative error ~2^-17; the dropped xl.wl term is ~2^-18).  A K step covers
// 32 input channels: the staged B row is [xh 32 | xl 32] (converted while
// staging), the packed A row [wh 32 | wl 32] (ops/conv.py pack_weight_split),
// and the three products are three MFMAs over the same LDS rows -- 3x the
// MFMA work of bf16, no extra passes over the activations.
//
// KG > 1: intra-block split-K (as conv_buf_kernel): KG groups of 4 waves over
// the same output tile, group g staging and multiplying K steps g, g + KG, ...
// through its own double buffer, partial tiles summed in LDS by group 0.  The
// register-staged K loop exposes one global-load latency per step; at the
// batch-1 shapes (STIR 1x64x80: 160 blocks, 72 K steps of the ConvGRU) that
// latency, not the MFMAs, set the kernel time.
template <int BM, int BN, int WAVES_M, int WAVES_N, int BK, bool GEO = false, bool F32 = false, int KG = 1>
__global__ __launch_bounds__(256 * KG) void conv_lds_kernel(Args a) {
  static_assert(WAVES_M * WAVES_N == 4, "4 waves");
  static_assert(KG == 1 || KG == 2 || KG == 4, "KG");
  static_assert(BK == 32 || BK == 64, "BK");
  static_assert(!F32 || BK == 64, "F32: 64-wide staged rows ([hi 32 | lo 32])");
  constexpr int CPR = BK / 8;  // 16-byte chunks per staged row
  constexpr int WM = BM / WAVES_M / 16, WN = BN / WAVES_N / 16;
  constexpr int NA = BM * CPR / 256, NB = F32 ? BN * 4 / 256 : BN * CPR / 256;  // F32: 8-channel units
  static_assert(NA >= 1 && NB >= 1, "BM, BN must be multiples of 64");
  __shared__ uint4 lds_[KG * 2][(BM + BN) * CPR];

  const int kg = KG == 1 ? 0 : __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 8);
  uint4 (*lds)[(BM + BN) * CPR] = lds_ + kg * 2;  // this K group's double buffer
  const int t = threadIdx.x & 255, lane = t & 63, wave = t >> 6;
  const int wm = wave % WAVES_M, wn = wave / WAVES_M;
  const int bm0 = blockIdx.y * BM, bn0 = blockIdx.x * BN;
  const int m0 = bm0 + wm * WM * 16, n0 = bn0 + wn * WN * 16;
  const int H = a.H, W = a.W, KW = a.KW, PH = a.PH, PW = a.PW, Ktot = a.Ktot;
  const int taps = a.KH * KW;
  const int HW = H * W;
  // input grid and stride (GEO), else the output grid at stride 1
  const int Hi = GEO ? a.Hi : H, Wi = GEO ? a.Wi : W, SY = GEO ? a.SY : 1, SX = GEO ? a.SX : 1;

  // this thread's staging rows
  const bf16_t* arow[NA];
  int acol[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int id = t + 256 * i;
    arow[i] = a.w + (size_t)(bm0 + id / CPR) * taps * Ktot + (id % CPR) * 8;
    acol[i] = id % CPR;
  }
  constexpr int BCPR = F32 ? 4 : CPR;  // B staging units per row
  int sb[NB], sy[NB], sx[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int id = t + 256 * i;
    const int p = bn0 + id / BCPR;
    if (p < a.P) {
      sb[i] = p / HW;
      const int q = p - sb[i] * HW;
      sy[i] = q / W;
      sx[i] = q - sy[i] * W;
    } else {
      sb[i] = -1;
      sy[i] = sx[i] = 0;
    }
  }

  const Seg s0 = a.seg[0], s1 = a.seg[1], s2 = a.seg[2];
  constexpr int SH = (BK == 32 || F32) ? 5 : 6;  // input channels per K step: 32 (BK 32, F32) or 64
  constexpr int KSTEP = F32 ? 32 : BK;
  constexpr int WMUL = F32 ? 2 : 1;               // packed weight K per input channel ([wh | wl])
  const int e1 = taps * (s0.C >> SH);
  const int e2 = e1 + (a.nseg > 1 ? taps * (s1.C >> SH) : 0);
  const int nsteps = e2 + (a.nseg > 2 ? taps * (s2.C >> SH) : 0);
  const int nst = (nsteps + KG - 1) / KG;  // block-uniform trip count; a group's steps past the end stage zeros
  const uint4 zero = make_uint4(0, 0, 0, 0);

  uint4 ra[NA], rb[NB], rl[F32 ? NB : 1];
#define RS_GLOAD(STEP)                                                                          \
  do {                                                                                          \
    const int step_ = (STEP) * KG + kg;                                                         \
    if (KG > 1 && step_ >= nsteps) {                                                            \
      _Pragma("unroll") for (int i = 0; i < NA; ++i) ra[i] = zero;                              \
      _Pragma("unroll") for (int i = 0; i < NB; ++i) { rb[i] = zero; if constexpr (F32) rl[i] = zero; } \
      break;                                                                                    \
    }                                                                                           \
    const int si = (step_ >= e1) + (step_ >= e2);                                               \
    const bf16_t* sp = si == 0 ? s0.ptr : (si == 1 ? s1.ptr : s2.ptr);                          \
    const int sC = si == 0 ? s0.C : (si == 1 ? s1.C : s2.C);                                    \
    const int sst = si == 0 ? s0.stride : (si == 1 ? s1.stride : s2.stride);                    \
    const int kseg = si == 0 ? 0 : (si == 1 ? s0.C : s0.C + s1.C);                              \
    const int local = step_ - (si == 0 ? 0 : (si == 1 ? e1 : e2));                             \
    const int chunks = sC >> SH;                                                                \
    const int tap = local / chunks;                                                             \
    const int c0 = (local - tap * chunks) * KSTEP;                                              \
    const int dy = tap / KW - PH, dx = tap % KW - PW;                                           \
    _Pragma("unroll") for (int i = 0; i < NA; ++i)                                              \
      ra[i] = ld16(arow[i] + (size_t)tap * Ktot + (kseg + c0) * WMUL);                          \
    _Pragma("unroll") for (int i = 0; i < NB; ++i) {                                            \
      const int yy = sy[i] * SY + dy, xx = sx[i] * SX + dx;                                     \
      const bool ok = sb[i] >= 0 && yy >= 0 && yy < Hi && xx >= 0 && xx < Wi;                  \
      const size_t pix_ = (size_t)(sb[i] * Hi + yy) * Wi + xx;                                  \
      if constexpr (F32) {                                                                      \
        const float* fp_ = reinterpret_cast<const float*>(sp) + pix_ * sst + c0 + ((t + 256 * i) % 4) * 8; \
        float4 q0 = make_float4(0.f, 0.f, 0.f, 0.f), q1 = q0;                                   \
        if (ok) {                                                                               \
          q0 = *reinterpret_cast<const float4*>(fp_);                                           \
          q1 = *reinterpret_cast<const float4*>(fp_ + 4);                                       \
        }                                                                                       \
        split8(q0, q1, rb[i], rl[i]);                                                           \
      } else {                                                                                  \
        rb[i] = ok ? ld16(sp + pix_ * sst + c0 + ((t + 256 * i) % CPR) * 8) : zero;             \
      }                                                                                         \
    }                                                                                           \
  } while (0)
#define RS_LSTORE(BUF)                                                                          \
  do {                                                                                          \
    _Pragma("unroll") for (int i = 0; i < NA; ++i) {                                            \
      const int id = t + 256 * i;                                                               \
      lds[BUF][swz<CPR>(id / CPR, acol[i])] = ra[i];                                            \
    }                                                                                           \
    _Pragma("unroll") for (int i = 0; i < NB; ++i) {                                            \
      const int id = t + 256 * i;                                                               \
      if constexpr (F32) {  /* unit j of the row: hi -> chunk j, lo -> chunk j + 4 */           \
        lds[BUF][BM * CPR + swz<CPR>(id / 4, id % 4)] = rb[i];                                  \
        lds[BUF][BM * CPR + swz<CPR>(id / 4, id % 4 + 4)] = rl[i];                              \
      } else {                                                                                  \
        lds[BUF][BM * CPR + swz<CPR>(id / CPR, id % CPR)] = rb[i];                              \
      }                                                                                         \
    }                                                                                           \
  } while (0)

  f32x4_t acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int lr = lane & 15, lc = lane >> 4;
  RS_GLOAD(0);
  RS_LSTORE(0);
  __syncthreads();
  for (int step = 0; step < nst; ++step) {
    const int buf = step & 1;
    if (step + 1 < nst) RS_GLOAD(step + 1);
    // (A half, B half) per MFMA pass: bf16 -> the two 32-deep halves of the
    // 64-deep step; F32 -> (wh, xh), (wh, xl), (wl, xh)
    constexpr int NPASS = F32 ? 3 : BK / 32;
#pragma unroll
    for (int ps = 0; ps < NPASS; ++ps) {
      const int ka = F32 ? (ps == 2 ? 1 : 0) : ps, kb = F32 ? (ps == 1 ? 1 : 0) : ps;
      uint4 fa[WM], fb[WN];
#pragma unroll
      for (int mt = 0; mt < WM; ++mt) fa[mt] = lds[buf][swz<CPR>(wm * WM * 16 + mt * 16 + lr, ka * 4 + lc)];
#pragma unroll
      for (int nt = 0; nt < WN; ++nt)
        fb[nt] = lds[buf][BM * CPR + swz<CPR>(wn * WN * 16 + nt * 16 + lr, kb * 4 + lc)];
#pragma unroll
      for (int mt = 0; mt < WM; ++mt)
#pragma unroll
        for (int nt = 0; nt < WN; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[mt]),
                                                                __builtin_bit_cast(bf16x8_t, fb[nt]),
                                                                acc[mt][nt], 0, 0, 0);
    }
    if (step + 1 < nst) RS_LSTORE(buf ^ 1);
    __syncthreads();
  }
#undef RS_GLOAD
#undef RS_LSTORE
  if constexpr (KG > 1) {
    // groups 1.. park their partial tiles in LDS (free after the loop's last
    // barrier), group 0 adds them in group order
    constexpr int NE = WM * WN * 4;
    static_assert((KG - 1) * NE * 256 * 4 <= KG * 2 * (BM + BN) * CPR * 16, "split-K reduction buffer");
    float* red = reinterpret_cast<float*>(&lds_[0][0]);
    if (kg > 0) {
#pragma unroll
      for (int mt = 0; mt < WM; ++mt)
#pragma unroll
        for (int nt = 0; nt < WN; ++nt)
#pragma unroll
          for (int j = 0; j < 4; ++j) red[((kg - 1) * NE + (mt * WN + nt) * 4 + j) * 256 + t] = acc[mt][nt][j];
    }
    __syncthreads();
    if (kg > 0) return;
#pragma unroll
    for (int g = 0; g < KG - 1; ++g)
#pragma unroll
      for (int mt = 0; mt < WM; ++mt)
#pragma unroll
        for (int nt = 0; nt < WN; ++nt)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[mt][nt][j] += red[(g * NE + (mt * WN + nt) * 4 + j) * 256 + t];
  }

  int pb[WN], py[WN], px[WN];
#pragma unroll
  for (int nt = 0; nt < WN; ++nt) {
    const int p = n0 + nt * 16 + lr;
    if (p < a.P) {
      pb[nt] = p / HW;
      const int q = p - pb[nt] * HW;
      py[nt] = q / W;
      px[nt] = q - py[nt] * W;
    } else {
      pb[nt] = -1;
      py[nt] = px[nt] = 0;
    }
  }
  int pp[WN];
#pragma unroll
  for (int nt = 0; nt < WN; ++nt)
    pp[nt] = GEO ? (pb[nt] * a.oH + py[nt] * a.OSY + a.OOY) * a.oW + px[nt] * a.OSX + a.OOX
                 : n0 + nt * 16 + lr;
  if constexpr (F32)
    epilogue_pix_f32<WM, WN>(a, acc, m0, lane, pp, pb);
  else
    epilogue_pix<WM, WN>(a, acc, m0, lane, pp, pb, py, px);
}

// ------------------------------------------------------------------ direct-to-LDS variant
// Same tile as conv_lds_kernel (BM output channels x BN pixels, 64-deep K
// steps, st-XOR-swizzled 128-B LDS rows) but the tiles are copied global ->
// LDS by global_load_lds_dwordx4 (no VGPR round trip, no ds_write), through a
// 3-stage ring: loads of step k+2 are issued while step k is computed, and a
// counted `s_waitcnt vmcnt` retires only step k's copies before the barrier.
// The LDS destination of one wave-instruction is lane-linear, so the swizzle
// is applied to the per-lane SOURCE chunk instead.  Out-of-image pixels read a
// zero page.  Blocks are remapped so that each XCD (private L2) walks a
// contiguous run of pixel tiles with all their output-channel tiles: the
// halo rows of neighbouring tiles and the activation panel shared by the
// Cout tiles of one pixel tile are L2 hits instead of cross-XCD refetches.
__device__ uint4 g_zero_page[8];
template <int BM, int BN, int WAVES_M, int WAVES_N, int BK, int STAGES>
__global__ __launch_bounds__(256) void conv_glds_kernel(Args a) {
  static_assert(WAVES_M * WAVES_N == 4, "4 waves");
  static_assert(BK == 32 || BK == 64, "BK");
  static_assert(STAGES >= 2 && STAGES <= 4, "STAGES");
  constexpr int CPR = BK / 8;     // 16-B chunks per LDS row
  constexpr int RB = CPR * 16;    // LDS row bytes
  constexpr int SH = BK == 32 ? 5 : 6;
  constexpr int WM = BM / WAVES_M / 16, WN = BN / WAVES_N / 16;
  constexpr int NA = BM * CPR / 256, NB = BN * CPR / 256;
  constexpr int NLD = NA + NB;    // DMA instructions per thread per K step
  static_assert(NA >= 1 && NB >= 1, "tile too small for 256 threads");
  __shared__ uint4 lds[STAGES][(BM + BN) * CPR];

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave % WAVES_M, wn = wave / WAVES_M;
  const int nct = cdiv(a.Cout, BM);
  const int lid = a.xcd_remap ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int bm0 = (lid % nct) * BM, bn0 = (lid / nct) * BN;
  const int m0 = bm0 + wm * WM * 16, n0 = bn0 + wn * WN * 16;
  const int H = a.H, W = a.W, KW = a.KW, PH = a.PH, PW = a.PW, Ktot = a.Ktot;
  const int taps = a.KH * KW;
  const int HW = H * W;

  // staging: thread t, instruction i fills LDS chunk id = t + 256 i, i.e.
  // row id / CPR at physical slot id % CPR, which holds the logical chunk
  // slot ^ xor(row) of swz<CPR>
  auto xrow = [](int r) { return CPR == 4 ? (r >> 2) & 3 : (r >> 1) & 7; };
  const bf16_t* arow[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int id = t + 256 * i, r = id / CPR;
    arow[i] = a.w + (size_t)(bm0 + r) * taps * Ktot + (((id % CPR) ^ xrow(r)) * 8);
  }
  int sb[NB], sy[NB], sx[NB], sc[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int id = t + 256 * i, r = id / CPR;
    const int p = bn0 + r;
    sc[i] = ((id % CPR) ^ xrow(r)) * 8;
    if (p < a.P) {
      sb[i] = p / HW;
      const int q = p - sb[i] * HW;
      sy[i] = q / W;
      sx[i] = q - sy[i] * W;
    } else {
      sb[i] = -1;
      sy[i] = sx[i] = 0;
    }
  }
  const int wbase = wave * 64;

  const Seg s0 = a.seg[0], s1 = a.seg[1], s2 = a.seg[2];
  const int e1 = taps * (s0.C >> SH);
  const int e2 = e1 + (a.nseg > 1 ? taps * (s1.C >> SH) : 0);
  const int nsteps = e2 + (a.nseg > 2 ? taps * (s2.C >> SH) : 0);

#define RS_ISSUE(STEP, BUF)                                                                     \
  do {                                                                                          \
    const int step_ = (STEP);                                                                   \
    const int si = (step_ >= e1) + (step_ >= e2);                                               \
    const bf16_t* sp = si == 0 ? s0.ptr : (si == 1 ? s1.ptr : s2.ptr);                          \
    const int sC = si == 0 ? s0.C : (si == 1 ? s1.C : s2.C);                                    \
    const int sst = si == 0 ? s0.stride : (si == 1 ? s1.stride : s2.stride);                    \
    const int kseg = si == 0 ? 0 : (si == 1 ? s0.C : s0.C + s1.C);                              \
    const int local = step_ - (si == 0 ? 0 : (si == 1 ? e1 : e2));                             \
    const int chunks = sC >> SH;                                                                \
    const int tap = local / chunks;                                                             \
    const int c0 = (local - tap * chunks) * BK;                                                 \
    const int dy = tap / KW - PH, dx = tap % KW - PW;                                           \
    uint4* dst_ = lds[BUF];                                                                     \
    _Pragma("unroll") for (int i = 0; i < NA; ++i)                                              \
      glds16(arow[i] + (size_t)tap * Ktot + kseg + c0, dst_ + wbase + 256 * i);                 \
    _Pragma("unroll") for (int i = 0; i < NB; ++i) {                                            \
      const int yy = sy[i] + dy, xx = sx[i] + dx;                                               \
      const bool ok = sb[i] >= 0 && yy >= 0 && yy < H && xx >= 0 && xx < W;                    \
      const void* src_ = ok ? (const void*)(sp + ((size_t)(sb[i] * H + yy) * W + xx) * sst + c0 + sc[i]) \
                            : (const void*)g_zero_page;                                         \
      glds16(src_, dst_ + BM * CPR + wbase + 256 * i);                                          \
    }                                                                                           \
  } while (0)

  f32x4_t acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int lr = lane & 15, lc = lane >> 4;
  // Fragment reads are inline-asm ds_read_b128: the compiler cannot prove
  // they miss the in-flight LDS DMA and would otherwise drain vmcnt to 0 in
  // front of them, collapsing the ring to one step of lookahead.  For this
  // lane the row XOR term is xrow(lr) (tile rows start at multiples of 16).
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) uint4*)&lds[0][0];
  constexpr uint32_t kStage = (BM + BN) * RB;
  constexpr int KK = BK / 32;
  uint32_t abase[KK], bbase[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) {
    abase[kk] = lds0 + (uint32_t)((wm * WM * 16 + lr) * RB + (((kk * 4 + lc) ^ xrow(lr)) * 16));
    bbase[kk] = lds0 + (uint32_t)(BM * RB + (wn * WN * 16 + lr) * RB + (((kk * 4 + lc) ^ xrow(lr)) * 16));
  }
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nsteps) RS_ISSUE(s, s);
  int buf = 0;
  for (int step = 0; step < nsteps; ++step) {
    // retire this step's copies; keep up to STAGES-2 later steps in flight
    const int ahead = min(STAGES - 2, nsteps - 1 - step);
    if (STAGES >= 4 && ahead >= 2) wait_vmcnt<2 * NLD>();
    else if (STAGES >= 3 && ahead >= 1) wait_vmcnt<NLD>();
    else wait_vmcnt<0>();
    asm volatile("s_barrier" ::: "memory");  // all waves' copies landed; buffer step-1 is free
    const uint32_t so = buf * kStage;
    u32x4_t fa[KK][WM], fb[KK][WN];
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
#pragma unroll
      for (int mt = 0; mt < WM; ++mt)
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(fa[kk][mt]) : "v"(abase[kk] + so), "i"(mt * 16 * RB)
                     : "memory");
#pragma unroll
      for (int nt = 0; nt < WN; ++nt)
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(fb[kk][nt]) : "v"(bbase[kk] + so), "i"(nt * 16 * RB)
                     : "memory");
    }
    if (step + STAGES - 1 < nsteps) RS_ISSUE(step + STAGES - 1, buf == 0 ? STAGES - 1 : buf - 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
#pragma unroll
      for (int mt = 0; mt < WM; ++mt) asm volatile("" : "+v"(fa[kk][mt]));
#pragma unroll
      for (int nt = 0; nt < WN; ++nt) asm volatile("" : "+v"(fb[kk][nt]));
    }
#pragma unroll
    for (int kk = 0; kk < KK; ++kk)
#pragma unroll
      for (int mt = 0; mt < WM; ++mt)
#pragma unroll
        for (int nt = 0; nt < WN; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[kk][mt]),
                                                                __builtin_bit_cast(bf16x8_t, fb[kk][nt]),
                                                                acc[mt][nt], 0, 0, 0);
    buf = buf == STAGES - 1 ? 0 : buf + 1;
  }
#undef RS_ISSUE

  int pb[WN], py[WN], px[WN];
#pragma unroll
  for (int nt = 0; nt < WN; ++nt) {
    const int p = n0 + nt * 16 + lr;
    if (p < a.P) {
      pb[nt] = p / HW;
      const int q = p - pb[nt] * HW;
      py[nt] = q / W;
      px[nt] = q - py[nt] * W;
    } else {
      pb[nt] = -1;
      py[nt] = px[nt] = 0;
    }
  }
  epilogue<WM, WN>(a, acc, m0, n0, lane, pb, py, px);
}

// ------------------------------------------------------------------ buffer-DMA variant
// conv_glds_kernel spends most of its issue slots on per-lane address
// arithmetic (segment / tap / chunk decode with integer divisions, 64-bit
// pointer math and bounds tests for every staged row at every K step): with
// one or two waves per SIMD that VALU work, not the MFMAs, set the step time.
// Here the per-step work is almost all scalar:
//  * the (segment, tap, chunk) walk is a scalar counter, no divisions;
//  * tiles are copied with buffer_load_dwordx4 ... lds through per-segment
//    buffer descriptors: the weight tile's step offset is the scalar SOFFSET
//    (zero VALU per A row), a pixel row's offset is its precomputed base + the
//    scalar tap shift (one add);
//  * zero padding: each staged pixel row keeps a bitmask of the taps that
//    land inside the image (built once per block); a row outside gets an
//    offset past the buffer's end, which the buffer unit returns as zeros.

// 4 or 8 waves.  8-wave tiles (256x96, 192x96, 128x96) are sized for the
// training shape (P = 22816): one block per CU covers the whole pixel range in
// ~one round, and every staged byte feeds 1.6x more MFMA work than the 4-wave
// 128x64 tile with 3 blocks per CU (the kernel is L2->LDS bound there,
// profiles/conv_tiles_r1.md).  When BN*8 chunks are not a multiple of the
// thread count, the last B staging instruction of the surplus waves is a
// zero-fill of a 1 KiB pad (every wave issues the same number of loads, so
// the vmcnt bookkeeping stays uniform).
//
// KG > 1: intra-block split-K for small grids (batch-1 inference: 7480 pixels,
// ~470 64x64 tiles for 256 CUs, < 2 waves per SIMD, every K step waits on
// L2 latency).  The block holds KG groups of WAVES_M x WAVES_N waves over the
// SAME output tile; group g stages and multiplies K steps g, g + KG, ... into
// its own slice of each stage buffer, so KG x as many waves and loads are in
// flight per tile and the serial K loop is KG x shorter.  At the end groups
// 1..KG-1 park their accumulators in LDS and group 0 sums them (fixed order)
// and runs the epilogue.
template <int BM, int BN, int WAVES_M, int WAVES_N, int STAGES, int KG = 1>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N * KG) void conv_buf_kernel(Args a) {
  constexpr int NT = 64 * WAVES_M * WAVES_N;  // threads per K group
  static_assert(NT == 256 || NT == 512, "4 or 8 waves");
  static_assert(KG == 1 || KG == 2 || KG == 4, "KG");
  static_assert(STAGES >= 2 && STAGES <= 4, "STAGES");
  constexpr int BK = 64, CPR = 8, RB = 128;
  static_assert(BM % (WAVES_M * 16) == 0 && BN % (WAVES_N * 16) == 0, "wave tiles");
  constexpr int WM = BM / WAVES_M / 16, WN = BN / WAVES_N / 16;
  static_assert((BM * CPR) % NT == 0, "A staging");
  constexpr int NBC = BN * CPR;                 // B chunks per stage
  constexpr int NA = BM * CPR / NT, NB = (NBC + NT - 1) / NT;
  constexpr bool BPART = (NBC % NT) != 0;       // last B instruction only partly real
  constexpr int PAD = BPART ? 64 : 0;
  constexpr int NLD = NA + NB;
  constexpr int kFar = 0x7ffffff0;  // past every buffer: reads as zero
  constexpr int GSLOT = (BM + BN) * CPR + PAD;  // uint4 slots of one K group's slice of a stage
  __shared__ uint4 lds[STAGES][KG * GSLOT];

  const int kg = KG == 1 ? 0 : __builtin_amdgcn_readfirstlane((int)threadIdx.x / NT);
  const int t = threadIdx.x - kg * NT, lane = t & 63, wave = t >> 6;  // within the K group
  const int wm = wave % WAVES_M, wn = wave / WAVES_M;
  const int nct = cdiv(a.Cout, BM);
  const int lid = a.xcd_remap ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int bm0 = (lid % nct) * BM, bn0 = (lid / nct) * BN;
  const int m0 = bm0 + wm * WM * 16, n0 = bn0 + wn * WN * 16;
  const int H = a.H, W = a.W, KW = a.KW, Ktot = a.Ktot;
  const int taps = a.KH * KW;
  const int HW = H * W;

  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, a.w_bytes, 0x00020000);
  const Seg s0 = a.seg[0], s1 = a.seg[1], s2 = a.seg[2];
  const __amdgpu_buffer_rsrc_t rs0 =
      __builtin_amdgcn_make_buffer_rsrc((void*)s0.ptr, (short)0, a.seg_bytes[0], 0x00020000);
  const __amdgpu_buffer_rsrc_t rs1 =
      __builtin_amdgcn_make_buffer_rsrc((void*)s1.ptr, (short)0, a.seg_bytes[1], 0x00020000);
  const __amdgpu_buffer_rsrc_t rs2 =
      __builtin_amdgcn_make_buffer_rsrc((void*)s2.ptr, (short)0, a.seg_bytes[2], 0x00020000);

  // staging slot (thread t, instruction i) = LDS chunk t + 256 i: row r, physical
  // slot id % 8 holding logical chunk slot ^ ((r >> 1) & 7)  (swz<8>)
  int aoff[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int id = t + NT * i, r = id / CPR;
    aoff[i] = ((bm0 + r) * taps * Ktot + (((id % CPR) ^ ((r >> 1) & 7)) * 8)) * 2;
  }
  // pixel rows: offset (elements, stride-free) of pixel (y - PH, x - PW) and the valid-tap mask
  int bpix[NB], bch[NB];
  unsigned bmask[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int id = t + NT * i, r = id / CPR;
    const int p = bn0 + r;
    bch[i] = ((id % CPR) ^ ((r >> 1) & 7)) * 8;
    bmask[i] = 0u;
    bpix[i] = 0;
    if (p < a.P && id < NBC) {
      const int b = p / HW, q = p - b * HW, y = q / W, x = q - y * W;
      bpix[i] = (b * H + y - a.PH) * W + (x - a.PW);
      for (int tp = 0, ty = 0, tx = 0; tp < taps; ++tp) {
        const int yy = y + ty - a.PH, xx = x + tx - a.PW;
        if (yy >= 0 && yy < H && xx >= 0 && xx < W) bmask[i] |= 1u << tp;
        if (++tx == KW) { tx = 0; ++ty; }
      }
    }
  }
  const int wbase = wave * 64;
  const int e1 = taps * (s0.C >> 6);
  const int e2 = e1 + (a.nseg > 1 ? taps * (s1.C >> 6) : 0);
  const int nsteps = e2 + (a.nseg > 2 ? taps * (s2.C >> 6) : 0);
  const int nst = (nsteps + KG - 1) / KG;  // stages; stage s holds K steps s * KG + (0 .. KG-1)

  // scalar walk of this group's K steps: segment si, tap (ty, tx), channel chunk c0
  int si = 0, tap = 0, ty = 0, tx = 0, c0 = 0, kseg = 0, kstep = 0;
#define RS_BADV()                                                                               \
  do {                                                                                          \
    const int sC_ = si == 0 ? s0.C : (si == 1 ? s1.C : s2.C);                                   \
    ++kstep;                                                                                    \
    c0 += BK;                                                                                   \
    if (c0 == sC_) {                                                                            \
      c0 = 0;                                                                                   \
      ++tap;                                                                                    \
      if (++tx == KW) { tx = 0; ++ty; }                                                         \
      if (tap == taps) { tap = 0; ty = 0; kseg += sC_; ++si; }                                  \
    }                                                                                           \
  } while (0)
  for (int g = 0; g < kg; ++g) RS_BADV();
  // (a macro, not a lambda: capturing the staging arrays by reference would
  // take their address and move them to scratch).  A K step past the end
  // (the last stage of a split walk) stages zeros: every wave still issues
  // NLD loads per stage, so the vmcnt bookkeeping stays uniform.
#define RS_BISSUE(BUF)                                                                          \
  do {                                                                                          \
    const bool live_ = kstep < nsteps;                                                          \
    const int sst = si == 0 ? s0.stride : (si == 1 ? s1.stride : s2.stride);                    \
    const __amdgpu_buffer_rsrc_t rb = si == 0 ? rs0 : (si == 1 ? rs1 : rs2);                    \
    uint4* dst = lds[BUF] + kg * GSLOT;                                                         \
    const int asoff = live_ ? (tap * Ktot + kseg + c0) * 2 : 0;                                 \
    _Pragma("unroll") for (int i = 0; i < NA; ++i)                                              \
      bdma16(rw, dst + wbase + NT * i, live_ ? aoff[i] : kFar, asoff);                          \
    const int tsh = ty * W + tx;                                                                \
    _Pragma("unroll") for (int i = 0; i < NB; ++i) {                                            \
      const int v = (live_ && ((bmask[i] >> tap) & 1u)) ? ((bpix[i] + tsh) * sst + c0 + bch[i]) * 2 : kFar; \
      const bool pad = BPART && i == NB - 1 && wbase + NT * i >= NBC;                           \
      bdma16(rb, dst + BM * CPR + (pad ? NBC : wbase + NT * i), v, 0);                          \
    }                                                                                           \
    _Pragma("unroll") for (int g_ = 0; g_ < KG; ++g_) RS_BADV(); /* this group's next K step */ \
  } while (0)


  f32x4_t acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int lr = lane & 15, lc = lane >> 4;
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) uint4*)&lds[0][0] + kg * GSLOT * 16;
  constexpr uint32_t kStage = KG * GSLOT * 16;
  uint32_t abase[2], bbase[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    abase[kk] = lds0 + (uint32_t)((wm * WM * 16 + lr) * RB + (((kk * 4 + lc) ^ ((lr >> 1) & 7)) * 16));
    bbase[kk] = lds0 + (uint32_t)(BM * RB + (wn * WN * 16 + lr) * RB + (((kk * 4 + lc) ^ ((lr >> 1) & 7)) * 16));
  }
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nst) RS_BISSUE(s);
  int buf = 0;
  for (int step = 0; step < nst; ++step) {
    // retire this step's copies; keep up to STAGES-2 later steps in flight
    const int ahead = min(STAGES - 2, nst - 1 - step);
    if (STAGES >= 4 && ahead >= 2) wait_vmcnt<2 * NLD>();
    else if (STAGES >= 3 && ahead >= 1) wait_vmcnt<NLD>();
    else wait_vmcnt<0>();
    asm volatile("s_barrier" ::: "memory");
    const uint32_t so = buf * kStage;
    u32x4_t fa[2][WM], fb[2][WN];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int mt = 0; mt < WM; ++mt)
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(fa[kk][mt]) : "v"(abase[kk] + so), "i"(mt * 16 * RB)
                     : "memory");
#pragma unroll
      for (int nt = 0; nt < WN; ++nt)
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(fb[kk][nt]) : "v"(bbase[kk] + so), "i"(nt * 16 * RB)
                     : "memory");
    }
    if (step + STAGES - 1 < nst) RS_BISSUE(buf == 0 ? STAGES - 1 : buf - 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int mt = 0; mt < WM; ++mt) asm volatile("" : "+v"(fa[kk][mt]));
#pragma unroll
      for (int nt = 0; nt < WN; ++nt) asm volatile("" : "+v"(fb[kk][nt]));
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int mt = 0; mt < WM; ++mt)
#pragma unroll
        for (int nt = 0; nt < WN; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[kk][mt]),
                                                                __builtin_bit_cast(bf16x8_t, fb[kk][nt]),
                                                                acc[mt][nt], 0, 0, 0);
    buf = buf == STAGES - 1 ? 0 : buf + 1;
  }

#undef RS_BISSUE
#undef RS_BADV
  if constexpr (KG > 1) {
    // groups 1.. park their partial tiles in the (now free) stage buffers,
    // lane-linear per accumulator element; group 0 adds them in group order
    constexpr int NE = WM * WN * 4;  // accumulator floats per lane
    static_assert((KG - 1) * NE * NT * 4 <= STAGES * KG * GSLOT * 16, "split-K reduction buffer");
    float* red = reinterpret_cast<float*>(&lds[0][0]);
    __syncthreads();  // every wave is done with the stage buffers
    if (kg > 0) {
#pragma unroll
      for (int mt = 0; mt < WM; ++mt)
#pragma unroll
        for (int nt = 0; nt < WN; ++nt)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            red[((size_t)((kg - 1) * NE + (mt * WN + nt) * 4 + j) * NT) + t] = acc[mt][nt][j];
    }
    __syncthreads();
    if (kg > 0) return;
#pragma unroll
    for (int g = 0; g < KG - 1; ++g)
#pragma unroll
      for (int mt = 0; mt < WM; ++mt)
#pragma unroll
        for (int nt = 0; nt < WN; ++nt)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[mt][nt][j] += red[((size_t)(g * NE + (mt * WN + nt) * 4 + j) * NT) + t];
  }

  int pb[WN], py[WN], px[WN];
#pragma unroll
  for (int nt = 0; nt < WN; ++nt) {
    const int p = n0 + nt * 16 + lr;
    if (p < a.P) {
      pb[nt] = p / HW;
      const int q = p - pb[nt] * HW;
      py[nt] = q / W;
      px[nt] = q - py[nt] * W;
    } else {
      pb[nt] = -1;
      py[nt] = px[nt] = 0;
    }
  }
  epilogue<WM, WN>(a, acc, m0, n0, lane, pb, py, px);
}

// ------------------------------------------------------------------ halo (patch) variant
// conv_buf_kernel stages a fresh BN-pixel x 64-channel tile for EVERY (tap,
// chunk) K step: a 3x3 conv fetches each input row 9 times from L2, and at
// the training shape the kernel runs at the L2 -> LDS rate (~11 TB/s,
// profiles/conv_tiles_r1.md), not at the MFMA rate.  Here the pixel tile is a
// TH x 16 patch of ONE image.  Per 64-channel chunk the block stages the
// patch's (TH+KH-1) x (16+KW-1) halo once -- pixels outside the image read
// past the buffer end, i.e. as zeros, so padding needs no per-tap masks --
// and every tap reads its shifted window of it from LDS.  Per K step only the
// weight tile is fetched; the halo costs ~1/taps of a pixel tile.
// K walk: segment -> chunk -> tap (tap innermost).  Two-stage weight ring;
// the halo is double-buffered and issued together with the weights of its
// chunk's first tap (one step ahead); the buffer it overwrites was last read
// two chunks back, i.e. before the previous step's barrier.
template <int BM, int TH, int HCAP>
__global__ __launch_bounds__(256) void conv_halo_kernel(Args a) {
  constexpr int TW = 16, BN = TH * TW;
  constexpr int WM = BM / 2 / 16, WN = BN / 2 / 16;  // 2 x 2 waves
  constexpr int NA = BM * 8 / 256, NH = HCAP * 8 / 256;
  constexpr int AST = BM * 8, HST = HCAP * 8;  // 16-B chunks per weight stage / halo buffer
  constexpr int kFar = 0x7ffffff0;
  __shared__ uint4 lds[2 * AST + 2 * HST];

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int H = a.H, W = a.W, KW = a.KW, Ktot = a.Ktot;
  const int taps = a.KH * KW;
  const int hw = TW + KW - 1;               // halo row width
  const int hrows = (TH + a.KH - 1) * hw;   // halo pixels (<= HCAP, host-checked)
  const int ntx = cdiv(W, TW), npb = cdiv(H, TH) * ntx;
  const int nct = cdiv(a.Cout, BM);
  const int lid = a.xcd_remap ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int bm0 = (lid % nct) * BM;
  const int pt = lid / nct;
  const int img = pt / npb, pq = pt - img * npb;
  const int pty = pq / ntx;
  const int y0 = pty * TH, x0 = (pq - pty * ntx) * TW;
  const int m0 = bm0 + wm * WM * 16;

  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, a.w_bytes, 0x00020000);
  const Seg s0 = a.seg[0], s1 = a.seg[1], s2 = a.seg[2];
  const __amdgpu_buffer_rsrc_t rs0 =
      __builtin_amdgcn_make_buffer_rsrc((void*)s0.ptr, (short)0, a.seg_bytes[0], 0x00020000);
  const __amdgpu_buffer_rsrc_t rs1 =
      __builtin_amdgcn_make_buffer_rsrc((void*)s1.ptr, (short)0, a.seg_bytes[1], 0x00020000);
  const __amdgpu_buffer_rsrc_t rs2 =
      __builtin_amdgcn_make_buffer_rsrc((void*)s2.ptr, (short)0, a.seg_bytes[2], 0x00020000);

  // staging slot (thread t, instruction i) = chunk t + 256 i: row r = slot / 8,
  // physical 16-B slot holding logical chunk (slot % 8) ^ ((r >> 1) & 7)
  int aoff[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int id = t + 256 * i, r = id >> 3;
    aoff[i] = ((bm0 + r) * taps * Ktot + (((id & 7) ^ ((r >> 1) & 7)) * 8)) * 2;
  }
  int hpix[NH], hch[NH];
#pragma unroll
  for (int i = 0; i < NH; ++i) {
    const int id = t + 256 * i, r = id >> 3;
    hch[i] = ((id & 7) ^ ((r >> 1) & 7)) * 8;
    hpix[i] = -1;
    if (r < hrows) {
      const int hy = r / hw, hx = r - hy * hw;
      const int y = y0 + hy - a.PH, x = x0 + hx - a.PW;
      if (y >= 0 && y < H && x >= 0 && x < W) hpix[i] = (img * H + y) * W + x;
    }
  }
  const int wbase = wave * 64;
  const int nsteps =
      taps * ((s0.C >> 6) + (a.nseg > 1 ? (s1.C >> 6) : 0) + (a.nseg > 2 ? (s2.C >> 6) : 0));

  // issue-side scalar walk: segment si, channel chunk c0, tap itap
  int si = 0, c0 = 0, kseg = 0, itap = 0, ichunk = 0, istep = 0;
#define RS_HISSUE()                                                                                 \
  do {                                                                                              \
    const int sC = si == 0 ? s0.C : (si == 1 ? s1.C : s2.C);                                        \
    if (itap == 0) {                                                                                \
      const int sst = si == 0 ? s0.stride : (si == 1 ? s1.stride : s2.stride);                      \
      const __amdgpu_buffer_rsrc_t rb = si == 0 ? rs0 : (si == 1 ? rs1 : rs2);                      \
      uint4* hd = lds + 2 * AST + (ichunk & 1) * HST;                                               \
      _Pragma("unroll") for (int i = 0; i < NH; ++i) {                                              \
        const int v = hpix[i] >= 0 ? (hpix[i] * sst + c0 + hch[i]) * 2 : kFar;                      \
        bdma16(rb, hd + wbase + 256 * i, v, 0);                                                     \
      }                                                                                             \
    }                                                                                               \
    uint4* ad = lds + (istep & 1) * AST;                                                            \
    const int asoff = (itap * Ktot + kseg + c0) * 2;                                                \
    _Pragma("unroll") for (int i = 0; i < NA; ++i) bdma16(rw, ad + wbase + 256 * i, aoff[i], asoff); \
    ++istep;                                                                                        \
    if (++itap == taps) {                                                                           \
      itap = 0;                                                                                     \
      ++ichunk;                                                                                     \
      c0 += 64;                                                                                     \
      if (c0 == sC) { c0 = 0; kseg += sC; ++si; }                                                   \
    }                                                                                               \
  } while (0)

  f32x4_t acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int lr = lane & 15, lc = lane >> 4;
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) uint4*)&lds[0];
  uint32_t abase[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
    abase[kk] = lds0 + (uint32_t)((wm * WM * 16 + lr) * 128 + (((kk * 4 + lc) ^ ((lr >> 1) & 7)) * 16));
  int rbn[WN];  // halo row of this lane's pixel (patch row wn*WN + nt, column lr) at tap (0, 0)
#pragma unroll
  for (int nt = 0; nt < WN; ++nt) rbn[nt] = (wn * WN + nt) * hw + lr;

  RS_HISSUE();
  int ctap = 0, cty = 0, ctx = 0, cchunk = 0;
  for (int step = 0; step < nsteps; ++step) {
    wait_vmcnt<0>();
    asm volatile("s_barrier" ::: "memory");  // step's weights + halo landed; buffers of step-1 free
    const uint32_t so = (step & 1) * AST * 16;
    const uint32_t hb = lds0 + (uint32_t)((2 * AST + (cchunk & 1) * HST) * 16);
    const int toff = cty * hw + ctx;
    uint32_t brow[WN], bsw[WN];
#pragma unroll
    for (int nt = 0; nt < WN; ++nt) {
      const int row = rbn[nt] + toff;
      brow[nt] = hb + (uint32_t)(row * 128);
      bsw[nt] = (uint32_t)((row >> 1) & 7);
    }
    u32x4_t fa[2][WM], fb[2][WN];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int mt = 0; mt < WM; ++mt)
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(fa[kk][mt]) : "v"(abase[kk] + so), "i"(mt * 16 * 128)
                     : "memory");
#pragma unroll
      for (int nt = 0; nt < WN; ++nt)
        asm volatile("ds_read_b128 %0, %1" : "=v"(fb[kk][nt])
                     : "v"(brow[nt] + ((((uint32_t)(kk * 4 + lc)) ^ bsw[nt]) << 4)) : "memory");
    }
    if (step + 1 < nsteps) RS_HISSUE();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int mt = 0; mt < WM; ++mt) asm volatile("" : "+v"(fa[kk][mt]));
#pragma unroll
      for (int nt = 0; nt < WN; ++nt) asm volatile("" : "+v"(fb[kk][nt]));
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int mt = 0; mt < WM; ++mt)
#pragma unroll
        for (int nt = 0; nt < WN; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[kk][mt]),
                                                                __builtin_bit_cast(bf16x8_t, fb[kk][nt]),
                                                                acc[mt][nt], 0, 0, 0);
    if (++ctx == KW) { ctx = 0; ++cty; }
    if (++ctap == taps) { ctap = 0; cty = 0; ctx = 0; ++cchunk; }
  }
#undef RS_HISSUE

  int pp[WN], pb[WN], py[WN], px[WN];
#pragma unroll
  for (int nt = 0; nt < WN; ++nt) {
    const int y = y0 + wn * WN + nt, x = x0 + lr;
    if (y < H && x < W) {
      pb[nt] = img;
      py[nt] = y;
      px[nt] = x;
      pp[nt] = (img * H + y) * W + x;
    } else {
      pb[nt] = -1;
      py[nt] = px[nt] = pp[nt] = 0;
    }
  }
  epilogue_pix<WM, WN>(a, acc, m0, lane, pp, pb, py, px);
}

// ------------------------------------------------------------------ small-N variant
// Cout <= 16 (the flow head's 256 -> 2 conv): one 16x16 output tile per block
// (16 pixels), the K steps split over the 4 waves (step = wave mod 4), partial
// accumulators reduced through LDS, epilogue by wave 0.  Without the K split
// such a conv is one long dependent MFMA chain per 16 pixels.
__global__ __launch_bounds__(256) void conv_smalln_kernel(Args a) {
  __shared__ f32x4_t red[4][64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int n0 = blockIdx.x * 16;
  const int H = a.H, W = a.W, KW = a.KW, PH = a.PH, PW = a.PW, Ktot = a.Ktot;
  const int taps = a.KH * KW;
  const int HW = H * W;
  const int lr = lane & 15, lk = (lane >> 4) * 8;
  int pb[1], py[1], px[1];
  {
    const int p = n0 + lr;
    if (p < a.P) {
      pb[0] = p / HW;
      const int q = p - pb[0] * HW;
      py[0] = q / W;
      px[0] = q - py[0] * W;
    } else {
      pb[0] = -1;
      py[0] = px[0] = 0;
    }
  }
  const bf16_t* wrow = a.w + (size_t)lr * taps * Ktot + lk;
  const Seg s0 = a.seg[0], s1 = a.seg[1], s2 = a.seg[2];
  const int e1 = taps * (s0.C >> 5);
  const int e2 = e1 + (a.nseg > 1 ? taps * (s1.C >> 5) : 0);
  const int nsteps = e2 + (a.nseg > 2 ? taps * (s2.C >> 5) : 0);
  const uint4 zero = make_uint4(0, 0, 0, 0);
  f32x4_t acc[1][1];
  acc[0][0] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  for (int step = wave; step < nsteps; step += 4) {
    const int si = (step >= e1) + (step >= e2);
    const bf16_t* sp = si == 0 ? s0.ptr : (si == 1 ? s1.ptr : s2.ptr);
    const int sC = si == 0 ? s0.C : (si == 1 ? s1.C : s2.C);
    const int sst = si == 0 ? s0.stride : (si == 1 ? s1.stride : s2.stride);
    const int kseg = si == 0 ? 0 : (si == 1 ? s0.C : s0.C + s1.C);
    const int local = step - (si == 0 ? 0 : (si == 1 ? e1 : e2));
    const int chunks = sC >> 5;
    const int tap = local / chunks;
    const int c0 = (local - tap * chunks) * 32;
    const int dy = tap / KW - PH, dx = tap % KW - PW;
    const uint4 fa = ld16(wrow + (size_t)tap * Ktot + kseg + c0);
    const int yy = py[0] + dy, xx = px[0] + dx;
    const bool ok = pb[0] >= 0 && yy >= 0 && yy < H && xx >= 0 && xx < W;
    const uint4 fb = ok ? ld16(sp + ((size_t)(pb[0] * H + yy) * W + xx) * sst + c0 + lk) : zero;
    acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa),
                                                        __builtin_bit_cast(bf16x8_t, fb), acc[0][0], 0, 0, 0);
  }
  red[wave][lane] = acc[0][0];
  __syncthreads();
  if (wave == 0) {
    acc[0][0] = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
    epilogue<1, 1>(a, acc, 0, n0, lane, pb, py, px);
  }
}

// ------------------------------------------------------------------ GRU gate backward
// One ConvGRU pass h' = (1-z) h + z q~, q~ = tanh(q_pre), z = sigmoid(z_pre):
//   dq_pre = dh' z (1 - q~^2)        -> dq (bf16, the q-conv dgrad/wgrad operand)
//   dz_pre = dh' (q~ - h) z (1 - z)  -> dzr[:, 0:hd] (bf16)
//   dh    <- dh' (1 - z)             (fp32, in place; the conv dgrads add to it)
// T: the activations' type (bf16, or fp32 in the fp32 training engine).
template <typename T>
__global__ __launch_bounds__(256) void gru_gate_bwd_kernel(float* __restrict__ dh, int dhstr, const T* __restrict__ z,
                                                           int zstr, const T* __restrict__ q, int qstr,
                                                           const T* __restrict__ h, int hstr, int hoff,
                                                           T* __restrict__ dq, int dqstr,
                                                           T* __restrict__ dzr, int dzrstr, long P, int hd) {
  const long total = P * hd;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long p = i / hd;
    const int c = (int)(i - p * hd);
    const float g = dh[p * dhstr + c];
    const float zv = io<T>::ld(z + p * zstr + c), qv = io<T>::ld(q + p * qstr + c);
    const float hv = io<T>::ld(h + p * hstr + hoff + c);
    io<T>::st(dq + p * dqstr + c, g * zv * (1.f - qv * qv));
    io<T>::st(dzr + p * dzrstr + c, g * (qv - hv) * zv * (1.f - zv));
    dh[p * dhstr + c] = g * (1.f - zv);
  }
}

// Motion-encoder output gradient: d = G[:, off:off+n] * (act > 0) -> out (T, width
// ostr, channels >= n zeroed), then G[:, off:off+nz] = 0 (consumed).
template <typename T>
__global__ __launch_bounds__(256) void relu_take_kernel(float* __restrict__ G, int gstr, int goff, int n, int nz,
                                                        const T* __restrict__ act, int astr, int aoff,
                                                        T* __restrict__ out, int ostr, long P) {
  const long total = P * ostr;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long p = i / ostr;
    const int c = (int)(i - p * ostr);
    float v = 0.f;
    if (c < n) {
      const float g = G[p * gstr + goff + c];
      v = io<T>::ld(act + p * astr + aoff + c) > 0.f ? g : 0.f;
    }
    io<T>::st(out + i, v);
    if (c < nz) G[p * gstr + goff + c] = 0.f;
  }
}

}  // namespace conv

// ------------------------------------------------------------------ launchers
// conv_gemm1.hip: tile 70 (1x1, bf16, segments % 64 channels)
bool conv_1x1_launch(const conv::Args& a, int tile, hipStream_t stream);

struct ConvLaunch {
  const void* seg_ptr[3];
  int seg_C[3], seg_stride[3];
  int nseg;
  const void* w;
  const float* bias;
  int B, H, W, KH, KW, PH, PW, Cout, Cout_pad, Ktot;
  int epi;
  float scale;
  int hd;
  void* out; int ostr, ooff;
  void* out2; int o2str, o2off;
  void* out3; int o3str, o3off;
  const void* aux1; int a1str, a1off;
  const void* aux2; int a2str, a2off;
  int tile;  // kernel variant (ops/conv.py choose_tile)
  unsigned seg_bytes[3];  // bytes from seg_ptr to the end of its tensor (buffer range checks)
  unsigned w_bytes;
  int geo;  // 1: strided / remapped geometry below (conv_lds tiles 2-4, 6-8)
  int Hi, Wi, SY, SX, oH, oW, OSY, OSX, OOY, OOX;
  // EPI_NORM per-channel scale (conv_common.h Args)
  const float* chs;
  int f32;  // fp32 activations / outputs (split-bf16 tiles 6-8, conv_lds_kernel<..., F32>)
};

// false: the tile is not instantiated for this kernel size (the host raises)
bool conv_launch(const ConvLaunch& L, hipStream_t stream) {
  conv::Args a{};
  for (int s = 0; s < 3; ++s) {
    a.seg[s].ptr = static_cast<const bf16_t*>(L.seg_ptr[s]);
    a.seg[s].C = L.seg_C[s];
    a.seg[s].stride = L.seg_stride[s];
  }
  a.nseg = L.nseg;
  a.w = static_cast<const bf16_t*>(L.w);
  a.bias = L.bias;
  a.B = L.B; a.H = L.H; a.W = L.W; a.P = L.B * L.H * L.W;
  a.KH = L.KH; a.KW = L.KW; a.PH = L.PH; a.PW = L.PW;
  a.Cout = L.Cout; a.Ktot = L.Ktot;
  a.epi = L.epi; a.scale = L.scale; a.hd = L.hd;
  a.out = L.out; a.ostr = L.ostr; a.ooff = L.ooff;
  a.out2 = L.out2; a.o2str = L.o2str; a.o2off = L.o2off;
  a.out3 = L.out3; a.o3str = L.o3str; a.o3off = L.o3off;
  a.aux1 = static_cast<const bf16_t*>(L.aux1); a.a1str = L.a1str; a.a1off = L.a1off;
  a.aux2 = static_cast<const bf16_t*>(L.aux2); a.a2str = L.a2str; a.a2off = L.a2off;
  for (int s = 0; s < 3; ++s) a.seg_bytes[s] = L.seg_bytes[s];
  a.w_bytes = L.w_bytes;
  a.chs = L.chs;
  a.f32 = L.f32;
  a.xcd_remap = 1;
  if (L.geo) {
    a.Hi = L.Hi; a.Wi = L.Wi; a.SY = L.SY; a.SX = L.SX;
    a.oH = L.oH; a.oW = L.oW; a.OSY = L.OSY; a.OSX = L.OSX; a.OOY = L.OOY; a.OOX = L.OOX;
#define RS_GEO(BM_, BN_, WM_, WN_, BK_)                                                             \
  if (L.f32)                                                                                       \
    hipLaunchKernelGGL((conv::conv_lds_kernel<BM_, BN_, WM_, WN_, 64, true, true>),               \
                       dim3(cdiv(a.P, BN_), cdiv(L.Cout, BM_)), dim3(256), 0, stream, a);          \
  else                                                                                             \
    hipLaunchKernelGGL((conv::conv_lds_kernel<BM_, BN_, WM_, WN_, BK_, true>),                    \
                       dim3(cdiv(a.P, BN_), cdiv(L.Cout, BM_)), dim3(256), 0, stream, a)
    switch (L.tile) {
      case 2: RS_GEO(64, 128, 1, 4, 32); break;
      case 3: RS_GEO(64, 64, 2, 2, 32); break;
      case 6: RS_GEO(64, 64, 2, 2, 64); break;
      case 7: RS_GEO(128, 64, 2, 2, 64); break;
      case 8: RS_GEO(128, 128, 2, 2, 64); break;
      default: RS_GEO(128, 64, 2, 2, 32); break;  // 4
    }
#undef RS_GEO
    return true;
  }
  if (L.f32 && L.tile >= 81 && L.tile <= 85) {  // fp32 weight-streaming tiles (conv_v3f.hip)
    return conv_v3f_launch(a, L.tile, stream);
  }
  if (L.f32) {  // fp32 activations: split-bf16 register-staged tiles 6 / 7 / 8, split-K 38-40 (host-checked)
#define RS_F32(BM_, BN_, KG_)                                                                       \
  hipLaunchKernelGGL((conv::conv_lds_kernel<BM_, BN_, 2, 2, 64, false, true, KG_>),                \
                     dim3(cdiv(a.P, BN_), cdiv(L.Cout, BM_)), dim3(256 * KG_), 0, stream, a)
    if (L.tile == 6) RS_F32(64, 64, 1);
    else if (L.tile == 8) RS_F32(128, 128, 1);
    else if (L.tile == 38) RS_F32(64, 64, 4);
    else if (L.tile == 39) RS_F32(128, 64, 2);
    else if (L.tile == 40) RS_F32(64, 64, 2);
    else RS_F32(128, 64, 1);
#undef RS_F32
    return true;
  }
  if (L.tile == 41) {  // tile 3 (64x64, 32-deep K, register-staged) with 4-way intra-block split-K
    dim3 grid(cdiv(a.P, 64), cdiv(L.Cout, 64));
    hipLaunchKernelGGL((conv::conv_lds_kernel<64, 64, 2, 2, 32, false, false, 4>), grid, dim3(1024), 0, stream, a);
    return true;
  }
  if (L.tile >= 24 && L.tile <= 26) {  // halo (patch) tiles: grid = Cout tiles x (images x patch rows x patch columns)
    const int TH = L.tile == 26 ? 4 : 8, BM = L.tile == 25 ? 64 : 128;
    const dim3 grid(cdiv(L.Cout, BM) * L.B * cdiv(L.H, TH) * cdiv(L.W, 16));
    if (L.tile == 24) hipLaunchKernelGGL((conv::conv_halo_kernel<128, 8, 192>), grid, dim3(256), 0, stream, a);
    else if (L.tile == 25) hipLaunchKernelGGL((conv::conv_halo_kernel<64, 8, 192>), grid, dim3(256), 0, stream, a);
    else hipLaunchKernelGGL((conv::conv_halo_kernel<128, 4, 128>), grid, dim3(256), 0, stream, a);
    return true;
  }
  if (L.tile >= 42 && L.tile <= 54) {  // lean unrolled-tap tiles (conv_v2.hip)
    return conv_v2_launch(a, L.tile, stream);
  }
  if (L.tile == 70) {  // 1x1 convs as plain GEMMs (conv_gemm1.hip)
    return conv_1x1_launch(a, L.tile, stream);
  }
  if (L.tile >= 56) {  // weight-streaming tiles (conv_v3.hip), fragment-major weights
    return conv_v3_launch(a, L.tile, stream);
  }
  if (L.tile == 5) {
    hipLaunchKernelGGL(conv::conv_smalln_kernel, dim3(cdiv(a.P, 16)), dim3(256), 0, stream, a);
  } else if (L.tile >= 2) {
    if (L.tile == 2) {  // 64 co x 128 px, waves 1 x 4 (wave 64 x 32)
      dim3 grid(cdiv(a.P, 128), cdiv(L.Cout, 64));
      hipLaunchKernelGGL((conv::conv_lds_kernel<64, 128, 1, 4, 32>), grid, dim3(256), 0, stream, a);
    } else if (L.tile == 3) {  // 64 co x 64 px, waves 2 x 2 (wave 32 x 32)
      dim3 grid(cdiv(a.P, 64), cdiv(L.Cout, 64));
      hipLaunchKernelGGL((conv::conv_lds_kernel<64, 64, 2, 2, 32>), grid, dim3(256), 0, stream, a);
    } else if (L.tile == 4) {  // 128 co x 64 px, waves 2 x 2 (wave 64 x 32)
      dim3 grid(cdiv(a.P, 64), cdiv(L.Cout, 128));
      hipLaunchKernelGGL((conv::conv_lds_kernel<128, 64, 2, 2, 32>), grid, dim3(256), 0, stream, a);
    } else if (L.tile == 6) {  // tile 3 with 64-deep K steps
      dim3 grid(cdiv(a.P, 64), cdiv(L.Cout, 64));
      hipLaunchKernelGGL((conv::conv_lds_kernel<64, 64, 2, 2, 64>), grid, dim3(256), 0, stream, a);
    } else if (L.tile == 7) {  // tile 4 with 64-deep K steps
      dim3 grid(cdiv(a.P, 64), cdiv(L.Cout, 128));
      hipLaunchKernelGGL((conv::conv_lds_kernel<128, 64, 2, 2, 64>), grid, dim3(256), 0, stream, a);
    } else if (L.tile == 8) {  // 128 co x 128 px, waves 2 x 2 (wave 64 x 64), 64-deep K steps
      dim3 grid(cdiv(a.P, 128), cdiv(L.Cout, 128));
      hipLaunchKernelGGL((conv::conv_lds_kernel<128, 128, 2, 2, 64>), grid, dim3(256), 0, stream, a);
    } else {  // direct-to-LDS ring (conv_glds_kernel), grid 1-D over (pixel tile, Cout tile)
#define RS_GLDS(BM_, BN_, BK_, ST_)                                                                  \
  hipLaunchKernelGGL((conv::conv_glds_kernel<BM_, BN_, 2, 2, BK_, ST_>),                             \
                     dim3(cdiv(a.P, BN_) * cdiv(L.Cout, BM_)), dim3(256), 0, stream, a)
      switch (L.tile) {
        case 9: RS_GLDS(64, 64, 64, 3); break;
        case 10: RS_GLDS(128, 64, 64, 3); break;
        case 11: RS_GLDS(128, 64, 64, 2); break;
        case 12: RS_GLDS(128, 64, 32, 4); break;
        case 13: RS_GLDS(128, 64, 32, 3); break;
        case 14: RS_GLDS(64, 64, 32, 4); break;
        case 15: RS_GLDS(64, 64, 64, 2); break;
#define RS_BUF(BM_, BN_, ST_)                                                                        \
  hipLaunchKernelGGL((conv::conv_buf_kernel<BM_, BN_, 2, 2, ST_>), dim3(cdiv(a.P, BN_) * cdiv(L.Cout, BM_)), \
                     dim3(256), 0, stream, a)
        case 16: RS_BUF(128, 64, 2); break;
        case 17: RS_BUF(64, 64, 2); break;
        case 18: RS_BUF(128, 64, 3); break;
        case 19: RS_BUF(64, 64, 3); break;
        case 20: RS_BUF(128, 128, 2); break;  // wave tile 64x64: 1.5x fewer L2 bytes per FLOP than 128x64
        case 21: RS_BUF(64, 128, 2); break;
        case 22: RS_BUF(128, 128, 3); break;
        case 23: RS_BUF(64, 64, 4); break;    // deep ring for latency-bound small grids (inference)
#define RS_BUF8(BM_, BN_, ST_)                                                                       \
  hipLaunchKernelGGL((conv::conv_buf_kernel<BM_, BN_, 4, 2, ST_>), dim3(cdiv(a.P, BN_) * cdiv(L.Cout, BM_)), \
                     dim3(512), 0, stream, a)
        // 8-wave tiles for the training shape (one block per CU, ~one round)
        case 27: RS_BUF8(256, 96, 3); break;
        case 28: RS_BUF8(128, 96, 3); break;
        case 29: RS_BUF8(192, 96, 3); break;
        case 30: RS_BUF8(256, 96, 2); break;
        case 31: RS_BUF8(128, 96, 2); break;
        case 32: RS_BUF8(256, 192, 2); break;
        case 33: RS_BUF8(128, 192, 2); break;
#define RS_BUFK(BM_, BN_, ST_, KG_)                                                                  \
  hipLaunchKernelGGL((conv::conv_buf_kernel<BM_, BN_, 2, 2, ST_, KG_>),                                \
                     dim3(cdiv(a.P, BN_) * cdiv(L.Cout, BM_)), dim3(256 * KG_), 0, stream, a)
        // intra-block split-K tiles for small grids (batch-1 inference)
        case 34: RS_BUFK(64, 64, 2, 2); break;
        case 35: RS_BUFK(64, 64, 3, 2); break;
        case 36: RS_BUFK(128, 64, 2, 2); break;
        default: RS_BUFK(64, 64, 2, 4); break;  // 37
#undef RS_BUFK
#undef RS_BUF8
#undef RS_BUF
      }
#undef RS_GLDS
    }
  } else if (L.tile == 1) {
    constexpr int WM = 4, WN = 2, WAVES_M = 1, WAVES_N = 4;
    dim3 grid(cdiv(a.P, WN * 16 * WAVES_N), cdiv(L.Cout, WM * 16 * WAVES_M));
    hipLaunchKernelGGL((conv::conv_kernel<WM, WN, WAVES_M, WAVES_N>), grid, dim3(64 * WAVES_M * WAVES_N),
                       0, stream, a);
  } else {
    constexpr int WM = 2, WN = 2, WAVES_M = 1, WAVES_N = 4;
    dim3 grid(cdiv(a.P, WN * 16 * WAVES_N), cdiv(L.Cout, WM * 16 * WAVES_M));
    hipLaunchKernelGGL((conv::conv_kernel<WM, WN, WAVES_M, WAVES_N>), grid, dim3(64 * WAVES_M * WAVES_N),
                       0, stream, a);
  }
  return true;
}

static int egrid(long total) {
  const long g = (total + 255) / 256;
  return (int)(g < 16384 ? g : 16384);
}

void gru_gate_bwd_launch(float* dh, int dhstr, const void* z, int zstr, const void* q, int qstr, const void* h,
                         int hstr, int hoff, void* dq, int dqstr, void* dzr, int dzrstr, long P, int hd, bool f32,
                         hipStream_t stream) {
  if (f32)
    hipLaunchKernelGGL(conv::gru_gate_bwd_kernel<float>, dim3(egrid(P * hd)), dim3(256), 0, stream, dh, dhstr,
                       static_cast<const float*>(z), zstr, static_cast<const float*>(q), qstr,
                       static_cast<const float*>(h), hstr, hoff, static_cast<float*>(dq), dqstr,
                       static_cast<float*>(dzr), dzrstr, P, hd);
  else
    hipLaunchKernelGGL(conv::gru_gate_bwd_kernel<bf16_t>, dim3(egrid(P * hd)), dim3(256), 0, stream, dh, dhstr,
                       static_cast<const bf16_t*>(z), zstr, static_cast<const bf16_t*>(q), qstr,
                       static_cast<const bf16_t*>(h), hstr, hoff, static_cast<bf16_t*>(dq), dqstr,
                       static_cast<bf16_t*>(dzr), dzrstr, P, hd);
}

void relu_take_launch(float* G, int gstr, int goff, int n, int nz, const void* act, int astr, int aoff, void* out,
                      int ostr, long P, bool f32, hipStream_t stream) {
  if (f32)
    hipLaunchKernelGGL(conv::relu_take_kernel<float>, dim3(egrid(P * ostr)), dim3(256), 0, stream, G, gstr, goff, n,
                       nz, static_cast<const float*>(act), astr, aoff, static_cast<float*>(out), ostr, P);
  else
    hipLaunchKernelGGL(conv::relu_take_kernel<bf16_t>, dim3(egrid(P * ostr)), dim3(256), 0, stream, G, gstr, goff, n,
                       nz, static_cast<const bf16_t*>(act), astr, aoff, static_cast<bf16_t*>(out), ostr, P);
}


}  // namespace rs
