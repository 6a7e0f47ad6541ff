// The encoders' 7x7 / stride-2 / pad-3 stem convolution, 3 -> Cout (<= 64)
// (reference core/extractor.py:135 BasicEncoder.conv1, :212 SmallEncoder.conv1),
// forward and weight gradient on the matrix cores.
//
// A 3-channel input makes the generic implicit GEMM waste 29 of every 32 K
// lanes (K steps are 32 channels of ONE tap).  Here K runs over a whole 7-tap
// ROW instead: for output pixel (oy, ox) and kernel row ky the 7 input pixels
// 2*ox-3 .. 2*ox+3 of input row 2*oy-3+ky are 21 CONSECUTIVE values of the
// NHWC image (7 pixels x 3 channels), zero-padded to K = 32: one 16x16x32 MFMA
// per (16 channels, 16 pixels, ky), 7 K steps in all (147 of 224 K lanes
// live).  The im2col rows [px][ky][32] are staged in LDS per block (a 64-pixel
// run of one output row, all channels); the fp32 image is rounded to bf16 on
// the way in (what bf16 autocast feeds the reference conv), or split into
// hi / lo bf16 pairs for fp32 inference (x.w ~= xh.wh + xl.wh + xh.wl, as the
// F32 conv tiles).  The epilogue is the shared one of conv_common.h: plain
// store + normalisation statistics (instance / train-mode batch norm) or the
// eval-mode BatchNorm scale / shift + ReLU (EPI_NORM).
//
// Weight gradient: dW[co][ky][k] = sum_px dY[px][co] * im2col[px][ky][k], a
// 64 x 224 x P GEMM with K = pixels: each block reduces a contiguous pixel
// range through LDS-staged, transposed 32-pixel K slices of dY and of the
// im2col rows, writes its fp32 partial tile, and a second kernel sums the
// partials in a fixed order (deterministic).
#include "conv_common.h"

namespace rs {
namespace stem {

constexpr int PXB = 64;   // output pixels per forward block (one row run)
constexpr int KR = 32;    // K per kernel row (21 live)
constexpr int RS_ = KR + 8;  // LDS row stride (bf16): 80 B, 16-B aligned, rotates the 16-B bank slots

struct SArgs {
  const void* x;     // NHWC image, 3 channels, fp32 (x_bf16 = 0) or bf16
  int x_bf16;
  int B, Hi, Wi, Ho, Wo;
};

__device__ __forceinline__ float ldx(const SArgs& s, size_t i) {
  return s.x_bf16 ? bf2f(static_cast<const bf16_t*>(s.x)[i]) : static_cast<const float*>(s.x)[i];
}

// one im2col row (21 values of image row iy starting at pixel ix0), as bf16 hi / lo
template <bool F32>
__device__ __forceinline__ void im2col_row(const SArgs& s, int b, int iy, int ix0, bf16_t* hi, bf16_t* lo) {
  const bool rowok = iy >= 0 && iy < s.Hi;
  const size_t rbase = ((size_t)b * s.Hi + (rowok ? iy : 0)) * s.Wi;
#pragma unroll
  for (int k = 0; k < KR; ++k) {
    float v = 0.f;
    if (k < 21) {
      const int ix = ix0 + k / 3;
      if (rowok && ix >= 0 && ix < s.Wi) v = ldx(s, (rbase + ix) * 3 + k % 3);
    }
    const bf16_t h = f2bf(v);
    hi[k] = h;
    if constexpr (F32) lo[k] = f2bf(v - bf2f(h));
  }
}

// Forward.  Block = 64 output pixels (b, oy, ox0 .. ox0+63) x 64 channels;
// waves 2 x 2, wave tile 32 channels x 32 pixels (2 x 2 16x16 MFMA tiles).
// w: packed [64][7][32] bf16 ([64][7][64] = [wh 32 | wl 32] for F32).
// Staging: the 7 input rows the block reads are each ONE contiguous run of
// the NHWC image (134 pixels x 3 channels = 402 values from pixel 2*ox0 - 3),
// loaded coalesced and stored as bf16 (hi / lo) rows of XR elements; the
// im2col row of output pixel n and kernel row ky is then elements
// [6n, 6n + 21) of LDS row ky -- no per-(pixel, tap) gathers.  K lanes
// 21..31 read the next pixel's values; the packed weights are zero there.
constexpr int XR = 416;  // LDS row (elements): 402 live + the K-lane overhang of pixel 63 (6 * 63 + 32 = 410)

template <bool F32>
__global__ __launch_bounds__(256) void stem_fwd_kernel(SArgs s, conv::Args a) {
  __shared__ __attribute__((aligned(16))) bf16_t xs[(F32 ? 2 : 1) * 7 * XR];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int segs = cdiv(s.Wo, PXB);
  const int row = blockIdx.x / segs, ox0 = (blockIdx.x - row * segs) * PXB;
  const int b = row / s.Ho, oy = row - b * s.Ho;
  const int ix0 = 2 * ox0 - 3;
  // value pairs (2 consecutive elements of one row): 7 rows x 208 pairs
  for (int q = t; q < 7 * (XR / 2); q += 256) {
    const int ky = q / (XR / 2), e = (q - ky * (XR / 2)) * 2;
    const int iy = 2 * oy - 3 + ky;
    float v[2] = {0.f, 0.f};
    if (iy >= 0 && iy < s.Hi) {
      const size_t rbase = ((size_t)b * s.Hi + iy) * s.Wi * 3;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int ee = e + u, ix = ix0 + ee / 3;
        if (ee < 402 && ix >= 0 && ix < s.Wi) v[u] = ldx(s, rbase + (size_t)ix * 3 + ee % 3);
      }
    }
    const bf16_t h0 = f2bf(v[0]), h1 = f2bf(v[1]);
    *reinterpret_cast<uint32_t*>(xs + ky * XR + e) = uint32_t(h0) | (uint32_t(h1) << 16);
    if constexpr (F32) {
      const bf16_t l0 = f2bf(v[0] - bf2f(h0)), l1 = f2bf(v[1] - bf2f(h1));
      *reinterpret_cast<uint32_t*>(xs + 7 * XR + ky * XR + e) = uint32_t(l0) | (uint32_t(l1) << 16);
    }
  }
  __syncthreads();
  const int wm = wave & 1, wn = wave >> 1;
  const int lr = lane & 15, lc = lane >> 4;
  constexpr int WK = F32 ? 2 * KR : KR;  // packed weight K per kernel row
  f32x4_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // B fragment: 8 bf16 at element 6n + 8lc of row ky (4-byte aligned: four 32-bit reads)
  auto bfrag = [&](const bf16_t* base, int n, int ky) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(base + ky * XR + 6 * n + 8 * lc);
    return make_uint4(p[0], p[1], p[2], p[3]);
  };
#pragma unroll
  for (int ky = 0; ky < 7; ++ky) {
    uint4 fa[2][F32 ? 2 : 1], fb[2][F32 ? 2 : 1];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const bf16_t* wr = a.w + ((size_t)(wm * 32 + mt * 16 + lr) * 7 + ky) * WK + lc * 8;
      fa[mt][0] = conv::ld16(wr);
      if constexpr (F32) fa[mt][1] = conv::ld16(wr + KR);
    }
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int n = wn * 32 + nt * 16 + lr;
      fb[nt][0] = bfrag(xs, n, ky);
      if constexpr (F32) fb[nt][1] = bfrag(xs + 7 * XR, n, ky);
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[mt][0]),
                                                              __builtin_bit_cast(bf16x8_t, fb[nt][0]), acc[mt][nt],
                                                              0, 0, 0);
        if constexpr (F32) {
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[mt][0]),
                                                                __builtin_bit_cast(bf16x8_t, fb[nt][1]),
                                                                acc[mt][nt], 0, 0, 0);
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[mt][1]),
                                                                __builtin_bit_cast(bf16x8_t, fb[nt][0]),
                                                                acc[mt][nt], 0, 0, 0);
        }
      }
  }
  int pp[2], pb[2], py[2], px[2];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int ox = ox0 + wn * 32 + nt * 16 + lr;
    const bool ok = ox < s.Wo;
    pb[nt] = ok ? b : -1;
    py[nt] = oy;
    px[nt] = ox;
    pp[nt] = ok ? (b * s.Ho + oy) * s.Wo + ox : 0;
  }
  const int m0 = wm * 32;
  if constexpr (F32)
    conv::epilogue_pix_f32<2, 2>(a, acc, m0, lane, pp, pb);
  else
    conv::epilogue_pix<2, 2>(a, acc, m0, lane, pp, pb, py, px);
}

// Weight gradient partials.  Block = a contiguous range of output pixels
// (multiple of 32), all 64 channels x 8 kernel-row slots (7 live, K = 32
// each: N = 256).  Per 32-pixel K slice: dY^T [64 co][32 px] and the im2col
// rows transposed [256 n][32 px] are staged in LDS; wave w owns n-tiles
// 4w .. 4w+3 for all 4 channel tiles (16 16x16x32 MFMAs per slice).
constexpr int WKP = 32;            // pixels per K slice
constexpr int TS = WKP + 8;        // transposed LDS row stride (bf16)

__global__ __launch_bounds__(256) void stem_wgrad_kernel(SArgs s, const bf16_t* __restrict__ dy, int ystr, int Cout,
                                                         int px_per_block, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) bf16_t ys[64 * TS];    // [co][px]
  __shared__ __attribute__((aligned(16))) bf16_t xs[256 * TS];   // [ky*32 + k][px]
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int lr = lane & 15, lc = lane >> 4;
  const long P = (long)s.B * s.Ho * s.Wo;
  const long p0 = (long)blockIdx.x * px_per_block;
  const long p1 = p0 + px_per_block < P ? p0 + px_per_block : P;
  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  for (long q0 = p0; q0 < p1; q0 += WKP) {
    // dY slice, transposed: thread -> (pixel j = t / 8, channels 8 * (t % 8) .. +7)
    {
      const int j = t >> 3, c8 = (t & 7) * 8;
      const long p = q0 + j;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (p < p1 && c8 < Cout) v = *reinterpret_cast<const uint4*>(dy + p * ystr + c8);
      const bf16_t* e = reinterpret_cast<const bf16_t*>(&v);
#pragma unroll
      for (int i = 0; i < 8; ++i) ys[(c8 + i) * TS + j] = (c8 + i < Cout) ? e[i] : (bf16_t)0;
    }
    // im2col slice, transposed: thread -> (pixel j = t % 32, kernel row ky = t / 32 (7: zero))
    {
      const int j = t & 31, ky = t >> 5;
      const long p = q0 + j;
      bf16_t row[KR];
      if (ky < 7 && p < p1) {
        const int b = (int)(p / ((long)s.Ho * s.Wo));
        const int rem = (int)(p - (long)b * s.Ho * s.Wo);
        const int oy = rem / s.Wo, ox = rem - oy * s.Wo;
        im2col_row<false>(s, b, 2 * oy - 3 + ky, 2 * ox - 3, row, nullptr);
      } else {
#pragma unroll
        for (int k = 0; k < KR; ++k) row[k] = 0;
      }
#pragma unroll
      for (int k = 0; k < KR; ++k) xs[(ky * KR + k) * TS + j] = row[k];
    }
    __syncthreads();
    uint4 fa[4], fb[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) fa[mt] = *reinterpret_cast<const uint4*>(ys + (mt * 16 + lr) * TS + lc * 8);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
      fb[nt] = *reinterpret_cast<const uint4*>(xs + ((wave * 4 + nt) * 16 + lr) * TS + lc * 8);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[mt]),
                                                              __builtin_bit_cast(bf16x8_t, fb[nt]), acc[mt][nt],
                                                              0, 0, 0);
    __syncthreads();
  }
  // partial tile [64 co][224 n] of this block: C[co][n], co = mt*16 + 4*lc + j, n = (4w + nt)*16 + lr
  float* o = part + (size_t)blockIdx.x * 64 * 224;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int n = (wave * 4 + nt) * 16 + lr;
      if (n < 224)
#pragma unroll
        for (int j = 0; j < 4; ++j) o[(size_t)(mt * 16 + 4 * lc + j) * 224 + n] = acc[mt][nt][j];
    }
}

// dW[co][ci][ky][kx] (fp32, the conv weight's layout) = sum over blocks of the
// partials, in block order; k = kx * 3 + ci of kernel row ky
__global__ __launch_bounds__(256) void stem_wgrad_reduce_kernel(const float* __restrict__ part, int nblk, int Cout,
                                                                float* __restrict__ dw) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // over Cout * 147
  if (i >= Cout * 147) return;
  const int co = i / 147, r = i - co * 147;
  const int ci = r / 49, ky = (r / 7) % 7, kx = r % 7;
  const int n = ky * KR + kx * 3 + ci;
  float acc = 0.f;
  for (int blk = 0; blk < nblk; ++blk) acc += part[((size_t)blk * 64 + co) * 224 + n];
  dw[i] = acc;
}

}  // namespace stem

// host launch block (must match ops_conv.cpp)
struct StemLaunch {
  const void* x;
  int x_bf16, B, Hi, Wi, Ho, Wo;
  const void* w;  // packed [64][7][32] (F32: [64][7][64])
  const float* bias;
  int Cout, epi, relu;
  void* out;
  int ostr, ooff;
  const void* res;
  int rstr;
  const float* chs;
  int f32;
};

void stem_launch(const StemLaunch& L, hipStream_t stream) {
  conv::Args a{};
  a.w = static_cast<const bf16_t*>(L.w);
  a.bias = L.bias;
  a.B = L.B; a.H = L.Ho; a.W = L.Wo; a.P = L.B * L.Ho * L.Wo;
  a.Cout = L.Cout;
  a.epi = L.epi; a.hd = L.relu; a.scale = 1.f;
  a.out = L.out; a.ostr = L.ostr; a.ooff = L.ooff;
  a.aux1 = static_cast<const bf16_t*>(L.res); a.a1str = L.rstr; a.a1off = 0;
  a.chs = L.chs; a.f32 = L.f32;
  stem::SArgs s{L.x, L.x_bf16, L.B, L.Hi, L.Wi, L.Ho, L.Wo};
  const dim3 grid((unsigned)(L.B * L.Ho * cdiv(L.Wo, stem::PXB)));
  if (L.f32)
    hipLaunchKernelGGL(stem::stem_fwd_kernel<true>, grid, dim3(256), 0, stream, s, a);
  else
    hipLaunchKernelGGL(stem::stem_fwd_kernel<false>, grid, dim3(256), 0, stream, s, a);
}

int stem_wgrad_blocks(long P, int* px_per_block) {
  // ~2 blocks per CU, whole 32-pixel K slices per block
  long per = (P + 511) / 512;
  per = (per + 31) / 32 * 32;
  if (per < 32) per = 32;
  *px_per_block = (int)per;
  return (int)((P + per - 1) / per);
}

void stem_wgrad_launch(const void* x, bool x_bf16, int B, int Hi, int Wi, int Ho, int Wo, const bf16_t* dy, int ystr,
                       int Cout, float* part, int nblk, int px_per_block, float* dw, hipStream_t stream) {
  stem::SArgs s{x, x_bf16 ? 1 : 0, B, Hi, Wi, Ho, Wo};
  hipLaunchKernelGGL(stem::stem_wgrad_kernel, dim3(nblk), dim3(256), 0, stream, s, dy, ystr, Cout, px_per_block,
                     part);
  hipLaunchKernelGGL(stem::stem_wgrad_reduce_kernel, dim3(cdiv(Cout * 147, 256)), dim3(256), 0, stream, part, nblk,
                     Cout, dw);
}

}  // namespace rs
