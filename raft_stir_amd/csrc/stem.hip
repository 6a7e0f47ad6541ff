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

// Weight gradient partials: dW^T tile [64 co][7 ky x 32 k] = sum over pixels
// of dY[px][co] x im2col[px][ky][k] (k = kx * 3 + ci, 21 live), K = pixels.
// Block = 7 waves, wave ky owns kernel row ky (2 x v_mfma_f32_32x32x16_bf16
// accumulators: co 0-31 / 32-63 x 32 k), walking a contiguous range of
// 64-pixel chunks (b, oy, ox0 .. ox0+63) of the output grid.  Per chunk:
//  * dY rows (64 px x 64 co, zeros past the row / Cout) -> LDS [px][co], the
//    64-B halves of each 128-B row swapped on (px >> 1) & 1;
//  * the 7 input rows the chunk reads, each ONE contiguous 134-pixel run of
//    the NHWC image (402 values), -> LDS twice: the im2col row of pixel px and
//    kernel row ky is elements [6 px, 6 px + 32) of run ky, so the B fragment
//    (4 pixels of one column per lane, ds_read_b64_tr_b16) reads the runs in
//    place -- even pixels from copy A (element e at byte 2e: 8-B aligned rows),
//    odd pixels from copy B (element e at byte 2e + 4); columns 21..31 pick up
//    the next pixel's values and land in dW columns nobody reads;
//  * the next chunk's global loads are in flight while this chunk's MFMAs run
//    (register prefetch, fixed per-thread slots).
// Each block writes its fp32 partial tile; stem_wgrad_reduce_kernel adds the
// partials in block order (deterministic).
constexpr int WG_WAVES = 7, WG_T = 64 * WG_WAVES;
constexpr int WG_RAWP = 416;  // run row pitch (elements): 402 live, reads up to 6 * 63 + 31 + 2 = 411
constexpr int WG_RJ = (7 * 402 + WG_T - 1) / WG_T;  // run elements per thread

__global__ __launch_bounds__(WG_T) void stem_wgrad_kernel(SArgs s, const bf16_t* __restrict__ dy, int ystr, int Cout,
                                                          int chunks_per_block, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) uint8_t ylds[64 * 128];    // [px][co] bf16
  __shared__ __attribute__((aligned(16))) bf16_t runA[7 * WG_RAWP];  // element e at index e
  __shared__ __attribute__((aligned(16))) bf16_t runB[7 * WG_RAWP];  // element e at index e + 2
  const int t = threadIdx.x, lane = t & 63;
  const int ky = __builtin_amdgcn_readfirstlane(t >> 6);
  const int cpr = cdiv(s.Wo, 64);
  const int nchunk = s.B * s.Ho * cpr;
  const int c0 = blockIdx.x * chunks_per_block, c1 = min(nchunk, c0 + chunks_per_block);
  for (int i = t; i < 7 * 16; i += WG_T) {  // constant zeros past the live run values
    runA[(i >> 4) * WG_RAWP + 402 + (i & 15) % 14] = 0;
    runB[(i >> 4) * WG_RAWP + 404 + (i & 15) % 12] = 0;
  }
  // fixed staging slots: dY slots t and t + 448 (< 512); run elements t + 448 j
  int rr[WG_RJ], re[WG_RJ];
#pragma unroll
  for (int j = 0; j < WG_RJ; ++j) {
    const int qq = t + WG_T * j;
    rr[j] = qq < 7 * 402 ? qq / 402 : -1;
    re[j] = qq - (qq / 402) * 402;
  }
  uint4 ypre[2];
  float xpre[WG_RJ];
  auto prefetch = [&](int c) {
    const int rowid = c / cpr, ox0 = (c - rowid * cpr) * 64;
    const int b = rowid / s.Ho, oy = rowid - b * s.Ho;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int sl = t + WG_T * u;
      const int px = (sl >> 3) & 63, c16 = sl & 7;
      ypre[u] = make_uint4(0u, 0u, 0u, 0u);
      if (sl < 512 && ox0 + px < s.Wo && c16 * 8 < Cout)
        ypre[u] = *reinterpret_cast<const uint4*>(dy + ((size_t)rowid * s.Wo + ox0 + px) * ystr + c16 * 8);
    }
    const int ix0 = 2 * ox0 - 3;
#pragma unroll
    for (int j = 0; j < WG_RJ; ++j) {
      const int iy = 2 * oy - 3 + rr[j], ix = ix0 + re[j] / 3;
      xpre[j] = 0.f;
      if (rr[j] >= 0 && iy >= 0 && iy < s.Hi && ix >= 0 && ix < s.Wi)
        xpre[j] = ldx(s, (((size_t)b * s.Hi + iy) * s.Wi + ix) * 3 + re[j] % 3);
    }
  };

  // fragment read roles (tr16): 16-lane group g, lane 4q + p -> row q (+ 8h, + 4, + 16 KK), columns 4p .. 4p+3
  const int g = lane >> 4, gi = lane & 15, q = gi >> 2, p = gi & 3, h = lane >> 5;
  const uint32_t y0 = (uint32_t)(size_t)(__attribute__((address_space(3))) uint8_t*)ylds;
  // A (dY^T): row px = 16 KK + 8h + q (+4), co = 32 i + 16 (g & 1) + 4p: half i ^ ((q >> 1) & 1)
  uint32_t aaddr[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
    aaddr[i] = y0 + (8 * h + q) * 128 + ((i ^ ((q >> 1) & 1)) << 6) + 32 * (g & 1) + 8 * p;
  // B (run ky): pixel px = 8h + q (+4, + 16 KK) -> elements 6 px + 16 (g & 1) + 4p; parity of px = parity of q
  const uint32_t rb = (q & 1) ? (uint32_t)(size_t)(__attribute__((address_space(3))) bf16_t*)runB + 4
                              : (uint32_t)(size_t)(__attribute__((address_space(3))) bf16_t*)runA;
  const uint32_t baddr = rb + (ky * WG_RAWP + 6 * (8 * h + q) + 16 * (g & 1) + 4 * p) * 2;

  f32x16_t acc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;

  if (c0 < c1) prefetch(c0);
  for (int c = c0; c < c1; ++c) {
    __syncthreads();  // the previous chunk's fragments are read
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int sl = t + WG_T * u, px = (sl >> 3) & 63, c16 = sl & 7;
      if (sl < 512) *reinterpret_cast<uint4*>(ylds + px * 128 + ((c16 ^ (((px >> 1) & 1) << 2)) << 4)) = ypre[u];
    }
#pragma unroll
    for (int j = 0; j < WG_RJ; ++j) {
      if (rr[j] >= 0) {
        const bf16_t v = f2bf(xpre[j]);
        runA[rr[j] * WG_RAWP + re[j]] = v;
        runB[rr[j] * WG_RAWP + re[j] + 2] = v;
      }
    }
    __syncthreads();
    if (c + 1 < c1) prefetch(c + 1);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      typedef short v4s __attribute__((ext_vector_type(4)));
      v4s alo[2], ahi[2], blo, bhi;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        alo[i] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) v4s*)(size_t)(aaddr[i] + kk * 16 * 128));
        ahi[i] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) v4s*)(size_t)(aaddr[i] + (kk * 16 + 4) * 128));
      }
      blo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(size_t)(baddr + kk * 16 * 12));
      bhi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) v4s*)(size_t)(baddr + (kk * 16 + 4) * 12));
      const bf16x8_t bv = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(blo, bhi, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const bf16x8_t av =
            __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(alo[i], ahi[i], 0, 1, 2, 3, 4, 5, 6, 7));
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc[i], 0, 0, 0);
      }
    }
  }
  // partial tile [64 co][224 n]: acc[i] reg r -> co = 32 i + (r & 3) + 8 (r >> 2) + 4h, n = ky * 32 + lane & 31
  float* o = part + (size_t)blockIdx.x * 64 * 224;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r)
      o[(size_t)(32 * i + (r & 3) + 8 * (r >> 2) + 4 * h) * 224 + ky * 32 + (lane & 31)] = acc[i][r];
}

// dW[co][ci][ky][kx] (fp32, the conv weight's layout) = sum over blocks of the
// partials, k = kx * 3 + ci of kernel row ky.  Block = 64 outputs x 16 partial
// lanes: lane j sums partials j, j + 16, ... in order, then output o adds the
// 16 lane sums in lane order (deterministic; independent loads in flight
// instead of one serial chain of nblk loads per output).
constexpr int RD_O = 64, RD_L = 16;

__global__ __launch_bounds__(RD_O * RD_L) void stem_wgrad_reduce_kernel(const float* __restrict__ part, int nblk,
                                                                        int Cout, float* __restrict__ dw) {
  __shared__ float red[RD_L][RD_O];
  const int o = threadIdx.x % RD_O, j = threadIdx.x / RD_O;
  const int i = blockIdx.x * RD_O + o;  // over Cout * 147
  float acc = 0.f;
  if (i < Cout * 147) {
    const int co = i / 147, r = i - co * 147;
    const int ci = r / 49, ky = (r / 7) % 7, kx = r % 7;
    const size_t n = (size_t)co * 224 + ky * KR + kx * 3 + ci;
    int blk = j;
    for (; blk + 3 * RD_L < nblk; blk += 4 * RD_L) {
      const float v0 = part[(size_t)blk * 64 * 224 + n], v1 = part[(size_t)(blk + RD_L) * 64 * 224 + n];
      const float v2 = part[(size_t)(blk + 2 * RD_L) * 64 * 224 + n], v3 = part[(size_t)(blk + 3 * RD_L) * 64 * 224 + n];
      acc += v0;
      acc += v1;
      acc += v2;
      acc += v3;
    }
    for (; blk < nblk; blk += RD_L) acc += part[(size_t)blk * 64 * 224 + n];
  }
  red[j][o] = acc;
  __syncthreads();
  if (j == 0 && i < Cout * 147) {
    float t = 0.f;
#pragma unroll
    for (int l = 0; l < RD_L; ++l) t += red[l][o];
    dw[i] = t;
  }
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

// (B, Ho, Wo) -> blocks of chunks_per_block 64-pixel row chunks: ~2 blocks per CU
int stem_wgrad_blocks(int B, int Ho, int Wo, int* chunks_per_block) {
  const long nchunk = (long)B * Ho * cdiv(Wo, 64);
  long per = (nchunk + 511) / 512;
  if (per < 1) per = 1;
  *chunks_per_block = (int)per;
  return (int)((nchunk + per - 1) / per);
}

void stem_wgrad_launch(const void* x, bool x_bf16, int B, int Hi, int Wi, int Ho, int Wo, const bf16_t* dy, int ystr,
                       int Cout, float* part, int nblk, int chunks_per_block, float* dw, hipStream_t stream) {
  stem::SArgs s{x, x_bf16 ? 1 : 0, B, Hi, Wi, Ho, Wo};
  hipLaunchKernelGGL(stem::stem_wgrad_kernel, dim3(nblk), dim3(stem::WG_T), 0, stream, s, dy, ystr, Cout,
                     chunks_per_block, part);
  hipLaunchKernelGGL(stem::stem_wgrad_reduce_kernel, dim3(cdiv(Cout * 147, stem::RD_O)), dim3(stem::RD_O * stem::RD_L),
                     0, stream, part, nblk, Cout, dw);
}

}  // namespace rs
