// Weight gradient of RAFT-small's narrow encoder convs for training
// (reference core/extractor.py:60-116 BottleneckBlock, :195-267
// SmallEncoder: 1x1 / 3x3, stride 1 / 2, 8-256 channels), NHWC:
//
//   dW[co][ky][kx][ci] = sum_{b, oy, ox} dY[b, oy, ox, co] * X[b, oy*S + ky - P, ox*S + kx - P, ci]
//
// The forward and the input gradient run on csrc/sconv.hip (the input
// gradient as a stride-1 conv of dY -- zero-interleaved for stride 2 -- with
// the flipped, transposed weights; ops/enc_conv.py sconv_train).  These
// reductions have few outputs (Cout x taps x Cin <= ~25k) and many pixels, so
// a VALU reduction, no MFMA tile to fill:
//  * block = a contiguous range of output rows (b, oy); thread = a 4 output x
//    8 input channel tile of one tap x a pixel sub-lane (32 accumulators; per
//    pixel one 8-B dY load and one 16-B input load; threads sharing a pixel
//    hit the same lines);
//  * sub-lane sums combined in LDS in a fixed order, one fp32 partial row per
//    block; sconv_wgrad_reduce_kernel adds the blocks in a fixed order
//    (deterministic).
#include <stdlib.h>

#include <algorithm>

#include "common.h"

namespace rs {
namespace swg {

struct WArgs {
  const void* x;   // [B, Hi, Wi, xstr] (Cin channels used)
  const void* dy;  // [B, Ho, Wo, ystr] (Cout channels used)
  int xstr, ystr, Cin, Cout;
  int B, Hi, Wi, Ho, Wo, KH, KW, S, P;
  int rows_per_block;
  float* part;     // [nblk][Cout * KH * KW * Cin]
};

template <typename T>
__device__ __forceinline__ float ld1(const T* p);
template <>
__device__ __forceinline__ float ld1<bf16_t>(const bf16_t* p) {
  return __uint_as_float((uint32_t)(*reinterpret_cast<const uint16_t*>(p)) << 16);
}
template <>
__device__ __forceinline__ float ld1<float>(const float* p) { return *p; }

template <typename T>
__device__ __forceinline__ void ld8(const T* p, float (&v)[8]);
template <>
__device__ __forceinline__ void ld8<bf16_t>(const bf16_t* p, float (&v)[8]) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
template <>
__device__ __forceinline__ void ld8<float>(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

constexpr int THREADS = 256;

template <typename T>
__device__ __forceinline__ void ld4(const T* p, float (&v)[4]);
template <>
__device__ __forceinline__ void ld4<bf16_t>(const bf16_t* p, float (&v)[4]) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  v[0] = __uint_as_float(u.x << 16);
  v[1] = __uint_as_float(u.x & 0xffff0000u);
  v[2] = __uint_as_float(u.y << 16);
  v[3] = __uint_as_float(u.y & 0xffff0000u);
}
template <>
__device__ __forceinline__ void ld4<float>(const float* p, float (&v)[4]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
}

typedef float f32x2_t __attribute__((ext_vector_type(2)));

// thread tile: CO (4 or 8) output channels x 8 input channels of one tap
// (8 CO accumulators; per pixel one 2*CO-B dY load, one 16-B input load,
// 8 CO FMAs as packed v_pk_fma_f32 -- two fp32 FMAs per lane per issue; CO = 8
// halves the loads per FMA of this load-bound reduction)
template <typename T, int CO>
__global__ __launch_bounds__(THREADS) void sconv_wgrad_kernel(WArgs a) {
  __shared__ float red[THREADS * 8];
  const int t = threadIdx.x;
  const int T_ = a.KH * a.KW, C8 = a.Cin / 8, O4 = a.Cout / CO;
  const int ng_all = O4 * T_ * C8;               // 8*CO-output groups
  const int NG = ng_all < THREADS ? ng_all : THREADS;
  const int SL = THREADS / NG;                   // pixel sub-lanes per group
  const int gi = t % NG, sl = t / NG;
  const bool active = sl < SL;
  const int nrows = a.B * a.Ho;
  const int r0 = blockIdx.x * a.rows_per_block, r1 = min(nrows, r0 + a.rows_per_block);
  const T* x = static_cast<const T*>(a.x);
  const T* dy = static_cast<const T*>(a.dy);
  const int OUT = a.Cout * T_ * a.Cin;
  float* out = a.part + (size_t)blockIdx.x * OUT;
  for (int g0 = 0; g0 < ng_all; g0 += NG) {
    const int g = g0 + gi;
    f32x2_t acc[CO][4];
#pragma unroll
    for (int i = 0; i < CO; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x2_t{0.f, 0.f};
    int co0 = 0, tap = 0, c8 = 0;
    if (g < ng_all) {
      c8 = g % C8;
      const int ct = g / C8;
      tap = ct % T_;
      co0 = (ct / T_) * CO;
    }
    if (active && g < ng_all) {
      const int ky = tap / a.KW, kx = tap - ky * a.KW;
      for (int r = r0; r < r1; ++r) {
        const int b = r / a.Ho, oy = r - b * a.Ho;
        const int iy = oy * a.S + ky - a.P;
        if ((unsigned)iy >= (unsigned)a.Hi) continue;
        const T* xrow = x + (size_t)(b * a.Hi + iy) * a.Wi * a.xstr + c8 * 8;
        const T* dyrow = dy + (size_t)r * a.Wo * a.ystr + co0;
        for (int ox = sl; ox < a.Wo; ox += SL) {
          const int ix = ox * a.S + kx - a.P;
          if ((unsigned)ix >= (unsigned)a.Wi) continue;
          float d[CO], v[8];
          if constexpr (CO == 8)
            ld8<T>(dyrow + (size_t)ox * a.ystr, d);
          else
            ld4<T>(dyrow + (size_t)ox * a.ystr, d);
          ld8<T>(xrow + (size_t)ix * a.xstr, v);
#pragma unroll
          for (int i = 0; i < CO; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[i][j] = __builtin_elementwise_fma(f32x2_t{d[i], d[i]}, f32x2_t{v[2 * j], v[2 * j + 1]}, acc[i][j]);
        }
      }
    }
    // combine the sub-lanes in order, one output channel (8 values) at a time
#pragma unroll
    for (int i = 0; i < CO; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        red[t * 8 + 2 * j] = acc[i][j].x;
        red[t * 8 + 2 * j + 1] = acc[i][j].y;
      }
      __syncthreads();
      if (sl == 0 && g < ng_all) {
        float s[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] = 0.f;
        for (int q = 0; q < SL; ++q)
#pragma unroll
          for (int j = 0; j < 8; ++j) s[j] += red[(q * NG + gi) * 8 + j];
        // output order [co][tap][ci]
        float4* o = reinterpret_cast<float4*>(out + ((size_t)(co0 + i) * T_ + tap) * a.Cin + c8 * 8);
        o[0] = make_float4(s[0], s[1], s[2], s[3]);
        o[1] = make_float4(s[4], s[5], s[6], s[7]);
      }
      __syncthreads();
    }
  }
}

// dw[i] = sum over blocks of part[blk][i]: 64 outputs x 16 block lanes per
// block (lane j sums blocks j, j + 16, ... in order; the 16 lane sums are
// added in lane order -- deterministic)
constexpr int RD_O = 64, RD_L = 16;

__global__ __launch_bounds__(RD_O * RD_L) void sconv_wgrad_reduce_kernel(const float* __restrict__ part, int nblk,
                                                                         int OUT, float* __restrict__ dw) {
  __shared__ float red2[RD_L][RD_O];
  const int o = threadIdx.x % RD_O, j = threadIdx.x / RD_O;
  const int i = blockIdx.x * RD_O + o;
  float acc = 0.f;
  if (i < OUT) {
    int b = j;
    for (; b + 3 * RD_L < nblk; b += 4 * RD_L) {
      const float v0 = part[(size_t)b * OUT + i], v1 = part[(size_t)(b + RD_L) * OUT + i];
      const float v2 = part[(size_t)(b + 2 * RD_L) * OUT + i], v3 = part[(size_t)(b + 3 * RD_L) * OUT + i];
      acc += v0;
      acc += v1;
      acc += v2;
      acc += v3;
    }
    for (; b < nblk; b += RD_L) acc += part[(size_t)b * OUT + i];
  }
  red2[j][o] = acc;
  __syncthreads();
  if (j == 0 && i < OUT) {
    float s = 0.f;
#pragma unroll
    for (int l = 0; l < RD_L; ++l) s += red2[l][o];
    dw[i] = s;
  }
}

}  // namespace swg

struct SconvWgradLaunch {
  const void* x;
  const void* dy;
  int xstr, ystr, Cin, Cout, B, Hi, Wi, Ho, Wo, KH, KW, S, P;
  bool f32;
  float* dw;
  float* part;  // sconv_wgrad_workspace floats
};

// blocks: rows of the output grid split so that nblk * OUT stays <= ~4M floats
int sconv_wgrad_blocks(int B, int Ho, int OUT, int* rows_per_block) {
  const int nrows = B * Ho;
  int nblk = std::max(1, std::min(nrows, std::min(1024, (4 << 20) / std::max(1, OUT))));
  const int per = (nrows + nblk - 1) / nblk;
  *rows_per_block = per;
  return (nrows + per - 1) / per;
}

void sconv_wgrad_launch(const SconvWgradLaunch& L, int nblk, int rows_per_block, hipStream_t stream) {
  swg::WArgs a{L.x, L.dy, L.xstr, L.ystr, L.Cin, L.Cout, L.B, L.Hi, L.Wi, L.Ho, L.Wo, L.KH, L.KW, L.S, L.P,
               rows_per_block, L.part};
  static const int co_env = [] {
    const char* e = getenv("RS_SWG_CO");
    return e ? atoi(e) : 8;
  }();
  const bool co8 = co_env == 8 && L.Cout % 8 == 0;
  if (L.f32) {
    if (co8) hipLaunchKernelGGL((swg::sconv_wgrad_kernel<float, 8>), dim3(nblk), dim3(swg::THREADS), 0, stream, a);
    else hipLaunchKernelGGL((swg::sconv_wgrad_kernel<float, 4>), dim3(nblk), dim3(swg::THREADS), 0, stream, a);
  } else {
    if (co8) hipLaunchKernelGGL((swg::sconv_wgrad_kernel<bf16_t, 8>), dim3(nblk), dim3(swg::THREADS), 0, stream, a);
    else hipLaunchKernelGGL((swg::sconv_wgrad_kernel<bf16_t, 4>), dim3(nblk), dim3(swg::THREADS), 0, stream, a);
  }
  const int OUT = L.Cout * L.KH * L.KW * L.Cin;
  hipLaunchKernelGGL(swg::sconv_wgrad_reduce_kernel, dim3(cdiv(OUT, swg::RD_O)), dim3(swg::RD_O * swg::RD_L), 0, stream,
                     L.part, nblk, OUT, L.dw);
}

}  // namespace rs
