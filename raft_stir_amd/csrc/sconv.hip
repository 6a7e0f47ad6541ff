// Narrow-channel convolutions of RAFT-small's encoders (reference
// core/extractor.py:60-116 BottleneckBlock and :195-267 SmallEncoder: 1x1 and
// 3x3 convs, stride 1 / 2, with 8, 16, 24, 32, 64 or 96 channels) for
// inference, NHWC.
//
// These channel counts do not fill a 16- or 32-deep MFMA K step, and the
// convs are tiny (the STIR tracker's 1/2-res 3x3 8 -> 8 conv is 0.09 GFLOP):
// MIOpen runs them as implicit GEMMs of ~7-13 us each plus a separate bias
// kernel, and bf16 autocast adds a weight cast per call.  Here one VALU pass:
//  * a wave owns 64 consecutive output pixels x 8 output channels (one
//    channel group per wave: every lane reads the same weights, so the fp32
//    weight tile in LDS is read as broadcasts);
//  * per tap and 8-channel input chunk a lane loads 16 bytes of its input
//    pixel and does 64 FMAs; fp32 accumulation;
//  * epilogue: + bias, optional ReLU, optional residual add + ReLU (the
//    bottleneck's relu(x + relu(conv3(y))) when the encoder has no norm),
//    bf16 or fp32 NHWC store into a channel window.
#include <algorithm>

#include "common.h"

namespace rs {
namespace sconv {

struct SArgs {
  const void* x;
  int xstr, Cin;     // input pixel stride (elements), channels
  int B, Hi, Wi;
  const float* w;    // [Cout][KH][KW][Cin] fp32
  const float* bias; // [Cout] or null
  void* y;
  int ystr, yoff, Cout;
  int Ho, Wo, KH, KW, S, P;
  int relu;          // 1: relu(acc + b)
  const void* res;   // optional residual (same layout / dtype as y): y = relu(y + res)
  int rstr;
};

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

template <typename T>
__device__ __forceinline__ void st8(T* p, const float (&v)[8]);
template <>
__device__ __forceinline__ void st8<bf16_t>(bf16_t* p, const float (&v)[8]) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = uint32_t(f2bf(v[2 * i])) | (uint32_t(f2bf(v[2 * i + 1])) << 16);
  *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}
template <>
__device__ __forceinline__ void st8<float>(float* p, const float (&v)[8]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}

constexpr int kMaxW = 16384;  // fp32 weights per block (64 KiB of dynamic LDS)

// block = 4 waves = 4 output-channel groups of 8 over the same 64 pixels
template <typename T>
__global__ __launch_bounds__(256) void sconv_kernel(SArgs a) {
  extern __shared__ float4 ws4[];  // [ncg * 8][K] fp32, sized by the launch
  float* ws = reinterpret_cast<float*>(ws4);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int cg0 = blockIdx.y * 4;                 // first channel group of the block
  const int ncg = min(4, a.Cout / 8 - cg0);
  const int K = a.KH * a.KW * a.Cin;              // weights per output channel
  // stage this block's (<= 32) output channels' weights
  for (int i = t; i < ncg * 8 * K; i += 256) ws[i] = a.w[(size_t)cg0 * 8 * K + i];
  __syncthreads();
  if (wave >= ncg) return;
  const int p = blockIdx.x * 64 + lane;
  const int P = a.B * a.Ho * a.Wo;
  if (p >= P) return;
  const int b = p / (a.Ho * a.Wo), q = p - b * a.Ho * a.Wo;
  const int oy = q / a.Wo, ox = q - oy * a.Wo;
  const float* wg = ws + wave * 8 * K;            // [8 co][K]
  // even / odd input-channel partial sums per output channel: the 64 FMAs of
  // an 8-channel step as 32 packed v_pk_fma_f32 (two fp32 FMAs per lane per issue)
  typedef float f2_t __attribute__((ext_vector_type(2)));
  f2_t acc2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc2[j] = f2_t{0.f, 0.f};
  const T* x = static_cast<const T*>(a.x);
  for (int ky = 0; ky < a.KH; ++ky) {
    const int iy = oy * a.S + ky - a.P;
    if ((unsigned)iy >= (unsigned)a.Hi) continue;
    for (int kx = 0; kx < a.KW; ++kx) {
      const int ix = ox * a.S + kx - a.P;
      if ((unsigned)ix >= (unsigned)a.Wi) continue;
      const T* xp = x + ((size_t)(b * a.Hi + iy) * a.Wi + ix) * a.xstr;
      const float* wt = wg + (ky * a.KW + kx) * a.Cin;
      for (int c0 = 0; c0 < a.Cin; c0 += 8) {
        float v[8];
        ld8<T>(xp + c0, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          // same address in every lane: LDS broadcast; 32-B aligned (K, Cin, c0 % 8 == 0)
          const float4* wr = reinterpret_cast<const float4*>(wt + j * K + c0);
          const float4 w0 = wr[0], w1 = wr[1];
          acc2[j] = __builtin_elementwise_fma(f2_t{v[0], v[1]}, f2_t{w0.x, w0.y}, acc2[j]);
          acc2[j] = __builtin_elementwise_fma(f2_t{v[2], v[3]}, f2_t{w0.z, w0.w}, acc2[j]);
          acc2[j] = __builtin_elementwise_fma(f2_t{v[4], v[5]}, f2_t{w1.x, w1.y}, acc2[j]);
          acc2[j] = __builtin_elementwise_fma(f2_t{v[6], v[7]}, f2_t{w1.z, w1.w}, acc2[j]);
        }
      }
    }
  }
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = acc2[j].x + acc2[j].y;
  const int co = (cg0 + wave) * 8;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float v = acc[j] + (a.bias ? a.bias[co + j] : 0.f);
    acc[j] = a.relu ? fmaxf(v, 0.f) : v;
  }
  if (a.res) {
    float r[8];
    ld8<T>(static_cast<const T*>(a.res) + (size_t)p * a.rstr + co, r);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = fmaxf(acc[j] + r[j], 0.f);
  }
  st8<T>(static_cast<T*>(a.y) + (size_t)p * a.ystr + a.yoff + co, acc);
}

}  // namespace sconv

struct SconvLaunch {
  const void* x;
  int xstr, Cin, B, Hi, Wi;
  const float* w;
  const float* bias;
  void* y;
  int ystr, yoff, Cout, Ho, Wo, KH, KW, S, P, relu;
  const void* res;
  int rstr;
  bool f32;
};

int sconv_max_weights() { return sconv::kMaxW; }

void sconv_launch(const SconvLaunch& L, hipStream_t stream) {
  sconv::SArgs a{L.x, L.xstr, L.Cin, L.B, L.Hi, L.Wi, L.w, L.bias, L.y, L.ystr, L.yoff, L.Cout,
                 L.Ho, L.Wo, L.KH, L.KW, L.S, L.P, L.relu, L.res, L.rstr};
  const dim3 grid(cdiv(L.B * L.Ho * L.Wo, 64), cdiv(L.Cout / 8, 4));
  const size_t smem = (size_t)std::min(4, L.Cout / 8) * 8 * L.KH * L.KW * L.Cin * sizeof(float);
  if (L.f32)
    hipLaunchKernelGGL(sconv::sconv_kernel<float>, grid, dim3(256), smem, stream, a);
  else
    hipLaunchKernelGGL(sconv::sconv_kernel<bf16_t>, grid, dim3(256), smem, stream, a);
}

}  // namespace rs
