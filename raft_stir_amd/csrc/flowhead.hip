// Flow-head output convolution (reference core/update.py:6-14, FlowHead.conv2:
// 3x3, Cin = 256 (full) / 128 (small) -> 2 channels) and its input gradient.
//
// With only 2 output channels this conv is not GEMM-shaped: on the MFMA conv
// kernel 14 of the 16 output rows are padding and each 16-pixel block is one
// long dependent load->MFMA chain (28 us at the training shape), and its
// dgrad ran as a conv over a 64-channel zero-padded gradient (32 us).  Both
// are bandwidth problems (read the 256-channel hidden state once, write it
// once), so they are VALU kernels with the channels across the lanes:
//
//   forward : one wave = 8 consecutive pixels of a row; lane l holds channels
//             [CPL*l, CPL*l + CPL) of the 3 x 10 input neighbourhood (one
//             coalesced row read per input pixel) and fp32 weights for them;
//             the 8 x 2 per-lane partial sums are reduced across the wave by
//             a halving butterfly (17 shuffles instead of 96), then the
//             coords epilogue: crd = src + bias + conv (EPI_FLOW semantics).
//   dgrad   : one wave = 8 consecutive pixels; the fp32 flow gradient of the
//             3 x 10 neighbourhood is wave-uniform (scalar loads), lane l
//             produces channels [CPL*l, CPL*l + CPL) of each pixel's input
//             gradient, masked by the hidden ReLU (EPI_RELU_BWD semantics).
#include "common.h"

namespace rs {
namespace fh {

constexpr int PX = 8;  // pixels per wave

template <int CPL>
__device__ __forceinline__ void ldc(const bf16_t* p, float (&f)[CPL]) {
  if constexpr (CPL == 4) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    f[0] = bf2f((bf16_t)(u.x & 0xffffu));
    f[1] = bf2f((bf16_t)(u.x >> 16));
    f[2] = bf2f((bf16_t)(u.y & 0xffffu));
    f[3] = bf2f((bf16_t)(u.y >> 16));
  } else {
    const uint32_t u = *reinterpret_cast<const uint32_t*>(p);
    f[0] = bf2f((bf16_t)(u & 0xffffu));
    f[1] = bf2f((bf16_t)(u >> 16));
  }
}

// fp32 activations (the fp32 inference engine)
template <int CPL>
__device__ __forceinline__ void ldc(const float* p, float (&f)[CPL]) {
  if constexpr (CPL == 4) {
    const float4 u = *reinterpret_cast<const float4*>(p);
    f[0] = u.x; f[1] = u.y; f[2] = u.z; f[3] = u.w;
  } else {
    const float2 u = *reinterpret_cast<const float2*>(p);
    f[0] = u.x; f[1] = u.y;
  }
}

template <int CPL>
__device__ __forceinline__ void stc(bf16_t* p, const float (&f)[CPL]) {
  if constexpr (CPL == 4) {
    uint2 u;
    u.x = uint32_t(f2bf(f[0])) | (uint32_t(f2bf(f[1])) << 16);
    u.y = uint32_t(f2bf(f[2])) | (uint32_t(f2bf(f[3])) << 16);
    *reinterpret_cast<uint2*>(p) = u;
  } else {
    *reinterpret_cast<uint32_t*>(p) = uint32_t(f2bf(f[0])) | (uint32_t(f2bf(f[1])) << 16);
  }
}

template <int CPL>
__device__ __forceinline__ void stc(float* p, const float (&f)[CPL]) {
  if constexpr (CPL == 4)
    *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
  else
    *reinterpret_cast<float2*>(p) = make_float2(f[0], f[1]);
}

// x: NHWC bf16 or fp32 (pixel stride xstr, channel offset xoff), w: fp32
// [2][9][Cin], crd / src: (B, 2, H, W) fp32 (src may alias crd).
template <int CPL, typename XT>
__global__ __launch_bounds__(256) void flowhead_fwd_kernel(const XT* __restrict__ x, int xstr, int xoff,
                                                           const float* __restrict__ w,
                                                           const float* __restrict__ bias, int B, int H, int W,
                                                           float* crd, const float* src) {
  constexpr int CIN = 64 * CPL;
  const int lane = threadIdx.x & 63;
  const int segs_row = cdiv(W, PX);
  const int seg = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (seg >= B * H * segs_row) return;
  const int br = seg / segs_row, x0 = (seg - br * segs_row) * PX;
  const int b = br / H, y = br - b * H;
  float wr[2][9][CPL];
#pragma unroll
  for (int co = 0; co < 2; ++co)
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int j = 0; j < CPL; ++j) wr[co][t][j] = w[(co * 9 + t) * CIN + lane * CPL + j];
  float acc[PX * 2];
#pragma unroll
  for (int i = 0; i < PX * 2; ++i) acc[i] = 0.f;
  // all 3 x (PX + 2) neighbourhood loads are unconditional (clamped address,
  // 0/1 factor outside the image), so they are issued back to back and the
  // wave waits for memory once instead of once per load
  float v3[3][PX + 2][CPL];
#pragma unroll
  for (int ty = 0; ty < 3; ++ty) {
    const int yy = y + ty - 1;
    const bool iny = yy >= 0 && yy < H;
    const XT* row = x + ((size_t)(b * H + (iny ? yy : y)) * W) * xstr + xoff + lane * CPL;
#pragma unroll
    for (int c = 0; c < PX + 2; ++c) {
      const int xx = x0 + c - 1;
      const bool in = iny && xx >= 0 && xx < W;
      ldc<CPL>(row + (size_t)(in ? xx : x0) * xstr, v3[ty][c]);
      const float m = in ? 1.f : 0.f;
#pragma unroll
      for (int j = 0; j < CPL; ++j) v3[ty][c][j] *= m;
    }
  }
#pragma unroll
  for (int ty = 0; ty < 3; ++ty) {
#pragma unroll
    for (int c = 0; c < PX + 2; ++c) {
      const float (&v)[CPL] = v3[ty][c];
#pragma unroll
      for (int tx = 0; tx < 3; ++tx) {
        const int px = c - tx;  // output pixel x0 + px uses input column x0 + px + tx - 1
        if (px < 0 || px >= PX) continue;
#pragma unroll
        for (int co = 0; co < 2; ++co)
#pragma unroll
          for (int j = 0; j < CPL; ++j) acc[px * 2 + co] = fmaf(v[j], wr[co][ty * 3 + tx][j], acc[px * 2 + co]);
      }
    }
  }
  // halving butterfly: after the xor-32/16/8/4 steps lane l holds value (l >> 2) & 15 summed
  // over its 16-lane group; xor-2/1 finish the sum
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const bool hi = lane & 32;
    const float keep = hi ? acc[8 + i] : acc[i], send = hi ? acc[i] : acc[8 + i];
    acc[i] = keep + __shfl_xor(send, 32, 64);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bool hi = lane & 16;
    const float keep = hi ? acc[4 + i] : acc[i], send = hi ? acc[i] : acc[4 + i];
    acc[i] = keep + __shfl_xor(send, 16, 64);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const bool hi = lane & 8;
    const float keep = hi ? acc[2 + i] : acc[i], send = hi ? acc[i] : acc[2 + i];
    acc[i] = keep + __shfl_xor(send, 8, 64);
  }
  {
    const bool hi = lane & 4;
    const float keep = hi ? acc[1] : acc[0], send = hi ? acc[0] : acc[1];
    acc[0] = keep + __shfl_xor(send, 4, 64);
  }
  acc[0] += __shfl_xor(acc[0], 2, 64);
  acc[0] += __shfl_xor(acc[0], 1, 64);
  const int idx = (lane >> 2) & 15, px = idx >> 1, co = idx & 1;
  if ((lane & 3) == 0 && x0 + px < W) {
    const size_t o = ((size_t)(b * 2 + co) * H + y) * W + x0 + px;
    crd[o] = src[o] + bias[co] + acc[0];
  }
}

// dflow: (B, 2, H, W) fp32; w: fp32 [2][9][Cin]; act: NHWC T hidden (ReLU output,
// stride astr, offset aoff); out: NHWC T (stride ostr, offset ooff), Cin channels;
// T = bf16, or fp32 (the fp32 training engine).
template <int CPL, typename T>
__global__ __launch_bounds__(256) void flowhead_dgrad_kernel(const float* __restrict__ dflow,
                                                             const float* __restrict__ w, int B, int H, int W,
                                                             const T* __restrict__ act, int astr, int aoff,
                                                             T* __restrict__ out, int ostr, int ooff) {
  constexpr int CIN = 64 * CPL;
  const int lane = threadIdx.x & 63;
  const int segs_row = cdiv(W, PX);
  const int seg = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (seg >= B * H * segs_row) return;
  const int br = seg / segs_row, x0 = (seg - br * segs_row) * PX;
  const int b = br / H, y = br - b * H;
  float wr[2][9][CPL];
#pragma unroll
  for (int co = 0; co < 2; ++co)
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int j = 0; j < CPL; ++j) wr[co][t][j] = w[(co * 9 + t) * CIN + lane * CPL + j];
  // dx[q] = sum_{ty,tx} sum_co W[co][ty][tx] * dflow[q - (ty - 1, tx - 1)][co]
  float g[3][PX + 2][2];  // dflow at rows y-1..y+1, columns x0-1..x0+PX (wave-uniform)
  const size_t plane = (size_t)H * W;
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const int yy = y + r - 1;
#pragma unroll
    for (int c = 0; c < PX + 2; ++c) {
      const int xx = x0 + c - 1;
      const bool in = yy >= 0 && yy < H && xx >= 0 && xx < W;
      const size_t o = (size_t)b * 2 * plane + (size_t)(in ? yy : 0) * W + (in ? xx : 0);
      g[r][c][0] = in ? dflow[o] : 0.f;
      g[r][c][1] = in ? dflow[o + plane] : 0.f;
    }
  }
  // the hidden activations of the PX pixels (ReLU mask), loaded up front
  float av[PX][CPL];
#pragma unroll
  for (int px = 0; px < PX; ++px) {
    const int xc = x0 + px < W ? x0 + px : W - 1;
    ldc<CPL>(act + ((size_t)(b * H + y) * W + xc) * astr + aoff + lane * CPL, av[px]);
  }
#pragma unroll
  for (int px = 0; px < PX; ++px) {
    if (x0 + px >= W) break;
    float acc[CPL];
#pragma unroll
    for (int j = 0; j < CPL; ++j) acc[j] = 0.f;
#pragma unroll
    for (int ty = 0; ty < 3; ++ty)
#pragma unroll
      for (int tx = 0; tx < 3; ++tx) {
        // output pixel (y - (ty-1), x - (tx-1)) = neighbourhood row 2 - ty, column px + 2 - tx
        const float g0 = g[2 - ty][px + 2 - tx][0], g1 = g[2 - ty][px + 2 - tx][1];
#pragma unroll
        for (int j = 0; j < CPL; ++j)
          acc[j] = fmaf(g0, wr[0][ty * 3 + tx][j], fmaf(g1, wr[1][ty * 3 + tx][j], acc[j]));
      }
    const size_t p = (size_t)(b * H + y) * W + x0 + px;
#pragma unroll
    for (int j = 0; j < CPL; ++j) acc[j] = av[px][j] > 0.f ? acc[j] : 0.f;
    stc<CPL>(out + p * ostr + ooff + lane * CPL, acc);
  }
}

}  // namespace fh

void flowhead_fwd_launch(const void* x, int xstr, int xoff, int cin, const float* w, const float* bias, int B,
                         int H, int W, float* crd, const float* src, bool x_f32, hipStream_t s) {
  const int segs = B * H * cdiv(W, fh::PX);
  const dim3 grid(cdiv(segs, 4));
  if (x_f32) {
    const float* xf = static_cast<const float*>(x);
    if (cin == 256)
      hipLaunchKernelGGL((fh::flowhead_fwd_kernel<4, float>), grid, dim3(256), 0, s, xf, xstr, xoff, w, bias, B, H, W,
                         crd, src);
    else
      hipLaunchKernelGGL((fh::flowhead_fwd_kernel<2, float>), grid, dim3(256), 0, s, xf, xstr, xoff, w, bias, B, H, W,
                         crd, src);
    return;
  }
  const bf16_t* xb = static_cast<const bf16_t*>(x);
  if (cin == 256)
    hipLaunchKernelGGL((fh::flowhead_fwd_kernel<4, bf16_t>), grid, dim3(256), 0, s, xb, xstr, xoff, w, bias, B, H, W,
                       crd, src);
  else
    hipLaunchKernelGGL((fh::flowhead_fwd_kernel<2, bf16_t>), grid, dim3(256), 0, s, xb, xstr, xoff, w, bias, B, H, W,
                       crd, src);
}

void flowhead_dgrad_launch(const float* dflow, const float* w, int cin, int B, int H, int W, const void* act,
                           int astr, int aoff, void* out, int ostr, int ooff, bool f32, hipStream_t s) {
  const int segs = B * H * cdiv(W, fh::PX);
  const dim3 grid(cdiv(segs, 4));
  if (f32) {
    const float* ab = static_cast<const float*>(act);
    float* ob = static_cast<float*>(out);
    if (cin == 256)
      hipLaunchKernelGGL((fh::flowhead_dgrad_kernel<4, float>), grid, dim3(256), 0, s, dflow, w, B, H, W, ab, astr,
                         aoff, ob, ostr, ooff);
    else
      hipLaunchKernelGGL((fh::flowhead_dgrad_kernel<2, float>), grid, dim3(256), 0, s, dflow, w, B, H, W, ab, astr,
                         aoff, ob, ostr, ooff);
    return;
  }
  const bf16_t* ab = static_cast<const bf16_t*>(act);
  bf16_t* ob = static_cast<bf16_t*>(out);
  if (cin == 256)
    hipLaunchKernelGGL((fh::flowhead_dgrad_kernel<4, bf16_t>), grid, dim3(256), 0, s, dflow, w, B, H, W, ab, astr,
                       aoff, ob, ostr, ooff);
  else
    hipLaunchKernelGGL((fh::flowhead_dgrad_kernel<2, bf16_t>), grid, dim3(256), 0, s, dflow, w, B, H, W, ab, astr,
                       aoff, ob, ostr, ooff);
}

}  // namespace rs
