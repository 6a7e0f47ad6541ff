// fp32 -> (hi, lo) bf16 operand split in one pass: hi = bf16(x), lo = bf16(x - hi).
// The fp32 training engine (models/fused_train.py _conv_wgrad) runs its weight
// gradients as bf16 MFMA GEMMs over split operands (dYh.Xh + dYl.Xh + dYh.Xl);
// done with ATen this was four elementwise passes per operand (cast, upcast,
// subtract, cast -- ~13 ms of copy kernels per fp32 step at the Chairs crop,
// profiles/r4/train_fp32_kernel_stats_s14.csv), here one read and two
// half-width writes.
#include <algorithm>

#include "common.h"

namespace rs {
namespace splitk {

__device__ __forceinline__ void split4(const float4& v, uint2& h, uint2& l) {
  typedef float f2_t __attribute__((ext_vector_type(2)));
  typedef __bf16 b2_t __attribute__((ext_vector_type(2)));
  const f2_t p0 = {v.x, v.y}, p1 = {v.z, v.w};
  const uint32_t h0 = __builtin_bit_cast(uint32_t, __builtin_convertvector(p0, b2_t));
  const uint32_t h1 = __builtin_bit_cast(uint32_t, __builtin_convertvector(p1, b2_t));
  const f2_t r0 = p0 - f2_t{__uint_as_float(h0 << 16), __uint_as_float(h0 & 0xffff0000u)};
  const f2_t r1 = p1 - f2_t{__uint_as_float(h1 << 16), __uint_as_float(h1 & 0xffff0000u)};
  h = make_uint2(h0, h1);
  l = make_uint2(__builtin_bit_cast(uint32_t, __builtin_convertvector(r0, b2_t)),
                 __builtin_bit_cast(uint32_t, __builtin_convertvector(r1, b2_t)));
}

// four independent float4 per thread per step (loads in flight before any
// conversion), packed hardware conversions (split4)
__global__ __launch_bounds__(256) void split_bf16_kernel(const float* __restrict__ x, long n, bf16_t* __restrict__ hi,
                                                         bf16_t* __restrict__ lo) {
  const long n4 = n / 4;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i0 = (long)blockIdx.x * blockDim.x + threadIdx.x; i0 < n4; i0 += 4 * stride) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long i = i0 + u * stride;
      if (i < n4) v[u] = reinterpret_cast<const float4*>(x)[i];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long i = i0 + u * stride;
      if (i < n4) {
        uint2 h, l;
        split4(v[u], h, l);
        reinterpret_cast<uint2*>(hi)[i] = h;
        reinterpret_cast<uint2*>(lo)[i] = l;
      }
    }
  }
  // tail (n % 4 elements): the first threads of block 0
  if (blockIdx.x == 0 && threadIdx.x < n - 4 * n4) {
    const long i = 4 * n4 + threadIdx.x;
    const bf16_t h0 = f2bf(x[i]);
    hi[i] = h0;
    lo[i] = f2bf(x[i] - bf2f(h0));
  }
}

}  // namespace splitk

void split_bf16_launch(const float* x, long n, bf16_t* hi, bf16_t* lo, hipStream_t s) {
  const long n4 = n / 4;
  const int grid = (int)std::min<long>(std::max<long>((n4 + 1023) / 1024, 1), 4096);  // 4 float4 per thread
  hipLaunchKernelGGL(splitk::split_bf16_kernel, dim3(grid), dim3(256), 0, s, x, n, hi, lo);
}

}  // namespace rs
