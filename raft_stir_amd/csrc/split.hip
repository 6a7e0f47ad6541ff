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

__global__ __launch_bounds__(256) void split_bf16_kernel(const float* __restrict__ x, long n, bf16_t* __restrict__ hi,
                                                         bf16_t* __restrict__ lo) {
  const long n4 = n / 4;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    const float f[4] = {v.x, v.y, v.z, v.w};
    uint32_t h[2], l[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const bf16_t h0 = f2bf(f[2 * k]), h1 = f2bf(f[2 * k + 1]);
      const bf16_t l0 = f2bf(f[2 * k] - bf2f(h0)), l1 = f2bf(f[2 * k + 1] - bf2f(h1));
      h[k] = uint32_t(h0) | (uint32_t(h1) << 16);
      l[k] = uint32_t(l0) | (uint32_t(l1) << 16);
    }
    reinterpret_cast<uint2*>(hi)[i] = make_uint2(h[0], h[1]);
    reinterpret_cast<uint2*>(lo)[i] = make_uint2(l[0], l[1]);
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
  const int grid = (int)std::min<long>(std::max<long>((n4 + 255) / 256, 1), 8192);
  hipLaunchKernelGGL(splitk::split_bf16_kernel, dim3(grid), dim3(256), 0, s, x, n, hi, lo);
}

}  // namespace rs
