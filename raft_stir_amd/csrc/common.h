// Shared helpers for the gfx950 (CDNA4, MI355X) kernels of raft_stir_amd.
// Plain HIP; wave64; no CUDA compatibility layer.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rs {

constexpr int kWave = 64;

typedef __attribute__((ext_vector_type(8))) short bf16x8_t;   // 8 bf16 = 4 VGPRs
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;

typedef uint16_t bf16_t;  // raw bf16 bits

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}

// round-to-nearest-even f32 -> bf16 (NaN kept a NaN)
__device__ __forceinline__ bf16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return static_cast<bf16_t>((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<bf16_t>(u >> 16);
}

template <typename T> struct io;
template <> struct io<float> {
  __device__ __forceinline__ static float ld(const float* p) { return *p; }
  __device__ __forceinline__ static void st(float* p, float v) { *p = v; }
};
template <> struct io<bf16_t> {
  __device__ __forceinline__ static float ld(const bf16_t* p) { return bf2f(*p); }
  __device__ __forceinline__ static void st(bf16_t* p, float v) { *p = f2bf(v); }
};

// v_rcp_f32 (1 ulp) instead of an IEEE division (a ~12-instruction
// div_scale / div_fmas / div_fixup sequence per call in the conv epilogues)
__device__ __forceinline__ float rcpf_(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float sigmoidf_(float x) { return rcpf_(1.f + __expf(-x)); }
__device__ __forceinline__ float tanhf_(float x) {
  // tanh(x) = 1 - 2/(exp(2x)+1); saturates correctly for large |x|
  float e = __expf(2.f * x);
  return 1.f - 2.f * rcpf_(e + 1.f);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__host__ __device__ __forceinline__ int cdiv(int a, int b) { return (a + b - 1) / b; }
__host__ __device__ __forceinline__ int round_up(int a, int b) { return cdiv(a, b) * b; }

}  // namespace rs

