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

// round-to-nearest-even f32 -> bf16 (NaN kept a NaN): gfx950's
// v_cvt_pk_bf16_f32, one VALU op (the integer rounding it replaced took ~6
// per value, on every bf16 store of every epilogue)
__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, static_cast<__bf16>(f)); }

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

// Reduce-scatter across groups of L lanes (L a power of two; the lanes that
// differ only in their low log2(L) bits): every lane enters with N partial
// values and leaves with the group totals of N/L of them in v[0 .. N/L), the
// totals of entries (N/L) * (lane & (L-1)) + k.  log2(L) exchange steps, each
// sending half of the still-live values (N - N/L shuffles in all, instead of
// N * log2(L) for a butterfly all-reduce of every value).  All lanes of the
// wave must be active.
template <int N0, int n, int m>
__device__ __forceinline__ void rscat_step(float (&v)[N0], int lane) {
  if constexpr (m >= 1) {
    constexpr int half = n / 2;
    const bool up = (lane & m) != 0;
#pragma unroll
    for (int i = 0; i < half; ++i) {
      const float send = up ? v[i] : v[i + half];
      const float keep = up ? v[i + half] : v[i];
      v[i] = keep + __shfl_xor(send, m, 64);
    }
    rscat_step<N0, half, m / 2>(v, lane);
  }
}
template <int N, int L>
__device__ __forceinline__ void lane_reduce_scatter(float (&v)[N], int lane) {
  static_assert(N % L == 0 && (L & (L - 1)) == 0, "N must be a multiple of the power-of-two group size");
  rscat_step<N, N, L / 2>(v, lane);
}

__host__ __device__ __forceinline__ int cdiv(int a, int b) { return (a + b - 1) / b; }
__host__ __device__ __forceinline__ int round_up(int a, int b) { return cdiv(a, b) * b; }

}  // namespace rs

