// Memory-efficient ("alternate") correlation: forward + backward.
//
// Replaces reference alt_cuda_corr (correlation_kernel.cu K1/K2, 32-thread
// blocks, warp-synchronous LDS use without barriers, fp32 only, backward never
// wired to autograd -- SURVEY §2.3, defects B1-B4).  Semantics:
//
//   out[b, y, x, l*K2 + k] = scale * sum_c f1[b,y,x,c] * bilinear(f2_l[b,:,:,c], p + (dx,dy))
//
// with f2_l = avgpool^l(f2) (channels-last), p = coords/2^l, zero padding,
// k = (dx+r)*(2r+1) + (dy+r) (x-major).  Nothing of size HW x HW is stored.
//
// CDNA4 mapping: one wave64 per query pixel.  The (2r+2)^2 integer cells of a
// level are processed 8 at a time: lane = 8 * cell_slot + channel_slot, each
// lane holding C/8 channels of f1 in registers (4-wide interleaved so that
// the 8 lanes of a cell read one 128-B segment per instruction).  A cell's
// dot product is reduced across its 8 lanes with 3 xor-shuffles and parked in
// LDS; the (2r+1)^2 bilinear taps are then formed from LDS (each cell dot is
// computed ONCE and reused by up to 4 taps -- the K1 decomposition).
// Backward: per level, the cell gradients g(cell) are gathered from dout (same
// decomposition as corr_lookup's backward), then df1 accumulates in registers
// (plain store once per pixel: every pixel owns its df1 row) and df2_l
// receives g * f1 through float atomics (cells are shared between pixels).
// Deterministic mode (DET): the df2 contributions are rounded to 32.32
// fixed point and summed with 64-bit integer atomics -- integer addition is
// associative, so the sums do not depend on the order the waves arrive in
// (|df2| < 2^31, resolution 2^-32) -- then converted to fp32 by one pass.

#include <algorithm>
#include <type_traits>

#include "common.h"

namespace rs {
namespace otf {

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_v;

constexpr int WAVES = 4;
constexpr int MAXE2 = 100;  // (2r+2)^2 for r <= 4

template <typename T> __device__ __forceinline__ float4 ld4(const T* p);
template <> __device__ __forceinline__ float4 ld4<float>(const float* p) {
  return *reinterpret_cast<const float4*>(p);
}
template <> __device__ __forceinline__ float4 ld4<bf16_t>(const bf16_t* p) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                     __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
}

struct Lvl {
  const void* p[4];
  int H[4];
  int W[4];
};
struct LvlMut {
  float* p[4];
  int H[4];
  int W[4];
};

// CQ = C / 32: float4 groups per lane
template <typename T, typename OutT, int CQ>
__global__ __launch_bounds__(WAVES * 64) void otf_fwd_kernel(const T* __restrict__ f1, Lvl f2,
                                                             int levels,
                                                             const float* __restrict__ coords,
                                                             int B, int N1, int r, float scale,
                                                             OutT* __restrict__ out) {
  __shared__ float dots[WAVES][MAXE2];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long pix = (long)blockIdx.x * WAVES + wave;
  const bool active = pix < (long)B * N1;
  const long pixc = active ? pix : 0;
  const int b = (int)(pixc / N1), n = (int)(pixc % N1);
  constexpr int C = CQ * 32;
  const int slot = lane & 7, grp = lane >> 3;
  const int D = 2 * r + 1, K2 = D * D, E = D + 1, E2 = E * E, CH = levels * K2;

  // bf16: f1 stays packed and each 4-channel piece is two v_dot2_f32_bf16
  // (fp32 accumulation) instead of 4 unpacks + 4 FMAs
  constexpr bool BF = std::is_same<T, bf16_t>::value;
  float4 a[CQ];
  uint2 ab[CQ];
  const T* f1p = f1 + pixc * C;
#pragma unroll
  for (int q = 0; q < CQ; ++q) {
    if constexpr (BF)
      ab[q] = *reinterpret_cast<const uint2*>(f1p + q * 32 + slot * 4);
    else
      a[q] = ld4<T>(f1p + q * 32 + slot * 4);
  }

  const float cx0 = coords[((size_t)b * 2 + 0) * N1 + n];
  const float cy0 = coords[((size_t)b * 2 + 1) * N1 + n];

  for (int l = 0; l < levels; ++l) {
    const float inv = 1.f / (float)(1 << l);
    const float cx = cx0 * inv, cy = cy0 * inv;
    const float bx = floorf(cx), by = floorf(cy);
    const float fx = cx - bx, fy = cy - by;
    const int H = f2.H[l], W = f2.W[l];
    const T* f2b = static_cast<const T*>(f2.p[l]) + (size_t)b * H * W * C;
    for (int base = 0; base < E2; base += 8) {
      const int cell = base + grp;
      const int X = (int)bx - r + cell / E, Y = (int)by - r + cell % E;
      float s = 0.f;
      if (cell < E2 && X >= 0 && X < W && Y >= 0 && Y < H) {
        const T* row = f2b + ((size_t)Y * W + X) * C + slot * 4;
#pragma unroll
        for (int q = 0; q < CQ; ++q) {
          if constexpr (BF) {
            const uint2 v = *reinterpret_cast<const uint2*>(row + q * 32);
            s = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_v, ab[q].x),
                                                __builtin_bit_cast(bf16x2_v, v.x), s, false);
            s = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_v, ab[q].y),
                                                __builtin_bit_cast(bf16x2_v, v.y), s, false);
          } else {
            const float4 v = ld4<T>(row + q * 32);
            s += a[q].x * v.x + a[q].y * v.y + a[q].z * v.z + a[q].w * v.w;
          }
        }
      }
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      s += __shfl_xor(s, 4, 64);
      if (slot == 0 && cell < E2) dots[wave][cell] = s;
    }
    __syncthreads();
    if (active) {
      OutT* o = out + pix * CH + l * K2;
      for (int t = lane; t < K2; t += 64) {
        const int i = t / D, j = t % D;  // cell (a=i, c=j) is the tap's lower corner
        const float v = (1.f - fx) * (1.f - fy) * dots[wave][i * E + j] +
                        fx * (1.f - fy) * dots[wave][(i + 1) * E + j] +
                        (1.f - fx) * fy * dots[wave][i * E + j + 1] +
                        fx * fy * dots[wave][(i + 1) * E + j + 1];
        io<OutT>::st(o + t, v * scale);
      }
    }
    __syncthreads();
  }
}

__device__ __forceinline__ void fx_add(unsigned long long* p, float v) {
  atomicAdd(p, (unsigned long long)__double2ll_rn((double)v * 4294967296.0));
}

template <typename T, typename GT, int CQ, bool DET>
__global__ __launch_bounds__(WAVES * 64) void otf_bwd_kernel(const T* __restrict__ f1, Lvl f2,
                                                             int levels,
                                                             const float* __restrict__ coords,
                                                             int B, int N1, int r, float scale,
                                                             const GT* __restrict__ dout,
                                                             float* __restrict__ df1, LvlMut df2) {
  __shared__ float gs[WAVES][MAXE2];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long pix = (long)blockIdx.x * WAVES + wave;
  const bool active = pix < (long)B * N1;
  const long pixc = active ? pix : 0;
  const int b = (int)(pixc / N1), n = (int)(pixc % N1);
  constexpr int C = CQ * 32;
  const int slot = lane & 7, grp = lane >> 3;
  const int D = 2 * r + 1, K2 = D * D, E = D + 1, E2 = E * E, CH = levels * K2;

  float4 a[CQ], da[CQ];
  const T* f1p = f1 + pixc * C;
#pragma unroll
  for (int q = 0; q < CQ; ++q) {
    a[q] = ld4<T>(f1p + q * 32 + slot * 4);
    da[q] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const float cx0 = coords[((size_t)b * 2 + 0) * N1 + n];
  const float cy0 = coords[((size_t)b * 2 + 1) * N1 + n];

  for (int l = 0; l < levels; ++l) {
    const float inv = 1.f / (float)(1 << l);
    const float cx = cx0 * inv, cy = cy0 * inv;
    const float bx = floorf(cx), by = floorf(cy);
    const float fx = cx - bx, fy = cy - by;
    const int H = f2.H[l], W = f2.W[l];
    // gather cell gradients
    const GT* g = dout + pixc * CH + l * K2;
    for (int cell = lane; cell < E2; cell += 64) {
      const int ca = cell / E, cc = cell % E;
      float acc = 0.f;
#pragma unroll
      for (int di = 0; di < 2; ++di) {
        const int i = ca - di;
        if (i < 0 || i >= D) continue;
        const float wx = di == 0 ? (1.f - fx) : fx;
#pragma unroll
        for (int dj = 0; dj < 2; ++dj) {
          const int j = cc - dj;
          if (j < 0 || j >= D) continue;
          const float wy = dj == 0 ? (1.f - fy) : fy;
          acc += wx * wy * io<GT>::ld(g + i * D + j);
        }
      }
      gs[wave][cell] = active ? acc * scale : 0.f;
    }
    __syncthreads();
    const T* f2b = static_cast<const T*>(f2.p[l]) + (size_t)b * H * W * C;
    float* d2b = DET ? nullptr : df2.p[l] + (size_t)b * H * W * C;
    for (int base = 0; base < E2; base += 8) {
      const int cell = base + grp;
      const int X = (int)bx - r + cell / E, Y = (int)by - r + cell % E;
      if (active && cell < E2 && X >= 0 && X < W && Y >= 0 && Y < H) {
        const float gc = gs[wave][cell];
        if (gc != 0.f) {
          const size_t off = ((size_t)Y * W + X) * C + slot * 4;
#pragma unroll
          for (int q = 0; q < CQ; ++q) {
            const float4 v = ld4<T>(f2b + off + q * 32);
            da[q].x += gc * v.x; da[q].y += gc * v.y; da[q].z += gc * v.z; da[q].w += gc * v.w;
            if constexpr (DET) {  // df2.p[l]: int64 32.32 fixed-point accumulators
              unsigned long long* d = reinterpret_cast<unsigned long long*>(df2.p[l]) +
                                      (size_t)b * H * W * C + off + q * 32;
              fx_add(d + 0, gc * a[q].x);
              fx_add(d + 1, gc * a[q].y);
              fx_add(d + 2, gc * a[q].z);
              fx_add(d + 3, gc * a[q].w);
            } else {
              float* d = d2b + off + q * 32;
              atomicAdd(d + 0, gc * a[q].x);
              atomicAdd(d + 1, gc * a[q].y);
              atomicAdd(d + 2, gc * a[q].z);
              atomicAdd(d + 3, gc * a[q].w);
            }
          }
        }
      }
    }
    __syncthreads();
  }
  // reduce da over the 8 cell groups (lanes with equal slot)
#pragma unroll
  for (int q = 0; q < CQ; ++q) {
#pragma unroll
    for (int o = 8; o < 64; o <<= 1) {
      da[q].x += __shfl_xor(da[q].x, o, 64);
      da[q].y += __shfl_xor(da[q].y, o, 64);
      da[q].z += __shfl_xor(da[q].z, o, 64);
      da[q].w += __shfl_xor(da[q].w, o, 64);
    }
  }
  if (active && grp == 0) {
#pragma unroll
    for (int q = 0; q < CQ; ++q)
      *reinterpret_cast<float4*>(df1 + pix * C + q * 32 + slot * 4) = da[q];
  }
}

// 32.32 fixed point (int64) -> fp32
__global__ __launch_bounds__(256) void fx_to_f32_kernel(const long long* __restrict__ in, long n,
                                                        float* __restrict__ out) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    out[i] = (float)((double)in[i] * (1.0 / 4294967296.0));
}

}  // namespace otf

#define RS_OTF_DISPATCH_CQ(CQV, ...)                                  \
  switch (CQV) {                                                      \
    case 2: { constexpr int CQ = 2; __VA_ARGS__; } break;             \
    case 3: { constexpr int CQ = 3; __VA_ARGS__; } break;             \
    case 4: { constexpr int CQ = 4; __VA_ARGS__; } break;             \
    case 8: { constexpr int CQ = 8; __VA_ARGS__; } break;             \
    default: { constexpr int CQ = 1; __VA_ARGS__; } break;            \
  }

bool corr_otf_supported_channels(int C) {
  return C % 32 == 0 && (C / 32 == 1 || C / 32 == 2 || C / 32 == 3 || C / 32 == 4 || C / 32 == 8);
}

void corr_otf_fwd_launch(const void* f1, const void* const* f2, const int* Hs, const int* Ws,
                         int levels, bool fm_bf16, const float* coords, int B, int N1, int C,
                         int r, float scale, void* out, bool out_bf16, hipStream_t stream) {
  otf::Lvl p;
  for (int l = 0; l < 4; ++l) {
    p.p[l] = l < levels ? f2[l] : nullptr;
    p.H[l] = l < levels ? Hs[l] : 0;
    p.W[l] = l < levels ? Ws[l] : 0;
  }
  const long npix = (long)B * N1;
  dim3 grid((unsigned)cdiv((int)npix, otf::WAVES)), block(otf::WAVES * 64);
  const int cq = C / 32;
#define RS_L(T, OT)                                                                           \
  hipLaunchKernelGGL((otf::otf_fwd_kernel<T, OT, CQ>), grid, block, 0, stream,               \
                     static_cast<const T*>(f1), p, levels, coords, B, N1, r, scale,           \
                     static_cast<OT*>(out))
  if (fm_bf16) {
    if (out_bf16) { RS_OTF_DISPATCH_CQ(cq, RS_L(bf16_t, bf16_t)); }
    else { RS_OTF_DISPATCH_CQ(cq, RS_L(bf16_t, float)); }
  } else {
    if (out_bf16) { RS_OTF_DISPATCH_CQ(cq, RS_L(float, bf16_t)); }
    else { RS_OTF_DISPATCH_CQ(cq, RS_L(float, float)); }
  }
#undef RS_L
}

// det: df2[l] are int64 fixed-point accumulators (zeroed) of the level sizes;
// df2f[l] receive their fp32 values
void corr_otf_bwd_launch(const void* f1, const void* const* f2, const int* Hs, const int* Ws,
                         int levels, bool fm_bf16, const float* coords, int B, int N1, int C,
                         int r, float scale, const void* dout, bool dout_bf16, float* df1,
                         float* const* df2, bool det, float* const* df2f, hipStream_t stream) {
  otf::Lvl p;
  otf::LvlMut d;
  for (int l = 0; l < 4; ++l) {
    p.p[l] = l < levels ? f2[l] : nullptr;
    d.p[l] = l < levels ? df2[l] : nullptr;
    p.H[l] = d.H[l] = l < levels ? Hs[l] : 0;
    p.W[l] = d.W[l] = l < levels ? Ws[l] : 0;
  }
  const long npix = (long)B * N1;
  dim3 grid((unsigned)cdiv((int)npix, otf::WAVES)), block(otf::WAVES * 64);
  const int cq = C / 32;
#define RS_L(T, GT)                                                                          \
  if (det)                                                                                   \
    hipLaunchKernelGGL((otf::otf_bwd_kernel<T, GT, CQ, true>), grid, block, 0, stream,       \
                       static_cast<const T*>(f1), p, levels, coords, B, N1, r, scale,        \
                       static_cast<const GT*>(dout), df1, d);                                \
  else                                                                                       \
    hipLaunchKernelGGL((otf::otf_bwd_kernel<T, GT, CQ, false>), grid, block, 0, stream,      \
                       static_cast<const T*>(f1), p, levels, coords, B, N1, r, scale,        \
                       static_cast<const GT*>(dout), df1, d)
  if (fm_bf16) {
    if (dout_bf16) { RS_OTF_DISPATCH_CQ(cq, RS_L(bf16_t, bf16_t)); }
    else { RS_OTF_DISPATCH_CQ(cq, RS_L(bf16_t, float)); }
  } else {
    if (dout_bf16) { RS_OTF_DISPATCH_CQ(cq, RS_L(float, bf16_t)); }
    else { RS_OTF_DISPATCH_CQ(cq, RS_L(float, float)); }
  }
#undef RS_L
  if (det)
    for (int l = 0; l < levels; ++l) {
      const long n = (long)B * Hs[l] * Ws[l] * C;
      const int g = (int)std::min<long>((n + 255) / 256, 16384);
      hipLaunchKernelGGL(otf::fx_to_f32_kernel, dim3(g), dim3(256), 0, stream,
                         reinterpret_cast<const long long*>(df2[l]), n, df2f[l]);
    }
}

}  // namespace rs
