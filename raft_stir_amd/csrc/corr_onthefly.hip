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
// Default kernels (the per-query ones above serve fp32 features in the forward): 4 x 4
// query TILES -- the forward gathers the bounding box of the tile's 16
// windows once per level and computes the cell dots as a small GEMM on MFMA
// (otf_tile_kernel); the backward gathers the tile's cell gradients over the
// same box into LDS, accumulates df1 in registers and sums each box cell's
// df2 over the 16 queries before ONE atomic per (cell, channel)
// (otf_tile_bwd_kernel).
// Deterministic mode (DET): the df2 contributions are rounded to fixed point
// and summed with 64-bit integer atomics -- integer addition is associative,
// so the sums do not depend on the order the waves arrive in -- then
// converted to fp32 by one pass.  The scale is picked per call from max|dout|
// and max|f1| (fx_scan_kernel / fx_scale: every sum fits int64 with
// resolution relative to the data), and a non-finite input turns the whole
// df2 into NaN (integer sums would saturate it into a finite value).

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

// ------------------------------------------------------- tiled forward (MFMA)
// Block = 4 waves = a 4 x 4 tile of query pixels.  Per level the 16 windows
// of a tile nearly coincide under smooth flow (neighbouring centres differ by
// a fraction of a cell at the coarse levels), so the bounding box of their
// union, BW x BH cells (typically 120-170 at r = 4, <= MAXC), is gathered
// ONCE for the whole tile and the cell dots become a small GEMM on
// mfma_f32_16x16x32_bf16: A = the tile's 16 f1 rows (registers, loaded once
// for all levels), B = 16 bounding-box cells x 32 channels per MFMA, one
// 16-byte load per lane straight from the channels-last level (zero outside
// the image).  Each cell's C-vector is read once per tile instead of once per
// query: ~6x less gather traffic than otf_fwd_kernel at r = 4.  A level whose
// bounding box exceeds MAXC (motion boundaries, large flow differences inside
// the tile) falls back to otf_fwd_kernel's per-query v_dot2 cell loop, one
// query per wave at a time.  Both paths park the cell dots in LDS (the box
// layout, or the per-query E x E layout) and the bilinear taps are formed
// from there with the same arithmetic as otf_fwd_kernel.  Blocks are ordered
// XCD-major (block i runs on XCD i % 8), so each XCD's L2 sees a contiguous
// run of tiles whose windows overlap.
constexpr int TQ = 4;      // tile side, queries
constexpr int MAXC = 256;  // bounding-box cells on the MFMA path (16 chunks of 16)

template <typename OutT, int CQ>
__global__ __launch_bounds__(256) void otf_tile_kernel(const bf16_t* __restrict__ f1, Lvl f2, int levels,
                                                       const float* __restrict__ coords, int B, int H1, int W1,
                                                       int tiles_x, int tiles_y, int per_xcd, int r, float scale,
                                                       OutT* __restrict__ out) {
  __shared__ float dots[16][MAXC + 4];
  __shared__ int qoff[16];
  __shared__ float qfx[16], qfy[16];
  constexpr int C = CQ * 32;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tile = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  if (tile >= B * tiles_x * tiles_y) return;  // whole block, before any barrier
  const int b = tile / (tiles_x * tiles_y), t2 = tile % (tiles_x * tiles_y);
  const int ty = t2 / tiles_x, tx = t2 % tiles_x;
  const int N1 = H1 * W1;
  const int D = 2 * r + 1, K2 = D * D, E = D + 1, E2 = E * E, CH = levels * K2;
  const int r16 = lane & 15, q4 = lane >> 4;

  // lane's query = r16 (lanes 16.. mirror 0..15): the MFMA A row and the bounding-box input
  const int qy = ty * TQ + (r16 >> 2), qx = tx * TQ + (r16 & 3);
  const bool qact = qy < H1 && qx < W1;
  const int qn = qact ? qy * W1 + qx : 0;
  const float cx0 = coords[((size_t)b * 2 + 0) * N1 + qn];
  const float cy0 = coords[((size_t)b * 2 + 1) * N1 + qn];
  uint4 fa[CQ];  // A fragments: query r16, channels 32 s + 8 q4 .. + 8
  {
    const bf16_t* p = f1 + ((size_t)b * N1 + qn) * C + 8 * q4;
#pragma unroll
    for (int s = 0; s < CQ; ++s)
      fa[s] = qact ? *reinterpret_cast<const uint4*>(p + 32 * s) : make_uint4(0u, 0u, 0u, 0u);
  }

  for (int l = 0; l < levels; ++l) {
    const float inv = 1.f / (float)(1 << l);
    const float cx = cx0 * inv, cy = cy0 * inv;
    const float bx = floorf(cx), by = floorf(cy);
    const int X0 = (int)bx - r, Y0 = (int)by - r;
    int xmn = qact ? X0 : 0x7fffffff, ymn = qact ? Y0 : 0x7fffffff;
    int xmx = qact ? X0 : -0x7fffffff, ymx = qact ? Y0 : -0x7fffffff;
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) {  // within each 16-lane group: the tile's extremes
      xmn = min(xmn, __shfl_xor(xmn, o, 64));
      ymn = min(ymn, __shfl_xor(ymn, o, 64));
      xmx = max(xmx, __shfl_xor(xmx, o, 64));
      ymx = max(ymx, __shfl_xor(ymx, o, 64));
    }
    const int BW = xmx - xmn + E, BH = ymx - ymn + E;
    const bool tiled = BW * BH <= MAXC;  // identical in every wave
    const int sx = tiled ? 1 : E, sy = tiled ? BW : 1;
    if (wave == 0 && lane < 16) {
      qoff[lane] = tiled ? (Y0 - ymn) * BW + (X0 - xmn) : 0;
      qfx[lane] = cx - bx;
      qfy[lane] = cy - by;
    }
    const int H = f2.H[l], W = f2.W[l];
    const bf16_t* f2b = static_cast<const bf16_t*>(f2.p[l]) + (size_t)b * H * W * C;
    if (tiled) {
      const int ncell = BW * BH, nch = cdiv(ncell, 16);
      // two 16-cell chunks per pass (2 CQ loads in flight per lane)
      for (int c0 = wave; c0 < nch; c0 += 8) {
        uint4 fb[2][CQ];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int n = (c0 + 4 * h) * 16 + r16;
          const int X = xmn + n % BW, Y = ymn + n / BW;
          const bool ok = c0 + 4 * h < nch && n < ncell && X >= 0 && X < W && Y >= 0 && Y < H;
          const bf16_t* p = f2b + (size_t)(ok ? Y * W + X : 0) * C + 8 * q4;
#pragma unroll
          for (int s = 0; s < CQ; ++s)
            fb[h][s] = ok ? *reinterpret_cast<const uint4*>(p + 32 * s) : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          if (c0 + 4 * h >= nch) break;
          f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < CQ; ++s)
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[s]),
                                                          __builtin_bit_cast(bf16x8_t, fb[h][s]), acc, 0, 0, 0);
          // D[query 4 q4 + j][cell r16 of the chunk]
#pragma unroll
          for (int j = 0; j < 4; ++j) dots[4 * q4 + j][(c0 + 4 * h) * 16 + r16] = acc[j];
        }
      }
    } else {
      // per-query fallback (otf_fwd_kernel's layout: lane = 8 * cell slot + channel slot)
      const int slot = lane & 7, grp = lane >> 3;
      for (int qq = wave; qq < 16; qq += 4) {
        const int y = ty * TQ + (qq >> 2), x = tx * TQ + (qq & 3);
        if (y >= H1 || x >= W1) continue;  // wave-uniform
        const int qX0 = __shfl(X0, qq, 64), qY0 = __shfl(Y0, qq, 64);
        const bf16_t* f1p = f1 + ((size_t)b * N1 + y * W1 + x) * C + slot * 4;
        uint2 ab[CQ];
#pragma unroll
        for (int q = 0; q < CQ; ++q) ab[q] = *reinterpret_cast<const uint2*>(f1p + q * 32);
        for (int base = 0; base < E2; base += 8) {
          const int cell = base + grp;
          const int X = qX0 + cell / E, Y = qY0 + cell % E;
          float s = 0.f;
          if (cell < E2 && X >= 0 && X < W && Y >= 0 && Y < H) {
            const bf16_t* row = f2b + ((size_t)Y * W + X) * C + slot * 4;
#pragma unroll
            for (int q = 0; q < CQ; ++q) {
              const uint2 v = *reinterpret_cast<const uint2*>(row + q * 32);
              s = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_v, ab[q].x),
                                                  __builtin_bit_cast(bf16x2_v, v.x), s, false);
              s = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_v, ab[q].y),
                                                  __builtin_bit_cast(bf16x2_v, v.y), s, false);
            }
          }
          s += __shfl_xor(s, 1, 64);
          s += __shfl_xor(s, 2, 64);
          s += __shfl_xor(s, 4, 64);
          if (slot == 0 && cell < E2) dots[qq][cell] = s;
        }
      }
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < 16 * K2; idx += 256) {
      const int qq = idx / K2, t = idx % K2;
      const int y = ty * TQ + (qq >> 2), x = tx * TQ + (qq & 3);
      if (y >= H1 || x >= W1) continue;
      const int i = t / D, j = t % D;  // cell (X0 + i, Y0 + j) is the tap's lower corner
      const float* d = &dots[qq][qoff[qq] + i * sx + j * sy];
      const float fx = qfx[qq], fy = qfy[qq];
      const float v = (1.f - fx) * (1.f - fy) * d[0] + fx * (1.f - fy) * d[sx] + (1.f - fx) * fy * d[sy] +
                      fx * fy * d[sx + sy];
      io<OutT>::st(out + ((size_t)b * N1 + y * W1 + x) * CH + l * K2 + t, v * scale);
    }
    __syncthreads();
  }
}

// Deterministic mode's fixed-point scale, picked per call on the device
// (fx_scan_kernel): fxs = {bits of max|dout|, bits of max|f1|, non-finite
// flag}.  Every df2 cell sum is bounded by 4 * nq * max|dout| * max|f1| *
// |scale| (a query adds at most 4 bilinear weights <= 1 to one cell), so
// S = 2^(61 - ceil(log2 bound)) keeps every sum inside int64 with a
// resolution relative to the data (training-scale upstream gradients of
// ~1e-7 keep ~50 significant bits instead of 32.32's ~9).
__device__ __forceinline__ double fx_scale(const unsigned* fxs, long nq, float scale) {
  const double m = (double)__uint_as_float(fxs[0]) * (double)__uint_as_float(fxs[1]) * fabs((double)scale) *
                   4.0 * (double)nq;
  if (!(m > 0.0) || fxs[2]) return 4294967296.0;  // all-zero or non-finite input: any scale
  return ldexp(1.0, 61 - (int)ceil(log2(m)));
}

__device__ __forceinline__ void fx_add(unsigned long long* p, float v, double S) {
  atomicAdd(p, (unsigned long long)__double2ll_rn((double)v * S));
}

template <typename T, typename GT, int CQ, bool DET>
__global__ __launch_bounds__(WAVES * 64) void otf_bwd_kernel(const T* __restrict__ f1, Lvl f2,
                                                             int levels,
                                                             const float* __restrict__ coords,
                                                             int B, int N1, int r, float scale,
                                                             const GT* __restrict__ dout,
                                                             float* __restrict__ df1, LvlMut df2,
    const unsigned* __restrict__ fxs) {
  const double fxS = DET ? fx_scale(fxs, (long)B * N1, scale) : 0.0;
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
              fx_add(d + 0, gc * a[q].x, fxS);
              fx_add(d + 1, gc * a[q].y, fxS);
              fx_add(d + 2, gc * a[q].z, fxS);
              fx_add(d + 3, gc * a[q].w, fxS);
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

// ------------------------------------------------------- tiled backward
// The per-query backward (otf_bwd_kernel) scatters every cell gradient times
// the query's f1 into df2 with one atomic per (query, cell, channel): 16k
// atomics per query and level at r = 3, C = 128.  Here a block owns the same
// 4 x 4 query tile as otf_tile_kernel; per level:
//  * the tile's cell gradients G[q][cell] over the bounding box of the 16
//    windows are gathered into LDS (each window cell sums its <= 4 taps, the
//    reverse of the forward's bilinear taps -- no LDS atomics);
//  * per 32-channel chunk the box's f2 cells are staged in LDS (fp32), then
//    half the block accumulates df1[q][c] = sum_cell G[q][cell] f2[cell][c]
//    (registers, summed over chunks and levels, one plain store per query at
//    the end) while the other half forms df2[cell][c] = sum_q G[q][cell]
//    f1[q][c] for the box and issues ONE atomic per (cell, channel) for the
//    whole tile (fp32 atomics, or 32.32 fixed point in deterministic mode);
//  * a box wider than MAXC cells (incoherent flow inside the tile) is
//    processed one query window at a time with the same machinery.
template <typename T, typename GT, int CQ, bool DET>
__global__ __launch_bounds__(256) void otf_tile_bwd_kernel(const T* __restrict__ f1, Lvl f2, int levels,
                                                           const float* __restrict__ coords, int B, int H1,
                                                           int W1, int tiles_x, int tiles_y, int per_xcd, int r,
                                                           float scale, const GT* __restrict__ dout,
                                                           float* __restrict__ df1, LvlMut df2,
    const unsigned* __restrict__ fxs) {
  const double fxS = DET ? fx_scale(fxs, (long)B * H1 * W1, scale) : 0.0;
  constexpr int C = CQ * 32;
  __shared__ float Gs[16][MAXC];
  __shared__ __attribute__((aligned(16))) float f2s[MAXC][36];  // 16-B rows: one ds_read_b128 per 4 channels
  __shared__ __attribute__((aligned(16))) float f1s[16][C];
  __shared__ int qX0[16], qY0[16], qn[16];
  __shared__ float qfx[16], qfy[16];
  const int t = threadIdx.x;
  const int tile = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  if (tile >= B * tiles_x * tiles_y) return;  // whole block, before any barrier
  const int b = tile / (tiles_x * tiles_y), t2 = tile % (tiles_x * tiles_y);
  const int ty = t2 / tiles_x, tx = t2 % tiles_x;
  const int N1 = H1 * W1;
  const int D = 2 * r + 1, K2 = D * D, E = D + 1, E2 = E * E, CH = levels * K2;

  if (t < 16) {
    const int y = ty * TQ + (t >> 2), x = tx * TQ + (t & 3);
    qn[t] = (y < H1 && x < W1) ? y * W1 + x : -1;
  }
  __syncthreads();
  for (int i = t; i < 16 * C; i += 256) {
    const int q = i / C, c = i % C;
    f1s[q][c] = qn[q] >= 0 ? io<T>::ld(f1 + ((size_t)b * N1 + qn[q]) * C + c) : 0.f;
  }
  // df1 accumulators: threads 0..127 own query dq = t >> 3, channels 32 k + 4 cg .. + 4 of every chunk k
  float a1[CQ][4];
#pragma unroll
  for (int k = 0; k < CQ; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) a1[k][j] = 0.f;

  for (int l = 0; l < levels; ++l) {
    const int H = f2.H[l], W = f2.W[l];
    if (t < 16) {
      const int n = qn[t] >= 0 ? qn[t] : 0;
      const float inv = 1.f / (float)(1 << l);
      const float cx = coords[((size_t)b * 2 + 0) * N1 + n] * inv, cy = coords[((size_t)b * 2 + 1) * N1 + n] * inv;
      const float bx = floorf(cx), by = floorf(cy);
      qX0[t] = (int)bx - r;
      qY0[t] = (int)by - r;
      qfx[t] = cx - bx;
      qfy[t] = cy - by;
    }
    __syncthreads();
    int xmn = 0x7fffffff, ymn = 0x7fffffff, xmx = -0x7fffffff, ymx = -0x7fffffff;
#pragma unroll
    for (int q = 0; q < 16; ++q)
      if (qn[q] >= 0) {
        xmn = min(xmn, qX0[q]);
        xmx = max(xmx, qX0[q]);
        ymn = min(ymn, qY0[q]);
        ymx = max(ymx, qY0[q]);
      }
    const bool fallback = (xmx - xmn + E) * (ymx - ymn + E) > MAXC;  // identical in every thread
    const T* f2b = static_cast<const T*>(f2.p[l]) + (size_t)b * H * W * C;
    for (int sub = 0; sub < (fallback ? 16 : 1); ++sub) {
      if (fallback && qn[sub] < 0) continue;  // uniform
      const int bx0 = fallback ? qX0[sub] : xmn, by0 = fallback ? qY0[sub] : ymn;
      const int bw = fallback ? E : xmx - xmn + E, bh = fallback ? E : ymx - ymn + E;
      const int nc = bw * bh;
      for (int i = t; i < 16 * MAXC; i += 256) (&Gs[0][0])[i] = 0.f;
      __syncthreads();
      // G[q][box cell]: each window cell (ca along x, cc along y) sums its <= 4 taps
      for (int i = t; i < 16 * E2; i += 256) {
        const int q = i / E2, cell = i - q * E2;
        if (qn[q] < 0 || (fallback && q != sub)) continue;
        const int ca = cell / E, cc = cell - ca * E;
        const float fx = qfx[q], fy = qfy[q];
        const GT* g = dout + ((size_t)b * N1 + qn[q]) * CH + l * K2;
        float acc = 0.f;
#pragma unroll
        for (int di = 0; di < 2; ++di) {
          const int ii = ca - di;
          if (ii < 0 || ii >= D) continue;
          const float wx = di == 0 ? (1.f - fx) : fx;
#pragma unroll
          for (int dj = 0; dj < 2; ++dj) {
            const int jj = cc - dj;
            if (jj < 0 || jj >= D) continue;
            const float wy = dj == 0 ? (1.f - fy) : fy;
            acc += wx * wy * io<GT>::ld(g + ii * D + jj);
          }
        }
        Gs[q][(qY0[q] + cc - by0) * bw + (qX0[q] + ca - bx0)] = acc * scale;
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < CQ; ++k) {
        for (int i = t; i < nc * 8; i += 256) {  // f2 box cells, 32-channel chunk k, 4 channels per piece
          const int cell = i >> 3, pc = i & 7;
          const int X = bx0 + cell % bw, Y = by0 + cell / bw;
          float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
          if (X >= 0 && X < W && Y >= 0 && Y < H) v = ld4<T>(f2b + ((size_t)Y * W + X) * C + 32 * k + 4 * pc);
          *reinterpret_cast<float4*>(&f2s[cell][4 * pc]) = v;
        }
        __syncthreads();
        if (t < 128) {  // df1[q][32 k + 4 cg ..] += sum_cell G[q][cell] f2[cell][..]
          const int dq = t >> 3, cg = t & 7;
          float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
          for (int cell = 0; cell < nc; ++cell) {
            const float gv = Gs[dq][cell];
            const float4 fv = *reinterpret_cast<const float4*>(&f2s[cell][4 * cg]);
            s0 += gv * fv.x;
            s1 += gv * fv.y;
            s2 += gv * fv.z;
            s3 += gv * fv.w;
          }
          a1[k][0] += s0;
          a1[k][1] += s1;
          a1[k][2] += s2;
          a1[k][3] += s3;
        } else {  // df2[box cell][32 k + 4 cg ..] += sum_q G[q][cell] f1[q][..]: one atomic per element per tile
          const int u = t - 128, cg = u & 7;
          for (int cell = u >> 3; cell < nc; cell += 16) {
            const int X = bx0 + cell % bw, Y = by0 + cell / bw;
            if (X < 0 || X >= W || Y < 0 || Y >= H) continue;
            float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
            bool any = false;
#pragma unroll
            for (int q = 0; q < 16; ++q) {  // zero G entries (queries whose window misses the cell) add 0
              const float gv = Gs[q][cell];
              const float4 fv = *reinterpret_cast<const float4*>(&f1s[q][32 * k + 4 * cg]);
              any = any || gv != 0.f;
              s0 += gv * fv.x;
              s1 += gv * fv.y;
              s2 += gv * fv.z;
              s3 += gv * fv.w;
            }
            if (!any) continue;
            const size_t off = ((size_t)b * H * W + (size_t)Y * W + X) * C + 32 * k + 4 * cg;
            if constexpr (DET) {
              unsigned long long* d = reinterpret_cast<unsigned long long*>(df2.p[l]) + off;
              fx_add(d + 0, s0, fxS);
              fx_add(d + 1, s1, fxS);
              fx_add(d + 2, s2, fxS);
              fx_add(d + 3, s3, fxS);
            } else {
              float* d = df2.p[l] + off;
              atomicAdd(d + 0, s0);
              atomicAdd(d + 1, s1);
              atomicAdd(d + 2, s2);
              atomicAdd(d + 3, s3);
            }
          }
        }
        __syncthreads();
      }
    }
  }
  if (t < 128) {
    const int dq = t >> 3, cg = t & 7;
    if (qn[dq] >= 0) {
      float* o = df1 + ((size_t)b * N1 + qn[dq]) * C;
#pragma unroll
      for (int k = 0; k < CQ; ++k)
        *reinterpret_cast<float4*>(o + 32 * k + 4 * cg) = make_float4(a1[k][0], a1[k][1], a1[k][2], a1[k][3]);
    }
  }
}

// ------------------------------------------------- tiled backward on MFMA
// bf16 features, C % 64 == 0 (RAFT C = 256, RAFT-small C = 128).  Same 4 x 4
// query tile, box and per-query fallback as otf_tile_bwd_kernel, but both
// contractions run on MFMA:
//   df1[q][c]    += sum_cell G[q][cell] f2[cell][c]   mfma_f32_16x16x32_bf16,
//                   K = box cells (32 per step), 16 channels per wave and
//                   64-channel chunk, accumulated in registers over levels;
//   df2[cell][c]  = sum_q G[q][cell] f1[q][c]         mfma_f32_16x16x16_bf16,
//                   K = the 16 queries, then ONE atomic per (cell, channel)
//                   straight from the accumulators.
// G is split into bf16 hi + lo (two MFMAs per product, fp32 accumulation), so
// the gradient keeps ~16 mantissa bits -- the fp32 VALU kernel's accuracy at a
// fraction of its LDS traffic.  Every operand stays in its natural row-major
// layout in LDS -- G [q][cell], f2's box chunk [cell][c], f1 [q][c], all
// staged with plain 16-byte copies -- and the operands whose K runs down the
// rows (G^T for df2, f2 for df1, f1 for df2) are gathered by
// ds_read_b64_tr_b16 (lane 4q+p of a 16-lane group addresses row q, columns
// 4p..4p+3; lane i receives column i of the 4 rows).
constexpr int GQP = MAXC + 8;  // G row pitch (bf16): the 16-B reads of 16 rows cover the banks
constexpr int F2C = 32;        // f2 box chunk: 32 channels (the block fits three times per CU)
constexpr int F2P = 48;        // f2 chunk row pitch (bf16, 96 B): the tr16 reads of 4 rows hit disjoint banks

typedef short v4s_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4s_t otf_tr16(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) v4s_t*)((__attribute__((address_space(3))) bf16_t*)p));
}

template <typename GT, int CQ, bool DET>
__global__ __launch_bounds__(256) void otf_tile_bwd_mma_kernel(const bf16_t* __restrict__ f1, Lvl f2, int levels,
                                                               const float* __restrict__ coords, int B, int H1,
                                                               int W1, int tiles_x, int tiles_y, int per_xcd, int r,
                                                               float scale, const GT* __restrict__ dout,
                                                               float* __restrict__ df1, LvlMut df2,
    const unsigned* __restrict__ fxs) {
  const double fxS = DET ? fx_scale(fxs, (long)B * H1 * W1, scale) : 0.0;
  constexpr int C = CQ * 32, NCH = C / F2C;
  constexpr int F1P = C + 16;  // f1 row pitch (bf16): rows 8 banks apart for the tr16 reads
  static_assert(C % 64 == 0, "C % 64");
  __shared__ __attribute__((aligned(16))) bf16_t Gq[2][16][GQP];  // [hi / lo][query][box cell]
  __shared__ __attribute__((aligned(16))) bf16_t F2s[MAXC][F2P];  // f2 box, one 32-channel chunk, [cell][c]
  __shared__ __attribute__((aligned(16))) bf16_t F1s[16][F1P];    // the tile's f1, [query][c]
  __shared__ uint8_t live[MAXC];  // box cell with a nonzero gradient
  __shared__ int qX0[16], qY0[16], qn[16];
  __shared__ float qfx[16], qfy[16];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int r16 = lane & 15, q4 = lane >> 4;
  const int tq = r16 >> 2, tp = r16 & 3;  // tr16 address roles: row tq, columns 4 tp .. + 4
  const int tile = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  if (tile >= B * tiles_x * tiles_y) return;  // whole block, before any barrier
  const int b = tile / (tiles_x * tiles_y), t2 = tile % (tiles_x * tiles_y);
  const int ty = t2 / tiles_x, tx = t2 % tiles_x;
  const int N1 = H1 * W1;
  const int D = 2 * r + 1, K2 = D * D, E = D + 1, E2 = E * E, CH = levels * K2;

  if (t < 16) {
    const int y = ty * TQ + (t >> 2), x = tx * TQ + (t & 3);
    qn[t] = (y < H1 && x < W1) ? y * W1 + x : -1;
  }
  __syncthreads();
  for (int i = t; i < 16 * (C / 8); i += 256) {  // f1 rows (zero for queries outside the image)
    const int q = i / (C / 8), cg = i % (C / 8);
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (qn[q] >= 0) v = *reinterpret_cast<const uint4*>(f1 + ((size_t)b * N1 + qn[q]) * C + 8 * cg);
    *reinterpret_cast<uint4*>(&F1s[q][8 * cg]) = v;
  }
  // df1: query 4 q4 + j, channel 32 k + 16 (wave & 1) + r16; waves 0-1 and 2-3 take
  // alternate 32-cell K steps of the same tiles (summed in LDS at the end)
  const int wn = wave & 1, wk = wave >> 1;
  f32x4_t a1[NCH];
#pragma unroll
  for (int k = 0; k < NCH; ++k) a1[k] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  for (int l = 0; l < levels; ++l) {
    const int H = f2.H[l], W = f2.W[l];
    __syncthreads();  // the previous level's readers of q* / G / F2s are done
    if (t < 16) {
      const int n = qn[t] >= 0 ? qn[t] : 0;
      const float inv = 1.f / (float)(1 << l);
      const float cx = coords[((size_t)b * 2 + 0) * N1 + n] * inv, cy = coords[((size_t)b * 2 + 1) * N1 + n] * inv;
      const float bx = floorf(cx), by = floorf(cy);
      qX0[t] = (int)bx - r;
      qY0[t] = (int)by - r;
      qfx[t] = cx - bx;
      qfy[t] = cy - by;
    }
    __syncthreads();
    int xmn = 0x7fffffff, ymn = 0x7fffffff, xmx = -0x7fffffff, ymx = -0x7fffffff;
#pragma unroll
    for (int q = 0; q < 16; ++q)
      if (qn[q] >= 0) {
        xmn = min(xmn, qX0[q]);
        xmx = max(xmx, qX0[q]);
        ymn = min(ymn, qY0[q]);
        ymx = max(ymx, qY0[q]);
      }
    const bool fallback = (xmx - xmn + E) * (ymx - ymn + E) > MAXC;  // identical in every thread
    const bf16_t* f2b = static_cast<const bf16_t*>(f2.p[l]) + (size_t)b * H * W * C;
    for (int sub = 0; sub < (fallback ? 16 : 1); ++sub) {
      if (fallback && qn[sub] < 0) continue;  // uniform
      const int bx0 = fallback ? qX0[sub] : xmn, by0 = fallback ? qY0[sub] : ymn;
      const int bw = fallback ? E : xmx - xmn + E, bh = fallback ? E : ymx - ymn + E;
      const int nc = bw * bh, ncp = round_up(nc, 32);
      if (sub > 0) __syncthreads();  // the previous window's readers are done
      for (int i = t; i < 16 * ncp / 2; i += 256) {  // zero G over the padded box
        const int q = i / (ncp / 2), c2 = i % (ncp / 2);
        reinterpret_cast<uint32_t*>(&Gq[0][q][0])[c2] = 0u;
        reinterpret_cast<uint32_t*>(&Gq[1][q][0])[c2] = 0u;
      }
      for (int i = t; i < ncp; i += 256) live[i] = 0;
      __syncthreads();
      // G[q][box cell]: each window cell (ca along x, cc along y) sums its <= 4 taps
      for (int i = t; i < 16 * E2; i += 256) {
        const int q = i / E2, cell = i - q * E2;
        if (qn[q] < 0 || (fallback && q != sub)) continue;
        const int ca = cell / E, cc = cell - ca * E;
        const float fx = qfx[q], fy = qfy[q];
        const GT* g = dout + ((size_t)b * N1 + qn[q]) * CH + l * K2;
        float acc = 0.f;
#pragma unroll
        for (int di = 0; di < 2; ++di) {
          const int ii = ca - di;
          if (ii < 0 || ii >= D) continue;
          const float wx = di == 0 ? (1.f - fx) : fx;
#pragma unroll
          for (int dj = 0; dj < 2; ++dj) {
            const int jj = cc - dj;
            if (jj < 0 || jj >= D) continue;
            const float wy = dj == 0 ? (1.f - fy) : fy;
            acc += wx * wy * io<GT>::ld(g + ii * D + jj);
          }
        }
        acc *= scale;
        const bf16_t hi = f2bf(acc), lo = f2bf(acc - bf2f(hi));
        const int bc = (qY0[q] + cc - by0) * bw + (qX0[q] + ca - bx0);
        Gq[0][q][bc] = hi;
        Gq[1][q][bc] = lo;
        if (acc != 0.f) live[bc] = 1;
      }
      __syncthreads();
      // df2[box cell][c] = sum_q G[q][cell] f1[q][c]: wave = channel tiles wave, wave + 4, ..
      for (int m = 0; m < ncp / 16; ++m) {
        // A = G^T: rows (queries) 4 q4 + tq, columns (cells) 16 m + 4 tp
        const v4s_t ahi = otf_tr16(&Gq[0][4 * q4 + tq][16 * m + 4 * tp]);
        const v4s_t alo = otf_tr16(&Gq[1][4 * q4 + tq][16 * m + 4 * tp]);
        int cl[4];
        bool ok[4], any = false;
#pragma unroll
        for (int j = 0; j < 4; ++j) {  // D rows of this lane: cells 16 m + 4 q4 + j
          const int cell = 16 * m + 4 * q4 + j;
          const int X = bx0 + cell % bw, Y = by0 + cell / bw;
          ok[j] = cell < nc && live[cell] && X >= 0 && X < W && Y >= 0 && Y < H;
          cl[j] = ok[j] ? Y * W + X : 0;
          any = any || ok[j];
        }
        if (!__builtin_amdgcn_ballot_w64(any)) continue;  // wave-uniform: a dead 16-cell group
        for (int n = wave; n < C / 16; n += 4) {
          const v4s_t bf = otf_tr16(&F1s[4 * q4 + tq][16 * n + 4 * tp]);  // B = f1: rows = queries
          f32x4_t d = {0.f, 0.f, 0.f, 0.f};
          d = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ahi, bf, d, 0, 0, 0);
          d = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(alo, bf, d, 0, 0, 0);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (!ok[j]) continue;
            const size_t off = ((size_t)b * H * W + cl[j]) * C + 16 * n + r16;
            if constexpr (DET)
              fx_add(reinterpret_cast<unsigned long long*>(df2.p[l]) + off, d[j], fxS);
            else
              atomicAdd(df2.p[l] + off, d[j]);
          }
        }
      }
      // df1[q][c] += sum_cell G[q][cell] f2[cell][c], per 32-channel chunk of f2's box
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        if (k > 0) __syncthreads();  // the previous chunk's MFMA reads of F2s are done
        for (int i = t; i < ncp * 4; i += 256) {
          const int cell = i >> 2, pc = i & 3;
          const int X = bx0 + cell % bw, Y = by0 + cell / bw;
          uint4 v = make_uint4(0u, 0u, 0u, 0u);
          if (cell < nc && X >= 0 && X < W && Y >= 0 && Y < H)
            v = *reinterpret_cast<const uint4*>(f2b + ((size_t)Y * W + X) * C + F2C * k + 8 * pc);
          *reinterpret_cast<uint4*>(&F2s[cell][8 * pc]) = v;
        }
        __syncthreads();
        for (int kc = wk; kc < ncp / 32; kc += 2) {
          const bf16x8_t ahi = *reinterpret_cast<const bf16x8_t*>(&Gq[0][r16][32 * kc + 8 * q4]);
          const bf16x8_t alo = *reinterpret_cast<const bf16x8_t*>(&Gq[1][r16][32 * kc + 8 * q4]);
          // B = f2: rows (cells) 32 kc + 8 q4 + tq (+ 4), columns 16 wn + 4 tp
          const v4s_t b0 = otf_tr16(&F2s[32 * kc + 8 * q4 + tq][16 * wn + 4 * tp]);
          const v4s_t b1 = otf_tr16(&F2s[32 * kc + 8 * q4 + 4 + tq][16 * wn + 4 * tp]);
          const bf16x8_t bv = bf16x8_t{b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
          a1[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, bv, a1[k], 0, 0, 0);
          a1[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo, bv, a1[k], 0, 0, 0);
        }
      }
    }
  }
  // df1: waves 2-3 hand their K-half to waves 0-1 through LDS (the F2s area), fixed order
  __syncthreads();
  float* red = reinterpret_cast<float*>(&F2s[0][0]);  // [2 waves][NCH][4][64 lanes]
  static_assert(2 * NCH * 4 * 64 * 4 <= (int)sizeof(F2s), "df1 hand-off fits in F2s");
  if (wk == 1) {
#pragma unroll
    for (int k = 0; k < NCH; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) red[((wn * NCH + k) * 4 + j) * 64 + lane] = a1[k][j];
  }
  __syncthreads();
  if (wk == 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = 4 * q4 + j;
      if (qn[q] < 0) continue;
      float* o = df1 + ((size_t)b * N1 + qn[q]) * C + 16 * wn + r16;
#pragma unroll
      for (int k = 0; k < NCH; ++k) o[F2C * k] = a1[k][j] + red[((wn * NCH + k) * 4 + j) * 64 + lane];
    }
  }
}

// max |dout|, max |f1| (as order-independent uint atomicMax of the
// non-negative float bits) and a non-finite flag: the inputs of fx_scale
template <typename T>
__device__ __forceinline__ float absf_(T v);
template <>
__device__ __forceinline__ float absf_<float>(float v) { return fabsf(v); }
template <>
__device__ __forceinline__ float absf_<bf16_t>(bf16_t v) { return fabsf(bf2f(v)); }

template <typename TD, typename TF>
__global__ __launch_bounds__(256) void fx_scan_kernel(const TD* __restrict__ dout, long nd, const TF* __restrict__ f1,
                                                      long nf, unsigned* __restrict__ fxs) {
  float md = 0.f, mf = 0.f;
  unsigned bad = 0;
  const long st = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nd; i += st) {
    const float v = absf_<TD>(dout[i]);
    bad |= !(v <= 3.0e38f);  // NaN or Inf
    md = fmaxf(md, v);
  }
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nf; i += st) {
    const float v = absf_<TF>(f1[i]);
    bad |= !(v <= 3.0e38f);
    mf = fmaxf(mf, v);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    md = fmaxf(md, __shfl_xor(md, o));
    mf = fmaxf(mf, __shfl_xor(mf, o));
    bad |= __shfl_xor(bad, o);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMax(fxs + 0, __float_as_uint(md));
    atomicMax(fxs + 1, __float_as_uint(mf));
    if (bad) atomicOr(fxs + 2, 1u);
  }
}

// fixed point (int64, scale fx_scale) -> fp32; NaN everywhere when an input was
// not finite (the integer sums cannot carry it), so the step's non-finite check sees it
__global__ __launch_bounds__(256) void fx_to_f32_kernel(const long long* __restrict__ in, long n,
                                                        float* __restrict__ out, const unsigned* __restrict__ fxs,
                                                        long nq, float scale) {
  const double inv = 1.0 / fx_scale(fxs, nq, scale);
  const bool bad = fxs[2] != 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    out[i] = bad ? __builtin_nanf("") : (float)((double)in[i] * inv);
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
                         int levels, bool fm_bf16, const float* coords, int B, int H1, int W1, int C,
                         int r, float scale, void* out, bool out_bf16, hipStream_t stream) {
  otf::Lvl p;
  for (int l = 0; l < 4; ++l) {
    p.p[l] = l < levels ? f2[l] : nullptr;
    p.H[l] = l < levels ? Hs[l] : 0;
    p.W[l] = l < levels ? Ws[l] : 0;
  }
  const int N1 = H1 * W1;
  const int cq = C / 32;
  if (fm_bf16 && (2 * r + 2) * (2 * r + 2) <= otf::MAXC) {
    const int tiles_x = cdiv(W1, otf::TQ), tiles_y = cdiv(H1, otf::TQ);
    const int per_xcd = cdiv(B * tiles_x * tiles_y, 8);
#define RS_L(OT)                                                                                        \
  hipLaunchKernelGGL((otf::otf_tile_kernel<OT, CQ>), dim3(8 * per_xcd), dim3(256), 0, stream,           \
                     static_cast<const bf16_t*>(f1), p, levels, coords, B, H1, W1, tiles_x, tiles_y,    \
                     per_xcd, r, scale, static_cast<OT*>(out))
    if (out_bf16) { RS_OTF_DISPATCH_CQ(cq, RS_L(bf16_t)); }
    else { RS_OTF_DISPATCH_CQ(cq, RS_L(float)); }
#undef RS_L
    return;
  }
  const long npix = (long)B * N1;
  dim3 grid((unsigned)cdiv((int)npix, otf::WAVES)), block(otf::WAVES * 64);
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
                         int levels, bool fm_bf16, const float* coords, int B, int H1, int W1, int C,
                         int r, float scale, const void* dout, bool dout_bf16, float* df1,
                         float* const* df2, bool det, float* const* df2f, unsigned* fxs, hipStream_t stream) {
  const int N1 = H1 * W1;
  if (det) {  // fxs (zeroed by the caller): the fixed-point scale's inputs
    const long nd = (long)B * N1 * levels * (2 * r + 1) * (2 * r + 1), nf = (long)B * N1 * C;
    const int g = (int)std::min<long>((nd + 255) / 256, 1024);
#define RS_FS(TD, TF) \
  hipLaunchKernelGGL((otf::fx_scan_kernel<TD, TF>), dim3(g), dim3(256), 0, stream, static_cast<const TD*>(dout), nd, \
                     static_cast<const TF*>(f1), nf, fxs)
    if (dout_bf16) {
      if (fm_bf16) RS_FS(bf16_t, bf16_t); else RS_FS(bf16_t, float);
    } else {
      if (fm_bf16) RS_FS(float, bf16_t); else RS_FS(float, float);
    }
#undef RS_FS
  }
  otf::Lvl p;
  otf::LvlMut d;
  for (int l = 0; l < 4; ++l) {
    p.p[l] = l < levels ? f2[l] : nullptr;
    d.p[l] = l < levels ? df2[l] : nullptr;
    p.H[l] = d.H[l] = l < levels ? Hs[l] : 0;
    p.W[l] = d.W[l] = l < levels ? Ws[l] : 0;
  }
  const int cq = C / 32;
  if (fm_bf16 && C % 64 == 0 && (2 * r + 2) * (2 * r + 2) <= otf::MAXC) {
    const int tiles_x = cdiv(W1, otf::TQ), tiles_y = cdiv(H1, otf::TQ);
    const int per_xcd = cdiv(B * tiles_x * tiles_y, 8);
    const bf16_t* f1b = static_cast<const bf16_t*>(f1);
#define RS_LM(GT)                                                                                          \
  if (det)                                                                                                 \
    hipLaunchKernelGGL((otf::otf_tile_bwd_mma_kernel<GT, CQ, true>), dim3(8 * per_xcd), dim3(256), 0, stream, \
                       f1b, p, levels, coords, B, H1, W1, tiles_x, tiles_y, per_xcd, r, scale,                \
                       static_cast<const GT*>(dout), df1, d, fxs);                                               \
  else                                                                                                     \
    hipLaunchKernelGGL((otf::otf_tile_bwd_mma_kernel<GT, CQ, false>), dim3(8 * per_xcd), dim3(256), 0, stream, \
                       f1b, p, levels, coords, B, H1, W1, tiles_x, tiles_y, per_xcd, r, scale,                \
                       static_cast<const GT*>(dout), df1, d, fxs)
    switch (cq) {
      case 2: { constexpr int CQ = 2; if (dout_bf16) { RS_LM(bf16_t); } else { RS_LM(float); } } break;
      case 4: { constexpr int CQ = 4; if (dout_bf16) { RS_LM(bf16_t); } else { RS_LM(float); } } break;
      default: { constexpr int CQ = 8; if (dout_bf16) { RS_LM(bf16_t); } else { RS_LM(float); } } break;
    }
#undef RS_LM
  } else if ((2 * r + 2) * (2 * r + 2) <= otf::MAXC) {
    const int tiles_x = cdiv(W1, otf::TQ), tiles_y = cdiv(H1, otf::TQ);
    const int per_xcd = cdiv(B * tiles_x * tiles_y, 8);
#define RS_LT(T, GT)                                                                                      \
  if (det)                                                                                                \
    hipLaunchKernelGGL((otf::otf_tile_bwd_kernel<T, GT, CQ, true>), dim3(8 * per_xcd), dim3(256), 0, stream, \
                       static_cast<const T*>(f1), p, levels, coords, B, H1, W1, tiles_x, tiles_y, per_xcd, r, \
                       scale, static_cast<const GT*>(dout), df1, d, fxs);                                       \
  else                                                                                                    \
    hipLaunchKernelGGL((otf::otf_tile_bwd_kernel<T, GT, CQ, false>), dim3(8 * per_xcd), dim3(256), 0, stream, \
                       static_cast<const T*>(f1), p, levels, coords, B, H1, W1, tiles_x, tiles_y, per_xcd, r, \
                       scale, static_cast<const GT*>(dout), df1, d, fxs)
    if (fm_bf16) {
      if (dout_bf16) { RS_OTF_DISPATCH_CQ(cq, RS_LT(bf16_t, bf16_t)); }
      else { RS_OTF_DISPATCH_CQ(cq, RS_LT(bf16_t, float)); }
    } else {
      if (dout_bf16) { RS_OTF_DISPATCH_CQ(cq, RS_LT(float, bf16_t)); }
      else { RS_OTF_DISPATCH_CQ(cq, RS_LT(float, float)); }
    }
#undef RS_LT
  } else {
  const long npix = (long)B * N1;
  dim3 grid((unsigned)cdiv((int)npix, otf::WAVES)), block(otf::WAVES * 64);
#define RS_L(T, GT)                                                                          \
  if (det)                                                                                   \
    hipLaunchKernelGGL((otf::otf_bwd_kernel<T, GT, CQ, true>), grid, block, 0, stream,       \
                       static_cast<const T*>(f1), p, levels, coords, B, N1, r, scale,        \
                       static_cast<const GT*>(dout), df1, d, fxs);                                \
  else                                                                                       \
    hipLaunchKernelGGL((otf::otf_bwd_kernel<T, GT, CQ, false>), grid, block, 0, stream,      \
                       static_cast<const T*>(f1), p, levels, coords, B, N1, r, scale,        \
                       static_cast<const GT*>(dout), df1, d, fxs)
  if (fm_bf16) {
    if (dout_bf16) { RS_OTF_DISPATCH_CQ(cq, RS_L(bf16_t, bf16_t)); }
    else { RS_OTF_DISPATCH_CQ(cq, RS_L(bf16_t, float)); }
  } else {
    if (dout_bf16) { RS_OTF_DISPATCH_CQ(cq, RS_L(float, bf16_t)); }
    else { RS_OTF_DISPATCH_CQ(cq, RS_L(float, float)); }
  }
#undef RS_L
  }
  if (det)
    for (int l = 0; l < levels; ++l) {
      const long n = (long)B * Hs[l] * Ws[l] * C;
      const int g = (int)std::min<long>((n + 255) / 256, 16384);
      hipLaunchKernelGGL(otf::fx_to_f32_kernel, dim3(g), dim3(256), 0, stream,
                         reinterpret_cast<const long long*>(df2[l]), n, df2f[l], fxs, (long)B * N1, scale);
    }
}

}  // namespace rs
