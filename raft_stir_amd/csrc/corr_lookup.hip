// Multi-scale correlation-pyramid window lookup (forward + backward).
//
// Replaces reference core/corr.py:29-50 (per level: linspace/meshgrid, then
// grid_sample(align_corners=True, zero padding) of a (2r+1)^2 window around
// coords/2^l, cat, permute) with one launch per direction.
//
// Forward: out[b, y, x, l*K2 + k] (channels-last, fp32 or bf16) where
//   k = (dx + r) * (2r+1) + (dy + r)   (x-offset-major, as the reference)
// One thread per output element; consecutive threads walk one pixel's 4*K2
// channels, so the NHWC store is contiguous and the 4 bilinear taps of
// neighbouring threads fall in the same cache lines of that pixel's own row
// of the volume.
//
// Backward (training): every window tap (dx, dy) shares the SAME fractional
// offset (fx, fy) at a level because dx, dy are integers, so the (2r+1)^2
// bilinear taps touch exactly the (2r+2)^2 integer cells
//   X = floor(cx/2^l) - r + a,  Y = floor(cy/2^l) - r + c,  a, c in [0, 2r+1].
// We launch one thread per CELL and gather its <= 4 contributing taps:
//   g(a,c) = sum_{i in {a-1,a}, j in {c-1,c}} wx(i) wy(j) dout[i, j]
// Cells of one pixel are distinct and a pixel only ever touches its own row
// of the volume, so the accumulation into the pyramid gradient is a plain
// read-modify-write: no atomics, deterministic.  The lookup is called once
// per refinement iteration against the same pyramid, so the gradient of all
// iterations accumulates in one pyramid-shaped buffer; `pyr_grad_fold` then
// applies the avg-pool backward (level l cell -> its 2^l x 2^l level-0 block,
// weight 4^-l) and the 1/sqrt(C) scale once.

#include <algorithm>

#include "common.h"

namespace rs {
namespace lookup {

// Pyramid levels: element (b*N1 + pix, y, x) of level l at p[l] + pix*S[l] + y*W[l] + x
// (S = row pitch >= H*W).  Pyr elements are fp32 or bf16 (template PT of the
// forward kernels, RAFTConfig.corr_dtype); the gradient pyramid is fp32.
struct Pyr {
  const void* p[4];
  int H[4];
  int W[4];
  int S[4];
};
struct PyrMut {
  float* p[4];
  int H[4];
  int W[4];
  int S[4];
};

template <typename PT, typename OutT>
__global__ __launch_bounds__(256) void lookup_fwd_kernel(Pyr pyr, int levels,
                                                         const float* __restrict__ coords, int B,
                                                         int H1, int W1, int r,
                                                         OutT* __restrict__ out, long total,
                                                         int ostride) {
  const int D = 2 * r + 1, K2 = D * D, CH = levels * K2;
  const int N1 = H1 * W1;
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const int ch = (int)(idx % ostride);
    const long pix = idx / ostride;  // b * N1 + n
    if (ch >= CH) {  // zero the channel padding of a padded (K-aligned) output row
      io<OutT>::st(out + idx, 0.f);
      continue;
    }
    const int b = (int)(pix / N1), n = (int)(pix % N1);
    const int l = ch / K2, k = ch % K2;
    const int i = k / D, j = k % D;  // i: dx index, j: dy index
    const float inv = 1.f / (float)(1 << l);
    const float cx = coords[((size_t)b * 2 + 0) * N1 + n] * inv;
    const float cy = coords[((size_t)b * 2 + 1) * N1 + n] * inv;
    const float x = cx + (float)(i - r), y = cy + (float)(j - r);
    const float x0f = floorf(x), y0f = floorf(y);
    const float fx = x - x0f, fy = y - y0f;
    const int x0 = (int)x0f, y0 = (int)y0f;
    const int H = pyr.H[l], W = pyr.W[l];
    const PT* row = static_cast<const PT*>(pyr.p[l]) + pix * (size_t)pyr.S[l];
    float v = 0.f;
    const bool xin0 = x0 >= 0 && x0 < W, xin1 = x0 + 1 >= 0 && x0 + 1 < W;
    if (y0 >= 0 && y0 < H) {
      const PT* rr = row + (size_t)y0 * W;
      if (xin0) v += (1.f - fx) * (1.f - fy) * io<PT>::ld(rr + x0);
      if (xin1) v += fx * (1.f - fy) * io<PT>::ld(rr + x0 + 1);
    }
    if (y0 + 1 >= 0 && y0 + 1 < H) {
      const PT* rr = row + (size_t)(y0 + 1) * W;
      if (xin0) v += (1.f - fx) * fy * io<PT>::ld(rr + x0);
      if (xin1) v += fx * fy * io<PT>::ld(rr + x0 + 1);
    }
    io<OutT>::st(out + idx, v);
  }
}

template <typename GT>
__global__ __launch_bounds__(256) void lookup_bwd_kernel(PyrMut gpyr, int levels,
                                                         const float* __restrict__ coords, int B,
                                                         int H1, int W1, int r,
                                                         const GT* __restrict__ dout, long total,
                                                         int dstride) {
  const int D = 2 * r + 1, K2 = D * D;
  const int E = D + 1, E2 = E * E;  // integer cells per level
  const int N1 = H1 * W1;
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const int cell = (int)(idx % E2);
    const long pl = idx / E2;  // (b*N1 + n) * levels + l
    const int l = (int)(pl % levels);
    const long pix = pl / levels;
    const int b = (int)(pix / N1), n = (int)(pix % N1);
    const int a = cell / E, c = cell % E;  // a: x cell index, c: y cell index
    const float inv = 1.f / (float)(1 << l);
    const float cx = coords[((size_t)b * 2 + 0) * N1 + n] * inv;
    const float cy = coords[((size_t)b * 2 + 1) * N1 + n] * inv;
    const float bx = floorf(cx), by = floorf(cy);
    const float fx = cx - bx, fy = cy - by;
    const int X = (int)bx - r + a, Y = (int)by - r + c;
    const int H = gpyr.H[l], W = gpyr.W[l];
    if (X < 0 || X >= W || Y < 0 || Y >= H) continue;
    const GT* g = dout + pix * dstride + l * K2;
    float acc = 0.f;
    // tap i = a uses this cell as its lower x-corner (weight 1-fx); tap a-1 as upper (fx)
#pragma unroll
    for (int di = 0; di < 2; ++di) {
      const int i = a - di;
      if (i < 0 || i >= D) continue;
      const float wx = di == 0 ? (1.f - fx) : fx;
#pragma unroll
      for (int dj = 0; dj < 2; ++dj) {
        const int j = c - dj;
        if (j < 0 || j >= D) continue;
        const float wy = dj == 0 ? (1.f - fy) : fy;
        acc += wx * wy * io<GT>::ld(g + i * D + j);
      }
    }
    float* dst = gpyr.p[l] + pix * (size_t)gpyr.S[l] + (size_t)Y * W + X;
    *dst += acc;
  }
}

// ---------------------------------------------------------------- wave-per-pixel variants
// (radius 3 / 4, the RAFT-small / RAFT configurations).  One wave owns one
// pixel; per level the (2r+2)^2 integer cells its window touches are staged
// in LDS with x-fastest (row-coalesced) loads, then each lane produces output
// channels from LDS with the level's shared bilinear weights (every tap has
// the same fractional offset).  All index math is 32-bit with compile-time
// divisors.  Backward mirrors it: the pixel's dout slice is staged in LDS and
// each lane gathers the <= 4 taps of one cell, then updates its pyramid-
// gradient row with x-fastest (coalesced) read-modify-writes.
template <typename P>
__device__ __forceinline__ auto lvl_ptr(const P& pyr, int l) {
  return l == 0 ? pyr.p[0] : (l == 1 ? pyr.p[1] : (l == 2 ? pyr.p[2] : pyr.p[3]));
}
template <typename P>
__device__ __forceinline__ int lvl_S(const P& pyr, int l) {
  return l == 0 ? pyr.S[0] : (l == 1 ? pyr.S[1] : (l == 2 ? pyr.S[2] : pyr.S[3]));
}
template <typename P>
__device__ __forceinline__ int lvl_H(const P& pyr, int l) {
  return l == 0 ? pyr.H[0] : (l == 1 ? pyr.H[1] : (l == 2 ? pyr.H[2] : pyr.H[3]));
}
template <typename P>
__device__ __forceinline__ int lvl_W(const P& pyr, int l) {
  return l == 0 ? pyr.W[0] : (l == 1 ? pyr.W[1] : (l == 2 ? pyr.W[2] : pyr.W[3]));
}

template <int R, typename PT, typename OutT>
__global__ __launch_bounds__(256) void lookup_fwd_wave_kernel(Pyr pyr, int levels, const float* __restrict__ coords,
                                                              int N1, int P, OutT* __restrict__ out, int ostride) {
  constexpr int D = 2 * R + 1, K2 = D * D, E = D + 1, E2 = E * E;
  __shared__ float win[4][4][E2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int pix = blockIdx.x * 4 + w;
  if (pix >= P) return;
  const int b = pix / N1, n = pix - b * N1;
  const float cx0 = coords[(size_t)(b * 2) * N1 + n], cy0 = coords[(size_t)(b * 2 + 1) * N1 + n];
  float fxs[4], fys[4];
#pragma unroll
  for (int l = 0; l < 4; ++l) {
    if (l >= levels) break;
    const float inv = 1.f / (float)(1 << l);
    const float cx = cx0 * inv, cy = cy0 * inv;
    const float bx = floorf(cx), by = floorf(cy);
    fxs[l] = cx - bx;
    fys[l] = cy - by;
    const int X0 = (int)bx - R, Y0 = (int)by - R;
    const int H = lvl_H(pyr, l), W = lvl_W(pyr, l);
    const PT* row = static_cast<const PT*>(lvl_ptr(pyr, l)) + (size_t)pix * lvl_S(pyr, l);
    for (int idx = lane; idx < E2; idx += 64) {
      const int c = idx / E, a = idx - c * E;
      const int X = X0 + a, Y = Y0 + c;
      win[w][l][idx] = (X >= 0 && X < W && Y >= 0 && Y < H) ? io<PT>::ld(row + (size_t)Y * W + X) : 0.f;
    }
  }
  // each wave only touches its own LDS slice: a wave-level ordering point suffices
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  const int CH = levels * K2;
  OutT* o = out + (size_t)pix * ostride;
  for (int ch = lane; ch < ostride; ch += 64) {
    float v = 0.f;
    if (ch < CH) {
      const int l = ch / K2, k = ch - l * K2;
      const int i = k / D, j = k - i * D;  // i: x tap, j: y tap
      const float fx = l == 0 ? fxs[0] : (l == 1 ? fxs[1] : (l == 2 ? fxs[2] : fxs[3]));
      const float fy = l == 0 ? fys[0] : (l == 1 ? fys[1] : (l == 2 ? fys[2] : fys[3]));
      const float* L = win[w][l] + j * E + i;
      v = (1.f - fy) * ((1.f - fx) * L[0] + fx * L[1]) + fy * ((1.f - fx) * L[E] + fx * L[E + 1]);
    }
    io<OutT>::st(o + ch, v);
  }
}

template <int R, typename GT>
__global__ __launch_bounds__(256) void lookup_bwd_wave_kernel(PyrMut gpyr, int levels, const float* __restrict__ coords,
                                                              int N1, int P, const GT* __restrict__ dout,
                                                              int dstride) {
  constexpr int D = 2 * R + 1, K2 = D * D, E = D + 1, E2 = E * E;
  __shared__ float gs[4][4][K2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int pix = blockIdx.x * 4 + w;
  if (pix >= P) return;
  const int b = pix / N1, n = pix - b * N1;
  const float cx0 = coords[(size_t)(b * 2) * N1 + n], cy0 = coords[(size_t)(b * 2 + 1) * N1 + n];
  const GT* g = dout + (size_t)pix * dstride;
  for (int idx = lane; idx < levels * K2; idx += 64) gs[w][idx / K2][idx % K2] = io<GT>::ld(g + idx);
  // each wave only touches its own LDS slice: a wave-level ordering point suffices
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int l = 0; l < 4; ++l) {
    if (l >= levels) break;
    const float inv = 1.f / (float)(1 << l);
    const float cx = cx0 * inv, cy = cy0 * inv;
    const float bx = floorf(cx), by = floorf(cy);
    const float fx = cx - bx, fy = cy - by;
    const int X0 = (int)bx - R, Y0 = (int)by - R;
    const int H = lvl_H(gpyr, l), W = lvl_W(gpyr, l);
    float* row = lvl_ptr(gpyr, l) + (size_t)pix * lvl_S(gpyr, l);
    const float* G = gs[w][l];  // G[i * D + j], i: x tap, j: y tap
    for (int idx = lane; idx < E2; idx += 64) {
      const int c = idx / E, a = idx - c * E;  // cell (x = a, y = c), x fastest
      const int X = X0 + a, Y = Y0 + c;
      if (X < 0 || X >= W || Y < 0 || Y >= H) continue;
      float acc = 0.f;
      // tap i = a uses this cell as its lower x-corner (1 - fx), tap a - 1 as its upper (fx)
      if (a < D) {
        if (c < D) acc += (1.f - fx) * (1.f - fy) * G[a * D + c];
        if (c > 0) acc += (1.f - fx) * fy * G[a * D + c - 1];
      }
      if (a > 0) {
        if (c < D) acc += fx * (1.f - fy) * G[(a - 1) * D + c];
        if (c > 0) acc += fx * fy * G[(a - 1) * D + c - 1];
      }
      row[(size_t)Y * W + X] += acc;
    }
  }
}

// G0 = scale * (g0 + g1/4 + g2/16 + g3/64) expanded to level-0 cells, in place.
__global__ __launch_bounds__(256) void pyr_fold_kernel(PyrMut g, int levels, long rows,
                                                       float scale, bf16_t* __restrict__ out_bf16) {
  const int H0 = g.H[0], W0 = g.W[0];
  const long total = rows * H0 * W0;
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const int x = (int)(idx % W0);
    const int y = (int)((idx / W0) % H0);
    const long row = idx / ((long)H0 * W0);
    const size_t o0 = row * (size_t)g.S[0] + (size_t)y * W0 + x;
    float v = g.p[0][o0];
    float w = 1.f;
#pragma unroll
    for (int l = 1; l < 4; ++l) {
      if (l >= levels) break;
      w *= 0.25f;
      const int yl = y >> l, xl = x >> l;
      if (yl < g.H[l] && xl < g.W[l])
        v += w * g.p[l][row * (size_t)g.S[l] + (size_t)yl * g.W[l] + xl];
    }
    if (out_bf16)
      out_bf16[idx] = f2bf(v * scale);  // GEMM operand for the fmap gradients (compact rows)
    else
      g.p[0][o0] = v * scale;
  }
}

// Same fold, 4 consecutive row elements per thread: grid (row chunks, rows),
// 32-bit in-row index math only (the flat kernel above spends most of its time
// in 64-bit div/mod per element: 469 us for the 477 MB of the training-shape
// fold), one 16-B level-0 load, one 8-B bf16 store (or 16-B in-place store).
// Needs S[0] % 4 == 0 (pyramid rows are padded to 128 B).  bf16 rows have
// pitch OP >= E = H0*W0 (columns E..OP-1 are written as zeros: the padded
// operand of the corr_bwd.hip GEMMs); 8-B stores need OP % 4 == 0.
template <bool BF16>
__global__ __launch_bounds__(256) void pyr_fold4_kernel(PyrMut g, int levels, int rows, float scale,
                                                        bf16_t* __restrict__ out_bf16, int OP) {
  const int H0 = g.H[0], W0 = g.W[0], E = H0 * W0;
  const int span = BF16 ? OP : E;  // elements written per row
  const int E4 = (span + 3) >> 2;
  const bool vec_out = (OP & 3) == 0;
  for (int row = blockIdx.y; row < rows; row += gridDim.y) {
    float* r0 = g.p[0] + (size_t)row * g.S[0];
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < E4; q += gridDim.x * blockDim.x) {
      const int e = q * 4;
      const bool full = e + 4 <= E;
      float v[4];
      if (full) {
        const float4 t = *reinterpret_cast<const float4*>(r0 + e);
        v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = e + j < E ? r0[e + j] : 0.f;
      }
      if (e < E) {
        int ys[4], xs[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          ys[j] = (e + j) / W0;
          xs[j] = e + j - ys[j] * W0;
        }
        float w = 1.f;
#pragma unroll
        for (int l = 1; l < 4; ++l) {
          if (l >= levels) break;
          w *= 0.25f;
          const float* rl = g.p[l] + (size_t)row * g.S[l];
          const int Hl = g.H[l], Wl = g.W[l];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int yl = ys[j] >> l, xl = xs[j] >> l;
            if (e + j < E && yl < Hl && xl < Wl) v[j] += w * rl[yl * Wl + xl];
          }
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] *= scale;
      if (BF16) {
        bf16_t* o = out_bf16 + (size_t)row * OP + e;
        if (e + 4 <= OP && vec_out) {
          const uint2 pk = make_uint2(uint32_t(f2bf(v[0])) | (uint32_t(f2bf(v[1])) << 16),
                                      uint32_t(f2bf(v[2])) | (uint32_t(f2bf(v[3])) << 16));
          *reinterpret_cast<uint2*>(o) = pk;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (e + j < OP) o[j] = f2bf(v[j]);
        }
      } else if (full) {
        *reinterpret_cast<float4*>(r0 + e) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (e + j < E) r0[e + j] = v[j];
      }
    }
  }
}

// Padded bf16 fold (the operand of the corr_bwd.hip GEMMs): one block per
// row.  The coarse levels' cells of the row (<= 1 KB at the training shape)
// are staged in LDS first (coalesced), so each level-0 quad costs one 16-B
// load, 3 x 4 LDS reads and one 8-B store; columns E .. OP-1 are zeros.
// Needs OP % 4 == 0, OP <= 6144 and the coarse levels' cells <= FOLD_LDS
// floats; vec0: 16-B aligned level-0 rows (S[0] % 4 == 0), else scalar loads.
constexpr int FOLD_LDS = 4096;

__global__ __launch_bounds__(256) void pyr_fold_rows_kernel(PyrMut g, int levels, float scale,
                                                            bf16_t* __restrict__ out, bf16_t* __restrict__ out_lo,
                                                            int OP, int vec0) {
  __shared__ float cl[FOLD_LDS];
  const int row = blockIdx.x;
  const int H0 = g.H[0], W0 = g.W[0], E = H0 * W0;
  const float* r0 = g.p[0] + (size_t)row * g.S[0];
  // level-0 quads of this thread, loads issued before the LDS staging
  const int nq = OP >> 2;
  constexpr int QPT = 6;  // quads per thread (OP <= 6144 elements)
  float4 v[QPT];
#pragma unroll
  for (int j = 0; j < QPT; ++j) {
    const int e = (threadIdx.x + 256 * j) * 4;
    v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (e + 4 <= E && vec0) {
      v[j] = *reinterpret_cast<const float4*>(r0 + e);
    } else if (e + 4 <= E) {
      v[j] = make_float4(r0[e], r0[e + 1], r0[e + 2], r0[e + 3]);
    } else if (e < E) {
      v[j].x = r0[e];
      if (e + 1 < E) v[j].y = r0[e + 1];
      if (e + 2 < E) v[j].z = r0[e + 2];
    }
  }
  int off[4] = {0, 0, 0, 0};
  {
    int o = 0;
#pragma unroll
    for (int l = 1; l < 4; ++l) {
      off[l] = o;
      if (l < levels) {
        const int n = g.H[l] * g.W[l];
        const float* rl = g.p[l] + (size_t)row * g.S[l];
        for (int i = threadIdx.x; i < n; i += 256) cl[o + i] = rl[i];
        o += n;
      }
    }
  }
  __syncthreads();
  const float inv_w = 1.f / (float)W0;
#pragma unroll
  for (int j = 0; j < QPT; ++j) {
    const int q = threadIdx.x + 256 * j;
    if (q >= nq) break;
    const int e = q * 4;
    float f[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
    if (e < E) {
      int y = (int)(((float)e + 0.5f) * inv_w), x = e - y * W0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (e + k < E) {
          float w = 1.f;
#pragma unroll
          for (int l = 1; l < 4; ++l) {
            if (l >= levels) break;
            w *= 0.25f;
            const int yl = y >> l, xl = x >> l;
            if (yl < g.H[l] && xl < g.W[l]) f[k] += w * cl[off[l] + yl * g.W[l] + xl];
          }
        }
        if (++x == W0) {
          x = 0;
          ++y;
        }
      }
    }
    bf16_t hv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f[k] *= scale;
      hv[k] = f2bf(f[k]);
    }
    *reinterpret_cast<uint2*>(out + (size_t)row * OP + e) =
        make_uint2(uint32_t(hv[0]) | (uint32_t(hv[1]) << 16), uint32_t(hv[2]) | (uint32_t(hv[3]) << 16));
    if (out_lo != nullptr) {  // split-bf16 operand: lo = bf16(x - hi)
      bf16_t lv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) lv[k] = f2bf(f[k] - bf2f(hv[k]));
      *reinterpret_cast<uint2*>(out_lo + (size_t)row * OP + e) =
          make_uint2(uint32_t(lv[0]) | (uint32_t(lv[1]) << 16), uint32_t(lv[2]) | (uint32_t(lv[3]) << 16));
    }
  }
}

// Wave-per-row form of the padded bf16 fold (the training shape's operand of
// corr_bwd.hip: 22,816 rows of 2,852 level-0 cells): each wave owns one row,
// issues ALL its level-0 loads (QW float4 per lane, 16-B coalesced) and the
// row's coarse cells (staged in the wave's own LDS slice, no block barrier)
// before it computes; four rows per 256-thread block.  The block-per-row
// kernel above issued <= 3 loads per thread behind a block-wide barrier and
// ran at ~1.7 TB/s (profiles/r2/README.md); this one is bound by the HBM
// stream (profiles/r6/README.md).
constexpr int FW_LDS = 1024;  // coarse cells per row (wave): training shape 953
template <int QW>
__global__ __launch_bounds__(256) void pyr_fold_wave_kernel(PyrMut g, int levels, float scale,
                                                            bf16_t* __restrict__ out, int OP, int rows) {
  __shared__ float cl[4][FW_LDS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row = blockIdx.x * 4 + wave;
  if (row >= rows) return;  // whole wave (no block-level barrier below)
  const int H0 = g.H[0], W0 = g.W[0], E = H0 * W0;
  const float* r0 = g.p[0] + (size_t)row * g.S[0];
  float4 v[QW];
#pragma unroll
  for (int j = 0; j < QW; ++j) {
    const int e = (lane + 64 * j) * 4;
    v[j] = e + 4 <= E ? *reinterpret_cast<const float4*>(r0 + e) : make_float4(0.f, 0.f, 0.f, 0.f);
    if (e < E && e + 4 > E) {  // the row's ragged tail
      v[j].x = r0[e];
      if (e + 1 < E) v[j].y = r0[e + 1];
      if (e + 2 < E) v[j].z = r0[e + 2];
    }
  }
  int off[4] = {0, 0, 0, 0};
  {
    int o = 0;
#pragma unroll
    for (int l = 1; l < 4; ++l) {
      off[l] = o;
      if (l < levels) {
        const int n = g.H[l] * g.W[l];
        const float* rl = g.p[l] + (size_t)row * g.S[l];
        for (int i = lane; i < n; i += 64) cl[wave][o + i] = rl[i];
        o += n;
      }
    }
  }
  // the wave's own LDS slice: order its stores before the other lanes' reads
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const float inv_w = 1.f / (float)W0;
#pragma unroll
  for (int j = 0; j < QW; ++j) {
    const int e = (lane + 64 * j) * 4;
    if (e >= OP) break;
    float f[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
    if (e < E) {
      int y = (int)(((float)e + 0.5f) * inv_w), x = e - y * W0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (e + k < E) {
          float w = 1.f;
#pragma unroll
          for (int l = 1; l < 4; ++l) {
            if (l >= levels) break;
            w *= 0.25f;
            const int yl = y >> l, xl = x >> l;  // (floor pooling: the last odd row / column has no parent)
            if (yl < g.H[l] && xl < g.W[l]) f[k] += w * cl[wave][off[l] + yl * g.W[l] + xl];
          }
        }
        if (++x == W0) {
          x = 0;
          ++y;
        }
      }
    }
    const uint2 pk = make_uint2(uint32_t(f2bf(f[0] * scale)) | (uint32_t(f2bf(f[1] * scale)) << 16),
                                uint32_t(f2bf(f[2] * scale)) | (uint32_t(f2bf(f[3] * scale)) << 16));
    *reinterpret_cast<uint2*>(out + (size_t)row * OP + e) = pk;
  }
}

inline int grid_for(long total) {
  long blocks = (total + 255) / 256;
  if (blocks > 65535L * 8) blocks = 65535L * 8;
  return (int)blocks;
}

}  // namespace lookup

void corr_lookup_fwd_launch(const void* const* pyr, bool pyr_bf16, const int* Hs, const int* Ws, const int* Ss,
                            int levels, const float* coords, int B, int H1, int W1, int r, void* out,
                            bool out_bf16, hipStream_t stream, int ostride) {
  lookup::Pyr p;
  for (int l = 0; l < 4; ++l) {
    p.p[l] = l < levels ? pyr[l] : nullptr;
    p.H[l] = l < levels ? Hs[l] : 0;
    p.W[l] = l < levels ? Ws[l] : 0;
    p.S[l] = l < levels ? Ss[l] : 0;
  }
  const int CH = levels * (2 * r + 1) * (2 * r + 1);
  if (ostride <= 0) ostride = CH;
  const long total = (long)B * H1 * W1 * ostride;
  if (total == 0) return;
  const long P = (long)B * H1 * W1;
  if ((r == 3 || r == 4) && P < (1L << 30)) {
    const dim3 g((unsigned)((P + 3) / 4));
#define RS_LF(R_, PT_, T_)                                                                                    \
  hipLaunchKernelGGL((lookup::lookup_fwd_wave_kernel<R_, PT_, T_>), g, dim3(256), 0, stream, p, levels, coords, \
                     H1 * W1, (int)P, static_cast<T_*>(out), ostride)
#define RS_LF2(R_)                                                              \
  do {                                                                          \
    if (pyr_bf16) { if (out_bf16) RS_LF(R_, bf16_t, bf16_t); else RS_LF(R_, bf16_t, float); } \
    else { if (out_bf16) RS_LF(R_, float, bf16_t); else RS_LF(R_, float, float); } \
  } while (0)
    if (r == 3) RS_LF2(3);
    else RS_LF2(4);
#undef RS_LF2
#undef RS_LF
    return;
  }
  const int grid = lookup::grid_for(total);
#define RS_LG(PT_, T_)                                                                                     \
  hipLaunchKernelGGL((lookup::lookup_fwd_kernel<PT_, T_>), dim3(grid), dim3(256), 0, stream, p, levels, coords, \
                     B, H1, W1, r, static_cast<T_*>(out), total, ostride)
  if (pyr_bf16) { if (out_bf16) RS_LG(bf16_t, bf16_t); else RS_LG(bf16_t, float); }
  else { if (out_bf16) RS_LG(float, bf16_t); else RS_LG(float, float); }
#undef RS_LG
}

void corr_lookup_bwd_launch(float* const* gpyr, const int* Hs, const int* Ws, const int* Ss, int levels,
                            const float* coords, int B, int H1, int W1, int r, const void* dout,
                            bool dout_bf16, hipStream_t stream, int dstride) {
  if (dstride <= 0) dstride = levels * (2 * r + 1) * (2 * r + 1);
  lookup::PyrMut p;
  for (int l = 0; l < 4; ++l) {
    p.p[l] = l < levels ? gpyr[l] : nullptr;
    p.H[l] = l < levels ? Hs[l] : 0;
    p.W[l] = l < levels ? Ws[l] : 0;
    p.S[l] = l < levels ? Ss[l] : 0;
  }
  const long total = (long)B * H1 * W1 * levels * (2 * r + 2) * (2 * r + 2);
  if (total == 0) return;
  const long P = (long)B * H1 * W1;
  if ((r == 3 || r == 4) && P < (1L << 30)) {
    const dim3 g((unsigned)((P + 3) / 4));
#define RS_LB(R_, T_)                                                                                    \
  hipLaunchKernelGGL((lookup::lookup_bwd_wave_kernel<R_, T_>), g, dim3(256), 0, stream, p, levels, coords, \
                     H1 * W1, (int)P, static_cast<const T_*>(dout), dstride)
    if (r == 3) { if (dout_bf16) RS_LB(3, bf16_t); else RS_LB(3, float); }
    else { if (dout_bf16) RS_LB(4, bf16_t); else RS_LB(4, float); }
#undef RS_LB
    return;
  }
  const int grid = lookup::grid_for(total);
  if (dout_bf16)
    hipLaunchKernelGGL(lookup::lookup_bwd_kernel<bf16_t>, dim3(grid), dim3(256), 0, stream, p,
                       levels, coords, B, H1, W1, r, static_cast<const bf16_t*>(dout), total, dstride);
  else
    hipLaunchKernelGGL(lookup::lookup_bwd_kernel<float>, dim3(grid), dim3(256), 0, stream, p,
                       levels, coords, B, H1, W1, r, static_cast<const float*>(dout), total, dstride);
}

// out_lo (row fold only): the lo halves of a split-bf16 output
void pyr_grad_fold_launch(float* const* gpyr, const int* Hs, const int* Ws, const int* Ss, int levels, long rows,
                          float scale, hipStream_t stream, void* out_bf16, int opitch, void* out_lo) {
  lookup::PyrMut p;
  for (int l = 0; l < 4; ++l) {
    p.p[l] = l < levels ? gpyr[l] : nullptr;
    p.H[l] = l < levels ? Hs[l] : 0;
    p.W[l] = l < levels ? Ws[l] : 0;
    p.S[l] = l < levels ? Ss[l] : 0;
  }
  const long total = rows * Hs[0] * Ws[0];
  if (total == 0) return;
  const long E = (long)Hs[0] * Ws[0];
  if (opitch <= 0) opitch = (int)E;
  long coarse = 0;
  for (int l = 1; l < levels; ++l) coarse += (long)Hs[l] * Ws[l];
  const bool aligned0 = Ss[0] % 4 == 0 && reinterpret_cast<uintptr_t>(gpyr[0]) % 16 == 0;
  bool alignedc = true;
  for (int l = 1; l < levels; ++l) alignedc = alignedc && gpyr[l] != nullptr;
  if (out_bf16 && !out_lo && aligned0 && alignedc && opitch % 4 == 0 && opitch <= 64 * 4 * 12 &&
      coarse <= lookup::FW_LDS && rows < (1L << 31)) {
    const unsigned grid = (unsigned)((rows + 3) / 4);
    const int qw = (opitch + 255) / 256;  // float4 per lane
#define RS_FW(Q) hipLaunchKernelGGL((lookup::pyr_fold_wave_kernel<Q>), dim3(grid), dim3(256), 0, stream, p, levels, \
                                    scale, static_cast<bf16_t*>(out_bf16), opitch, (int)rows)
    if (qw <= 4) RS_FW(4);
    else if (qw <= 8) RS_FW(8);
    else RS_FW(12);
#undef RS_FW
    return;
  }
  if (out_bf16 && opitch % 4 == 0 && opitch <= 6144 && coarse <= lookup::FOLD_LDS && rows < (1L << 31)) {
    const int vec0 = Ss[0] % 4 == 0 && reinterpret_cast<uintptr_t>(gpyr[0]) % 16 == 0;
    hipLaunchKernelGGL(lookup::pyr_fold_rows_kernel, dim3((unsigned)rows), dim3(256), 0, stream, p, levels, scale,
                       static_cast<bf16_t*>(out_bf16), static_cast<bf16_t*>(out_lo), opitch, vec0);
    return;
  }
  if (Ss[0] % 4 == 0 && reinterpret_cast<uintptr_t>(gpyr[0]) % 16 == 0 && rows < (1L << 31) &&
      E < (1L << 30)) {
    const long span = out_bf16 ? opitch : E;
    const int bx = (int)std::min<long>((span + 4 * 256 - 1) / (4 * 256), 64);
    const dim3 grid(bx, (unsigned)std::min<long>(rows, 65535));
    if (out_bf16)
      hipLaunchKernelGGL(lookup::pyr_fold4_kernel<true>, grid, dim3(256), 0, stream, p, levels, (int)rows, scale,
                         static_cast<bf16_t*>(out_bf16), opitch);
    else
      hipLaunchKernelGGL(lookup::pyr_fold4_kernel<false>, grid, dim3(256), 0, stream, p, levels, (int)rows, scale,
                         nullptr, opitch);
    return;
  }
  // (the flat kernel writes compact rows: callers asking for a padded pitch check the aligned case above)
  hipLaunchKernelGGL(lookup::pyr_fold_kernel, dim3(lookup::grid_for(total)), dim3(256), 0, stream,
                     p, levels, rows, scale, static_cast<bf16_t*>(out_bf16));
}

}  // namespace rs
