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

#include "common.h"

namespace rs {
namespace lookup {

struct Pyr {
  const float* p[4];
  int H[4];
  int W[4];
};
struct PyrMut {
  float* p[4];
  int H[4];
  int W[4];
};

template <typename OutT>
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
    const float* row = pyr.p[l] + pix * (size_t)H * W;
    float v = 0.f;
    const bool xin0 = x0 >= 0 && x0 < W, xin1 = x0 + 1 >= 0 && x0 + 1 < W;
    if (y0 >= 0 && y0 < H) {
      const float* rr = row + (size_t)y0 * W;
      if (xin0) v += (1.f - fx) * (1.f - fy) * rr[x0];
      if (xin1) v += fx * (1.f - fy) * rr[x0 + 1];
    }
    if (y0 + 1 >= 0 && y0 + 1 < H) {
      const float* rr = row + (size_t)(y0 + 1) * W;
      if (xin0) v += (1.f - fx) * fy * rr[x0];
      if (xin1) v += fx * fy * rr[x0 + 1];
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
    float* dst = gpyr.p[l] + pix * (size_t)H * W + (size_t)Y * W + X;
    *dst += acc;
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
    float v = g.p[0][idx];
    float w = 1.f;
#pragma unroll
    for (int l = 1; l < 4; ++l) {
      if (l >= levels) break;
      w *= 0.25f;
      const int yl = y >> l, xl = x >> l;
      if (yl < g.H[l] && xl < g.W[l])
        v += w * g.p[l][row * (size_t)g.H[l] * g.W[l] + (size_t)yl * g.W[l] + xl];
    }
    if (out_bf16)
      out_bf16[idx] = f2bf(v * scale);  // GEMM operand for the fmap gradients
    else
      g.p[0][idx] = v * scale;
  }
}

inline int grid_for(long total) {
  long blocks = (total + 255) / 256;
  if (blocks > 65535L * 8) blocks = 65535L * 8;
  return (int)blocks;
}

}  // namespace lookup

void corr_lookup_fwd_launch(const float* const* pyr, const int* Hs, const int* Ws, int levels,
                            const float* coords, int B, int H1, int W1, int r, void* out,
                            bool out_bf16, hipStream_t stream, int ostride) {
  lookup::Pyr p;
  for (int l = 0; l < 4; ++l) {
    p.p[l] = l < levels ? pyr[l] : nullptr;
    p.H[l] = l < levels ? Hs[l] : 0;
    p.W[l] = l < levels ? Ws[l] : 0;
  }
  const int CH = levels * (2 * r + 1) * (2 * r + 1);
  if (ostride <= 0) ostride = CH;
  const long total = (long)B * H1 * W1 * ostride;
  if (total == 0) return;
  const int grid = lookup::grid_for(total);
  if (out_bf16)
    hipLaunchKernelGGL(lookup::lookup_fwd_kernel<bf16_t>, dim3(grid), dim3(256), 0, stream, p,
                       levels, coords, B, H1, W1, r, static_cast<bf16_t*>(out), total, ostride);
  else
    hipLaunchKernelGGL(lookup::lookup_fwd_kernel<float>, dim3(grid), dim3(256), 0, stream, p,
                       levels, coords, B, H1, W1, r, static_cast<float*>(out), total, ostride);
}

void corr_lookup_bwd_launch(float* const* gpyr, const int* Hs, const int* Ws, int levels,
                            const float* coords, int B, int H1, int W1, int r, const void* dout,
                            bool dout_bf16, hipStream_t stream, int dstride) {
  if (dstride <= 0) dstride = levels * (2 * r + 1) * (2 * r + 1);
  lookup::PyrMut p;
  for (int l = 0; l < 4; ++l) {
    p.p[l] = l < levels ? gpyr[l] : nullptr;
    p.H[l] = l < levels ? Hs[l] : 0;
    p.W[l] = l < levels ? Ws[l] : 0;
  }
  const long total = (long)B * H1 * W1 * levels * (2 * r + 2) * (2 * r + 2);
  if (total == 0) return;
  const int grid = lookup::grid_for(total);
  if (dout_bf16)
    hipLaunchKernelGGL(lookup::lookup_bwd_kernel<bf16_t>, dim3(grid), dim3(256), 0, stream, p,
                       levels, coords, B, H1, W1, r, static_cast<const bf16_t*>(dout), total, dstride);
  else
    hipLaunchKernelGGL(lookup::lookup_bwd_kernel<float>, dim3(grid), dim3(256), 0, stream, p,
                       levels, coords, B, H1, W1, r, static_cast<const float*>(dout), total, dstride);
}

void pyr_grad_fold_launch(float* const* gpyr, const int* Hs, const int* Ws, int levels, long rows,
                          float scale, hipStream_t stream, void* out_bf16) {
  lookup::PyrMut p;
  for (int l = 0; l < 4; ++l) {
    p.p[l] = l < levels ? gpyr[l] : nullptr;
    p.H[l] = l < levels ? Hs[l] : 0;
    p.W[l] = l < levels ? Ws[l] : 0;
  }
  const long total = rows * Hs[0] * Ws[0];
  if (total == 0) return;
  hipLaunchKernelGGL(lookup::pyr_fold_kernel, dim3(lookup::grid_for(total)), dim3(256), 0, stream,
                     p, levels, rows, scale, static_cast<bf16_t*>(out_bf16));
}

}  // namespace rs
