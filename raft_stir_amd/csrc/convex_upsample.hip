// Convex upsampling x8 (forward + backward).
//
// Replaces reference core/raft.py:72-83 (view -> softmax over 9 taps ->
// F.unfold(8*flow, 3x3, pad 1) -> weighted sum -> 6-D permute -> reshape),
// which materialises a (N, 2, 9, 8, 8, H, W) intermediate, with one kernel.
//
//   up[n, c, 8y+a, 8x+b] = sum_k softmax_k(mask[n, y, x, 64k + 8a + b]) * 8*flow[n, c, y+ky-1, x+kx-1]
//   (k = 3*ky + kx, zero padding outside the coarse grid)
//
// Work mapping: one thread per (coarse pixel, fine row a): it owns the 8
// sub-pixels b = 0..7 of that row, so every mask read is one 16-byte load
// (8 bf16 of tap k) and every output write 32 contiguous bytes per channel.
// A wave = 8 coarse pixels x 8 rows (lane = 8a + xo), a 256-thread block 32
// consecutive coarse pixels of one coarse row (grid = (W/32, H, N): no index
// divisions); the 8 lanes of one a write 256 contiguous bytes of a fine row.
// The mask is channels-last (the 1x1 mask-head conv writes NHWC).  Backward
// recomputes the softmax (nothing saved but inputs), writes dmask in the same
// layout, and reduces the 9x2 flow-neighbour partial sums of each coarse
// pixel over its 64 sub-pixels (8 in-thread, 8 rows by xor shuffles); a
// second tiny kernel gathers them into dflow (deterministic, no atomics).

#include <algorithm>
#include <cmath>

#include "common.h"

namespace rs {
namespace cvx {

constexpr int XW = 8;   // coarse pixels per wave
constexpr int WPB = 4;  // waves per block
constexpr int XB = XW * WPB;

__device__ __forceinline__ void ld8(const bf16_t* p, float (&f)[8]) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = bf2f((bf16_t)(w[i] & 0xffffu));
    f[2 * i + 1] = bf2f((bf16_t)(w[i] >> 16));
  }
}
__device__ __forceinline__ void ld8(const float* p, float (&f)[8]) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w;
  f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}
__device__ __forceinline__ void st8(bf16_t* p, const float (&f)[8]) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = uint32_t(f2bf(f[2 * i])) | (uint32_t(f2bf(f[2 * i + 1])) << 16);
  *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}
__device__ __forceinline__ void st8(float* p, const float (&f)[8]) {
  reinterpret_cast<float4*>(p)[0] = make_float4(f[0], f[1], f[2], f[3]);
  reinterpret_cast<float4*>(p)[1] = make_float4(f[4], f[5], f[6], f[7]);
}

// p[k][b] = softmax over k of m[64k + b] (m points at row a: mask + 8a)
template <typename MT>
__device__ __forceinline__ void softmax9x8(const MT* __restrict__ m, float (&p)[9][8]) {
#pragma unroll
  for (int k = 0; k < 9; ++k) ld8(m + 64 * k, p[k]);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    float mx = p[0][b];
#pragma unroll
    for (int k = 1; k < 9; ++k) mx = fmaxf(mx, p[k][b]);
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      p[k][b] = __expf(p[k][b] - mx);
      s += p[k][b];
    }
    const float inv = 1.f / s;
#pragma unroll
    for (int k = 0; k < 9; ++k) p[k][b] *= inv;
  }
}

__device__ __forceinline__ void neighbours(const float* __restrict__ flow, int n, int y, int x,
                                           int H, int W, float (&u)[9], float (&v)[9]) {
  const size_t plane = (size_t)H * W;
  const float* fu = flow + (size_t)n * 2 * plane;
  const float* fv = fu + plane;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int yy = y + k / 3 - 1, xx = x + k % 3 - 1;
    const bool in = yy >= 0 && yy < H && xx >= 0 && xx < W;
    u[k] = in ? 8.f * fu[(size_t)yy * W + xx] : 0.f;
    v[k] = in ? 8.f * fv[(size_t)yy * W + xx] : 0.f;
  }
}

template <typename MT>
__global__ __launch_bounds__(WPB * 64) void convex_up_fwd_kernel(
    const float* __restrict__ flow, const MT* __restrict__ mask, int N, int H, int W,
    float* __restrict__ out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int a = lane >> 3, x = blockIdx.x * XB + wave * XW + (lane & 7), y = blockIdx.y, n = blockIdx.z;
  if (x >= W) return;
  const size_t cp = ((size_t)n * H + y) * W + x;
  float p[9][8], u[9], v[9];
  softmax9x8(mask + cp * 576 + 8 * a, p);
  neighbours(flow, n, y, x, H, W, u, v);
  float su[8], sv[8];
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    su[b] = 0.f;
    sv[b] = 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      su[b] += p[k][b] * u[k];
      sv[b] += p[k][b] * v[k];
    }
  }
  const size_t W8 = (size_t)W * 8, plane = (size_t)H * 8 * W8;
  float* o = out + (size_t)n * 2 * plane + (size_t)(8 * y + a) * W8 + 8 * (size_t)x;
  st8(o, su);
  st8(o + plane, sv);
}

template <typename MT, typename GT>
__global__ __launch_bounds__(WPB * 64) void convex_up_bwd_kernel(
    const float* __restrict__ flow, const MT* __restrict__ mask, const GT* __restrict__ dup,
    int N, int H, int W, MT* __restrict__ dmask, int dpitch, float* __restrict__ partial) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int a = lane >> 3, x0 = blockIdx.x * XB + wave * XW + (lane & 7), y = blockIdx.y, n = blockIdx.z;
  const bool in = x0 < W;
  const int x = in ? x0 : W - 1;  // out-of-range lanes still join the shuffles (zero gradient)
  const size_t cp = ((size_t)n * H + y) * W + x;
  float p[9][8], u[9], v[9], gu[8], gv[8];
  softmax9x8(mask + cp * 576 + 8 * a, p);
  neighbours(flow, n, y, x, H, W, u, v);
  const size_t W8 = (size_t)W * 8, plane = (size_t)H * 8 * W8;
  const GT* g = dup + (size_t)n * 2 * plane + (size_t)(8 * y + a) * W8 + 8 * (size_t)x;
  ld8(g, gu);
  ld8(g + plane, gv);
  if (!in) {
#pragma unroll
    for (int b = 0; b < 8; ++b) gu[b] = gv[b] = 0.f;
  }
  // softmax backward: dm_k = p_k (dp_k - sum_j p_j dp_j), dp_k = gu*u_k + gv*v_k
  float dm[9][8];
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      dm[k][b] = gu[b] * u[k] + gv[b] * v[k];
      dot += p[k][b] * dm[k][b];
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) dm[k][b] = p[k][b] * (dm[k][b] - dot);
  }
  if (in) {
    MT* d = dmask + cp * dpitch + 8 * a;
#pragma unroll
    for (int k = 0; k < 9; ++k) st8(d + 64 * k, dm[k]);
  }
  // neighbour partials: d(8*flow_c[nbr_k]) = sum over the 64 sub-pixels of p_k * g_c  (x8 for d flow):
  // the 8 b in-thread, the 8 rows a (lanes 8 apart) by xor shuffles
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    float su = 0.f, sv = 0.f;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      su += p[k][b] * gu[b];
      sv += p[k][b] * gv[b];
    }
#pragma unroll
    for (int m = 8; m < 64; m <<= 1) {
      su += __shfl_xor(su, m, 64);
      sv += __shfl_xor(sv, m, 64);
    }
    if (a == 0 && in) {
      partial[cp * 18 + 2 * k] = 8.f * su;
      partial[cp * 18 + 2 * k + 1] = 8.f * sv;
    }
  }
}

// dflow[n, c, y, x] = sum_k partial[n, y - ky + 1, x - kx + 1, k, c]
__global__ __launch_bounds__(256) void convex_up_gather_kernel(const float* __restrict__ partial,
                                                                int N, int H, int W,
                                                                float* __restrict__ dflow) {
  const long total = (long)N * H * W;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int x = (int)(i % W), y = (int)((i / W) % H), n = (int)(i / ((long)H * W));
    float su = 0.f, sv = 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int yy = y - (k / 3 - 1), xx = x - (k % 3 - 1);
      if (yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
      const size_t src = (((size_t)n * H + yy) * W + xx) * 18 + 2 * k;
      su += partial[src];
      sv += partial[src + 1];
    }
    const size_t plane = (size_t)H * W;
    dflow[(size_t)n * 2 * plane + (size_t)y * W + x] = su;
    dflow[(size_t)n * 2 * plane + plane + (size_t)y * W + x] = sv;
  }
}

// Adjoint of RAFT-small's x8 bilinear upsampling with align_corners=True
// (reference core/utils/utils.py:80-82 upflow8, the training loss path):
//   dflow[n][c][i][j] = 8 * sum_I ah[I][i] * (sum_J aw[J][j] g[n][c][I][J])
// ah [8H][H], aw [8W][W]: the interpolation matrices (upsample_bilinear2d's
// float32 source-index arithmetic, models/fused_train.py _interp_matrix).
// Separable, two gather passes (deterministic, no atomics):
//   upflow8_cols_kernel: T[n][c][I][j] = sum_J aw[J][j] g[n][c][I][J]  (8W -> W)
//   upflow8_rows_kernel: dflow[n][c][i][j] = 8 sum_I ah[I][i] T[n][c][I][j]  (8H -> H)
// The nonzero rows of column j of aw lie in [floor((j - 1) r), ceil((j + 1) r)]
// for r = (8W - 1) / (W - 1); the loops run a window two wider on each side
// (zeros outside the band add nothing).
// The column pass reads each g row once, coalesced, into LDS: the band's
// weights differ per output column, so a direct gather from aw / g put every
// lane of a load on its own cache line (327 us per RAFT-small step, vs the
// 140 MB of g it has to read).  A block stages the W x L band weights once
// (wb[t][j] = aw[J0(j) + t][j]), then walks its rows RG at a time.
__device__ __forceinline__ void band(int j, int n, float r, int* lo, int* hi) {
  // (a single input row / column: every output row / column reads it)
  *lo = n > 1 ? max(0, (int)floorf((j - 1) * r) - 2) : 0;
  *hi = n > 1 ? min(8 * n - 1, (int)ceilf((j + 1) * r) + 2) : 8 * n - 1;
}

constexpr int UP_ROWS = 64;  // rows (n, c, I) per block of the column pass

__global__ __launch_bounds__(256) void upflow8_cols_kernel(const float* __restrict__ g, const float* __restrict__ aw,
                                                           long nrows, int W, int L, float* __restrict__ T) {
  extern __shared__ float sm[];
  const int W8 = 8 * W, t = threadIdx.x;
  const int RG = W >= 256 ? 1 : 256 / W;
  float* wb = sm;          // [L][W]
  float* gs = sm + L * W;  // [RG][8W]
  const float rw = W > 1 ? (float)(W8 - 1) / (float)(W - 1) : 0.f;
  for (int e = t; e < L * W; e += 256) {
    const int k = e / W, j = e - k * W;
    int J0, J1;
    band(j, W, rw, &J0, &J1);
    wb[e] = J0 + k <= J1 ? aw[(size_t)(J0 + k) * W + j] : 0.f;
  }
  const long rb = (long)blockIdx.x * UP_ROWS, re = min(nrows, rb + UP_ROWS);
  for (long r0 = rb; r0 < re; r0 += RG) {
    const int nr = (int)min((long)RG, re - r0);
    __syncthreads();  // wb staged / the previous rows consumed
    const float4* src = reinterpret_cast<const float4*>(g + (size_t)r0 * W8);
    for (int e = t; e < nr * W8 / 4; e += 256) reinterpret_cast<float4*>(gs)[e] = src[e];
    __syncthreads();
    for (int u = t; u < nr * W; u += 256) {
      const int rr = u / W, j = u - rr * W;
      int J0, J1;
      band(j, W, rw, &J0, &J1);
      const float* gr = gs + rr * W8 + J0;
      float acc = 0.f;
      for (int k = 0; k <= J1 - J0; ++k) acc += wb[k * W + j] * gr[k];
      T[(size_t)(r0 + rr) * W + j] = acc;
    }
  }
}

__global__ __launch_bounds__(256) void upflow8_rows_kernel(const float* __restrict__ T, const float* __restrict__ ah,
                                                           int NC, int H, int W, float* __restrict__ out) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)NC * H * W;
  if (idx >= total) return;
  const int j = (int)(idx % W), i = (int)((idx / W) % H), nc = (int)(idx / ((long)H * W));
  const int H8 = 8 * H;
  const float rh = H > 1 ? (float)(H8 - 1) / (float)(H - 1) : 0.f;
  int I0, I1;
  band(i, H, rh, &I0, &I1);
  const float* tp = T + (size_t)nc * H8 * W + j;
  float acc = 0.f;
  for (int I = I0; I <= I1; ++I) acc += ah[(size_t)I * H + i] * tp[(size_t)I * W];
  out[idx] = 8.f * acc;
}

}  // namespace cvx

// flow: (N,2,H,W) fp32; mask: (N,H,W,576) channels-last; out: (N,2,8H,8W) fp32
void convex_up_fwd_launch(const float* flow, const void* mask, bool mask_bf16, int N, int H, int W,
                          float* out, hipStream_t stream) {
  const long cps = (long)N * H * W;
  if (cps == 0) return;
  dim3 grid((unsigned)cdiv(W, cvx::XB), (unsigned)H, (unsigned)N), block(cvx::WPB * 64);
  if (mask_bf16)
    hipLaunchKernelGGL(cvx::convex_up_fwd_kernel<bf16_t>, grid, block, 0, stream, flow,
                       static_cast<const bf16_t*>(mask), N, H, W, out);
  else
    hipLaunchKernelGGL(cvx::convex_up_fwd_kernel<float>, grid, block, 0, stream, flow,
                       static_cast<const float*>(mask), N, H, W, out);
}

// partial: scratch (N*H*W*18) fp32; dmask: (N,H,W,dpitch), channels 0..575 written
void convex_up_bwd_launch(const float* flow, const void* mask, bool mask_bf16, const void* dup,
                          bool dup_bf16, int N, int H, int W, void* dmask, int dpitch, float* dflow,
                          float* partial, hipStream_t stream) {
  const long cps = (long)N * H * W;
  if (cps == 0) return;
  dim3 grid((unsigned)cdiv(W, cvx::XB), (unsigned)H, (unsigned)N), block(cvx::WPB * 64);
#define RS_L(MT, GT)                                                                         \
  hipLaunchKernelGGL((cvx::convex_up_bwd_kernel<MT, GT>), grid, block, 0, stream, flow,     \
                     static_cast<const MT*>(mask), static_cast<const GT*>(dup), N, H, W,     \
                     static_cast<MT*>(dmask), dpitch, partial)
  if (mask_bf16) {
    if (dup_bf16) RS_L(bf16_t, bf16_t); else RS_L(bf16_t, float);
  } else {
    if (dup_bf16) RS_L(float, bf16_t); else RS_L(float, float);
  }
#undef RS_L
  long g = (cps + 255) / 256;
  if (g > 65535) g = 65535;
  hipLaunchKernelGGL(cvx::convex_up_gather_kernel, dim3((unsigned)g), dim3(256), 0, stream,
                     partial, N, H, W, dflow);
}

// tmp: NC * 8H * W floats (the column pass)
int upflow8_band(int W) {  // band width bound of the column pass (cvx::band)
  if (W <= 1) return 8;
  const float rw = (float)(8 * W - 1) / (float)(W - 1);
  return std::min(8 * W, (int)std::ceil(2.f * rw) + 8);
}

size_t upflow8_cols_lds(int W) {
  const int RG = W >= 256 ? 1 : 256 / W;
  return (size_t)(upflow8_band(W) * W + RG * 8 * W) * sizeof(float);
}

void upflow8_bwd_launch(const float* g, const float* ah, const float* aw, int NC, int H, int W, float* tmp,
                        float* out, hipStream_t stream) {
  const long nrows = (long)NC * 8 * H, t2 = (long)NC * H * W;
  if (t2 == 0) return;
  hipLaunchKernelGGL(cvx::upflow8_cols_kernel, dim3((unsigned)((nrows + cvx::UP_ROWS - 1) / cvx::UP_ROWS)), dim3(256),
                     upflow8_cols_lds(W), stream, g, aw, nrows, W, upflow8_band(W), tmp);
  hipLaunchKernelGGL(cvx::upflow8_rows_kernel, dim3((unsigned)((t2 + 255) / 256)), dim3(256), 0, stream, tmp, ah, NC,
                     H, W, out);
}

}  // namespace rs
