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
    int N, int H, int W, MT* __restrict__ dmask, float* __restrict__ partial) {
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
    MT* d = dmask + cp * 576 + 8 * a;
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
//   dflow[n][c][i][j] = 8 * sum_{I, J} ah[I][i] aw[J][j] g[n][c][I][J]
// ah [8H][H], aw [8W][W]: the interpolation matrices (upsample_bilinear2d's
// float32 source-index arithmetic, models/fused_train.py _interp_matrix).
// Gather form, one output per thread: the nonzero rows of column i lie in
// [floor((i - 1) / r), ceil((i + 1) / r)] for r = (H - 1) / (8H - 1); the loop
// runs a window two wider on each side (zeros outside the band add nothing)
// -- deterministic, no atomics.
__global__ __launch_bounds__(256) void upflow8_bwd_kernel(const float* __restrict__ g, const float* __restrict__ ah,
                                                          const float* __restrict__ aw, int NC, int H, int W,
                                                          float* __restrict__ out) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)NC * H * W;
  if (idx >= total) return;
  const int j = (int)(idx % W), i = (int)((idx / W) % H), nc = (int)(idx / ((long)H * W));
  const int H8 = 8 * H, W8 = 8 * W;
  const float rh = H > 1 ? (float)(H8 - 1) / (float)(H - 1) : 0.f;  // output rows per input row
  const float rw = W > 1 ? (float)(W8 - 1) / (float)(W - 1) : 0.f;
  // (a single input row / column: every output row / column reads it)
  const int I0 = H > 1 ? max(0, (int)floorf((i - 1) * rh) - 2) : 0;
  const int I1 = H > 1 ? min(H8 - 1, (int)ceilf((i + 1) * rh) + 2) : H8 - 1;
  const int J0 = W > 1 ? max(0, (int)floorf((j - 1) * rw) - 2) : 0;
  const int J1 = W > 1 ? min(W8 - 1, (int)ceilf((j + 1) * rw) + 2) : W8 - 1;
  const float* gp = g + (size_t)nc * H8 * W8;
  float acc = 0.f;
  for (int I = I0; I <= I1; ++I) {
    const float a = ah[(size_t)I * H + i];
    if (a == 0.f) continue;
    float row = 0.f;
    for (int J = J0; J <= J1; ++J) row += aw[(size_t)J * W + j] * gp[(size_t)I * W8 + J];
    acc += a * row;
  }
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

// partial: scratch (N*H*W*18) fp32
void convex_up_bwd_launch(const float* flow, const void* mask, bool mask_bf16, const void* dup,
                          bool dup_bf16, int N, int H, int W, void* dmask, float* dflow,
                          float* partial, hipStream_t stream) {
  const long cps = (long)N * H * W;
  if (cps == 0) return;
  dim3 grid((unsigned)cdiv(W, cvx::XB), (unsigned)H, (unsigned)N), block(cvx::WPB * 64);
#define RS_L(MT, GT)                                                                         \
  hipLaunchKernelGGL((cvx::convex_up_bwd_kernel<MT, GT>), grid, block, 0, stream, flow,     \
                     static_cast<const MT*>(mask), static_cast<const GT*>(dup), N, H, W,     \
                     static_cast<MT*>(dmask), partial)
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

void upflow8_bwd_launch(const float* g, const float* ah, const float* aw, int NC, int H, int W, float* out,
                        hipStream_t stream) {
  const long total = (long)NC * H * W;
  if (total > 0)
    hipLaunchKernelGGL(cvx::upflow8_bwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, g, ah, aw,
                       NC, H, W, out);
}

}  // namespace rs
