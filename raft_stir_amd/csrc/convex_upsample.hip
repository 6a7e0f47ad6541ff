// Convex upsampling x8 (forward + backward).
//
// Replaces reference core/raft.py:72-83 (view -> softmax over 9 taps ->
// F.unfold(8*flow, 3x3, pad 1) -> weighted sum -> 6-D permute -> reshape),
// which materialises a (N, 2, 9, 8, 8, H, W) intermediate, with one kernel.
//
//   up[n, c, 8y+a, 8x+b] = sum_k softmax_k(mask[n, y, x, 64k + 8a + b]) * 8*flow[n, c, y+ky-1, x+kx-1]
//   (k = 3*ky + kx, zero padding outside the coarse grid)
//
// One wave64 per coarse pixel: lane = 8a + b owns one of its 64 sub-pixels.
// The mask is channels-last (the 1x1 mask-head conv writes NHWC), so the 9
// loads of a lane are 9 coalesced 64-lane rows; the 3x3 flow neighbourhood is
// wave-uniform.  Backward recomputes the softmax (nothing saved but inputs),
// writes dmask in the same coalesced layout, and reduces the 9x2 flow-
// neighbour partial sums across the wave; a second tiny kernel gathers them
// into dflow (deterministic, no atomics).

#include "common.h"

namespace rs {
namespace cvx {

constexpr int WAVES = 4;

template <typename MT>
__device__ __forceinline__ void softmax9(const MT* __restrict__ m, int lane, float (&p)[9]) {
  float mx = -INFINITY;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    p[k] = io<MT>::ld(m + 64 * k + lane);
    mx = fmaxf(mx, p[k]);
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    p[k] = __expf(p[k] - mx);
    s += p[k];
  }
  const float inv = 1.f / s;
#pragma unroll
  for (int k = 0; k < 9; ++k) p[k] *= inv;
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
__global__ __launch_bounds__(WAVES * 64) void convex_up_fwd_kernel(
    const float* __restrict__ flow, const MT* __restrict__ mask, int N, int H, int W,
    float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const long cp = (long)blockIdx.x * WAVES + (threadIdx.x >> 6);  // coarse pixel id
  if (cp >= (long)N * H * W) return;
  const int x = (int)(cp % W), y = (int)((cp / W) % H), n = (int)(cp / ((long)H * W));
  float p[9], u[9], v[9];
  softmax9(mask + cp * 576, lane, p);
  neighbours(flow, n, y, x, H, W, u, v);
  float su = 0.f, sv = 0.f;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    su += p[k] * u[k];
    sv += p[k] * v[k];
  }
  const int a = lane >> 3, b = lane & 7;
  const size_t W8 = (size_t)W * 8, plane = (size_t)H * 8 * W8;
  const size_t o = (size_t)(8 * y + a) * W8 + 8 * x + b;
  out[(size_t)n * 2 * plane + o] = su;
  out[(size_t)n * 2 * plane + plane + o] = sv;
}

template <typename MT, typename GT>
__global__ __launch_bounds__(WAVES * 64) void convex_up_bwd_kernel(
    const float* __restrict__ flow, const MT* __restrict__ mask, const GT* __restrict__ dup,
    int N, int H, int W, MT* __restrict__ dmask, float* __restrict__ partial) {
  const int lane = threadIdx.x & 63;
  const long cp = (long)blockIdx.x * WAVES + (threadIdx.x >> 6);
  if (cp >= (long)N * H * W) return;
  const int x = (int)(cp % W), y = (int)((cp / W) % H), n = (int)(cp / ((long)H * W));
  float p[9], u[9], v[9];
  softmax9(mask + cp * 576, lane, p);
  neighbours(flow, n, y, x, H, W, u, v);
  const int a = lane >> 3, b = lane & 7;
  const size_t W8 = (size_t)W * 8, plane = (size_t)H * 8 * W8;
  const size_t o = (size_t)(8 * y + a) * W8 + 8 * x + b;
  const float gu = io<GT>::ld(dup + (size_t)n * 2 * plane + o);
  const float gv = io<GT>::ld(dup + (size_t)n * 2 * plane + plane + o);
  // softmax backward: dm_k = p_k (dp_k - sum_j p_j dp_j), dp_k = gu*u_k + gv*v_k
  float dp[9], dot = 0.f;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    dp[k] = gu * u[k] + gv * v[k];
    dot += p[k] * dp[k];
  }
  MT* dm = dmask + cp * 576;
#pragma unroll
  for (int k = 0; k < 9; ++k) io<MT>::st(dm + 64 * k + lane, p[k] * (dp[k] - dot));
  // neighbour partials: d(8*flow_c[nbr_k]) = sum_lanes p_k * g_c  -> x8 for d flow
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    float su = wave_sum(p[k] * gu);
    float sv = wave_sum(p[k] * gv);
    if (lane == 0) {
      partial[cp * 18 + 2 * k + 0] = 8.f * su;
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

}  // namespace cvx

// flow: (N,2,H,W) fp32; mask: (N,H,W,576) channels-last; out: (N,2,8H,8W) fp32
void convex_up_fwd_launch(const float* flow, const void* mask, bool mask_bf16, int N, int H, int W,
                          float* out, hipStream_t stream) {
  const long cps = (long)N * H * W;
  if (cps == 0) return;
  dim3 grid((unsigned)((cps + cvx::WAVES - 1) / cvx::WAVES)), block(cvx::WAVES * 64);
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
  dim3 grid((unsigned)((cps + cvx::WAVES - 1) / cvx::WAVES)), block(cvx::WAVES * 64);
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

}  // namespace rs
