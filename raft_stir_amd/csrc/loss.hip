// Fused RAFT sequence loss (reference train.py:47-72):
//
//   loss = sum_i gamma^(N-1-i) * mean_{b,c,y,x}( valid[b,y,x] * |pred_i[b,c,y,x] - gt[b,c,y,x]| )
//   valid = (valid_in >= 0.5) & (|gt| < max_flow)
//
// The reference evaluates it as ~6 elementwise/reduction kernels per
// prediction (12 predictions -> ~70 launches forward, as many backward), each
// re-reading the full-resolution ground truth.  Here: one pass over all N
// predictions (ground truth and the valid mask read once per pixel and kept
// in registers across the N predictions), per-block partial sums reduced
// deterministically by a second tiny kernel; the backward is one pass that
// writes every prediction's gradient w_i * valid * sign(pred_i - gt) / M.
// The same forward pass also forms the training metrics of the last
// prediction (reference train.py:62-70: mean EPE and the 1 / 3 / 5 px
// accuracies over the valid pixels), which took ~40 small ATen launches.
#include "common.h"

namespace rs {
namespace loss {

constexpr int THREADS = 256;

constexpr int NACC = 6;  // loss, EPE, < 1 px, < 3 px, < 5 px, valid count

// grid-stride over (b, y, x); B planes of HW pixels.  preds: [N][B][2][HW];
// partial: [gridDim.x][NACC]
__global__ __launch_bounds__(THREADS) void seq_loss_fwd_kernel(const float* __restrict__ preds,
                                                                const float* __restrict__ gt,
                                                                const float* __restrict__ valid, int N,
                                                                int B, long HW, float gamma, float max_flow,
                                                                float inv_m, float* __restrict__ partial) {
  const long P = (long)B * HW;
  float acc[NACC] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (long p = (long)blockIdx.x * THREADS + threadIdx.x; p < P; p += (long)gridDim.x * THREADS) {
    const long b = p / HW, q = p - b * HW;
    const long g0 = b * 2 * HW + q;
    const float gu = gt[g0], gv = gt[g0 + HW];
    const bool ok = valid[p] >= 0.5f && sqrtf(gu * gu + gv * gv) < max_flow;
    if (!ok) continue;
    float w = 1.f, s = 0.f;
    for (int i = N - 1; i >= 0; --i) {  // weight gamma^(N-1-i)
      const float* pr = preds + (size_t)i * B * 2 * HW + g0;
      const float du = pr[0] - gu, dv = pr[HW] - gv;
      s += w * (fabsf(du) + fabsf(dv));
      if (i == N - 1) {  // metrics of the final prediction
        const float epe = sqrtf(du * du + dv * dv);
        acc[1] += epe;
        acc[2] += epe < 1.f ? 1.f : 0.f;
        acc[3] += epe < 3.f ? 1.f : 0.f;
        acc[4] += epe < 5.f ? 1.f : 0.f;
      }
      w *= gamma;
    }
    acc[0] += s;
    acc[5] += 1.f;
  }
  __shared__ float sm[NACC][THREADS / 64];
#pragma unroll
  for (int k = 0; k < NACC; ++k) {
    const float v = wave_sum(acc[k]);
    if ((threadIdx.x & 63) == 0) sm[k][threadIdx.x >> 6] = v;
  }
  __syncthreads();
  if (threadIdx.x < NACC) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < THREADS / 64; ++w) t += sm[threadIdx.x][w];
    partial[blockIdx.x * NACC + threadIdx.x] = threadIdx.x == 0 ? t * inv_m : t;
  }
}

// out[0] = loss; out[1..4] = EPE, 1 / 3 / 5 px accuracy (means over the valid
// pixels, 0 when there are none): fixed-order fp64 sums of the block partials
__global__ __launch_bounds__(THREADS) void sum_kernel(const float* __restrict__ partial, int n,
                                                      float* __restrict__ out) {
  __shared__ double sm[NACC][THREADS];
  double t[NACC] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  for (int i = threadIdx.x; i < n; i += THREADS)
#pragma unroll
    for (int k = 0; k < NACC; ++k) t[k] += partial[i * NACC + k];
#pragma unroll
  for (int k = 0; k < NACC; ++k) sm[k][threadIdx.x] = t[k];
  __syncthreads();
  for (int s = THREADS / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s)
#pragma unroll
      for (int k = 0; k < NACC; ++k) sm[k][threadIdx.x] += sm[k][threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double cnt = sm[5][0] > 1.0 ? sm[5][0] : 1.0;
    out[0] = (float)sm[0][0];
#pragma unroll
    for (int k = 1; k < 5; ++k) out[k] = (float)(sm[k][0] / cnt);
  }
}

__global__ __launch_bounds__(THREADS) void seq_loss_bwd_kernel(const float* __restrict__ preds,
                                                                const float* __restrict__ gt,
                                                                const float* __restrict__ valid, int N,
                                                                int B, long HW, float gamma, float max_flow,
                                                                float inv_m, const float* __restrict__ gout,
                                                                float* __restrict__ grad) {
  const long P = (long)B * HW;
  const float go = gout[0] * inv_m;
  for (long p = (long)blockIdx.x * THREADS + threadIdx.x; p < P; p += (long)gridDim.x * THREADS) {
    const long b = p / HW, q = p - b * HW;
    const long g0 = b * 2 * HW + q;
    const float gu = gt[g0], gv = gt[g0 + HW];
    const bool ok = valid[p] >= 0.5f && sqrtf(gu * gu + gv * gv) < max_flow;
    float w = go;
    for (int i = N - 1; i >= 0; --i) {
      const size_t o = (size_t)i * B * 2 * HW + g0;
      float du = 0.f, dv = 0.f;
      if (ok) {
        const float eu = preds[o] - gu, ev = preds[o + HW] - gv;
        du = eu > 0.f ? w : (eu < 0.f ? -w : 0.f);
        dv = ev > 0.f ? w : (ev < 0.f ? -w : 0.f);
      }
      grad[o] = du;
      grad[o + HW] = dv;
      w *= gamma;
    }
  }
}

}  // namespace loss

static int loss_grid(long P) {
  const long g = (P + loss::THREADS - 1) / loss::THREADS;
  return (int)(g < 2048 ? g : 2048);
}

// partial: nblocks * loss::NACC floats; out: 5 floats (loss, EPE, 1 / 3 / 5 px)
void seq_loss_fwd_launch(const float* preds, const float* gt, const float* valid, int N, int B, long HW,
                         float gamma, float max_flow, float* partial, int nblocks, float* out,
                         hipStream_t s) {
  const float inv_m = 1.f / (float)((double)B * 2 * HW);
  hipLaunchKernelGGL(loss::seq_loss_fwd_kernel, dim3(nblocks), dim3(loss::THREADS), 0, s, preds, gt, valid,
                     N, B, HW, gamma, max_flow, inv_m, partial);
  hipLaunchKernelGGL(loss::sum_kernel, dim3(1), dim3(loss::THREADS), 0, s, partial, nblocks, out);
}

int seq_loss_blocks(long P) { return loss_grid(P); }
int seq_loss_partials(long P) { return loss_grid(P) * loss::NACC; }

void seq_loss_bwd_launch(const float* preds, const float* gt, const float* valid, int N, int B, long HW,
                         float gamma, float max_flow, const float* gout, float* grad, hipStream_t s) {
  const float inv_m = 1.f / (float)((double)B * 2 * HW);
  hipLaunchKernelGGL(loss::seq_loss_bwd_kernel, dim3(loss_grid((long)B * HW)), dim3(loss::THREADS), 0, s,
                     preds, gt, valid, N, B, HW, gamma, max_flow, inv_m, gout, grad);
}

}  // namespace rs
