// Fused gradient clipping + AdamW over every parameter of the model in two
// launches (reference train.py:173-181: clip_grad_norm_(model.parameters(),
// clip) then AdamW.step(), core/utils ... optim.AdamW(lr, wdecay, eps)).
//
// The stock path is clip_grad_norm_ (per-dtype foreach norms, a stack, a
// norm, a clamp, a foreach multiply) followed by the fused AdamW's Python
// bookkeeping over ~120 tensors and its multi-tensor launches: ~1 ms of host
// time at the tail of every step, while the GPU has nothing queued.  Here the
// parameter list is one kernel argument (device pointers, prefix offsets into
// one flat element space -- <= 128 tensors per launch group) and:
//
//   sumsq_kernel : block b reduces the squares of the gradient elements
//                  [b * CH, (b + 1) * CH) of the concatenated space (crossing
//                  tensor boundaries) into partial[b] -- plain stores;
//   adamw_kernel : every block first sums ALL partials in the same fixed
//                  order (deterministic, bitwise equal in every block), forms
//                  the clip coefficient min(max_norm / (||g|| + 1e-6), 1)
//                  (PyTorch's clip_grad_norm_), then updates its element range:
//                    g  = grad * coef            (the .grad tensors are left unclipped)
//                    p *= 1 - lr * wd
//                    m  = b1 m + (1 - b1) g ;  v = b2 v + (1 - b2) g^2
//                    p -= lr / bc1 * m / (sqrt(v) / sqrt(bc2) + eps)
//                  (torch.optim.AdamW's update).  A non-finite norm leaves
//                  parameters and moments untouched (the trainer's
//                  device-side skip of a non-finite step).
//
// Parameters and gradients are fp32 with identical dense strides (the memory
// of each is walked as a flat array); the moments are two flat fp32 buffers
// in the same concatenated order.  lr may live in device memory (hipGraph
// capture with a scheduler that writes it in place).
#include "common.h"
#include "optim.h"

namespace rs {
namespace optim {

constexpr int THREADS = 256;

// first tensor whose range contains element e (off[i] <= e < off[i+1])
__device__ __forceinline__ int find_tensor(const TList& L, long long e) {
  int lo = 0, hi = L.n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (L.off[mid] <= e) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ float block_sum(float v, float* sm) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) sm[wave] = v;
  __syncthreads();
  float t = 0.f;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int w = 0; w < THREADS / 64; ++w) t += sm[w];
    sm[THREADS / 64] = t;
  }
  __syncthreads();
  t = sm[THREADS / 64];
  __syncthreads();
  return t;
}

// state[0]: completed steps, state[1]: 1 if the previous call's update ran
// (finite norm) -- folded into the count here, i.e. before this call's
// adamw_kernel reads it, so a skipped step does not advance the bias
// corrections (torch's fused AdamW with found_inf)
__global__ __launch_bounds__(THREADS) void sumsq_kernel(TList L, float* __restrict__ partial, float* __restrict__ state) {
  __shared__ float sm[THREADS / 64 + 1];
  if (blockIdx.x == 0 && L.pbase == 0 && threadIdx.x == 0) {
    state[0] += state[1];
    state[1] = 0.f;
  }
  const long long e0 = (long long)blockIdx.x * CH;
  const long long e1 = min(e0 + CH, L.off[L.n]);
  float acc = 0.f;
  int ti = find_tensor(L, e0);
  for (long long s = e0; s < e1; ti++) {
    const long long te = min(e1, L.off[ti + 1]);
    const float* g = L.g[ti] - L.off[ti];
    for (long long e = s + threadIdx.x; e < te; e += THREADS) {
      const float v = g[e];
      acc += v * v;
    }
    s = te;
  }
  const float tot = block_sum(acc, sm);
  if (threadIdx.x == 0) partial[L.pbase + blockIdx.x] = tot;
}

struct Hyper {
  const float* lr_dev;  // device lr (capturable) or null
  float lr, beta1, beta2, eps, wd, max_norm;
  int nparts;           // partials over the whole flat space
  int clip;             // apply the clip coefficient
};

__global__ __launch_bounds__(THREADS) void adamw_kernel(TList L, const float* __restrict__ partial,
                                                        float* __restrict__ m, float* __restrict__ v, Hyper h,
                                                        float* __restrict__ state, float* __restrict__ norm_out) {
  __shared__ float sm[THREADS / 64 + 1];
  // ||g||^2: every block sums all partials in the same order -> identical coef everywhere
  float t = 0.f;
  for (int i = threadIdx.x; i < h.nparts; i += THREADS) t += partial[i];
  const float sq = block_sum(t, sm);
  const float norm = sqrtf(sq);
  const bool finite = isfinite(norm);
  const float step = state[0] + 1.f;  // (state[0] is only written by sumsq_kernel)
  __syncthreads();
  if (blockIdx.x == 0 && L.pbase == 0 && threadIdx.x == 0) {
    if (norm_out) *norm_out = norm;
    state[1] = finite ? 1.f : 0.f;
  }
  if (!finite) return;  // skip the step (uniform over the grid)
  const float bc1 = 1.f - powf(h.beta1, step);
  const float bc2_sqrt = sqrtf(1.f - powf(h.beta2, step));
  const float coef = h.clip ? fminf(h.max_norm / (norm + 1e-6f), 1.f) : 1.f;
  const float lr = h.lr_dev ? *h.lr_dev : h.lr;
  const float decay = 1.f - lr * h.wd;
  const float step_size = lr / bc1;
  const float ob1 = 1.f - h.beta1, ob2 = 1.f - h.beta2;

  const long long e0 = (long long)blockIdx.x * CH;
  const long long e1 = min(e0 + CH, L.off[L.n]);
  int ti = find_tensor(L, e0);
  for (long long s = e0; s < e1; ti++) {
    const long long te = min(e1, L.off[ti + 1]);
    float* p = L.p[ti] - L.off[ti];
    float* g = L.g[ti] - L.off[ti];
    float* mm = m + (L.moff[ti] - L.off[ti]);
    float* vv = v + (L.moff[ti] - L.off[ti]);
    for (long long e = s + threadIdx.x; e < te; e += THREADS) {
      const float gv = g[e] * coef;
      float pv = p[e] * decay;
      const float mv = h.beta1 * mm[e] + ob1 * gv;
      const float vvv = h.beta2 * vv[e] + ob2 * gv * gv;
      mm[e] = mv;
      vv[e] = vvv;
      const float denom = sqrtf(vvv) / bc2_sqrt + h.eps;
      pv -= step_size * (mv / denom);
      p[e] = pv;
    }
    s = te;
  }
}

}  // namespace optim

// groups: launch-group tables filled by the host op (ops_optim.cpp); total_blocks:
// block partials over all groups (= the length of `partial` that is used)
void clip_adamw_launch(const optim::TList* groups, int ngroups, long long total_blocks, float* partial, float* m,
                       float* v, const float* lr_dev, float lr, float beta1, float beta2, float eps, float wd,
                       float max_norm, bool clip, float* state, float* norm_out, hipStream_t s) {
  for (int gi = 0; gi < ngroups; ++gi) {
    const optim::TList& L = groups[gi];
    const int nb = (int)((L.off[L.n] + optim::CH - 1) / optim::CH);
    hipLaunchKernelGGL(optim::sumsq_kernel, dim3(nb), dim3(optim::THREADS), 0, s, L, partial, state);
  }
  optim::Hyper h{lr_dev, lr, beta1, beta2, eps, wd, max_norm, (int)total_blocks, clip ? 1 : 0};
  for (int gi = 0; gi < ngroups; ++gi) {
    const optim::TList& L = groups[gi];
    const int nb = (int)((L.off[L.n] + optim::CH - 1) / optim::CH);
    hipLaunchKernelGGL(optim::adamw_kernel, dim3(nb), dim3(optim::THREADS), 0, s, L, partial, m, v, h, state,
                       norm_out);
  }
}

}  // namespace rs
