// Channels-last (NHWC) normalisation + activation, fused, for the encoders.
//
// Replaces the stock InstanceNorm2d / BatchNorm2d + ReLU (+ residual add +
// ReLU) chains of reference core/extractor.py:6-116.  PyTorch's instance_norm
// reshapes to (1, B*C, H, W) and needs NCHW-contiguous memory, so on
// channels_last activations it copies the feature map out and back (the
// largest tensors of the encoders: 16 x 64 x 184 x 248 at the Chairs crop);
// here statistics and the normalised output are computed in place in NHWC:
//
//   stats    : per (group, channel) mean / rstd, group = sample (instance
//              norm) or the whole batch (batch norm); two-level reduction
//              (per-block partials -> fp64 finalize), deterministic.
//   apply    : y = act(gamma * (x - mean) * rstd + beta)  [+ residual, ReLU]
//   backward : S1 = sum g, S2 = sum g*xhat  (same two-level reduction), then
//              dx = gamma * rstd * (g - S1/N - xhat * S2/N), d(residual).
//
// x is viewed as (B, P, C) with P = H*W; vectors of 16 bytes along C.
#include "common.h"

namespace rs {
namespace norm {

constexpr int THREADS = 256;

template <typename T> struct Vec;
template <> struct Vec<float> {
  static constexpr int N = 4;
  __device__ static void load(const float* p, float* v) {
    float4 q = *reinterpret_cast<const float4*>(p);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  }
  __device__ static void store(float* p, const float* v) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
};
template <> struct Vec<bf16_t> {
  static constexpr int N = 8;
  __device__ static void load(const bf16_t* p, float* v) {
    uint4 q = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  __device__ static void store(bf16_t* p, const float* v) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = uint32_t(f2bf(v[2 * i])) | (uint32_t(f2bf(v[2 * i + 1])) << 16);
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
};

struct Args {
  const void* x;
  const void* dy;
  const void* res;
  const float* mean;   // (G, C)
  const float* rstd;   // (G, C)
  const float* gamma;  // (C) or null
  const float* beta;   // (C) or null
  const float* s1;     // (G, C) bwd sums
  const float* s2;
  void* y;
  void* dx;
  void* dres;
  float* ws;           // partials (B, S, C, 2)
  int B, P, C, S, G;
  int relu;
  float inv_n;
};

// --------------------------------------------------------------- reductions
// MODE 0: (x, x^2).  MODE 1: (g, g * xhat) with g the gradient reaching the
// pre-activation a = gamma * xhat + beta.
template <typename T, int MODE>
__global__ __launch_bounds__(THREADS) void reduce_kernel(Args a) {
  using V = Vec<T>;
  constexpr int VN = V::N;
  const int CV = a.C / VN;
  const int rows = THREADS / CV;
  const int tid = threadIdx.x;
  const int row = tid / CV, col = tid % CV;
  const int b = blockIdx.y, s = blockIdx.x;
  const int chunk = cdiv(a.P, a.S);
  const int p0 = s * chunk, p1 = min(a.P, p0 + chunk);
  float acc0[VN], acc1[VN];
#pragma unroll
  for (int i = 0; i < VN; ++i) acc0[i] = acc1[i] = 0.f;
  const int g = a.G == 1 ? 0 : b;
  float mu[VN], rs_[VN], ga[VN], be[VN];
  if (MODE == 1 && row < rows) {
#pragma unroll
    for (int i = 0; i < VN; ++i) {
      const int c = col * VN + i;
      mu[i] = a.mean[g * a.C + c];
      rs_[i] = a.rstd[g * a.C + c];
      ga[i] = a.gamma ? a.gamma[c] : 1.f;
      be[i] = a.beta ? a.beta[c] : 0.f;
    }
  }
  if (row < rows) {
    const T* x = static_cast<const T*>(a.x) + (size_t)b * a.P * a.C;
    const T* dy = static_cast<const T*>(a.dy) + (size_t)b * a.P * a.C;
    const T* res = a.res ? static_cast<const T*>(a.res) + (size_t)b * a.P * a.C : nullptr;
    for (int p = p0 + row; p < p1; p += rows) {
      const size_t off = (size_t)p * a.C + col * VN;
      float xv[VN];
      V::load(x + off, xv);
      if (MODE == 0) {
#pragma unroll
        for (int i = 0; i < VN; ++i) {
          acc0[i] += xv[i];
          acc1[i] += xv[i] * xv[i];
        }
      } else {
        float dv[VN], rv[VN];
        V::load(dy + off, dv);
        if (res) V::load(res + off, rv);
#pragma unroll
        for (int i = 0; i < VN; ++i) {
          const float xh = (xv[i] - mu[i]) * rs_[i];
          const float pre = ga[i] * xh + be[i];
          const float y1 = a.relu ? fmaxf(pre, 0.f) : pre;
          float gg = dv[i];
          if (res && rv[i] + y1 <= 0.f) gg = 0.f;
          if (a.relu && pre <= 0.f) gg = 0.f;
          acc0[i] += gg;
          acc1[i] += gg * xh;
        }
      }
    }
  }
  __shared__ float sm[THREADS * 8 * 2];
  const int rr = row < rows ? row : rows;  // idle threads park outside
#pragma unroll
  for (int i = 0; i < VN; ++i) {
    if (row < rows) {
      sm[(rr * a.C + col * VN + i) * 2] = acc0[i];
      sm[(rr * a.C + col * VN + i) * 2 + 1] = acc1[i];
    }
  }
  __syncthreads();
  for (int c = tid; c < a.C; c += THREADS) {
    float t0 = 0.f, t1 = 0.f;
    for (int r = 0; r < rows; ++r) {
      t0 += sm[(r * a.C + c) * 2];
      t1 += sm[(r * a.C + c) * 2 + 1];
    }
    float* w = a.ws + (((size_t)b * a.S + s) * a.C + c) * 2;
    w[0] = t0;
    w[1] = t1;
  }
}

// Combine partials: MODE 0 -> mean/rstd, MODE 1 -> s1/s2.
// Block (g, 32-channel chunk): 8 row-groups of 32 lanes each sum a strided
// share of the (b, s) partials in fp64, then an LDS reduction across groups.
template <int MODE>
__global__ __launch_bounds__(256) void finalize_kernel(const float* ws, int B, int S, int C, int G,
                                                       float eps, float inv_n, float* o0, float* o1) {
  const int g = blockIdx.x;
  const int c = blockIdx.y * 32 + (threadIdx.x & 31);
  const int part = threadIdx.x >> 5;
  const int b0 = G == 1 ? 0 : g, nb = G == 1 ? B : 1;
  double t0 = 0.0, t1 = 0.0;
  if (c < C) {
    for (int i = part; i < nb * S; i += 8) {
      const int b = b0 + i / S, s = i % S;
      const float* w = ws + (((size_t)b * S + s) * C + c) * 2;
      t0 += w[0];
      t1 += w[1];
    }
  }
  __shared__ double sm[2][8][32];
  sm[0][part][threadIdx.x & 31] = t0;
  sm[1][part][threadIdx.x & 31] = t1;
  __syncthreads();
  if (part == 0 && c < C) {
    for (int p = 1; p < 8; ++p) {
      t0 += sm[0][p][threadIdx.x];
      t1 += sm[1][p][threadIdx.x];
    }
    const int idx = g * C + c;
    if (MODE == 0) {
      const double m = t0 * inv_n;
      double var = t1 * inv_n - m * m;
      var = var < 0.0 ? 0.0 : var;
      o0[idx] = (float)m;
      o1[idx] = (float)(1.0 / sqrt(var + (double)eps));
    } else {
      o0[idx] = (float)t0;
      o1[idx] = (float)t1;
    }
  }
}

// --------------------------------------------------------------- elementwise
template <typename T>
__global__ __launch_bounds__(THREADS) void apply_fwd_kernel(Args a) {
  using V = Vec<T>;
  constexpr int VN = V::N;
  const size_t nvec = (size_t)a.B * a.P * a.C / VN;
  const int CV = a.C / VN;
  for (size_t v = blockIdx.x * (size_t)THREADS + threadIdx.x; v < nvec;
       v += (size_t)gridDim.x * THREADS) {
    const int c0 = (int)(v % CV) * VN;
    const int b = (int)(v / ((size_t)a.P * CV));
    const int g = a.G == 1 ? 0 : b;
    float xv[VN], rv[VN], out[VN];
    V::load(static_cast<const T*>(a.x) + v * VN, xv);
    if (a.res) V::load(static_cast<const T*>(a.res) + v * VN, rv);
#pragma unroll
    for (int i = 0; i < VN; ++i) {
      const int c = c0 + i;
      const float xh = (xv[i] - a.mean[g * a.C + c]) * a.rstd[g * a.C + c];
      float y = (a.gamma ? a.gamma[c] : 1.f) * xh + (a.beta ? a.beta[c] : 0.f);
      if (a.relu) y = fmaxf(y, 0.f);
      if (a.res) y = fmaxf(y + rv[i], 0.f);
      out[i] = y;
    }
    V::store(static_cast<T*>(a.y) + v * VN, out);
  }
}

template <typename T>
__global__ __launch_bounds__(THREADS) void apply_bwd_kernel(Args a) {
  using V = Vec<T>;
  constexpr int VN = V::N;
  const size_t nvec = (size_t)a.B * a.P * a.C / VN;
  const int CV = a.C / VN;
  for (size_t v = blockIdx.x * (size_t)THREADS + threadIdx.x; v < nvec;
       v += (size_t)gridDim.x * THREADS) {
    const int c0 = (int)(v % CV) * VN;
    const int b = (int)(v / ((size_t)a.P * CV));
    const int g = a.G == 1 ? 0 : b;
    float xv[VN], dv[VN], rv[VN], dxo[VN], dro[VN];
    V::load(static_cast<const T*>(a.x) + v * VN, xv);
    V::load(static_cast<const T*>(a.dy) + v * VN, dv);
    if (a.res) V::load(static_cast<const T*>(a.res) + v * VN, rv);
#pragma unroll
    for (int i = 0; i < VN; ++i) {
      const int c = c0 + i;
      const float m = a.mean[g * a.C + c], r = a.rstd[g * a.C + c];
      const float ga = a.gamma ? a.gamma[c] : 1.f;
      const float xh = (xv[i] - m) * r;
      const float pre = ga * xh + (a.beta ? a.beta[c] : 0.f);
      const float y1 = a.relu ? fmaxf(pre, 0.f) : pre;
      float gout = dv[i];
      if (a.res && rv[i] + y1 <= 0.f) gout = 0.f;
      dro[i] = gout;
      float gg = gout;
      if (a.relu && pre <= 0.f) gg = 0.f;
      dxo[i] = ga * r * (gg - a.s1[g * a.C + c] * a.inv_n - xh * a.s2[g * a.C + c] * a.inv_n);
    }
    V::store(static_cast<T*>(a.dx) + v * VN, dxo);
    if (a.dres) V::store(static_cast<T*>(a.dres) + v * VN, dro);
  }
}

int pick_splits(int B, int P, int C, int vn) {
  const int rows = THREADS / (C / vn);
  int S = cdiv(512, B);
  S = max(1, min(S, cdiv(P, rows * 8)));
  return S;
}

int grid_elem(size_t nvec) {
  size_t g = (nvec + THREADS - 1) / THREADS;
  return (int)(g < 8192 ? g : 8192);
}

}  // namespace norm

// ------------------------------------------------------------------ launchers
int norm_ws_floats(int B, int P, int C, bool bf16) {
  const int S = norm::pick_splits(B, P, C, bf16 ? 8 : 4);
  return B * S * C * 2;
}

void norm_stats_launch(bool bf16, const void* x, int B, int P, int C, int G, float eps, float* ws,
                       float* mean, float* rstd, hipStream_t s) {
  norm::Args a{};
  a.x = x;
  a.B = B; a.P = P; a.C = C; a.G = G;
  a.S = norm::pick_splits(B, P, C, bf16 ? 8 : 4);
  a.ws = ws;
  dim3 grid(a.S, B);
  if (bf16)
    hipLaunchKernelGGL((norm::reduce_kernel<bf16_t, 0>), grid, dim3(norm::THREADS), 0, s, a);
  else
    hipLaunchKernelGGL((norm::reduce_kernel<float, 0>), grid, dim3(norm::THREADS), 0, s, a);
  const float inv_n = 1.f / (float)((G == 1 ? (double)B : 1.0) * P);
  hipLaunchKernelGGL(norm::finalize_kernel<0>, dim3(G, cdiv(C, 32)), dim3(256), 0, s, ws, B, a.S,
                     C, G, eps, inv_n, mean, rstd);
}

void norm_fwd_launch(bool bf16, const void* x, const void* res, const float* mean,
                     const float* rstd, const float* gamma, const float* beta, int B, int P, int C,
                     int G, bool relu, void* y, hipStream_t s) {
  norm::Args a{};
  a.x = x; a.res = res; a.mean = mean; a.rstd = rstd; a.gamma = gamma; a.beta = beta; a.y = y;
  a.B = B; a.P = P; a.C = C; a.G = G; a.relu = relu;
  const size_t nvec = (size_t)B * P * C / (bf16 ? 8 : 4);
  if (bf16)
    hipLaunchKernelGGL(norm::apply_fwd_kernel<bf16_t>, dim3(norm::grid_elem(nvec)),
                       dim3(norm::THREADS), 0, s, a);
  else
    hipLaunchKernelGGL(norm::apply_fwd_kernel<float>, dim3(norm::grid_elem(nvec)),
                       dim3(norm::THREADS), 0, s, a);
}

void norm_bwd_launch(bool bf16, const void* x, const void* dy, const void* res, const float* mean,
                     const float* rstd, const float* gamma, const float* beta, int B, int P, int C,
                     int G, bool relu, bool batch_stats, float* ws, float* s1, float* s2, void* dx,
                     void* dres, hipStream_t s) {
  norm::Args a{};
  a.x = x; a.dy = dy; a.res = res; a.mean = mean; a.rstd = rstd; a.gamma = gamma; a.beta = beta;
  a.B = B; a.P = P; a.C = C; a.G = G; a.relu = relu; a.ws = ws;
  a.S = norm::pick_splits(B, P, C, bf16 ? 8 : 4);
  dim3 grid(a.S, B);
  if (bf16)
    hipLaunchKernelGGL((norm::reduce_kernel<bf16_t, 1>), grid, dim3(norm::THREADS), 0, s, a);
  else
    hipLaunchKernelGGL((norm::reduce_kernel<float, 1>), grid, dim3(norm::THREADS), 0, s, a);
  hipLaunchKernelGGL(norm::finalize_kernel<1>, dim3(G, cdiv(C, 32)), dim3(256), 0, s, ws, B, a.S,
                     C, G, 0.f, 0.f, s1, s2);
  a.s1 = s1; a.s2 = s2; a.dx = dx; a.dres = dres;
  a.inv_n = batch_stats ? 1.f / (float)((G == 1 ? (double)B : 1.0) * P) : 0.f;
  const size_t nvec = (size_t)B * P * C / (bf16 ? 8 : 4);
  if (bf16)
    hipLaunchKernelGGL(norm::apply_bwd_kernel<bf16_t>, dim3(norm::grid_elem(nvec)),
                       dim3(norm::THREADS), 0, s, a);
  else
    hipLaunchKernelGGL(norm::apply_bwd_kernel<float>, dim3(norm::grid_elem(nvec)),
                       dim3(norm::THREADS), 0, s, a);
}

}  // namespace rs
