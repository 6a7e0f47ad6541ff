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

#include <cstdlib>

namespace rs {
namespace norm {

constexpr int THREADS = 256;

template <typename T> struct Vec;
template <> struct Vec<float> {
  static constexpr int N = 4;
  typedef float4 raw;
  __device__ static raw ldraw(const float* p) { return *reinterpret_cast<const float4*>(p); }
  __device__ static void cvt(const raw& q, float* v) {
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  }
  __device__ static void load(const float* p, float* v) {
    float4 q = *reinterpret_cast<const float4*>(p);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  }
  __device__ static void store(float* p, const float* v) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
  __device__ static float rnd(float v) { return v; }
};
template <> struct Vec<bf16_t> {
  static constexpr int N = 8;
  typedef uint4 raw;
  __device__ static raw ldraw(const bf16_t* p) { return *reinterpret_cast<const uint4*>(p); }
  __device__ static void cvt(const raw& q, float* v) {
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
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
  __device__ static float rnd(float v) { return bf2f(f2bf(v)); }  // the value store() keeps
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
  // second upstream gradient (backward), added to dy on the fly: the skip
  // path's gradient of a residual block's input
  const void* dy2;
  // affine residual: res is a RAW tensor normalised on the fly,
  // r = (res - rmean) * rrstd * rgamma + rbeta (the downsample shortcut's
  // norm, no ReLU); backward: its (sum g, sum g * xhat) partials go to ws2,
  // apply_bwd writes its input gradient (rs1 / rs2 = its finalized sums) to dres
  const float* rmean;
  const float* rrstd;
  const float* rgamma;
  const float* rbeta;
  const float* rs1;
  const float* rs2;
  float* ws2;
  // staged output gradient (plain residual): the reduction stores the
  // residual's gradient gout = mask(dy + dy2) to dres in the tensor dtype and
  // takes its sums over those rounded values; apply_bwd then reads x and dres
  // only (not dy, dy2, res again) and leaves dres alone
  int gstage;
};

// BatchNorm running-statistics update, applied by finalize_kernel<0> for
// batch statistics (reference nn.BatchNorm2d train mode, momentum form):
//   running_mean = (1-m) running_mean + m (mean + bias)
//   running_var  = (1-m) running_var  + m var * n/(n-1),  var = rstd^-2 - eps
struct Running {
  float* rm;            // null: no update
  float* rv;
  long long* nbt;
  const float* bias;
  float mom, unb;
};

// --------------------------------------------------------------- reductions
// MODE 0: (x, x^2).  MODE 1: (g, g * xhat) with g the gradient reaching the
// pre-activation a = gamma * xhat + beta.
// AFF (MODE 1 only): the affine residual's constants and partial set are
// compiled in only where they are used -- as a run-time branch they held ~50
// VGPRs through the loop of every backward reduction and kept it at two waves
// per SIMD.  RU: pixel rows in flight per thread (MODE 0 reads one tensor).
template <typename T, int MODE, bool AFF = false>
__global__ __launch_bounds__(THREADS) void reduce_kernel(Args a) {
  constexpr int RU = MODE == 0 ? 8 : 4;
  using V = Vec<T>;
  constexpr int VN = V::N;
  const int CV = a.C / VN;
  const int rows = THREADS / CV;
  const int tid = threadIdx.x;
  const int row = tid / CV, col = tid % CV;
  const int b = blockIdx.y, s = blockIdx.x;
  const int chunk = cdiv(a.P, a.S);
  const int p0 = s * chunk, p1 = min(a.P, p0 + chunk);
  float acc0[VN], acc1[VN], racc0[VN], racc1[VN];
#pragma unroll
  for (int i = 0; i < VN; ++i) acc0[i] = acc1[i] = racc0[i] = racc1[i] = 0.f;
  const int g = a.G == 1 ? 0 : b;
  constexpr bool aff = MODE == 1 && AFF;  // affine residual (+ its own partials)
  float mu[VN], rs_[VN], ga[VN], be[VN], rmu[VN], rrs[VN], rsc[VN], rsh[VN];
  if (MODE == 1 && row < rows) {
#pragma unroll
    for (int i = 0; i < VN; ++i) {
      const int c = col * VN + i;
      mu[i] = a.mean[g * a.C + c];
      rs_[i] = a.rstd[g * a.C + c];
      ga[i] = a.gamma ? a.gamma[c] : 1.f;
      be[i] = a.beta ? a.beta[c] : 0.f;
      if (aff) {
        rmu[i] = a.rmean[g * a.C + c];
        rrs[i] = a.rrstd[g * a.C + c];
        rsc[i] = (a.rgamma ? a.rgamma[c] : 1.f) * rrs[i];
        rsh[i] = (a.rbeta ? a.rbeta[c] : 0.f) - rmu[i] * rsc[i];
      }
    }
  }
  if (row < rows) {
    const T* x = static_cast<const T*>(a.x) + (size_t)b * a.P * a.C;
    const T* dy = static_cast<const T*>(a.dy) + (size_t)b * a.P * a.C;
    const T* dy2 = a.dy2 ? static_cast<const T*>(a.dy2) + (size_t)b * a.P * a.C : nullptr;
    const T* res = a.res ? static_cast<const T*>(a.res) + (size_t)b * a.P * a.C : nullptr;
    T* gst = MODE == 1 && a.gstage ? static_cast<T*>(a.dres) + (size_t)b * a.P * a.C : nullptr;
    for (int p = p0 + row; p < p1; p += rows * RU) {
      typename V::raw xq[RU], dq[RU], rq[RU], eq[RU];
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const int pp = p + u * rows;
        if (pp < p1) {
          const size_t off = (size_t)pp * a.C + col * VN;
          xq[u] = V::ldraw(x + off);
          if (MODE == 1) {
            dq[u] = V::ldraw(dy + off);
            if (dy2) eq[u] = V::ldraw(dy2 + off);
            if (res) rq[u] = V::ldraw(res + off);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        if (p + u * rows >= p1) break;
        float xv[VN];
        V::cvt(xq[u], xv);
        if (MODE == 0) {
#pragma unroll
          for (int i = 0; i < VN; ++i) {
            acc0[i] += xv[i];
            acc1[i] += xv[i] * xv[i];
          }
        } else {
          float dv[VN], rv[VN], ev[VN];
          V::cvt(dq[u], dv);
          if (dy2) {
            V::cvt(eq[u], ev);
#pragma unroll
            for (int i = 0; i < VN; ++i) dv[i] += ev[i];
          }
          if (res) V::cvt(rq[u], rv);
#pragma unroll
          for (int i = 0; i < VN; ++i) {
            const float xh = (xv[i] - mu[i]) * rs_[i];
            const float pre = ga[i] * xh + be[i];
            const float y1 = a.relu ? fmaxf(pre, 0.f) : pre;
            float gg = dv[i];
            if (res && (aff ? rv[i] * rsc[i] + rsh[i] : rv[i]) + y1 <= 0.f) gg = 0.f;
            if (gst) gg = dv[i] = V::rnd(gg);  // dv: the staged values
            if (aff) {  // the residual branch's gradient, before the main branch's ReLU mask
              racc0[i] += gg;
              racc1[i] += gg * ((rv[i] - rmu[i]) * rrs[i]);
            }
            if (a.relu && pre <= 0.f) gg = 0.f;
            acc0[i] += gg;
            acc1[i] += gg * xh;
          }
          if (gst) V::store(gst + (size_t)(p + u * rows) * a.C + col * VN, dv);
        }
      }
    }
  }
  __shared__ float sm[THREADS * 8 * 2];
  const int rr = row < rows ? row : rows;  // idle threads park outside
  for (int set = 0; set < (aff ? 2 : 1); ++set) {
    if (set) __syncthreads();  // the first set's combine is done with sm
#pragma unroll
    for (int i = 0; i < VN; ++i) {
      if (row < rows) {
        sm[(rr * a.C + col * VN + i) * 2] = set ? racc0[i] : acc0[i];
        sm[(rr * a.C + col * VN + i) * 2 + 1] = set ? racc1[i] : acc1[i];
      }
    }
    __syncthreads();
    for (int c = tid; c < a.C; c += THREADS) {
      float t0 = 0.f, t1 = 0.f;
      for (int r = 0; r < rows; ++r) {
        t0 += sm[(r * a.C + c) * 2];
        t1 += sm[(r * a.C + c) * 2 + 1];
      }
      float* w = (set ? a.ws2 : a.ws) + (((size_t)b * a.S + s) * a.C + c) * 2;
      w[0] = t0;
      w[1] = t1;
    }
  }
}

// Combine partials: MODE 0 -> mean/rstd, MODE 1 -> s1/s2.
// Block (g, 8-channel chunk): 32 row-groups of 8 lanes each sum a strided
// share of the (b, s) partials in fp64, then an LDS tree across the groups
// (short serial chains: batch-norm groups have B * S partials per channel).
template <int MODE>
__global__ __launch_bounds__(256) void finalize_kernel(const float* ws, int B, int S, int C, int G,
                                                       float eps, float inv_n, float* o0, float* o1, Running run,
                                                       const float* ws2 = nullptr, float* o2 = nullptr,
                                                       float* o3 = nullptr) {
  if (blockIdx.z) {  // the second partial set (MODE 1 with an affine residual)
    ws = ws2;
    o0 = o2;
    o1 = o3;
  }
  const int g = blockIdx.x;
  const int c = blockIdx.y * 8 + (threadIdx.x & 7);
  const int part = threadIdx.x >> 3;
  const int b0 = G == 1 ? 0 : g, nb = G == 1 ? B : 1;
  double t0 = 0.0, t1 = 0.0;
  if (c < C) {
    // 4 independent partial loads in flight per thread: the chain of one
    // dependent load per partial made this kernel latency-bound (8 us per
    // batch-norm call at 512 partials); the summation order is unchanged
    // within each thread's strided share, so the result stays deterministic
    const int n = nb * S;
    for (int i = part; i < n; i += 32 * 4) {
      float2 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = i + 32 * u;
        v[u] = make_float2(0.f, 0.f);
        if (k < n) {
          const int b = b0 + k / S, s = k % S;
          v[u] = *reinterpret_cast<const float2*>(ws + (((size_t)b * S + s) * C + c) * 2);
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        t0 += v[u].x;
        t1 += v[u].y;
      }
    }
  }
  __shared__ double sm[2][256];
  sm[0][threadIdx.x] = t0;
  sm[1][threadIdx.x] = t1;
  __syncthreads();
  for (int st = 128; st >= 8; st >>= 1) {
    if (threadIdx.x < st) {
      sm[0][threadIdx.x] += sm[0][threadIdx.x + st];
      sm[1][threadIdx.x] += sm[1][threadIdx.x + st];
    }
    __syncthreads();
  }
  if (threadIdx.x < 8 && c < C) {
    t0 = sm[0][threadIdx.x];
    t1 = sm[1][threadIdx.x];
    const int idx = g * C + c;
    if (MODE == 0) {
      const double m = t0 * inv_n;
      double var = t1 * inv_n - m * m;
      var = var < 0.0 ? 0.0 : var;
      const float r = (float)(1.0 / sqrt(var + (double)eps));
      o0[idx] = (float)m;
      o1[idx] = r;
      if (run.rm != nullptr) {  // G == 1 (checked by the host)
        const float vf = fmaxf(1.f / (r * r) - eps, 0.f);
        const float bm = (float)m + (run.bias ? run.bias[c] : 0.f);
        run.rm[c] = (1.f - run.mom) * run.rm[c] + run.mom * bm;
        run.rv[c] = (1.f - run.mom) * run.rv[c] + run.mom * vf * run.unb;
        if (c == 0 && run.nbt != nullptr) run.nbt[0] += 1;
      }
    } else {
      o0[idx] = (float)t0;
      o1[idx] = (float)t1;
    }
  }
}

// --------------------------------------------------------------- elementwise
// Grid (S, B): block (s, b) streams pixels [p0, p1) of sample b.  Thread t
// owns channel vector t % CV for its whole life, so its per-channel constants
// are folded once into registers (scale = gamma*rstd, shift = beta -
// mean*scale, ...) instead of being re-gathered per element; the pixel loop
// is unrolled UNR deep so that many 16-B loads are in flight per thread.
constexpr int UNR = 4;

// AFF / K: compile-time variants, as for reduce_kernel (registers): apply_bwd
// K = 0 plain (dy2 / res at run time), 1 affine residual, 2 staged gradient,
// 3 neither dy2 nor res (x and dy only)
template <typename T, bool AFF>
__global__ __launch_bounds__(THREADS) void apply_fwd_kernel(Args a) {
  using V = Vec<T>;
  constexpr int VN = V::N;
  const int CV = a.C / VN;
  const int rows = THREADS / CV;
  const int row = threadIdx.x / CV, col = threadIdx.x % CV;
  if (row >= rows) return;
  const int b = blockIdx.y, g = a.G == 1 ? 0 : b;
  const int chunk = cdiv(a.P, a.S);
  const int p0 = blockIdx.x * chunk, p1 = min(a.P, p0 + chunk);
  float sc[VN], sh[VN], rsc[VN], rsh[VN];
  constexpr bool aff = AFF;
#pragma unroll
  for (int i = 0; i < VN; ++i) {
    const int c = col * VN + i;
    const float r = a.rstd[g * a.C + c];
    sc[i] = (a.gamma ? a.gamma[c] : 1.f) * r;
    sh[i] = (a.beta ? a.beta[c] : 0.f) - a.mean[g * a.C + c] * sc[i];
    rsc[i] = 1.f;
    rsh[i] = 0.f;
    if (aff) {
      rsc[i] = (a.rgamma ? a.rgamma[c] : 1.f) * a.rrstd[g * a.C + c];
      rsh[i] = (a.rbeta ? a.rbeta[c] : 0.f) - a.rmean[g * a.C + c] * rsc[i];
    }
  }
  const size_t base = (size_t)b * a.P * a.C + col * VN;
  const T* x = static_cast<const T*>(a.x) + base;
  const T* res = a.res ? static_cast<const T*>(a.res) + base : nullptr;
  T* y = static_cast<T*>(a.y) + base;
  const bool relu = a.relu;
  for (int p = p0 + row; p < p1; p += rows * UNR) {
    typename V::raw xq[UNR], rq[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int pp = p + u * rows;
      if (pp < p1) {
        xq[u] = V::ldraw(x + (size_t)pp * a.C);
        if (res) rq[u] = V::ldraw(res + (size_t)pp * a.C);
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int pp = p + u * rows;
      if (pp >= p1) break;
      float out[VN], xv[1][VN], rv[1][VN];
      V::cvt(xq[u], xv[0]);
      if (res) V::cvt(rq[u], rv[0]);
#pragma unroll
      for (int i = 0; i < VN; ++i) {
        float v = xv[0][i] * sc[i] + sh[i];
        if (relu) v = fmaxf(v, 0.f);
        if (res) v = fmaxf(v + rv[0][i] * rsc[i] + rsh[i], 0.f);
        out[i] = v;
      }
      V::store(y + (size_t)pp * a.C, out);
    }
  }
}

template <typename T, int K>
__global__ __launch_bounds__(THREADS) void apply_bwd_kernel(Args a) {
  using V = Vec<T>;
  constexpr int VN = V::N;
  const int CV = a.C / VN;
  const int rows = THREADS / CV;
  const int row = threadIdx.x / CV, col = threadIdx.x % CV;
  if (row >= rows) return;
  const int b = blockIdx.y, g = a.G == 1 ? 0 : b;
  const int chunk = cdiv(a.P, a.S);
  const int p0 = blockIdx.x * chunk, p1 = min(a.P, p0 + chunk);
  // pre = x*sc + sh ; dx = k1*gg - k1*m1 - (x - mean)*k2  with
  // k1 = gamma*rstd, m1 = s1/N, k2 = gamma*rstd^2*s2/N
  float sc[VN], sh[VN], k0[VN], k2[VN], mu[VN];
  float rsc[VN], rsh[VN], rk0[VN], rk2[VN], rmu[VN];
  constexpr bool aff = K == 1;
#pragma unroll
  for (int i = 0; i < VN; ++i) {
    const int c = col * VN + i;
    const float r = a.rstd[g * a.C + c];
    const float ga = a.gamma ? a.gamma[c] : 1.f;
    mu[i] = a.mean[g * a.C + c];
    sc[i] = ga * r;
    sh[i] = (a.beta ? a.beta[c] : 0.f) - mu[i] * sc[i];
    k0[i] = sc[i] * a.s1[g * a.C + c] * a.inv_n;
    k2[i] = sc[i] * r * a.s2[g * a.C + c] * a.inv_n;
    rsc[i] = 1.f;
    rsh[i] = rk0[i] = rk2[i] = rmu[i] = 0.f;
    if (aff) {  // the residual's own normalisation (forward constants, backward sums)
      const float rr = a.rrstd[g * a.C + c];
      rmu[i] = a.rmean[g * a.C + c];
      rsc[i] = (a.rgamma ? a.rgamma[c] : 1.f) * rr;
      rsh[i] = (a.rbeta ? a.rbeta[c] : 0.f) - rmu[i] * rsc[i];
      rk0[i] = rsc[i] * a.rs1[g * a.C + c] * a.inv_n;
      rk2[i] = rsc[i] * rr * a.rs2[g * a.C + c] * a.inv_n;
    }
  }
  const size_t base = (size_t)b * a.P * a.C + col * VN;
  const T* x = static_cast<const T*>(a.x) + base;
  // staged: dy := the masked residual gradient the reduction left in dres
  constexpr bool st = K == 2;
  const T* dy = static_cast<const T*>(st ? a.dres : a.dy) + base;
  const T* dy2 = K != 3 && a.dy2 && !st ? static_cast<const T*>(a.dy2) + base : nullptr;
  const T* res = K != 3 && a.res && !st ? static_cast<const T*>(a.res) + base : nullptr;
  T* dx = static_cast<T*>(a.dx) + base;
  T* dres = a.dres && !st ? static_cast<T*>(a.dres) + base : nullptr;
  const bool relu = a.relu;
  for (int p = p0 + row; p < p1; p += rows * UNR) {
    typename V::raw xq[UNR], dq[UNR], rq[UNR], eq[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int pp = p + u * rows;
      if (pp < p1) {
        xq[u] = V::ldraw(x + (size_t)pp * a.C);
        dq[u] = V::ldraw(dy + (size_t)pp * a.C);
        if (dy2) eq[u] = V::ldraw(dy2 + (size_t)pp * a.C);
        if (res) rq[u] = V::ldraw(res + (size_t)pp * a.C);
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int pp = p + u * rows;
      if (pp >= p1) break;
      float dxo[VN], dro[VN], xv[VN], dv[VN], rv[VN], ev[VN];
      V::cvt(xq[u], xv);
      V::cvt(dq[u], dv);
      if (dy2) {
        V::cvt(eq[u], ev);
#pragma unroll
        for (int i = 0; i < VN; ++i) dv[i] += ev[i];
      }
      if (res) V::cvt(rq[u], rv);
#pragma unroll
      for (int i = 0; i < VN; ++i) {
        const float pre = xv[i] * sc[i] + sh[i];
        const float y1 = relu ? fmaxf(pre, 0.f) : pre;
        float gout = dv[i];
        if (res && rv[i] * rsc[i] + rsh[i] + y1 <= 0.f) gout = 0.f;
        // residual input gradient: the skip gradient itself, or through the
        // residual's normalisation (affine residual)
        dro[i] = aff ? rsc[i] * gout - rk0[i] - (rv[i] - rmu[i]) * rk2[i] : gout;
        const float gg = (relu && pre <= 0.f) ? 0.f : gout;
        dxo[i] = sc[i] * gg - k0[i] - (xv[i] - mu[i]) * k2[i];
      }
      V::store(dx + (size_t)pp * a.C, dxo);
      if (dres) V::store(dres + (size_t)pp * a.C, dro);
    }
  }
}

// blocks per sample for the elementwise passes: ~2048 blocks in total, at
// least UNR*2 pixel rows per thread
int pick_apply_splits(int B, int P, int C, int vn) {
  const int rows = THREADS / (C / vn);
  int S = cdiv(2048, B);
  return max(1, min(S, cdiv(P, rows * UNR * 2)));
}

// total reduction blocks (larger grids measured slower in situ, round 4);
// norm_set_reduce_blocks: in-situ A/B of the target (RS_NORM_REDUCE_BLOCKS)
int g_reduce_target = 512;

// block target of the statistics pass (MODE 0), RS_NORM_STATS_BLOCKS to
// compare: 512 / 1024 / 2048 measured the same alone (18.6 / 18.5 / 19.8 us
// at 16 x 184 x 248 x 64 with RU = 8), 2048 slightly slower in situ
// (profiles/r6/ab_norm_reduce_aff_s43.txt)
int stats_target() {
  static const int t = [] {
    const char* e = getenv("RS_NORM_STATS_BLOCKS");
    return e && atoi(e) > 0 ? atoi(e) : 512;
  }();
  return t;
}

int pick_splits(int B, int P, int C, int vn, bool stats = false) {
  const int target = stats ? stats_target() : g_reduce_target;
  const int rows = THREADS / (C / vn);
  int S = cdiv(target, B);
  S = max(1, min(S, cdiv(P, rows * 8)));
  return S;
}

int grid_elem(size_t nvec) {
  size_t g = (nvec + THREADS - 1) / THREADS;
  return (int)(g < 8192 ? g : 8192);
}

}  // namespace norm

void norm_set_reduce_blocks(int n) { norm::g_reduce_target = n > 0 ? n : 512; }

// ------------------------------------------------------------------ launchers
int norm_ws_floats(int B, int P, int C, bool bf16, bool stats) {
  const int S = norm::pick_splits(B, P, C, bf16 ? 8 : 4, stats);
  return B * S * C * 2;
}

// rm / rv / nbt / rbias: the BatchNorm running update (G == 1; rm null: none)
void norm_stats_launch(bool bf16, const void* x, int B, int P, int C, int G, float eps, float* ws,
                       float* mean, float* rstd, float* rm, float* rv, long long* nbt, const float* rbias,
                       float mom, float unb, hipStream_t s) {
  norm::Args a{};
  a.x = x;
  a.B = B; a.P = P; a.C = C; a.G = G;
  a.S = norm::pick_splits(B, P, C, bf16 ? 8 : 4, true);
  a.ws = ws;
  dim3 grid(a.S, B);
  if (bf16)
    hipLaunchKernelGGL((norm::reduce_kernel<bf16_t, 0>), grid, dim3(norm::THREADS), 0, s, a);
  else
    hipLaunchKernelGGL((norm::reduce_kernel<float, 0>), grid, dim3(norm::THREADS), 0, s, a);
  const float inv_n = 1.f / (float)((G == 1 ? (double)B : 1.0) * P);
  const norm::Running run{rm, rv, nbt, rbias, mom, unb};
  hipLaunchKernelGGL(norm::finalize_kernel<0>, dim3(G, cdiv(C, 8)), dim3(256), 0, s, ws, B, a.S,
                     C, G, eps, inv_n, mean, rstd, run);
}

// rnorm (4 pointers or null): the residual is raw and normalised with
// (mean, rstd, gamma, beta) = rnorm[0..3] (affine residual, no ReLU)
void norm_fwd_launch(bool bf16, const void* x, const void* res, const float* mean,
                     const float* rstd, const float* gamma, const float* beta, int B, int P, int C,
                     int G, bool relu, void* y, const float* const* rnorm, hipStream_t s) {
  norm::Args a{};
  a.x = x; a.res = res; a.mean = mean; a.rstd = rstd; a.gamma = gamma; a.beta = beta; a.y = y;
  if (rnorm) { a.rmean = rnorm[0]; a.rrstd = rnorm[1]; a.rgamma = rnorm[2]; a.rbeta = rnorm[3]; }
  a.B = B; a.P = P; a.C = C; a.G = G; a.relu = relu;
  a.S = norm::pick_apply_splits(B, P, C, bf16 ? 8 : 4);
  const dim3 grid(a.S, B);
  if (bf16) {
    if (rnorm)
      hipLaunchKernelGGL((norm::apply_fwd_kernel<bf16_t, true>), grid, dim3(norm::THREADS), 0, s, a);
    else
      hipLaunchKernelGGL((norm::apply_fwd_kernel<bf16_t, false>), grid, dim3(norm::THREADS), 0, s, a);
  } else {
    if (rnorm)
      hipLaunchKernelGGL((norm::apply_fwd_kernel<float, true>), grid, dim3(norm::THREADS), 0, s, a);
    else
      hipLaunchKernelGGL((norm::apply_fwd_kernel<float, false>), grid, dim3(norm::THREADS), 0, s, a);
  }
}

// dy2: second upstream gradient (added on the fly) or null.  rnorm: as in
// norm_fwd_launch; then ws2 (same size as ws) and rs1 / rs2 receive the
// residual normalisation's sums and dres its input gradient.
void norm_bwd_launch(bool bf16, const void* x, const void* dy, const void* res, const float* mean,
                     const float* rstd, const float* gamma, const float* beta, int B, int P, int C,
                     int G, bool relu, bool batch_stats, float* ws, float* s1, float* s2, void* dx,
                     void* dres, const void* dy2, const float* const* rnorm, float* ws2, float* rs1,
                     float* rs2, hipStream_t s) {
  norm::Args a{};
  a.x = x; a.dy = dy; a.res = res; a.mean = mean; a.rstd = rstd; a.gamma = gamma; a.beta = beta;
  a.B = B; a.P = P; a.C = C; a.G = G; a.relu = relu; a.ws = ws; a.dy2 = dy2;
  if (rnorm) {
    a.rmean = rnorm[0]; a.rrstd = rnorm[1]; a.rgamma = rnorm[2]; a.rbeta = rnorm[3];
    a.ws2 = ws2;
  }
  // plain residual: stage the residual gradient in dres during the reduction
  // (RS_NORM_GSTAGE=0: recompute it in apply_bwd from dy, dy2 and res)
  static const bool gstage_on = [] {
    const char* e = getenv("RS_NORM_GSTAGE");
    return !(e && e[0] == '0');
  }();
  a.gstage = gstage_on && res != nullptr && rnorm == nullptr && dres != nullptr;
  if (a.gstage) a.dres = dres;
  a.S = norm::pick_splits(B, P, C, bf16 ? 8 : 4);
  dim3 grid(a.S, B);
  if (bf16) {
    if (rnorm)
      hipLaunchKernelGGL((norm::reduce_kernel<bf16_t, 1, true>), grid, dim3(norm::THREADS), 0, s, a);
    else
      hipLaunchKernelGGL((norm::reduce_kernel<bf16_t, 1>), grid, dim3(norm::THREADS), 0, s, a);
  } else {
    if (rnorm)
      hipLaunchKernelGGL((norm::reduce_kernel<float, 1, true>), grid, dim3(norm::THREADS), 0, s, a);
    else
      hipLaunchKernelGGL((norm::reduce_kernel<float, 1>), grid, dim3(norm::THREADS), 0, s, a);
  }
  hipLaunchKernelGGL(norm::finalize_kernel<1>, dim3(G, cdiv(C, 8), rnorm ? 2 : 1), dim3(256), 0, s, ws, B, a.S,
                     C, G, 0.f, 0.f, s1, s2, norm::Running{}, ws2, rs1, rs2);
  a.s1 = s1; a.s2 = s2; a.dx = dx; a.dres = dres; a.rs1 = rs1; a.rs2 = rs2;
  a.inv_n = batch_stats ? 1.f / (float)((G == 1 ? (double)B : 1.0) * P) : 0.f;
  a.S = norm::pick_apply_splits(B, P, C, bf16 ? 8 : 4);
  const dim3 agrid(a.S, B);
  const int kind = rnorm ? 1 : (a.gstage ? 2 : (!res && !dy2 ? 3 : 0));
#define RS_NORM_APPLY_BWD(TT)                                                                        \
  do {                                                                                               \
    if (kind == 1)                                                                                   \
      hipLaunchKernelGGL((norm::apply_bwd_kernel<TT, 1>), agrid, dim3(norm::THREADS), 0, s, a);     \
    else if (kind == 2)                                                                              \
      hipLaunchKernelGGL((norm::apply_bwd_kernel<TT, 2>), agrid, dim3(norm::THREADS), 0, s, a);     \
    else if (kind == 3)                                                                              \
      hipLaunchKernelGGL((norm::apply_bwd_kernel<TT, 3>), agrid, dim3(norm::THREADS), 0, s, a);     \
    else                                                                                             \
      hipLaunchKernelGGL((norm::apply_bwd_kernel<TT, 0>), agrid, dim3(norm::THREADS), 0, s, a);     \
  } while (0)
  if (bf16)
    RS_NORM_APPLY_BWD(bf16_t);
  else
    RS_NORM_APPLY_BWD(float);
#undef RS_NORM_APPLY_BWD
}

}  // namespace rs
