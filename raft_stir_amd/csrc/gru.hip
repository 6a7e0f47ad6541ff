// Fused ConvGRU gate kernels (forward + backward), channels-last.
//
// Reference core/update.py:16-60 computes, per GRU pass,
//   hx = cat[h, x]; z = sigmoid(convz(hx)); r = sigmoid(convr(hx));
//   q = tanh(convq(cat[r*h, x])); h' = (1-z)*h + z*q
// as ~10 separate elementwise/cat kernels around 3 convolutions.  The engine
// runs z and r as ONE convolution with concatenated weights (2*hdim output
// channels) and fuses everything else into these kernels:
//   gate_zr : zr_pre, h, x -> z, r (saved), rhx = [r*h | x]  (q-conv input)
//   gate_q  : q_pre, z, h  -> h', q~ = tanh(q_pre) (saved)
// Backward (hand-written, see ops/gru.py for the chain):
//   bwd_q   : dh', z, h, q~ -> dq_pre, dz_pre (into dzr[:, :hd]), dh_direct
//   bwd_r   : drhx (q-conv dgrad), h, r -> dr_pre (into dzr[:, hd:])
//   bwd_fin : dh_direct, drhx, r, dhx (zr-conv dgrad) -> dh, dx
// All tensors are NHWC rows of P = B*H*W pixels; math in fp32, storage T.

#include "common.h"

namespace rs {
namespace gru {

template <typename T>
__global__ __launch_bounds__(256) void gate_zr_kernel(const T* __restrict__ zr,
                                                      const T* __restrict__ h,
                                                      const T* __restrict__ x, long P, int hd,
                                                      int cin, T* __restrict__ z,
                                                      T* __restrict__ r, T* __restrict__ rhx) {
  const int ct = hd + cin;
  const long total = P * ct;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long p = i / ct;
    const int c = (int)(i - p * ct);
    if (c < hd) {
      const float zv = sigmoidf_(io<T>::ld(zr + p * 2 * hd + c));
      const float rv = sigmoidf_(io<T>::ld(zr + p * 2 * hd + hd + c));
      const float hv = io<T>::ld(h + p * hd + c);
      io<T>::st(z + p * hd + c, zv);
      io<T>::st(r + p * hd + c, rv);
      io<T>::st(rhx + i, rv * hv);
    } else {
      rhx[i] = x[p * cin + (c - hd)];
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void gate_q_kernel(const T* __restrict__ q,
                                                     const T* __restrict__ z,
                                                     const T* __restrict__ h, long total,
                                                     T* __restrict__ hn, T* __restrict__ qt) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const float qv = tanhf_(io<T>::ld(q + i));
    const float zv = io<T>::ld(z + i), hv = io<T>::ld(h + i);
    io<T>::st(qt + i, qv);
    io<T>::st(hn + i, (1.f - zv) * hv + zv * qv);
  }
}

template <typename T, typename GT>
__global__ __launch_bounds__(256) void bwd_q_kernel(const GT* __restrict__ dhn,
                                                    const T* __restrict__ z,
                                                    const T* __restrict__ h,
                                                    const T* __restrict__ qt, long P, int hd,
                                                    T* __restrict__ dq, T* __restrict__ dzr,
                                                    float* __restrict__ dh) {
  const long total = P * hd;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long p = i / hd;
    const int c = (int)(i - p * hd);
    const float g = io<GT>::ld(dhn + i);
    const float zv = io<T>::ld(z + i), hv = io<T>::ld(h + i), qv = io<T>::ld(qt + i);
    io<T>::st(dq + i, g * zv * (1.f - qv * qv));
    io<T>::st(dzr + p * 2 * hd + c, g * (qv - hv) * zv * (1.f - zv));
    dh[i] = g * (1.f - zv);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void bwd_r_kernel(const T* __restrict__ drhx,
                                                    const T* __restrict__ h,
                                                    const T* __restrict__ r, long P, int hd,
                                                    int cin, T* __restrict__ dzr) {
  const long total = P * hd;
  const int ct = hd + cin;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long p = i / hd;
    const int c = (int)(i - p * hd);
    const float g = io<T>::ld(drhx + p * ct + c);
    const float rv = io<T>::ld(r + i), hv = io<T>::ld(h + i);
    io<T>::st(dzr + p * 2 * hd + hd + c, g * hv * rv * (1.f - rv));
  }
}

template <typename T>
__global__ __launch_bounds__(256) void bwd_fin_kernel(const float* __restrict__ dhd,
                                                      const T* __restrict__ drhx,
                                                      const T* __restrict__ r,
                                                      const T* __restrict__ dhx, long P, int hd,
                                                      int cin, T* __restrict__ dh,
                                                      T* __restrict__ dx) {
  const int ct = hd + cin;
  const long total = P * ct;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long p = i / ct;
    const int c = (int)(i - p * ct);
    if (c < hd) {
      const long o = p * hd + c;
      const float v = dhd[o] + io<T>::ld(drhx + i) * io<T>::ld(r + o) + io<T>::ld(dhx + i);
      io<T>::st(dh + o, v);
    } else {
      io<T>::st(dx + p * cin + (c - hd), io<T>::ld(drhx + i) + io<T>::ld(dhx + i));
    }
  }
}

// Context features of the update block (reference core/raft.py:108-110):
// net, inp = split(cnet); net = tanh(net); inp = relu(inp), written straight
// into the fused engine's hidden-state slot and context buffer (row pitches
// hxp / ip), and the adjoint from the engine's fp32 gradient rows G (pitch gp):
//   dcnet = [G_h * (1 - tanh^2) | G_inp * (inp > 0)]
// -- one pass each way instead of split / tanh / relu / copies forward and
// casts / tanh / relu backward / cat backward.
template <typename T>
__global__ __launch_bounds__(256) void ctx_act_kernel(const T* __restrict__ cn, long P, int hd, int cd,
                                                      T* __restrict__ hx, int hxp, T* __restrict__ inp, int ip) {
  const int ct = hd + cd;
  const long total = P * ct;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long p = i / ct;
    const int c = (int)(i - p * ct);
    const float v = io<T>::ld(cn + i);
    if (c < hd)
      io<T>::st(hx + p * hxp + c, tanhf_(v));
    else
      io<T>::st(inp + p * ip + (c - hd), fmaxf(v, 0.f));
  }
}

template <typename T>
__global__ __launch_bounds__(256) void ctx_act_bwd_kernel(const float* __restrict__ G, int gp,
                                                          const T* __restrict__ hx, int hxp,
                                                          const T* __restrict__ inp, int ip, long P, int hd,
                                                          int cd, T* __restrict__ dcn) {
  const int ct = hd + cd;
  const long total = P * ct;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long p = i / ct;
    const int c = (int)(i - p * ct);
    const float g = G[p * gp + c];
    float d;
    if (c < hd) {
      const float t = io<T>::ld(hx + p * hxp + c);
      d = g * (1.f - t * t);
    } else {
      d = io<T>::ld(inp + p * ip + (c - hd)) > 0.f ? g : 0.f;
    }
    io<T>::st(dcn + i, d);
  }
}

inline unsigned grid_for(long total) {
  long g = (total + 255) / 256;
  if (g > 65535L * 4) g = 65535L * 4;
  return (unsigned)(g < 1 ? 1 : g);
}

}  // namespace gru

#define RS_GRU_T(BF, ...)                 \
  if (BF) {                               \
    using T = bf16_t;                     \
    __VA_ARGS__;                          \
  } else {                                \
    using T = float;                      \
    __VA_ARGS__;                          \
  }

void gru_gate_zr_launch(bool bf, const void* zr, const void* h, const void* x, long P, int hd,
                        int cin, void* z, void* r, void* rhx, hipStream_t s) {
  const long total = P * (hd + cin);
  RS_GRU_T(bf, hipLaunchKernelGGL(gru::gate_zr_kernel<T>, dim3(gru::grid_for(total)), dim3(256), 0,
                                  s, (const T*)zr, (const T*)h, (const T*)x, P, hd, cin, (T*)z,
                                  (T*)r, (T*)rhx));
}

void gru_gate_q_launch(bool bf, const void* q, const void* z, const void* h, long P, int hd,
                       void* hn, void* qt, hipStream_t s) {
  const long total = P * hd;
  RS_GRU_T(bf, hipLaunchKernelGGL(gru::gate_q_kernel<T>, dim3(gru::grid_for(total)), dim3(256), 0,
                                  s, (const T*)q, (const T*)z, (const T*)h, total, (T*)hn,
                                  (T*)qt));
}

void gru_bwd_q_launch(bool bf, const void* dhn, bool dhn_bf, const void* z, const void* h,
                      const void* qt, long P, int hd, void* dq, void* dzr, float* dh,
                      hipStream_t s) {
  const long total = P * hd;
  if (dhn_bf) {
    RS_GRU_T(bf, hipLaunchKernelGGL((gru::bwd_q_kernel<T, bf16_t>), dim3(gru::grid_for(total)),
                                    dim3(256), 0, s, (const bf16_t*)dhn, (const T*)z,
                                    (const T*)h, (const T*)qt, P, hd, (T*)dq, (T*)dzr, dh));
  } else {
    RS_GRU_T(bf, hipLaunchKernelGGL((gru::bwd_q_kernel<T, float>), dim3(gru::grid_for(total)),
                                    dim3(256), 0, s, (const float*)dhn, (const T*)z, (const T*)h,
                                    (const T*)qt, P, hd, (T*)dq, (T*)dzr, dh));
  }
}

void gru_bwd_r_launch(bool bf, const void* drhx, const void* h, const void* r, long P, int hd,
                      int cin, void* dzr, hipStream_t s) {
  const long total = P * hd;
  RS_GRU_T(bf, hipLaunchKernelGGL(gru::bwd_r_kernel<T>, dim3(gru::grid_for(total)), dim3(256), 0,
                                  s, (const T*)drhx, (const T*)h, (const T*)r, P, hd, cin,
                                  (T*)dzr));
}

void gru_bwd_fin_launch(bool bf, const float* dhd, const void* drhx, const void* r,
                        const void* dhx, long P, int hd, int cin, void* dh, void* dx,
                        hipStream_t s) {
  const long total = P * (hd + cin);
  RS_GRU_T(bf, hipLaunchKernelGGL(gru::bwd_fin_kernel<T>, dim3(gru::grid_for(total)), dim3(256),
                                  0, s, dhd, (const T*)drhx, (const T*)r, (const T*)dhx, P, hd,
                                  cin, (T*)dh, (T*)dx));
}

void ctx_act_launch(bool bf, const void* cn, long P, int hd, int cd, void* hx, int hxp, void* inp, int ip,
                    hipStream_t s) {
  const long total = P * (hd + cd);
  RS_GRU_T(bf, hipLaunchKernelGGL(gru::ctx_act_kernel<T>, dim3(gru::grid_for(total)), dim3(256), 0, s,
                                  (const T*)cn, P, hd, cd, (T*)hx, hxp, (T*)inp, ip));
}

void ctx_act_bwd_launch(bool bf, const float* G, int gp, const void* hx, int hxp, const void* inp, int ip, long P,
                        int hd, int cd, void* dcn, hipStream_t s) {
  const long total = P * (hd + cd);
  RS_GRU_T(bf, hipLaunchKernelGGL(gru::ctx_act_bwd_kernel<T>, dim3(gru::grid_for(total)), dim3(256), 0, s, G,
                                  gp, (const T*)hx, hxp, (const T*)inp, ip, P, hd, cd, (T*)dcn));
}

}  // namespace rs
