// Shared pieces of the implicit-GEMM convolution kernels (conv.hip, conv_v2.hip):
// epilogue kinds, the launch-argument block, the fused epilogues and the
// staging helpers (buffer / global LDS-DMA, counted vmcnt waits, XCD remap).
#pragma once
#include "common.h"

#include <stdlib.h>

namespace rs {
namespace conv {

enum Epi : int {
  EPI_BIAS = 0,
  EPI_RELU = 1,
  EPI_SCALE = 2,   // (acc + b) * scale
  EPI_GRU_ZR = 3,  // co < hd: z -> out ; co >= hd: r*h -> out2 (r -> out3 if set)
  EPI_GRU_Q = 4,   // h' = (1-z) h + z tanh(acc + b) -> out (q~ -> out2 if set)
  EPI_FLOW = 5,    // coords (fp32 NCHW) = (out2 ? out2 : coords) + acc + b   (co < 2)
  // backward (dgrad) epilogues
  EPI_RELU_BWD = 6,  // out(bf16) = v * (aux1 > 0)            (through the producer's ReLU)
  EPI_ACC_F32 = 7,   // out(fp32) += v                        (gradient accumulation)
  EPI_GRU_QBWD = 8,  // co < hd: drh = v -> out2(bf16)[co] = drh*h*r*(1-r) (dr_pre), out[co] += drh*r
                     // co >= hd: out(fp32)[co] += v          (h = aux1, r = aux2)
  // encoder normalisation folded into the conv (eval-mode BatchNorm):
  EPI_NORM = 9,  // v = acc * chs[co] + bias[co]; hd != 0: ReLU; aux1: v = relu(v + aux1) -> out (bf16)
};

struct Seg {
  const bf16_t* ptr;
  int C;       // channels read (multiple of 32)
  int stride;  // row stride in elements (multiple of 8)
};

struct Args {
  Seg seg[3];
  int nseg;
  const bf16_t* w;  // [Cout_pad][taps][Ktot]
  const float* bias;
  int B, H, W, P;
  int KH, KW, PH, PW;
  int Cout, Ktot;
  int epi;
  float scale;
  int hd;
  // outputs (element strides/offsets)
  void* out;
  int ostr, ooff;
  void* out2;
  int o2str, o2off;
  void* out3;
  int o3str, o3off;
  // aux inputs (bf16 NHWC)
  const bf16_t* aux1;  // h
  int a1str, a1off;
  const bf16_t* aux2;  // z
  int a2str, a2off;
  int xcd_remap;  // conv_glds_kernel: remap block ids so each XCD walks contiguous tiles
  unsigned seg_bytes[3];
  unsigned w_bytes;
  // strided / remapped geometry (conv_lds_kernel<..., GEO = true> only): the
  // GEMM pixel grid is B x H x W; GEMM pixel (b, y, x) reads input pixel
  // (b, y*SY + tap_dy, x*SX + tap_dx) of the Hi x Wi segment grid and writes
  // output pixel ((b*oH + y*OSY + OOY)*oW + x*OSX + OOX)
  int Hi, Wi, SY, SX;
  int oH, oW, OSY, OSX, OOY, OOX;
  // EPI_NORM per-channel scale
  const float* chs;
  int f32;  // fp32 activations / outputs (conv_lds_kernel<..., F32>, epilogue_pix_f32)
};

// fp32 -> (hi, lo) bf16 pairs for 8 consecutive channels: hi = rne(x),
// lo = rne(x - hi) (F32 tiles: x.w ~= xh.wh + xl.wh + xh.wl).  The packed
// gfx950 conversion (v_cvt_pk_bf16_f32, RNE) and one v_pk_add_f32 per pair:
// 5 VALU ops per 2 values instead of the integer rounding of f2bf
typedef float f32x2v_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split8(const float4& a, const float4& b, uint4& hi, uint4& lo) {
  const float x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  uint32_t h[4], l[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f32x2v_t v = {x[2 * i], x[2 * i + 1]};
    const uint32_t hu = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2v_t));
    const f32x2v_t hf = {__uint_as_float(hu << 16), __uint_as_float(hu & 0xffff0000u)};
    h[i] = hu;
    l[i] = __builtin_bit_cast(uint32_t, __builtin_convertvector(v - hf, bf16x2v_t));
  }
  hi = make_uint4(h[0], h[1], h[2], h[3]);
  lo = make_uint4(l[0], l[1], l[2], l[3]);
}

__device__ __forceinline__ uint4 ld16(const bf16_t* p) { return *reinterpret_cast<const uint4*>(p); }

// Shared epilogue: acc[mt][nt][j] holds output channel m0 + mt*16 + 4*(lane>>4) + j
// of flat pixel pp[nt] = (pb*H + py)*W + px (pb < 0: no pixel).  The epilogue
// kind is a template parameter of the fragment loop (dispatched once, outside
// it): with a runtime switch inside, the 16-fragment loops of the 4x4 wave
// tiles were too large to unroll and the accumulators went to scratch.
// 4 consecutive channels per lane: one 8-byte (bf16) / 16-byte (fp32) access
// when every epilogue base, offset and stride is a multiple of 4 elements
// (checked once per launch, see epi_loop); the element-wise forms otherwise.
__device__ __forceinline__ void ld4(const bf16_t* p, float (&f)[4]) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  f[0] = bf2f((bf16_t)(u.x & 0xffffu));
  f[1] = bf2f((bf16_t)(u.x >> 16));
  f[2] = bf2f((bf16_t)(u.y & 0xffffu));
  f[3] = bf2f((bf16_t)(u.y >> 16));
}
__device__ __forceinline__ void st4(bf16_t* p, const float (&f)[4]) {
  typedef float f2_t __attribute__((ext_vector_type(2)));
  typedef __bf16 b2_t __attribute__((ext_vector_type(2)));
  uint2 pk;  // two packed conversions (v_cvt_pk_bf16_f32)
  pk.x = __builtin_bit_cast(uint32_t, __builtin_convertvector((f2_t{f[0], f[1]}), b2_t));
  pk.y = __builtin_bit_cast(uint32_t, __builtin_convertvector((f2_t{f[2], f[3]}), b2_t));
  *reinterpret_cast<uint2*>(p) = pk;
}
__device__ __forceinline__ void acc4(float* p, const float (&f)[4]) {
  float4 o = *reinterpret_cast<float4*>(p);
  o.x += f[0];
  o.y += f[1];
  o.z += f[2];
  o.w += f[3];
  *reinterpret_cast<float4*>(p) = o;
}

template <int E>
__device__ __forceinline__ void epi_frag(const Args& a, float (&v)[4], int cb, int p, int pb, int py, int px,
                                         int HW, bool vec) {
  const bool full = cb + 3 < a.Cout;
  if constexpr (E == EPI_FLOW) {  // coords (+)= delta; out2 (if set) is the source coords
    float* crd = static_cast<float*>(a.out);
    const float* src = a.out2 ? static_cast<const float*>(a.out2) : crd;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int co = cb + j;
      if (co < a.Cout && co < 2) {
        const size_t o = ((size_t)pb * 2 + co) * HW + (size_t)py * a.W + px;
        crd[o] = src[o] + v[j];
      }
    }
  } else if constexpr (E == EPI_GRU_ZR) {
    if (cb < a.hd) {
      bf16_t* z = static_cast<bf16_t*>(a.out) + (size_t)p * a.ostr + a.ooff + cb;
      float zv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) zv[j] = sigmoidf_(v[j]);
      if (vec) {
        st4(z, zv);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) z[j] = f2bf(zv[j]);
      }
    } else {
      const int c = cb - a.hd;
      const bf16_t* h = a.aux1 + (size_t)p * a.a1str + a.a1off + c;
      bf16_t* rh = static_cast<bf16_t*>(a.out2) + (size_t)p * a.o2str + a.o2off + c;
      bf16_t* rs_ = a.out3 ? static_cast<bf16_t*>(a.out3) + (size_t)p * a.o3str + a.o3off + c : nullptr;
      float hv[4], rv[4], rhv[4];
      if (vec) {
        ld4(h, hv);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) hv[j] = bf2f(h[j]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        rv[j] = sigmoidf_(v[j]);
        rhv[j] = rv[j] * hv[j];
      }
      if (vec) {
        st4(rh, rhv);
        if (rs_) st4(rs_, rv);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          rh[j] = f2bf(rhv[j]);
          if (rs_) rs_[j] = f2bf(rv[j]);
        }
      }
    }
  } else if constexpr (E == EPI_GRU_Q) {
    const bf16_t* h = a.aux1 + (size_t)p * a.a1str + a.a1off + cb;
    const bf16_t* z = a.aux2 + (size_t)p * a.a2str + a.a2off + cb;
    bf16_t* hn = static_cast<bf16_t*>(a.out) + (size_t)p * a.ostr + a.ooff + cb;
    bf16_t* qs = a.out2 ? static_cast<bf16_t*>(a.out2) + (size_t)p * a.o2str + a.o2off + cb : nullptr;
    float hv[4], zv[4], qv[4], nv[4];
    if (vec) {
      ld4(h, hv);
      ld4(z, zv);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        hv[j] = bf2f(h[j]);
        zv[j] = bf2f(z[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      qv[j] = tanhf_(v[j]);
      nv[j] = (1.f - zv[j]) * hv[j] + zv[j] * qv[j];
    }
    if (vec) {
      st4(hn, nv);
      if (qs) st4(qs, qv);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        hn[j] = f2bf(nv[j]);
        if (qs) qs[j] = f2bf(qv[j]);
      }
    }
  } else if constexpr (E == EPI_RELU_BWD) {
    const bf16_t* act = a.aux1 + (size_t)p * a.a1str + a.a1off + cb;
    bf16_t* o = static_cast<bf16_t*>(a.out) + (size_t)p * a.ostr + a.ooff + cb;
    if (vec && full) {
      float av[4], ov[4];
      ld4(act, av);
#pragma unroll
      for (int j = 0; j < 4; ++j) ov[j] = av[j] > 0.f ? v[j] : 0.f;
      st4(o, ov);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (cb + j < a.Cout) o[j] = f2bf(bf2f(act[j]) > 0.f ? v[j] : 0.f);
    }
  } else if constexpr (E == EPI_ACC_F32) {
    float* o = static_cast<float*>(a.out) + (size_t)p * a.ostr + a.ooff + cb;
    if (vec && full) {
      acc4(o, v);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (cb + j < a.Cout) o[j] += v[j];
    }
  } else if constexpr (E == EPI_GRU_QBWD) {
    float* o = static_cast<float*>(a.out) + (size_t)p * a.ostr + a.ooff + cb;
    if (cb < a.hd) {
      const bf16_t* h = a.aux1 + (size_t)p * a.a1str + a.a1off + cb;
      const bf16_t* r = a.aux2 + (size_t)p * a.a2str + a.a2off + cb;
      bf16_t* drp = static_cast<bf16_t*>(a.out2) + (size_t)p * a.o2str + a.o2off + cb;
      float hv[4], rv[4], dv[4], gv[4];
      if (vec) {
        ld4(h, hv);
        ld4(r, rv);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          hv[j] = bf2f(h[j]);
          rv[j] = bf2f(r[j]);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dv[j] = v[j] * hv[j] * rv[j] * (1.f - rv[j]);
        gv[j] = v[j] * rv[j];
      }
      if (vec) {
        st4(drp, dv);
        acc4(o, gv);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          drp[j] = f2bf(dv[j]);
          o[j] += gv[j];
        }
      }
    } else {
      if (vec && full) {
        acc4(o, v);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (cb + j < a.Cout) o[j] += v[j];
      }
    }
  } else if constexpr (E == EPI_NORM) {
    if (a.hd) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
    }
    bf16_t* o = static_cast<bf16_t*>(a.out) + (size_t)p * a.ostr + a.ooff + cb;
    const bf16_t* r = a.aux1 ? a.aux1 + (size_t)p * a.a1str + a.a1off + cb : nullptr;
    if (vec && full) {
      if (r) {
        float rv[4];
        ld4(r, rv);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j] + rv[j], 0.f);
      }
      st4(o, v);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (cb + j < a.Cout) o[j] = f2bf(r ? fmaxf(v[j] + bf2f(r[j]), 0.f) : v[j]);
    }
  } else {  // EPI_BIAS / EPI_RELU / EPI_SCALE -> bf16
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr (E == EPI_RELU) v[j] = fmaxf(v[j], 0.f);
      if constexpr (E == EPI_SCALE) v[j] *= a.scale;
    }
    bf16_t* o = static_cast<bf16_t*>(a.out) + (size_t)p * a.ostr + a.ooff + cb;
    if (vec && full) {
      st4(o, v);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (cb + j < a.Cout) o[j] = f2bf(v[j]);
    }
  }
}

template <int WM, int WN, int E>
__device__ __forceinline__ void epi_loop(const Args& a, const f32x4_t (&acc)[WM][WN], int m0, int lane,
                                         const int (&pp)[WN], const int (&pb)[WN], const int (&py)[WN],
                                         const int (&px)[WN]) {
  const int HW = a.H * a.W;
  const int cq = (lane >> 4) * 4;
  // wave-uniform: every epilogue tensor 4-element aligned (vector accesses)
  const bool vec =
      ((a.ooff | a.ostr | a.o2off | a.o2str | a.o3off | a.o3str | a.a1off | a.a1str | a.a2off | a.a2str) & 3) == 0 &&
      (((uintptr_t)a.out | (uintptr_t)a.out2 | (uintptr_t)a.out3 | (uintptr_t)a.aux1 | (uintptr_t)a.aux2) & 15) == 0;
  const bool bvec = a.bias && (((uintptr_t)a.bias) & 15) == 0;
#pragma unroll
  for (int nt = 0; nt < WN; ++nt) {
    if (pb[nt] < 0) continue;
#pragma unroll
    for (int mt = 0; mt < WM; ++mt) {
      const int cb = m0 + mt * 16 + cq;
      if (cb >= a.Cout) continue;
      float v[4];
      if constexpr (E == EPI_NORM) {  // host-checked: chs / bias hold round_up(Cout, 4), 16-B aligned
        const float4 sv = *reinterpret_cast<const float4*>(a.chs + cb);
        const float4 bv = *reinterpret_cast<const float4*>(a.bias + cb);
        v[0] = acc[mt][nt][0] * sv.x + bv.x;
        v[1] = acc[mt][nt][1] * sv.y + bv.y;
        v[2] = acc[mt][nt][2] * sv.z + bv.z;
        v[3] = acc[mt][nt][3] * sv.w + bv.w;
      } else if (bvec && cb + 3 < a.Cout) {
        const float4 bv = *reinterpret_cast<const float4*>(a.bias + cb);
        v[0] = acc[mt][nt][0] + bv.x;
        v[1] = acc[mt][nt][1] + bv.y;
        v[2] = acc[mt][nt][2] + bv.z;
        v[3] = acc[mt][nt][3] + bv.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = acc[mt][nt][j] + (cb + j < a.Cout && a.bias ? a.bias[cb + j] : 0.f);
      }
      epi_frag<E>(a, v, cb, pp[nt], pb[nt], py[nt], px[nt], HW, vec);
    }
  }
}

template <int WM, int WN>
__device__ __forceinline__ void epilogue_pix(const Args& a, const f32x4_t (&acc)[WM][WN], int m0, int lane,
                                             const int (&pp)[WN], const int (&pb)[WN], const int (&py)[WN],
                                             const int (&px)[WN]) {
  switch (a.epi) {
#define RS_EPI(E) \
  case E: epi_loop<WM, WN, E>(a, acc, m0, lane, pp, pb, py, px); break
    RS_EPI(EPI_FLOW);
    RS_EPI(EPI_GRU_ZR);
    RS_EPI(EPI_GRU_Q);
    RS_EPI(EPI_RELU_BWD);
    RS_EPI(EPI_ACC_F32);
    RS_EPI(EPI_GRU_QBWD);
    RS_EPI(EPI_RELU);
    RS_EPI(EPI_SCALE);
    RS_EPI(EPI_NORM);
#undef RS_EPI
    default: epi_loop<WM, WN, EPI_BIAS>(a, acc, m0, lane, pp, pb, py, px); break;
  }
}

// ---------------------------------------------------------------- fp32 epilogues
// The F32 tiles' epilogues: the forward kinds of the inference engine and
// the encoders (bias / ReLU / scale, ConvGRU gates and update, eval-BN
// EPI_NORM with residual) and the dgrad kinds of the fp32 training engine
// (ReLU backward, fp32 accumulation, the q-conv r-gate backward) on fp32 NHWC
// outputs and aux inputs (every "bf16_t*" of Args is read as float*), plus
// the normalisation statistics of the unrounded output.
__device__ __forceinline__ void ld4f(const bf16_t* p, float (&f)[4]) {
  const float4 v = *reinterpret_cast<const float4*>(p);
  f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w;
}
__device__ __forceinline__ void st4f(void* p, const float (&f)[4]) {
  *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
}

template <int E>
__device__ __forceinline__ void epi_frag_f32(const Args& a, float (&v)[4], int cb, int p, bool vec) {
  const bool full = cb + 3 < a.Cout;
  auto fo = [](void* b, int str, int off, int p_, int c) { return static_cast<float*>(b) + (size_t)p_ * str + off + c; };
  auto fi = [](const bf16_t* b, int str, int off, int p_, int c) {
    return reinterpret_cast<const float*>(b) + (size_t)p_ * str + off + c;
  };
  if constexpr (E == EPI_GRU_ZR) {
    if (cb < a.hd) {
      float* z = fo(a.out, a.ostr, a.ooff, p, cb);
#pragma unroll
      for (int j = 0; j < 4; ++j) z[j] = sigmoidf_(v[j]);
    } else {
      const int c = cb - a.hd;
      const float* h = fi(a.aux1, a.a1str, a.a1off, p, c);
      float* rh = fo(a.out2, a.o2str, a.o2off, p, c);
      float* r = a.out3 ? fo(a.out3, a.o3str, a.o3off, p, c) : nullptr;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float rv = sigmoidf_(v[j]);
        rh[j] = rv * h[j];
        if (r) r[j] = rv;
      }
    }
  } else if constexpr (E == EPI_GRU_Q) {
    const float* h = fi(a.aux1, a.a1str, a.a1off, p, cb);
    const float* z = fi(a.aux2, a.a2str, a.a2off, p, cb);
    float* hn = fo(a.out, a.ostr, a.ooff, p, cb);
    float* qs = a.out2 ? fo(a.out2, a.o2str, a.o2off, p, cb) : nullptr;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float q = tanhf(v[j]);
      hn[j] = (1.f - z[j]) * h[j] + z[j] * q;
      if (qs) qs[j] = q;
    }
  } else if constexpr (E == EPI_RELU_BWD) {  // out = v * (act > 0)
    const float* act = fi(a.aux1, a.a1str, a.a1off, p, cb);
    float* o = fo(a.out, a.ostr, a.ooff, p, cb);
    if (vec && full) {
      const float4 av = *reinterpret_cast<const float4*>(act);
      *reinterpret_cast<float4*>(o) = make_float4(av.x > 0.f ? v[0] : 0.f, av.y > 0.f ? v[1] : 0.f,
                                                  av.z > 0.f ? v[2] : 0.f, av.w > 0.f ? v[3] : 0.f);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (cb + j < a.Cout) o[j] = act[j] > 0.f ? v[j] : 0.f;
    }
  } else if constexpr (E == EPI_ACC_F32) {  // out += v
    float* o = fo(a.out, a.ostr, a.ooff, p, cb);
    if (vec && full) {
      acc4(o, v);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (cb + j < a.Cout) o[j] += v[j];
    }
  } else if constexpr (E == EPI_GRU_QBWD) {  // as the bf16 form, fp32 dr_pre / h / r
    float* o = fo(a.out, a.ostr, a.ooff, p, cb);
    if (cb < a.hd) {
      const float* h = fi(a.aux1, a.a1str, a.a1off, p, cb);
      const float* r = fi(a.aux2, a.a2str, a.a2off, p, cb);
      float* drp = fo(a.out2, a.o2str, a.o2off, p, cb);
      float gv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        drp[j] = v[j] * h[j] * r[j] * (1.f - r[j]);
        gv[j] = v[j] * r[j];
      }
      if (vec) {
        acc4(o, gv);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] += gv[j];
      }
    } else if (vec && full) {
      acc4(o, v);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (cb + j < a.Cout) o[j] += v[j];
    }
  } else {  // EPI_BIAS / EPI_RELU / EPI_SCALE / EPI_NORM
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr (E == EPI_RELU) v[j] = fmaxf(v[j], 0.f);
      if constexpr (E == EPI_SCALE) v[j] *= a.scale;
      if constexpr (E == EPI_NORM)
        if (a.hd) v[j] = fmaxf(v[j], 0.f);
    }
    float* o = fo(a.out, a.ostr, a.ooff, p, cb);
    const float* r = (E == EPI_NORM && a.aux1) ? fi(a.aux1, a.a1str, a.a1off, p, cb) : nullptr;
    if (vec && full) {
      if (r) {
        float rv[4];
        ld4f(reinterpret_cast<const bf16_t*>(r), rv);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j] + rv[j], 0.f);
      }
      st4f(o, v);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (cb + j < a.Cout) o[j] = r ? fmaxf(v[j] + r[j], 0.f) : v[j];
    }
  }
}

template <int WM, int WN, int E>
__device__ __forceinline__ void epi_loop_f32(const Args& a, const f32x4_t (&acc)[WM][WN], int m0, int lane,
                                             const int (&pp)[WN], const int (&pb)[WN]) {
  const int cq = (lane >> 4) * 4;
  const bool vec =
      ((a.ooff | a.ostr | a.o2off | a.o2str | a.o3off | a.o3str | a.a1off | a.a1str | a.a2off | a.a2str) & 3) == 0 &&
      (((uintptr_t)a.out | (uintptr_t)a.out2 | (uintptr_t)a.out3 | (uintptr_t)a.aux1 | (uintptr_t)a.aux2) & 15) == 0;
#pragma unroll
  for (int nt = 0; nt < WN; ++nt) {
    if (pb[nt] < 0) continue;
#pragma unroll
    for (int mt = 0; mt < WM; ++mt) {
      const int cb = m0 + mt * 16 + cq;
      if (cb >= a.Cout) continue;
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = cb + j;
        const bool in = c < a.Cout;
        const float sc = (E == EPI_NORM && in) ? a.chs[c] : 1.f;
        v[j] = acc[mt][nt][j] * sc + (in && a.bias ? a.bias[c] : 0.f);
      }
      epi_frag_f32<E>(a, v, cb, pp[nt], vec);
    }
  }
}

template <int WM, int WN>
__device__ __forceinline__ void epilogue_pix_f32(const Args& a, const f32x4_t (&acc)[WM][WN], int m0, int lane,
                                                 const int (&pp)[WN], const int (&pb)[WN]) {
  switch (a.epi) {
#define RS_EPI32(E) \
  case E: epi_loop_f32<WM, WN, E>(a, acc, m0, lane, pp, pb); break
    RS_EPI32(EPI_GRU_ZR);
    RS_EPI32(EPI_GRU_Q);
    RS_EPI32(EPI_RELU_BWD);
    RS_EPI32(EPI_ACC_F32);
    RS_EPI32(EPI_GRU_QBWD);
    RS_EPI32(EPI_RELU);
    RS_EPI32(EPI_SCALE);
    RS_EPI32(EPI_NORM);
#undef RS_EPI32
    default: epi_loop_f32<WM, WN, EPI_BIAS>(a, acc, m0, lane, pp, pb); break;
  }
}

// Linear pixel tiles: the B columns of n-tile nt are pixels n0 + nt*16 + (lane&15).
template <int WM, int WN>
__device__ __forceinline__ void epilogue(const Args& a, const f32x4_t (&acc)[WM][WN], int m0, int n0,
                                         int lane, const int (&pb)[WN], const int (&py)[WN],
                                         const int (&px)[WN]) {
  int pp[WN];
#pragma unroll
  for (int nt = 0; nt < WN; ++nt) pp[nt] = n0 + nt * 16 + (lane & 15);
  epilogue_pix<WM, WN>(a, acc, m0, lane, pp, pb, py, px);
}

template <int WM, int WN, int WAVES_M, int WAVES_N>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) void conv_kernel(Args a) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave % WAVES_M, wn = wave / WAVES_M;
  const int m0 = (blockIdx.y * WAVES_M + wm) * WM * 16;  // first output channel of this wave
  const int n0 = (blockIdx.x * WAVES_N + wn) * WN * 16;  // first pixel of this wave
  const int lr = lane & 15, lk = (lane >> 4) * 8;
  const int taps = a.KH * a.KW;
  const int HW = a.H * a.W;

  // pixel coordinates of this lane's B columns
  int pb[WN], py[WN], px[WN];
#pragma unroll
  for (int nt = 0; nt < WN; ++nt) {
    const int p = n0 + nt * 16 + lr;
    if (p < a.P) {
      pb[nt] = p / HW;
      const int q = p - pb[nt] * HW;
      py[nt] = q / a.W;
      px[nt] = q - py[nt] * a.W;
    } else {
      pb[nt] = -1;
      py[nt] = px[nt] = 0;
    }
  }
  // weight row pointers of this lane's A rows
  const bf16_t* wrow[WM];
#pragma unroll
  for (int mt = 0; mt < WM; ++mt)
    wrow[mt] = a.w + (size_t)(m0 + mt * 16 + lr) * taps * a.Ktot + lk;

  f32x4_t acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // flattened K steps: (segment, tap, 32-channel chunk).  Segment fields are
  // selected with wave-uniform compares (no dynamic indexing of the kernarg
  // array, which would go through scratch).
  const Seg s0 = a.seg[0], s1 = a.seg[1], s2 = a.seg[2];
  const int e1 = taps * (s0.C >> 5);
  const int e2 = e1 + (a.nseg > 1 ? taps * (s1.C >> 5) : 0);
  const int nsteps = e2 + (a.nseg > 2 ? taps * (s2.C >> 5) : 0);

  // plain locals: a lambda capturing the byval kernarg struct by reference
  // would force a copy of it into scratch.
  const int H = a.H, W = a.W, KW = a.KW, PH = a.PH, PW = a.PW, Ktot = a.Ktot;
  const uint4 zero = make_uint4(0, 0, 0, 0);
#define RS_CONV_LOAD(STEP, FA, FB)                                                           \
  do {                                                                                       \
    const int step_ = (STEP);                                                                \
    const int si = (step_ >= e1) + (step_ >= e2);                                            \
    const bf16_t* sp = si == 0 ? s0.ptr : (si == 1 ? s1.ptr : s2.ptr);                       \
    const int sC = si == 0 ? s0.C : (si == 1 ? s1.C : s2.C);                                 \
    const int sst = si == 0 ? s0.stride : (si == 1 ? s1.stride : s2.stride);                 \
    const int kseg = si == 0 ? 0 : (si == 1 ? s0.C : s0.C + s1.C);                           \
    const int local = step_ - (si == 0 ? 0 : (si == 1 ? e1 : e2));                          \
    const int chunks = sC >> 5;                                                              \
    const int tap = local / chunks;                                                          \
    const int c0 = (local - tap * chunks) * 32;                                              \
    const int dy = tap / KW - PH, dx = tap % KW - PW;                                        \
    _Pragma("unroll") for (int mt = 0; mt < WM; ++mt)                                        \
      FA[mt] = ld16(wrow[mt] + (size_t)tap * Ktot + kseg + c0);                              \
    _Pragma("unroll") for (int nt = 0; nt < WN; ++nt) {                                      \
      const int yy = py[nt] + dy, xx = px[nt] + dx;                                          \
      const bool ok = pb[nt] >= 0 && yy >= 0 && yy < H && xx >= 0 && xx < W;                 \
      FB[nt] = ok ? ld16(sp + ((size_t)(pb[nt] * H + yy) * W + xx) * sst + c0 + lk) : zero;  \
    }                                                                                        \
  } while (0)

#define RS_CONV_MMA(FA, FB)                                                                       \
  _Pragma("unroll") for (int mt = 0; mt < WM; ++mt)                                               \
    _Pragma("unroll") for (int nt = 0; nt < WN; ++nt)                                             \
      acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(                                      \
          __builtin_bit_cast(bf16x8_t, FA[mt]), __builtin_bit_cast(bf16x8_t, FB[nt]), acc[mt][nt], \
          0, 0, 0)

  uint4 fa0[WM], fb0[WN], fa1[WM], fb1[WN];
  RS_CONV_LOAD(0, fa0, fb0);
  int step = 0;
  for (; step + 2 <= nsteps; step += 2) {
    RS_CONV_LOAD(step + 1, fa1, fb1);
    RS_CONV_MMA(fa0, fb0);
    if (step + 2 < nsteps) RS_CONV_LOAD(step + 2, fa0, fb0);
    RS_CONV_MMA(fa1, fb1);
  }
  if (step < nsteps) {
    RS_CONV_MMA(fa0, fb0);
  }
#undef RS_CONV_LOAD
#undef RS_CONV_MMA

  epilogue<WM, WN>(a, acc, m0, n0, lane, pb, py, px);
}

// staging helpers
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

__device__ __forceinline__ void glds16(const void* src, uint4* lds_base) {
  __builtin_amdgcn_global_load_lds(
      (const __attribute__((address_space(1))) void*)src, (__attribute__((address_space(3))) void*)lds_base, 16,
      0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void bdma16(__amdgpu_buffer_rsrc_t r, uint4* lds_base, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_base, 16, voff, soff,
                                           0, 0);
}

template <int N>
__device__ __forceinline__ void wait_lgkm() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}

// 32x32x16 accumulator -> the shared epilogue (4 consecutive channels per call)
template <int E>
__device__ __forceinline__ void epi32(const Args& a, const f32x16_t& acc, int m0, int lane, int p, int pb, int py,
                                      int px, bool vec) {
  if (pb < 0) return;
  const int HW = a.H * a.W;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int cb = m0 + 8 * g + 4 * (lane >> 5);
    if (cb >= a.Cout) continue;
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = acc[4 * g + j] + (cb + j < a.Cout && a.bias ? a.bias[cb + j] : 0.f);
    epi_frag<E>(a, v, cb, p, pb, py, px, HW, vec);
  }
}

// Batched form of epi32 for a whole 32-row fragment inside Cout (the common
// case): every bias / aux / read-modify-write load of the NB accumulators is
// issued first, unconditionally (pixels outside the image read pixel 0 and
// store nothing), and the arithmetic + stores follow -- ONE memory round trip
// per group of NBC accumulators instead of one dependent L2 round trip per
// 4-channel group (the per-element form branches around every load and waits
// vmcnt(0) after each: ~24 serial round trips for a 6-row patch).
template <int NB, int E>
__device__ __forceinline__ void epi32_batch(const Args& a, const f32x16_t (&acc)[NB], int m0, int lane,
                                            const int (&pp)[NB], const int (&pb)[NB]) {
  const int h4 = 4 * (lane >> 5);
  float bz[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) bz[i] = a.bias ? a.bias[m0 + 8 * (i >> 2) + h4 + (i & 3)] : 0.f;
  // GRU_ZR / GRU_QBWD: the fragment lies wholly on one side of hd (host: hd % 32 == 0 on this path)
  const bool lo = m0 < a.hd;
  constexpr int NBC = NB > 3 ? 3 : NB;
#pragma unroll
  for (int n0 = 0; n0 < NB; n0 += NBC) {
    uint2 l1[NBC][4], l2[NBC][4];
    float4 lf[NBC][4];
    // ---- phase 1: loads
#pragma unroll
    for (int k = 0; k < NBC; ++k) {
      if (n0 + k >= NB) break;
      const size_t p = (size_t)(pb[n0 + k] >= 0 ? pp[n0 + k] : 0);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int cb = m0 + 8 * g + h4;
        if constexpr (E == EPI_GRU_ZR) {
          if (!lo) l1[k][g] = *reinterpret_cast<const uint2*>(a.aux1 + p * a.a1str + a.a1off + cb - a.hd);
        } else if constexpr (E == EPI_GRU_Q) {
          l1[k][g] = *reinterpret_cast<const uint2*>(a.aux1 + p * a.a1str + a.a1off + cb);
          l2[k][g] = *reinterpret_cast<const uint2*>(a.aux2 + p * a.a2str + a.a2off + cb);
        } else if constexpr (E == EPI_RELU_BWD) {
          l1[k][g] = *reinterpret_cast<const uint2*>(a.aux1 + p * a.a1str + a.a1off + cb);
        } else if constexpr (E == EPI_ACC_F32) {
          lf[k][g] = *reinterpret_cast<const float4*>(static_cast<const float*>(a.out) + p * a.ostr + a.ooff + cb);
        } else if constexpr (E == EPI_GRU_QBWD) {
          lf[k][g] = *reinterpret_cast<const float4*>(static_cast<const float*>(a.out) + p * a.ostr + a.ooff + cb);
          if (lo) {
            l1[k][g] = *reinterpret_cast<const uint2*>(a.aux1 + p * a.a1str + a.a1off + cb);
            l2[k][g] = *reinterpret_cast<const uint2*>(a.aux2 + p * a.a2str + a.a2off + cb);
          }
        }
      }
    }
    // ---- phase 2: arithmetic + stores
#pragma unroll
    for (int k = 0; k < NBC; ++k) {
      if (n0 + k >= NB) break;
      if (pb[n0 + k] < 0) continue;
      const size_t p = (size_t)pp[n0 + k];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int cb = m0 + 8 * g + h4;
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = acc[n0 + k][4 * g + j] + bz[4 * g + j];
        auto unpack = [](uint2 u, float (&f)[4]) {
          f[0] = bf2f((bf16_t)(u.x & 0xffffu));
          f[1] = bf2f((bf16_t)(u.x >> 16));
          f[2] = bf2f((bf16_t)(u.y & 0xffffu));
          f[3] = bf2f((bf16_t)(u.y >> 16));
        };
        if constexpr (E == EPI_GRU_ZR) {
          float r[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) r[j] = sigmoidf_(v[j]);
          if (lo) {
            st4(static_cast<bf16_t*>(a.out) + p * a.ostr + a.ooff + cb, r);
          } else {
            const int c = cb - a.hd;
            float hv[4], rh[4];
            unpack(l1[k][g], hv);
#pragma unroll
            for (int j = 0; j < 4; ++j) rh[j] = r[j] * hv[j];
            st4(static_cast<bf16_t*>(a.out2) + p * a.o2str + a.o2off + c, rh);
            if (a.out3) st4(static_cast<bf16_t*>(a.out3) + p * a.o3str + a.o3off + c, r);
          }
        } else if constexpr (E == EPI_GRU_Q) {
          float hv[4], zv[4], q[4], nv[4];
          unpack(l1[k][g], hv);
          unpack(l2[k][g], zv);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            q[j] = tanhf_(v[j]);
            nv[j] = (1.f - zv[j]) * hv[j] + zv[j] * q[j];
          }
          st4(static_cast<bf16_t*>(a.out) + p * a.ostr + a.ooff + cb, nv);
          if (a.out2) st4(static_cast<bf16_t*>(a.out2) + p * a.o2str + a.o2off + cb, q);
        } else if constexpr (E == EPI_RELU_BWD) {
          float av[4];
          unpack(l1[k][g], av);
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = av[j] > 0.f ? v[j] : 0.f;
          st4(static_cast<bf16_t*>(a.out) + p * a.ostr + a.ooff + cb, v);
        } else if constexpr (E == EPI_ACC_F32) {
          const float4 o = lf[k][g];
          *reinterpret_cast<float4*>(static_cast<float*>(a.out) + p * a.ostr + a.ooff + cb) =
              make_float4(o.x + v[0], o.y + v[1], o.z + v[2], o.w + v[3]);
        } else if constexpr (E == EPI_GRU_QBWD) {
          const float4 o = lf[k][g];
          float* op = static_cast<float*>(a.out) + p * a.ostr + a.ooff + cb;
          if (lo) {
            float hv[4], rv[4], dv[4];
            unpack(l1[k][g], hv);
            unpack(l2[k][g], rv);
#pragma unroll
            for (int j = 0; j < 4; ++j) dv[j] = v[j] * hv[j] * rv[j] * (1.f - rv[j]);
            st4(static_cast<bf16_t*>(a.out2) + p * a.o2str + a.o2off + cb, dv);
            *reinterpret_cast<float4*>(op) =
                make_float4(o.x + v[0] * rv[0], o.y + v[1] * rv[1], o.z + v[2] * rv[2], o.w + v[3] * rv[3]);
          } else {
            *reinterpret_cast<float4*>(op) = make_float4(o.x + v[0], o.y + v[1], o.z + v[2], o.w + v[3]);
          }
        } else {  // EPI_BIAS / EPI_RELU / EPI_SCALE
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if constexpr (E == EPI_RELU) v[j] = fmaxf(v[j], 0.f);
            if constexpr (E == EPI_SCALE) v[j] *= a.scale;
          }
          st4(static_cast<bf16_t*>(a.out) + p * a.ostr + a.ooff + cb, v);
        }
      }
    }
  }
}

template <int NB>
__device__ __forceinline__ void epilogue32(const Args& a, const f32x16_t (&acc)[NB], int m0, int lane,
                                           const int (&pp)[NB], const int (&pb)[NB], const int (&py)[NB],
                                           const int (&px)[NB]) {
  const bool vec =
      ((a.ooff | a.ostr | a.o2off | a.o2str | a.o3off | a.o3str | a.a1off | a.a1str | a.a2off | a.a2str) & 3) == 0 &&
      (((uintptr_t)a.out | (uintptr_t)a.out2 | (uintptr_t)a.out3 | (uintptr_t)a.aux1 | (uintptr_t)a.aux2) & 15) == 0;
  // whole fragment inside Cout, 4-aligned epilogue tensors, GRU split on a 32-row boundary
  const bool fast = vec && m0 + 32 <= a.Cout && (a.hd & 31) == 0;
  if (fast) {
    switch (a.epi) {
#define RS_EB(E) \
  case E: epi32_batch<NB, E>(a, acc, m0, lane, pp, pb); return
      RS_EB(EPI_GRU_ZR);
      RS_EB(EPI_GRU_Q);
      RS_EB(EPI_RELU_BWD);
      RS_EB(EPI_ACC_F32);
      RS_EB(EPI_GRU_QBWD);
      RS_EB(EPI_RELU);
      RS_EB(EPI_SCALE);
      RS_EB(EPI_BIAS);
#undef RS_EB
      default: break;  // EPI_FLOW: element-wise form below
    }
  }
  switch (a.epi) {
#define RS_E2(E)                                                                      \
  case E:                                                                             \
    _Pragma("unroll") for (int nb = 0; nb < NB; ++nb)                                 \
      epi32<E>(a, acc[nb], m0, lane, pp[nb], pb[nb], py[nb], px[nb], vec);            \
    break
    RS_E2(EPI_FLOW);
    RS_E2(EPI_GRU_ZR);
    RS_E2(EPI_GRU_Q);
    RS_E2(EPI_RELU_BWD);
    RS_E2(EPI_ACC_F32);
    RS_E2(EPI_GRU_QBWD);
    RS_E2(EPI_RELU);
    RS_E2(EPI_SCALE);
#undef RS_E2
    default:
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) epi32<EPI_BIAS>(a, acc[nb], m0, lane, pp[nb], pb[nb], py[nb], px[nb], vec);
      break;
  }
}

}  // namespace conv

// conv_v2.hip: tiles 42-45 (3x3 / 1x5 / 5x1 only); false if the kernel size is not instantiated
bool conv_v2_launch(const conv::Args& a, int tile, hipStream_t stream);
// conv_v3.hip: tiles 60-68 (3x3 / 1x5 / 5x1; weights in the fragment-major layout, ops/conv.py frag_weight)
bool conv_v3_launch(const conv::Args& a, int tile, hipStream_t stream);
// conv_v3f.hip: tiles 81-83 (fp32 activations; split fragment-major weights, ops/conv.py frag_weight_split)
bool conv_v3f_launch(const conv::Args& a, int tile, hipStream_t stream);
}  // namespace rs
