// Weight-streaming implicit-GEMM convolution for the update-block 3x3 / 1x5 /
// 5x1 convs (reference core/update.py:6-136: the motion encoder, the
// SepConvGRU, the flow and mask heads, and the input gradients of all of them),
// tiles 60-71 of conv_fused.
//
// Why a third design (profiles/r4/pmc_update_conv_r4_start.txt,
// profiles/r5/README.md): the conv_v2 tiles share one BM x 64 weight tile per
// K step through an LDS ring, so every K step costs a workgroup barrier and
// the ring (2-3 slots of 16-32 KB) keeps only 1-2 K steps of weights in flight
// -- far less than the ~1 us an L2 fill takes under load.  Here:
//  * the block's waves split the OUTPUT CHANNELS only: wave w owns rows
//    [bm0 + 32 MW w, +32 MW) and every pixel of the block's TH x 32 patch, so
//    no two waves ever read the same weights and the weights never touch LDS:
//    each wave streams its own A fragments global -> VGPR (buffer_load_dwordx4,
//    one fully coalesced 1 KB fragment per 16-deep K slice in the
//    fragment-major layout, ops/conv.py frag_weight) through a register ring
//    RA - 1 slices deep (~2 us of MFMA work in flight);
//  * the activations are the only shared operand: per 64-channel chunk the
//    patch's (TH + KH - 1) x (32 + KW - 1) halo is DMA'd into LDS once
//    (buffer_load ... lds; 144-B pixel rows, conflict-free for every tap
//    shift) and read by all T taps as shifted B fragments; two halo buffers,
//    the next chunk's pieces issued during the first slices of this one;
//  * ONE workgroup barrier per chunk (T * 4 slices), none per K step;
//  * small Cout tiles with large pixel tiles (128 Cout x 192 px at the
//    training shape): with the B operand reused over T taps, MACs per L2 byte
//    grow with the pixel tile, not the Cout tile (1x5: 144 vs 104 FLOP/B for
//    conv_v2's 128 x 128).
// The tap loop of a chunk is fully unrolled (every ring slot, LDS offset,
// DMA count and vmcnt immediate is a compile-time constant); the chunk loop
// is a runtime loop over the concatenated input segments.  Out-of-range A
// slices (past the last chunk / the last row block) and halo pieces past the
// last chunk are issued as zero-returning out-of-range loads so every slice
// has the same compile-time VMEM count.
#pragma once
#include "conv_common.h"

namespace rs {
namespace conv {

typedef int i32x4_t __attribute__((ext_vector_type(4)));

// raw buffer resource (gfx950 dword3) for the inline-asm loads
__device__ __forceinline__ i32x4_t raw_rsrc(const void* p, unsigned bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  i32x4_t r;
  r.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  r.y = __builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32) & 0xffff);
  r.z = __builtin_amdgcn_readfirstlane((int)bytes);
  r.w = 0x00020000;
  return r;
}

template <int KH, int KW, int NWM, int MW, int THW, int RA, int NWP>
struct V3 {
  static constexpr int T = KH * KW, NSL = 4 * T, D = RA - 1;
  static constexpr int TH = THW * NWP, NW = NWM * NWP;  // patch rows; waves (Cout x pixel rows)
  static constexpr int NT = 64 * NW, BM = 32 * MW * NWM, TW = 32;
  static constexpr int HH = TH + KH - 1, HWD = TW + KW - 1;
  static constexpr int PPR = (HWD * 9 + 63) / 64;   // DMA pieces (1 KB) per halo row
  static constexpr int ROWSL = PPR * 64;            // 16-B slots per halo row
  static constexpr int NHP = HH * PPR;               // halo pieces per chunk
  static constexpr int NHPW = (NHP + NW - 1) / NW;   // ... per wave (the last may be padding)
  static constexpr int HSL = NHPW * NW * 64;         // slots per halo buffer
  // halo pieces go at slice positions [0, LASTP): early enough that waiting
  // for the chunk's last A slice retires them, or (deep rings) all at position 0
  static constexpr int LASTP = NSL > RA ? NSL - RA : 1;
  static constexpr int PPP = (NHPW + LASTP - 1) / LASTP;  // ... this many per position
  static constexpr int LDS_SLOTS = 2 * HSL;
  static constexpr int hcnt(int j) {
    j = ((j % NSL) + NSL) % NSL;
    if (j >= LASTP) return 0;
    const int n = NHPW - j * PPP;
    return n < 0 ? 0 : (n > PPP ? PPP : n);
  }
  // VMEM instructions issued after the last A load of slice j (its own ring
  // slot was filled D positions earlier; the halo pieces of every position in
  // between ride along) -- the vmcnt that retires slice j
  static constexpr int nwait(int j) {
    int n = D * MW;
    for (int i = j - D; i <= j; ++i) n += hcnt(i);
    return n;
  }
  // the wait before the chunk's closing barrier: the last slice AND the halo
  static constexpr int bwait() {
    int last = 0;
    for (int j = 0; j < NSL; ++j)
      if (hcnt(j) > 0) last = j;
    const int after = (NSL - 1 - last) * MW;
    return nwait(NSL - 1) < after ? nwait(NSL - 1) : after;
  }
  static constexpr bool counts_ok() {
    for (int j = 0; j < NSL; ++j)
      if (nwait(j) > 63) return false;
    return true;
  }
};

template <int KH, int KW, int NWM, int MW, int THW, int RA, int NWP = 1>
__global__ __launch_bounds__(64 * NWM * NWP) void conv_v3_kernel(Args a) {
  using C = V3<KH, KW, NWM, MW, THW, RA, NWP>;
  constexpr int TH = C::TH, NW = C::NW;
  constexpr int T = C::T, NSL = C::NSL, D = C::D, BM = C::BM;
  constexpr int HWD = C::HWD, PPR = C::PPR, NHP = C::NHP, NHPW = C::NHPW, HSL = C::HSL;
  constexpr int ROWSL = C::ROWSL, PPP = C::PPP;
  constexpr int PH = KH / 2, PW = KW / 2;
  constexpr int kFar = 0x7ffffff0;
  static_assert(NSL % RA == 0, "ring slots must divide the slices of a chunk");
  static_assert(C::LASTP > 0 && C::counts_ok(), "halo schedule / vmcnt range");
  static_assert(MW == 1 || MW == 2, "MW");
  static_assert(T <= 9, "taps");
  __shared__ uint4 lds[C::LDS_SLOTS];

  const int t_ = threadIdx.x, lane = t_ & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t_ >> 6);
  // output-channel slice, patch-row group of this wave (NWP == 1: constants,
  // so the single-group tiles compile to the same code as before NWP existed)
  const int cw = NWP == 1 ? wave : wave % NWM, pw = NWP == 1 ? 0 : wave / NWM;
  const int H = a.H, W = a.W;
  const int ntx = cdiv(W, 32), npb = cdiv(H, TH) * ntx;
  const int nct = cdiv(a.Cout, BM);
  const int lid = a.xcd_remap ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int bm0 = (lid % nct) * BM;
  const int pt = lid / nct;
  const int img = pt / npb, pq = pt - img * npb;
  const int pty = pq / ntx;
  const int y0 = pty * TH, x0 = (pq - pty * ntx) * 32;

  const bf16_t *const sp0 = a.seg[0].ptr, *const sp1 = a.seg[1].ptr, *const sp2 = a.seg[2].ptr;
  const unsigned sb0 = a.seg_bytes[0], sb1 = a.seg_bytes[1], sb2 = a.seg_bytes[2];
  const int st0 = a.seg[0].stride, st1 = a.seg[1].stride, st2 = a.seg[2].stride;
  const int e1 = a.seg[0].C >> 6;
  const int e2 = e1 + (a.nseg > 1 ? (a.seg[1].C >> 6) : 0);
  const int nchunks = e2 + (a.nseg > 2 ? (a.seg[2].C >> 6) : 0);
  const int NS = nchunks * NSL;  // 16-deep K slices of the whole reduction

  // ---- A: this wave's fragment stream(s), 1 KB per slice, lane-linear
  const i32x4_t rsA = raw_rsrc(a.w, a.w_bytes);
  int vA[MW];
#pragma unroll
  for (int mw = 0; mw < MW; ++mw) vA[mw] = ((bm0 >> 5) + cw * MW + mw) * NS * 1024 + lane * 16;

  // ---- halo: piece q of this wave = slots g*64 .. +63 of a halo buffer, g = wave + NW q
  int hpix[NHPW], hch[NHPW];
#pragma unroll
  for (int q = 0; q < NHPW; ++q) {
    const int g = wave + NW * q;
    const int hr = g / PPR, sr = (g - hr * PPR) * 64 + lane;
    const int hc = sr / 9, ch = sr - hc * 9;
    hpix[q] = -1;
    hch[q] = ch * 8;
    if (g < NHP && ch < 8 && hc < HWD) {
      const int y = y0 + hr - PH, x = x0 + hc - PW;
      if (y >= 0 && y < H && x >= 0 && x < W) hpix[q] = (img * H + y) * W + x;
    }
  }
  const int wbase = wave * 64;
  // halo pieces [Q0, Q0 + NQ) of chunk CQ into the halo buffer at slot HBASE
#define V3_ISSUE_H(CQ, HBASE, Q0, NQ)                                                          \
  do {                                                                                         \
    const int cq_ = (CQ);                                                                      \
    const int si_ = cq_ < e1 ? 0 : (cq_ < e2 ? 1 : 2);                                         \
    const int c0_ = (cq_ - (si_ == 0 ? 0 : (si_ == 1 ? e1 : e2))) * 64;                        \
    const bool live_ = cq_ < nchunks;                                                          \
    const int sst_ = si_ == 0 ? st0 : (si_ == 1 ? st1 : st2);                                  \
    const __amdgpu_buffer_rsrc_t rb_ = __builtin_amdgcn_make_buffer_rsrc(                      \
        (void*)(si_ == 0 ? sp0 : (si_ == 1 ? sp1 : sp2)), (short)0,                            \
        si_ == 0 ? sb0 : (si_ == 1 ? sb1 : sb2), 0x00020000);                                  \
    _Pragma("unroll") for (int q = (Q0); q < (Q0) + (NQ); ++q) {                               \
      const int v_ = (live_ && hpix[q] >= 0) ? (hpix[q] * sst_ + hch[q]) * 2 : kFar;           \
      bdma16(rb_, lds + (HBASE) + wbase + NW * 64 * q, v_, c0_ * 2);                            \
    }                                                                                          \
  } while (0)

  // ---- B fragment read bases (bytes, LDS): halo buffer 0, patch row nb, column l32, chunk h
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) uint4*)&lds[0];
  const int h = lane >> 5, l32 = lane & 31;
  uint32_t bro[THW];
#pragma unroll
  for (int nb = 0; nb < THW; ++nb) bro[nb] = lds0 + (uint32_t)(((pw * THW + nb) * ROWSL + l32 * 9 + h) * 16);

  f32x16_t acc[MW][THW];
#pragma unroll
  for (int mw = 0; mw < MW; ++mw)
#pragma unroll
    for (int nb = 0; nb < THW; ++nb)
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[mw][nb][j] = 0.f;

  u32x4_t Ar[RA][MW];
  u32x4_t Bf[2][THW];

  // A fragments of slice (chunk base + SREL) into ring slot SL (vAc: chunk base offsets)
#define V3_LDA(SREL, SL)                                                                       \
  _Pragma("unroll") for (int mw = 0; mw < MW; ++mw)                                            \
    asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen"                                     \
                 : "=v"(Ar[SL][mw])                                                            \
                 : "v"(vAc[mw] + (SREL) * 1024), "s"(rsA)                                      \
                 : "memory")
  // B fragments of slice position J (tap J/4, 16-ch slice J%4) from the halo buffer at byte DB
#define V3_RDB(FB, DB, J)                                                                      \
  do {                                                                                         \
    constexpr int tp_ = (J) / 4, ks_ = (J) % 4;                                                \
    constexpr int toff_ = ((tp_ / KW) * ROWSL + (tp_ % KW) * 9 + 2 * ks_) * 16;                \
    _Pragma("unroll") for (int nb = 0; nb < THW; ++nb)                                          \
      asm volatile("ds_read_b128 %0, %1 offset:%2"                                             \
                   : "=v"(Bf[FB][nb]) : "v"(bro[nb] + (DB)), "i"(toff_) : "memory");           \
  } while (0)
#define V3_FENCE_A(SL)                                                                         \
  _Pragma("unroll") for (int mw = 0; mw < MW; ++mw) asm volatile("" : "+v"(Ar[SL][mw]))
#define V3_FENCE_B(FB)                                                                         \
  _Pragma("unroll") for (int nb = 0; nb < THW; ++nb) asm volatile("" : "+v"(Bf[FB][nb]))

  // ---- prologue: chunk-0 halo into buffer 0, A slices 0 .. D-1
  int vAc[MW];
#pragma unroll
  for (int mw = 0; mw < MW; ++mw) vAc[mw] = vA[mw];
  V3_ISSUE_H(0, 0, 0, NHPW);
#pragma unroll
  for (int sr = 0; sr < D; ++sr) V3_LDA(sr, sr);
  wait_vmcnt<D * MW>();
  asm volatile("s_barrier" ::: "memory");
  V3_RDB(0, 0u, 0);
  wait_lgkm<0>();
  V3_FENCE_B(0);

  // one slice at position J of chunk cc (halo buffer at byte dcur, the other at dnxt)
#define V3_SLICE(J)                                                                            \
  if constexpr ((J) < NSL) {                                                                   \
    constexpr int sa_ = ((J) + D) % RA, sc_ = (J) % RA, fb_ = (J) & 1;                         \
    V3_LDA((J) + D, sa_);                                                                      \
    if constexpr (C::hcnt(J) > 0) V3_ISSUE_H(cc + 1, hnxt, (J) * PPP, C::hcnt(J));             \
    if constexpr ((J) + 1 < NSL) V3_RDB(fb_ ^ 1, dcur, (J) + 1);                               \
    wait_vmcnt<(J) + 1 == NSL ? C::bwait() : C::nwait(J)>();                                   \
    V3_FENCE_A(sc_);                                                                           \
    if constexpr ((J) + 1 == NSL) {                                                            \
      if (cc + 1 < nchunks) {                                                                  \
        asm volatile("s_barrier" ::: "memory");                                                \
        V3_RDB(0, dnxt, 0);                                                                    \
      }                                                                                        \
    }                                                                                          \
    __builtin_amdgcn_sched_barrier(0);                                                         \
    _Pragma("unroll") for (int nb = 0; nb < THW; ++nb)                                          \
      _Pragma("unroll") for (int mw = 0; mw < MW; ++mw)                                        \
        acc[mw][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(                                 \
            __builtin_bit_cast(bf16x8_t, Ar[sc_][mw]), __builtin_bit_cast(bf16x8_t, Bf[fb_][nb]), \
            acc[mw][nb], 0, 0, 0);                                                             \
    __builtin_amdgcn_sched_barrier(0);                                                         \
    wait_lgkm<0>();                                                                            \
    V3_FENCE_B(fb_ ^ 1);                                                                       \
  }
#define V3_TAP(TT) V3_SLICE(4 * (TT)) V3_SLICE(4 * (TT) + 1) V3_SLICE(4 * (TT) + 2) V3_SLICE(4 * (TT) + 3)

  for (int cc = 0; cc < nchunks; ++cc) {
    const int hb = cc & 1;
    const uint32_t dcur = hb ? (uint32_t)(HSL * 16) : 0u, dnxt = hb ? 0u : (uint32_t)(HSL * 16);
    const int hnxt = hb ? 0 : HSL;  // slot base of the other halo buffer
#pragma unroll
    for (int mw = 0; mw < MW; ++mw) vAc[mw] = vA[mw] + cc * NSL * 1024;
    V3_TAP(0) V3_TAP(1) V3_TAP(2) V3_TAP(3) V3_TAP(4) V3_TAP(5) V3_TAP(6) V3_TAP(7) V3_TAP(8)
  }
#undef V3_TAP
#undef V3_SLICE
#undef V3_FENCE_B
#undef V3_FENCE_A
#undef V3_RDB
#undef V3_LDA
#undef V3_ISSUE_H
  // drain the trailing (out-of-range) A loads and halo pieces before the
  // workgroup ends (LDS-DMA must not land after the LDS is reallocated)
  wait_vmcnt<0>();

  // ---- epilogue: n-block nb = patch row nb, column l32
  int pp[THW], pb[THW], py[THW], px[THW];
#pragma unroll
  for (int nb = 0; nb < THW; ++nb) {
    const int y = y0 + pw * THW + nb, x = x0 + l32;
    if (y < H && x < W) {
      pb[nb] = img;
      py[nb] = y;
      px[nb] = x;
      pp[nb] = (img * H + y) * W + x;
    } else {
      pb[nb] = -1;
      py[nb] = px[nb] = pp[nb] = 0;
    }
  }
  epilogue32<THW>(a, acc[0], bm0 + cw * MW * 32, lane, pp, pb, py, px);
  if constexpr (MW > 1) epilogue32<THW>(a, acc[1], bm0 + (cw * MW + 1) * 32, lane, pp, pb, py, px);
}

}  // namespace conv

// tile -> (waves along Cout, 32-row fragments per wave, patch rows per wave, waves along the patch rows)
inline bool v3_geom(int tile, int* nwm, int* mw, int* thw, int* nwp) {
  *nwp = 1;
  *mw = 1;
  switch (tile) {
    case 56: *nwm = 4; *thw = 1; return true;  // one patch row: 4x the blocks of 61 (batch-1 grids)
    case 57: *nwm = 4; *thw = 2; return true;
    case 61: *nwm = 4; *thw = 3; return true;
    case 65: *nwm = 2; *thw = 3; return true;
    case 66: *nwm = 4; *thw = 3; *nwp = 2; return true;
    case 68: *nwm = 2; *thw = 3; *nwp = 4; return true;
    default: return false;  // (60, 62-64, 67: measured, never selected, dropped in round 6)
  }
}

// conv_v3_k{33,15,51}.hip: one translation unit per kernel shape (parallel build)
#define RS_V3_LAUNCHER(NAME, KH_, KW_)                                                             \
  bool NAME(const conv::Args& a, int tile, hipStream_t stream) {                                   \
    int nwm, mw, thw, nwp;                                                                         \
    if (!v3_geom(tile, &nwm, &mw, &thw, &nwp)) return false;                                       \
    const dim3 grid(cdiv(a.Cout, 32 * nwm * mw) * a.B * cdiv(a.H, thw * nwp) * cdiv(a.W, 32));     \
    const dim3 block(64 * nwm * nwp);                                                              \
    constexpr int R1 = KH_ * KW_ == 9 ? 12 : 10;                                                   \
    switch (tile) {                                                                                \
      case 56: hipLaunchKernelGGL((conv::conv_v3_kernel<KH_, KW_, 4, 1, 1, R1>), grid, block, 0, stream, a); break; \
      case 57: hipLaunchKernelGGL((conv::conv_v3_kernel<KH_, KW_, 4, 1, 2, R1>), grid, block, 0, stream, a); break; \
      case 61: hipLaunchKernelGGL((conv::conv_v3_kernel<KH_, KW_, 4, 1, 3, R1>), grid, block, 0, stream, a); break; \
      case 65: hipLaunchKernelGGL((conv::conv_v3_kernel<KH_, KW_, 2, 1, 3, R1>), grid, block, 0, stream, a); break; \
      case 66: hipLaunchKernelGGL((conv::conv_v3_kernel<KH_, KW_, 4, 1, 3, R1, 2>), grid, block, 0, stream, a); break; \
      default: hipLaunchKernelGGL((conv::conv_v3_kernel<KH_, KW_, 2, 1, 3, R1, 4>), grid, block, 0, stream, a); break; \
    }                                                                                              \
    return true;                                                                                   \
  }
bool conv_v3_launch_k33(const conv::Args& a, int tile, hipStream_t stream);
bool conv_v3_launch_k15(const conv::Args& a, int tile, hipStream_t stream);
bool conv_v3_launch_k51(const conv::Args& a, int tile, hipStream_t stream);
}  // namespace rs
