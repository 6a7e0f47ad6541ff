// fp32 weight-streaming convolution: the conv_v3.h design (each wave streams
// its own output channels' weight fragments global -> VGPR, the activation
// halo is the only shared LDS operand, one barrier per 64-channel chunk) for
// the fp32 engines' update-block 3x3 / 1x5 / 5x1 convs (reference
// core/update.py:6-136 at the reference's default fp32 precision), tiles 81-83
// of conv_fused.  The product is the split-bf16 one of the F32 register tiles,
//
//   x.w ~= xh.wh + xl.wh + xh.wl       (xh = rne(x), xl = rne(x - xh), same for w)
//
// three v_mfma_f32_32x32x16_bf16 per fragment pair with fp32 accumulation:
//  * the weights arrive pre-split in the fragment-major layout, hi blocks then
//    lo blocks (ops/conv.py frag_weight_split): two 1 KB A fragments per
//    16-deep K slice per wave, streamed through a register ring;
//  * the activations stay fp32 in memory: each 64-channel chunk's halo is
//    DMA'd into LDS as fp32 (17 x 16-B slots per pixel: 64 channels + one pad
//    slot, so the 32 pixels of a fragment read hit 16 distinct 4-bank groups
//    for any tap shift), then every lane splits the slots it DMA'd itself IN
//    PLACE, 4 fp32 -> [hi x4 | lo x4] bf16 (packed v_cvt_pk_bf16_f32 / one
//    v_pk_add_f32: 5 VALU ops per 2 values, once per halo element per chunk
//    instead of once per tap read), before the chunk's barrier; a B fragment
//    is then two ds_read_b128 whose halves ARE the hi and lo operands -- no
//    split pass over the activations in memory and no second halo;
//  * the fp32 epilogues of the F32 tiles (epi_frag_f32: bias / ReLU / scale,
//    ConvGRU gates and update, ReLU backward, fp32 accumulation, the q-conv
//    r-gate backward, eval-BN scale + shift (+ ReLU, + residual)) on fp32
//    outputs.
// Tiles: 81 = 4 waves x 3 patch rows (128 Cout x 96 px), 82 = 4 waves x 1 row
// (batch-1 grids), 83 = 4 waves x 2 rows, 84 = 2 x 2 waves (64 Cout x 4 rows:
// the 64-output encoder convs without a wasted half block), 85 = 84 with one
// halo buffer (Ktot = 64 only).
#include "conv_v3.h"

namespace rs {
namespace conv {

typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

template <int KH, int KW, int NWM, int THW, int RA, int NWP, int SB>
struct V3F {
  static constexpr int T = KH * KW, NSL = 4 * T, D = RA - 1;
  static constexpr int NW = NWM * NWP;  // waves: NWM along Cout x NWP along the patch rows
  static constexpr int TH = THW * NWP, TW = 32, BM = 32 * NWM;
  static constexpr int HH = TH + KH - 1, HWD = TW + KW - 1;
  static constexpr int PS = 17;                      // 16-B slots per halo pixel (64 fp32 + 1 pad)
  static constexpr int PPR = (HWD * PS + 63) / 64;   // DMA pieces (1 KB) per halo row
  static constexpr int ROWSL = PPR * 64;             // slots per halo row
  static constexpr int NHP = HH * PPR;               // halo pieces per chunk
  static constexpr int NHPW = (NHP + NW - 1) / NW;   // ... per wave (the last may be padding)
  static constexpr int HSL = NHPW * NW * 64;         // slots per halo buffer
  static constexpr int LASTP = NSL > RA ? NSL - RA : 1;
  static constexpr int PPP = (NHPW + LASTP - 1) / LASTP;
  // SB: ONE halo buffer (single-chunk convs, Ktot = 64: no next chunk to
  // prefetch) -- half the LDS, so two blocks share a CU and one block's halo
  // load overlaps the other's MFMAs
  static constexpr int LDS_SLOTS = SB ? HSL : 2 * HSL;
  static constexpr int hcnt(int j) {
    if (SB) return 0;  // no next-chunk halo pieces inside the slice loop
    j = ((j % NSL) + NSL) % NSL;
    if (j >= LASTP) return 0;
    const int n = NHPW - j * PPP;
    return n < 0 ? 0 : (n > PPP ? PPP : n);
  }
  // VMEM instructions issued after slice j's two A loads (see V3::nwait)
  static constexpr int nwait(int j) {
    int n = 2 * D;
    for (int i = j - D; i <= j; ++i) n += hcnt(i);
    return n;
  }
  static constexpr int bwait() {
    int last = 0;
    for (int j = 0; j < NSL; ++j)
      if (hcnt(j) > 0) last = j;
    const int after = (NSL - 1 - last) * 2;
    return nwait(NSL - 1) < after ? nwait(NSL - 1) : after;
  }
  static constexpr bool counts_ok() {
    for (int j = 0; j < NSL; ++j)
      if (nwait(j) > 63) return false;
    return true;
  }
};

// acc (32 Cout x 32 pixels per 32x32 block) -> the fp32 epilogue, 4 channels per call
template <int NB, int E>
__device__ __forceinline__ void epi32_f32(const Args& a, const f32x16_t (&acc)[NB], int m0, int lane,
                                          const int (&pp)[NB], const int (&pb)[NB], bool vec) {
  const int h4 = 4 * (lane >> 5);
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    if (pb[nb] < 0) continue;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int cb = m0 + 8 * g + h4;
      if (cb >= a.Cout) continue;
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool in = cb + j < a.Cout;
        const float sc = (E == EPI_NORM && in) ? a.chs[cb + j] : 1.f;  // eval-BN scale (EPI_NORM)
        v[j] = acc[nb][4 * g + j] * sc + (in && a.bias ? a.bias[cb + j] : 0.f);
      }
      epi_frag_f32<E>(a, v, cb, pp[nb], vec);
    }
  }
}

template <int NB>
__device__ __forceinline__ void epilogue32_f32(const Args& a, const f32x16_t (&acc)[NB], int m0, int lane,
                                               const int (&pp)[NB], const int (&pb)[NB]) {
  const bool vec =
      ((a.ooff | a.ostr | a.o2off | a.o2str | a.o3off | a.o3str | a.a1off | a.a1str | a.a2off | a.a2str) & 3) == 0 &&
      (((uintptr_t)a.out | (uintptr_t)a.out2 | (uintptr_t)a.out3 | (uintptr_t)a.aux1 | (uintptr_t)a.aux2) & 15) == 0;
  switch (a.epi) {
#define RS_E3(E) \
  case E: epi32_f32<NB, E>(a, acc, m0, lane, pp, pb, vec); break
    RS_E3(EPI_GRU_ZR);
    RS_E3(EPI_GRU_Q);
    RS_E3(EPI_RELU_BWD);
    RS_E3(EPI_ACC_F32);
    RS_E3(EPI_GRU_QBWD);
    RS_E3(EPI_RELU);
    RS_E3(EPI_SCALE);
    RS_E3(EPI_NORM);
#undef RS_E3
    default: epi32_f32<NB, EPI_BIAS>(a, acc, m0, lane, pp, pb, vec); break;
  }
}

template <int KH, int KW, int NWM, int THW, int RA, int NWP = 1, int SB = 0>
__global__ __launch_bounds__(64 * NWM * NWP) void conv_v3f_kernel(Args a) {
  using C = V3F<KH, KW, NWM, THW, RA, NWP, SB>;
  constexpr int NW = C::NW, TH = C::TH, T = C::T, NSL = C::NSL, D = C::D, BM = C::BM;
  constexpr int HWD = C::HWD, PS = C::PS, PPR = C::PPR, NHP = C::NHP, NHPW = C::NHPW, HSL = C::HSL;
  constexpr int ROWSL = C::ROWSL, PPP = C::PPP;
  constexpr int PH = KH / 2, PW = KW / 2;
  constexpr int kFar = 0x7ffffff0;
  static_assert(NSL % RA == 0, "ring slots must divide the slices of a chunk");
  static_assert(C::LASTP > 0 && C::counts_ok(), "halo schedule / vmcnt range");
  static_assert(T <= 9, "taps");
  static_assert(C::LDS_SLOTS * 16 <= 160 * 1024, "LDS");
  __shared__ uint4 lds[C::LDS_SLOTS];

  const int t_ = threadIdx.x, lane = t_ & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t_ >> 6);
  const int cw = NWP == 1 ? wave : wave % NWM, pw = NWP == 1 ? 0 : wave / NWM;  // Cout slice, patch-row group
  const int H = a.H, W = a.W;
  const int ntx = cdiv(W, 32), npb = cdiv(H, TH) * ntx;
  const int nct = cdiv(a.Cout, BM);
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int bm0 = (lid % nct) * BM;
  const int pt = lid / nct;
  const int img = pt / npb, pq = pt - img * npb;
  const int pty = pq / ntx;
  const int y0 = pty * TH, x0 = (pq - pty * ntx) * 32;

  const float *const sp0 = reinterpret_cast<const float*>(a.seg[0].ptr),
              *const sp1 = reinterpret_cast<const float*>(a.seg[1].ptr),
              *const sp2 = reinterpret_cast<const float*>(a.seg[2].ptr);
  const unsigned sb0 = a.seg_bytes[0], sb1 = a.seg_bytes[1], sb2 = a.seg_bytes[2];
  const int st0 = a.seg[0].stride, st1 = a.seg[1].stride, st2 = a.seg[2].stride;
  const int e1 = a.seg[0].C >> 6;
  const int e2 = e1 + (a.nseg > 1 ? (a.seg[1].C >> 6) : 0);
  const int nchunks = e2 + (a.nseg > 2 ? (a.seg[2].C >> 6) : 0);
  const int NS = nchunks * NSL;  // 16-deep K slices of the whole reduction

  // ---- A: this wave's hi and lo fragment streams, 1 KB per slice each
  const i32x4_t rsA = raw_rsrc(a.w, a.w_bytes);
  const int vA = ((bm0 >> 5) + cw) * NS * 1024 + lane * 16;
  const int loff = (int)(a.w_bytes >> 1);  // the lo blocks follow the hi blocks

  // ---- halo: piece q of this wave = slots g*64 .. +63 of a halo buffer, g = wave + NW q
  int hpix[NHPW], hch[NHPW];
#pragma unroll
  for (int q = 0; q < NHPW; ++q) {
    const int g = wave + NW * q;
    const int hr = g / PPR, sr = (g - hr * PPR) * 64 + lane;
    const int hc = sr / PS, ch = sr - hc * PS;
    hpix[q] = -1;
    hch[q] = ch * 4;  // fp32 channel of this 16-B slot
    if (g < NHP && ch < 16 && hc < HWD) {
      const int y = y0 + hr - PH, x = x0 + hc - PW;
      if (y >= 0 && y < H && x >= 0 && x < W) hpix[q] = (img * H + y) * W + x;
    }
  }
  const int wbase = wave * 64;
#define V3F_ISSUE_H(CQ, HBASE, Q0, NQ)                                                         \
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
      const int v_ = (live_ && hpix[q] >= 0) ? (hpix[q] * sst_ + hch[q]) * 4 : kFar;           \
      bdma16(rb_, lds + (HBASE) + wbase + NW * 64 * q, v_, c0_ * 4);                            \
    }                                                                                          \
  } while (0)

  // ---- B fragment read bases (bytes): patch row nb, column l32, fp32 channels 8h .. 8h+7 of the slice
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) uint4*)&lds[0];
  const int h = lane >> 5, l32 = lane & 31;
  uint32_t bro[THW];
#pragma unroll
  for (int nb = 0; nb < THW; ++nb) bro[nb] = lds0 + (uint32_t)(((pw * THW + nb) * ROWSL + l32 * PS + 2 * h) * 16);

  f32x16_t acc[THW];
#pragma unroll
  for (int nb = 0; nb < THW; ++nb)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[nb][j] = 0.f;

  u32x4_t Ah[RA], Al[RA];
  // B fragments of the current / next slice: per patch row the two 16-B halo
  // slots of the lane's 8 channels, each [hi x4 | lo x4] (split in LDS, below)
  u32x4_t Bs[2][THW][2];

#define V3F_LDA(SREL, SL)                                                                      \
  do {                                                                                         \
    asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen"                                     \
                 : "=v"(Ah[SL]) : "v"(vAc + (SREL) * 1024), "s"(rsA) : "memory");              \
    asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen"                                     \
                 : "=v"(Al[SL]) : "v"(vAc + loff + (SREL) * 1024), "s"(rsA) : "memory");       \
  } while (0)
#define V3F_RDB(FB, DB, J)                                                                     \
  do {                                                                                         \
    constexpr int tp_ = (J) / 4, ks_ = (J) % 4;                                                \
    constexpr int toff_ = ((tp_ / KW) * ROWSL + (tp_ % KW) * PS + 4 * ks_) * 16;               \
    _Pragma("unroll") for (int nb = 0; nb < THW; ++nb) {                                        \
      asm volatile("ds_read_b128 %0, %1 offset:%2"                                             \
                   : "=v"(Bs[FB][nb][0]) : "v"(bro[nb] + (DB)), "i"(toff_) : "memory");        \
      asm volatile("ds_read_b128 %0, %1 offset:%2"                                             \
                   : "=v"(Bs[FB][nb][1]) : "v"(bro[nb] + (DB)), "i"(toff_ + 16) : "memory");   \
    }                                                                                          \
  } while (0)
#define V3F_FENCE_A(SL) asm volatile("" : "+v"(Ah[SL]), "+v"(Al[SL]))
#define V3F_FENCE_B(FB)                                                                        \
  _Pragma("unroll") for (int nb = 0; nb < THW; ++nb) asm volatile("" : "+v"(Bs[FB][nb][0]), "+v"(Bs[FB][nb][1]))
  // hi / lo bf16x8 fragments from the two [hi x4 | lo x4] slots: register selection only
#define V3F_BH(FB, NB) (u32x4_t{Bs[FB][NB][0].x, Bs[FB][NB][0].y, Bs[FB][NB][1].x, Bs[FB][NB][1].y})
#define V3F_BL(FB, NB) (u32x4_t{Bs[FB][NB][0].z, Bs[FB][NB][0].w, Bs[FB][NB][1].z, Bs[FB][NB][1].w})
#define V3F_GROUP(AF, BSEL, FB)                                                                \
  _Pragma("unroll") for (int nb = 0; nb < THW; ++nb)                                            \
    acc[nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, AF),         \
                                                      __builtin_bit_cast(bf16x8_t, BSEL(FB, nb)), acc[nb], 0, 0, 0)
  // every lane converts the halo slots it DMA'd itself, in place: 4 fp32 -> [hi x4 | lo x4]
  // (its own LDS-DMA has landed at its vmcnt wait; the following barrier publishes the result)
#define V3F_CONVERT(HBASE)                                                                     \
  _Pragma("unroll") for (int q = 0; q < NHPW; ++q) {                                            \
    uint4* sl_ = lds + (HBASE) + wbase + NW * 64 * q + lane;                                   \
    const uint4 v_ = *sl_;                                                                     \
    const f32x2_t p0_ = {__builtin_bit_cast(float, v_.x), __builtin_bit_cast(float, v_.y)};     \
    const f32x2_t p1_ = {__builtin_bit_cast(float, v_.z), __builtin_bit_cast(float, v_.w)};     \
    const uint32_t h0_ = __builtin_bit_cast(uint32_t, __builtin_convertvector(p0_, bf16x2_t)); \
    const uint32_t h1_ = __builtin_bit_cast(uint32_t, __builtin_convertvector(p1_, bf16x2_t)); \
    const f32x2_t r0_ = p0_ - f32x2_t{__builtin_bit_cast(float, h0_ << 16),                    \
                                      __builtin_bit_cast(float, h0_ & 0xffff0000u)};           \
    const f32x2_t r1_ = p1_ - f32x2_t{__builtin_bit_cast(float, h1_ << 16),                    \
                                      __builtin_bit_cast(float, h1_ & 0xffff0000u)};           \
    *sl_ = make_uint4(h0_, h1_, __builtin_bit_cast(uint32_t, __builtin_convertvector(r0_, bf16x2_t)), \
                      __builtin_bit_cast(uint32_t, __builtin_convertvector(r1_, bf16x2_t)));   \
  }

  // ---- prologue: chunk-0 halo into buffer 0 (then split in place), A slices 0 .. D-1
  int vAc = vA;
  V3F_ISSUE_H(0, 0, 0, NHPW);
#pragma unroll
  for (int sr = 0; sr < D; ++sr) V3F_LDA(sr, sr);
  wait_vmcnt<2 * D>();
  V3F_CONVERT(0);
  __syncthreads();
  V3F_RDB(0, 0u, 0);
  wait_lgkm<0>();
  V3F_FENCE_B(0);

#define V3F_SLICE(J)                                                                           \
  if constexpr ((J) < NSL) {                                                                   \
    constexpr int sa_ = ((J) + D) % RA, sc_ = (J) % RA, fb_ = (J) & 1;                         \
    V3F_LDA((J) + D, sa_);                                                                     \
    if constexpr (C::hcnt(J) > 0) V3F_ISSUE_H(cc + 1, hnxt, (J) * PPP, C::hcnt(J));            \
    if constexpr ((J) + 1 < NSL) V3F_RDB(fb_ ^ 1, dcur, (J) + 1);                              \
    wait_vmcnt<(J) + 1 == NSL ? C::bwait() : C::nwait(J)>();                                   \
    V3F_FENCE_A(sc_);                                                                          \
    if constexpr ((J) + 1 == NSL) {                                                            \
      if (cc + 1 < nchunks) {  /* the next chunk's halo: landed (bwait), split, published */   \
        V3F_CONVERT(hnxt);                                                                     \
        __syncthreads();                                                                       \
        V3F_RDB(fb_ ^ 1, dnxt, 0);                                                             \
      }                                                                                        \
    }                                                                                          \
    __builtin_amdgcn_sched_barrier(0);                                                         \
    V3F_GROUP(Ah[sc_], V3F_BH, fb_);                                                           \
    V3F_GROUP(Al[sc_], V3F_BH, fb_);                                                           \
    V3F_GROUP(Ah[sc_], V3F_BL, fb_);                                                           \
    __builtin_amdgcn_sched_barrier(0);                                                         \
    wait_lgkm<0>();                                                                            \
    V3F_FENCE_B(fb_ ^ 1);                                                                      \
  }
#define V3F_TAP(TT) V3F_SLICE(4 * (TT)) V3F_SLICE(4 * (TT) + 1) V3F_SLICE(4 * (TT) + 2) V3F_SLICE(4 * (TT) + 3)

  for (int cc = 0; cc < nchunks; ++cc) {
    const int hb = cc & 1;
    const uint32_t dcur = hb ? (uint32_t)(HSL * 16) : 0u, dnxt = hb ? 0u : (uint32_t)(HSL * 16);
    const int hnxt = hb ? 0 : HSL;
    vAc = vA + cc * NSL * 1024;
    V3F_TAP(0) V3F_TAP(1) V3F_TAP(2) V3F_TAP(3) V3F_TAP(4) V3F_TAP(5) V3F_TAP(6) V3F_TAP(7) V3F_TAP(8)
  }
#undef V3F_TAP
#undef V3F_SLICE
#undef V3F_FENCE_A
#undef V3F_FENCE_B
#undef V3F_BH
#undef V3F_BL
#undef V3F_CONVERT
#undef V3F_GROUP
#undef V3F_RDB
#undef V3F_LDA
#undef V3F_ISSUE_H
  // the trailing (out-of-range) A loads and halo pieces land before the workgroup ends
  wait_vmcnt<0>();

  int pp[THW], pb[THW];
#pragma unroll
  for (int nb = 0; nb < THW; ++nb) {
    const int y = y0 + pw * THW + nb, x = x0 + l32;
    if (y < H && x < W) {
      pb[nb] = img;
      pp[nb] = (img * H + y) * W + x;
    } else {
      pb[nb] = -1;
      pp[nb] = 0;
    }
  }
  epilogue32_f32<THW>(a, acc, bm0 + cw * 32, lane, pp, pb);
}

template <int KH, int KW>
bool v3f_launch(const Args& a, int tile, hipStream_t stream) {
  constexpr int RA = KH * KW == 9 ? 9 : 10;  // ring slots: divide the 36 / 20 slices of a chunk
  // (waves along Cout, patch rows per wave, waves along the patch rows)
  const bool t64 = tile == 84 || tile == 85;
  const int nwm = t64 ? 2 : 4, thw = tile == 81 ? 3 : (tile == 82 ? 1 : 2), nwp = t64 ? 2 : 1;
  const dim3 grid(cdiv(a.Cout, 32 * nwm) * a.B * cdiv(a.H, thw * nwp) * cdiv(a.W, 32));
  const dim3 block(64 * nwm * nwp);
  switch (tile) {
    case 81: hipLaunchKernelGGL((conv_v3f_kernel<KH, KW, 4, 3, RA>), grid, block, 0, stream, a); break;
    case 82: hipLaunchKernelGGL((conv_v3f_kernel<KH, KW, 4, 1, RA>), grid, block, 0, stream, a); break;
    case 83: hipLaunchKernelGGL((conv_v3f_kernel<KH, KW, 4, 2, RA>), grid, block, 0, stream, a); break;
    case 84: hipLaunchKernelGGL((conv_v3f_kernel<KH, KW, 2, 2, RA, 2>), grid, block, 0, stream, a); break;
    case 85: hipLaunchKernelGGL((conv_v3f_kernel<KH, KW, 2, 2, RA, 2, 1>), grid, block, 0, stream, a); break;
    default: return false;
  }
  return true;
}

}  // namespace conv

bool conv_v3f_launch(const conv::Args& a, int tile, hipStream_t stream) {
  if (a.KH == 3 && a.KW == 3) return conv::v3f_launch<3, 3>(a, tile, stream);
  if (a.KH == 1 && a.KW == 5) return conv::v3f_launch<1, 5>(a, tile, stream);
  if (a.KH == 5 && a.KW == 1) return conv::v3f_launch<5, 1>(a, tile, stream);
  return false;
}

}  // namespace rs
