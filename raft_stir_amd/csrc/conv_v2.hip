// Lean implicit-GEMM convolution for the update-block 3x3 / 1x5 / 5x1 convs
// (reference core/update.py:6-136), tiles 42-45 of conv_fused.
//
// profiles/conv_tiles_r2.md: at the inference grid (~1 block per CU, one
// wave per SIMD) the earlier kernels are ISSUE bound -- ~100 scalar + ~60
// vector instructions of K-walk bookkeeping around 16 MFMA issue slots per
// K step.  This kernel is built so that the steady state is almost only
// MFMAs, ds_reads with immediate offsets and a few LDS-DMA pieces:
//  * (KH, KW) are template parameters: the tap loop is fully unrolled inside a
//    runtime loop over 64-channel chunks; every per-step quantity (tap shift,
//    ring slot of the halo, DMA piece counts, vmcnt immediates) is a
//    compile-time constant.
//  * v_mfma_f32_32x32x16_bf16 (32 issue cycles, 24 of them free for other
//    instructions); a wave owns 32 output channels x 64 pixels (two 32x32
//    accumulators).
//  * B (pixels): the block's TH x 32 patch of one image; per 64-channel chunk
//    its (TH+KH-1) x (32+KW-1) halo is copied once into LDS (buffer_load ...
//    lds; pixels outside the image read past the buffer end = zeros) and
//    every tap reads its shifted window from there.  Halo pixels are 144-B
//    LDS rows (8 data chunks + 1 pad chunk): 32 consecutive pixels then hit
//    32 distinct 16-B bank slots per lane group at ANY tap shift, so the tap
//    shift is a pure ds_read immediate.  Two halo buffers: the next chunk's
//    pieces ride along with the weight groups of taps S-1 .. T-1.
//  * A (weights): the only per-step stream, BM rows x 64 channels, an S-slot
//    ring (S-1 steps of lookahead), 128-B rows with the (row>>1)&7 chunk XOR
//    (conflict-free for the aligned 32-row A reads).
//  * fragments are double-buffered at K=16 granularity: the reads of the
//    next 16-deep slice are in flight while the MFMAs of this one run; the
//    one barrier per K step sits before the first slice of the next step.
//  * steps past the end and halo pieces past the last chunk are issued as
//    out-of-range (zero, no traffic) copies so every group has the same
//    compile-time DMA count.
#include "conv_common.h"

namespace rs {
namespace conv {

template <int KH, int KW, int NWM, int NWN, int S, int MW = 1>
struct V2 {
  static constexpr int T = KH * KW;
  static constexpr int NW = NWM * NWN, NT = 64 * NW;
  static constexpr int BM = 32 * NWM * MW;     // output channels per block (a wave: 32 MW)
  static constexpr int TH = 2 * NWN, TW = 32;  // pixel patch (a wave: 2 patch rows)
  static constexpr int HH = TH + KH - 1, HWD = TW + KW - 1;
  static constexpr int PPR = (HWD * 9 + 63) / 64;        // DMA pieces per halo row
  static constexpr int NHP = HH * PPR;                   // halo pieces per chunk
  static constexpr int NHPW = (NHP + NW - 1) / NW;       // ... per wave (last ones may be padding)
  static constexpr int HSL = NHPW * NW * 64;             // 16-B slots per halo buffer
  static constexpr int ROWSL = PPR * 64;                 // slots per halo row
  static constexpr int ASL = BM * 8;                     // slots per weight stage
  static constexpr int NAPW = ASL / 64 / NW;             // weight pieces per wave per step
  static constexpr int NTH = T - S + 1;                  // taps carrying next-chunk halo pieces
  static constexpr int LDS_SLOTS = S * ASL + 2 * HSL;
  static_assert(S >= 2 && T >= S, "ring depth vs taps");
  static_assert(ASL % (64 * NW) == 0, "weight pieces per wave");
  // halo piece q of a wave goes with tap S-1 + (q % NTH) (taps >= S-1: the
  // slot it overwrites was last read before that step's barrier)
  static constexpr int hp_at(int t) {
    int n = 0;
    for (int q = 0; q < NHPW; ++q)
      if (t >= S - 1 && S - 1 + (q % NTH) == t) ++n;
    return n;
  }
  static constexpr int group_cnt(int t) { return NAPW + hp_at(t); }
  // DMA instructions of groups d = 2 .. S-1 steps after tap t (allowed in flight
  // while waiting for the group one step after t)
  static constexpr int pend_after(int t) {
    int n = 0;
    for (int d = 2; d <= S - 1; ++d) n += group_cnt((t + d) % T);
    return n;
  }
  static constexpr int pend_prologue() {
    int n = 0;
    for (int d = 1; d <= S - 1; ++d) n += group_cnt(d % T);
    return n;
  }
};

template <int KH, int KW, int NWM, int NWN, int S, int MW = 1>
__global__ __launch_bounds__(64 * NWM * NWN) void conv_v2_kernel(Args a) {
  using C = V2<KH, KW, NWM, NWN, S, MW>;
  constexpr int T = C::T, NW = C::NW, NT = C::NT, BM = C::BM, TH = C::TH, TW = C::TW;
  constexpr int HWD = C::HWD, PPR = C::PPR, NHP = C::NHP, NHPW = C::NHPW, HSL = C::HSL;
  constexpr int ROWSL = C::ROWSL, ASL = C::ASL, NAPW = C::NAPW, NTH = C::NTH;
  constexpr int PH = KH / 2, PW = KW / 2;
  constexpr int kFar = 0x7ffffff0;
  __shared__ uint4 lds[C::LDS_SLOTS];

  const int t_ = threadIdx.x, lane = t_ & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t_ >> 6);
  const int wm = wave % NWM, wn = wave / NWM;
  const int H = a.H, W = a.W, Ktot = a.Ktot;
  const int ntx = cdiv(W, TW), npb = cdiv(H, TH) * ntx;
  const int nct = cdiv(a.Cout, BM);
  const int lid = a.xcd_remap ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int bm0 = (lid % nct) * BM;
  const int pt = lid / nct;
  const int img = pt / npb, pq = pt - img * npb;
  const int pty = pq / ntx;
  const int y0 = pty * TH, x0 = (pq - pty * ntx) * TW;

  // kernel arguments copied to scalars once; buffer descriptors are rebuilt
  // (4 SALU) at each use rather than selected among live descriptors
  const bf16_t* const wp = a.w;
  const unsigned wbytes = a.w_bytes;
  const bf16_t *const sp0 = a.seg[0].ptr, *const sp1 = a.seg[1].ptr, *const sp2 = a.seg[2].ptr;
  const unsigned sb0 = a.seg_bytes[0], sb1 = a.seg_bytes[1], sb2 = a.seg_bytes[2];
  const int st0 = a.seg[0].stride, st1 = a.seg[1].stride, st2 = a.seg[2].stride;
  const int e1 = a.seg[0].C >> 6;
  const int e2 = e1 + (a.nseg > 1 ? (a.seg[1].C >> 6) : 0);
  const int nchunks = e2 + (a.nseg > 2 ? (a.seg[2].C >> 6) : 0);

  // ---- per-lane DMA sources (fixed for the whole K loop)
  // weights: piece p of this wave = slots g*64 .. +63, g = wave + NW p: row g*8 + lane/8,
  // physical chunk lane%8 holding logical chunk (lane%8) ^ ((row>>1)&7)
  int aoff[NAPW];
#pragma unroll
  for (int p = 0; p < NAPW; ++p) {
    const int g = wave + NW * p, r = g * 8 + (lane >> 3);
    aoff[p] = ((bm0 + r) * T * Ktot + (((lane & 7) ^ ((r >> 1) & 7)) * 8)) * 2;
  }
  // halo: piece q of this wave = slots g*64 .. +63 of the halo buffer, g = wave + NW q:
  // halo row g / PPR, slot-in-row (g % PPR)*64 + lane -> pixel /9, chunk %9 (8 = pad)
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

  // chunk q -> (segment, channel offset inside it, K offset in the packed weights)
#define RS_CHUNK(Q, SI, C0, KK)                                                  \
  do {                                                                           \
    const int q_ = (Q);                                                          \
    SI = q_ < e1 ? 0 : (q_ < e2 ? 1 : 2);                                        \
    const int st_ = SI == 0 ? 0 : (SI == 1 ? e1 : e2);                           \
    C0 = (q_ - st_) * 64;                                                        \
    KK = q_ * 64;                                                                \
  } while (0)

  uint4* const ldsA = lds;
  uint4* const ldsH = lds + S * ASL;
  const int wbase = wave * 64;

  // weights of step (chunk q, tap t) into ring slot sl (q >= nchunks: zeros)
#define RS_ISSUE_A(Q, TAP, SL)                                                               \
  do {                                                                                       \
    const int kk_ = (Q) * 64;                                                                \
    const int so_ = (Q) < nchunks ? ((TAP) * Ktot + kk_) * 2 : kFar;                         \
    const __amdgpu_buffer_rsrc_t rw_ = __builtin_amdgcn_make_buffer_rsrc((void*)wp, (short)0, wbytes, 0x00020000); \
    _Pragma("unroll") for (int p = 0; p < NAPW; ++p)                                         \
      bdma16(rw_, ldsA + (SL) * ASL + wbase + NW * 64 * p, aoff[p], so_);                   \
  } while (0)
  // halo pieces q with P(q) true of chunk Q into halo buffer HB
#define RS_ISSUE_H(Q, HB, PRED)                                                              \
  do {                                                                                       \
    int si_, c0_, kq_;                                                                       \
    RS_CHUNK((Q), si_, c0_, kq_);                                                            \
    (void)kq_;                                                                               \
    const bool live_ = (Q) < nchunks;                                                        \
    const int sst_ = si_ == 0 ? st0 : (si_ == 1 ? st1 : st2);                                \
    const __amdgpu_buffer_rsrc_t rb_ = __builtin_amdgcn_make_buffer_rsrc(                    \
        (void*)(si_ == 0 ? sp0 : (si_ == 1 ? sp1 : sp2)), (short)0,                          \
        si_ == 0 ? sb0 : (si_ == 1 ? sb1 : sb2), 0x00020000);                                \
    _Pragma("unroll") for (int q = 0; q < NHPW; ++q) {                                       \
      if (PRED) {                                                                            \
        const int v_ = (live_ && hpix[q] >= 0) ? (hpix[q] * sst_ + hch[q]) * 2 : kFar;       \
        bdma16(rb_, ldsH + (HB) * HSL + wbase + NW * 64 * q, v_, c0_ * 2);                   \
      }                                                                                      \
    }                                                                                        \
  } while (0)

  // ---- fragment read addresses (bytes, LDS)
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) uint4*)&lds[0];
  const int h = lane >> 5, l32 = lane & 31;
  uint32_t aro[MW][4];  // A row (wm*32*MW + mw*32 + l32), chunk 2ks+h, XOR-swizzled; + slot base at read time
#pragma unroll
  for (int mw = 0; mw < MW; ++mw)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int r = (wm * MW + mw) * 32 + l32;
      aro[mw][ks] = lds0 + (uint32_t)(r * 128 + (((2 * ks + h) ^ ((r >> 1) & 7)) * 16));
    }
  uint32_t bro[2][2];  // [halo buffer][n-block]: halo pixel (patch row, column l32), chunk h
#pragma unroll
  for (int hb = 0; hb < 2; ++hb)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
      bro[hb][nb] = lds0 + (uint32_t)((S * ASL + hb * HSL + (wn * 2 + nb) * ROWSL + l32 * 9 + h) * 16);

  f32x16_t acc[MW][2];
#pragma unroll
  for (int mw = 0; mw < MW; ++mw)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[mw][nb][j] = 0.f;

  u32x4_t F[2][MW + 2];  // [buffer][A_0 .. A_MW-1, B0, B1]
  // read the K=16 slice ks of tap TAP from weight slot SL and halo buffer HB into F[FB]
#define RS_READ(FB, SL, HB, TAP, KS)                                                         \
  do {                                                                                       \
    constexpr int toff_ = (((TAP) / KW) * ROWSL + ((TAP) % KW) * 9 + 2 * (KS)) * 16;         \
    asm volatile("ds_read_b128 %0, %1" : "=v"(F[FB][0]) : "v"(aro[0][KS] + (SL) * ASL * 16) : "memory"); \
    if constexpr (MW > 1)                                                                    \
      asm volatile("ds_read_b128 %0, %1" : "=v"(F[FB][1]) : "v"(aro[1][KS] + (SL) * ASL * 16) : "memory"); \
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(F[FB][MW]) : "v"(bro[HB][0]), "i"(toff_) : "memory"); \
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(F[FB][MW + 1]) : "v"(bro[HB][1]), "i"(toff_) : "memory"); \
  } while (0)
#define RS_MMA1(FB, MI, NB)                                                                  \
  acc[MI][NB] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, F[FB][MI]),  \
                                                        __builtin_bit_cast(bf16x8_t, F[FB][MW + (NB)]), \
                                                        acc[MI][NB], 0, 0, 0)
#define RS_MMA(FB)                                                                           \
  do {                                                                                       \
    RS_MMA1(FB, 0, 0);                                                                       \
    RS_MMA1(FB, 0, 1);                                                                       \
    if constexpr (MW > 1) {                                                                  \
      RS_MMA1(FB, 1, 0);                                                                     \
      RS_MMA1(FB, 1, 1);                                                                     \
    }                                                                                        \
  } while (0)
#define RS_FENCE(FB)                                                                         \
  do {                                                                                       \
    asm volatile("" : "+v"(F[FB][0]), "+v"(F[FB][MW]), "+v"(F[FB][MW + 1]));                 \
    if constexpr (MW > 1) asm volatile("" : "+v"(F[FB][1]));                                  \
  } while (0)

  // ---- prologue: chunk-0 halo, groups 0 .. S-1 (all in chunk 0 since S <= T)
  RS_ISSUE_H(0, 0, true);
#pragma unroll
  for (int j = 0; j < S; ++j) {
    RS_ISSUE_A(0, j, j);
    RS_ISSUE_H(1, 1, j >= S - 1 && S - 1 + (q % NTH) == j);
  }
  wait_vmcnt<C::pend_prologue()>();
  asm volatile("s_barrier" ::: "memory");
  RS_READ(0, 0, 0, 0, 0);
  wait_lgkm<0>();
  RS_FENCE(0);

  // ---- main loop: runtime over chunks, unrolled over taps and K=16 slices.
  // Ring slot of step j = c*T + t is j % S; tracked as a scalar base (slot0 of
  // the chunk) so the per-tap slot is (slot0 + t) % S.
  // one K=16 slice: read the next slice (or, at ks 3, wait + barrier + refill
  // the ring + read the next step's first slice), then the MFMAs of this one
#define RS_KS(TT, KS)                                                                        \
  do {                                                                                       \
    constexpr int cur_ = (KS) & 1, nxt_ = cur_ ^ 1;                                          \
    if constexpr ((KS) < 3) {                                                                \
      RS_READ(nxt_, sl, hb, (TT), (KS) + 1);                                                 \
    } else {                                                                                 \
      if ((TT) + 1 < T || c + 1 < nchunks) {                                                 \
        wait_vmcnt<C::pend_after(TT)>();                                                     \
        asm volatile("s_barrier" ::: "memory");                                              \
        constexpr int tS_ = ((TT) + S) % T, dc_ = ((TT) + S) / T;                            \
        RS_ISSUE_A(c + dc_, tS_, sl);                                                        \
        RS_ISSUE_H(c + dc_ + 1, (c + dc_ + 1) & 1, tS_ >= S - 1 && S - 1 + (q % NTH) == tS_); \
        const int sn_ = sl + 1 == S ? 0 : sl + 1;                                            \
        if constexpr ((TT) + 1 < T) {                                                        \
          RS_READ(nxt_, sn_, hb, (TT) + 1, 0);                                               \
        } else {                                                                             \
          RS_READ(nxt_, sn_, hb ^ 1, 0, 0);                                                  \
        }                                                                                    \
      }                                                                                      \
    }                                                                                        \
    RS_MMA(cur_);                                                                            \
    __builtin_amdgcn_sched_barrier(0);                                                       \
    wait_lgkm<0>();                                                                          \
    RS_FENCE(nxt_);                                                                          \
  } while (0)
#define RS_TAP(TT)                                                                           \
  if constexpr ((TT) < T) {                                                                  \
    const int sl = (slot0 + (TT)) % S;                                                       \
    RS_KS(TT, 0);                                                                            \
    RS_KS(TT, 1);                                                                            \
    RS_KS(TT, 2);                                                                            \
    RS_KS(TT, 3);                                                                            \
  }
  static_assert(T <= 9, "taps");
  static_assert(MW == 1 || MW == 2, "MW");
  int slot0 = 0;
  for (int c = 0; c < nchunks; ++c) {
    const int hb = c & 1;
    RS_TAP(0) RS_TAP(1) RS_TAP(2) RS_TAP(3) RS_TAP(4) RS_TAP(5) RS_TAP(6) RS_TAP(7) RS_TAP(8)
    slot0 = (slot0 + T) % S;
  }
#undef RS_TAP
#undef RS_KS
#undef RS_FENCE
#undef RS_MMA
#undef RS_MMA1
#undef RS_READ
#undef RS_ISSUE_H
#undef RS_ISSUE_A
#undef RS_CHUNK

  // ---- epilogue: n-block nb = patch row wn*2 + nb, column l32
  int pp[2], pb[2], py[2], px[2];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    const int y = y0 + wn * 2 + nb, x = x0 + l32;
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
  epilogue32<2>(a, acc[0], bm0 + wm * MW * 32, lane, pp, pb, py, px);
  if constexpr (MW > 1) epilogue32<2>(a, acc[1], bm0 + (wm * MW + 1) * 32, lane, pp, pb, py, px);
}

}  // namespace conv

bool conv_v2_launch(const conv::Args& a, int tile, hipStream_t stream) {
  // tile 42: 2x2 waves (64 Cout x 4x32 px, 4-slot ring); 43: 1x4 (32 x 8x32);
  // 44: 4x1 (128 x 2x32); 45 / 46 / 47: 2x2 with a 3 / 5 / 6-slot ring (47: 5 for 5 taps)
  // 48 / 49: 2x2 waves of 64 Cout x 2x32 px (two A fragments per wave, 128 Cout x 4x32 px
  // per block; 3 / 2-slot ring); 50: 4x1 waves of 64 x 2x32 (256 Cout x 2x32 px, 3 slots)
  // 51 / 52: 4x2 waves of 64 Cout x 2x32 px (256 Cout x 4x32 px per block, 8 waves; 2 / 3-slot ring,
  // 5x1: 2 slots -- its 8-row halo leaves no room for a third); 53: 4x2 waves of 32 x 2x32 (128 x 4x32, 2 slots);
  // 54: 3x2 waves of 64 x 2x32 (192 Cout x 4x32 px, 6 waves, 3 / 2-slot ring) for the 192-channel convs
  // (convc2 forward and input gradients), which a 256-Cout tile pads by a third.
  // 51-53 stage each weight tile once for 128 pixels x all (or 128) output channels: the fewest staged bytes
  // per MAC of the family at the training grid (8 x 46 x 62: 192 blocks, one round on 256 CUs)
  const int mw = ((tile >= 48 && tile <= 52) || tile == 54) ? 2 : 1;
  const int nwm = tile == 43 ? 1 : tile == 54 ? 3 : (tile == 44 || tile >= 50) ? 4 : 2;
  const int nwn = tile == 43 ? 4 : (tile == 44 || tile == 50) ? 1 : 2;
  const int BM = 32 * nwm * mw, TH = 2 * nwn;
  const dim3 grid(cdiv(a.Cout, BM) * a.B * cdiv(a.H, TH) * cdiv(a.W, 32));
  const dim3 block(64 * nwm * nwn);
#define RS_V2(KH_, KW_)                                                                                  \
  switch (tile) {                                                                                        \
    case 42: hipLaunchKernelGGL((conv::conv_v2_kernel<KH_, KW_, 2, 2, 4>), grid, block, 0, stream, a); break; \
    case 43: hipLaunchKernelGGL((conv::conv_v2_kernel<KH_, KW_, 1, 4, 4>), grid, block, 0, stream, a); break; \
    case 44: hipLaunchKernelGGL((conv::conv_v2_kernel<KH_, KW_, 4, 1, 4>), grid, block, 0, stream, a); break; \
    case 46: hipLaunchKernelGGL((conv::conv_v2_kernel<KH_, KW_, 2, 2, 5>), grid, block, 0, stream, a); break; \
    case 47: hipLaunchKernelGGL((conv::conv_v2_kernel<KH_, KW_, 2, 2, (KH_ * KW_ >= 6 ? 6 : 5)>), grid, block, 0, stream, a); break; \
    case 48: hipLaunchKernelGGL((conv::conv_v2_kernel<KH_, KW_, 2, 2, 3, 2>), grid, block, 0, stream, a); break; \
    case 49: hipLaunchKernelGGL((conv::conv_v2_kernel<KH_, KW_, 2, 2, 2, 2>), grid, block, 0, stream, a); break; \
    case 50: hipLaunchKernelGGL((conv::conv_v2_kernel<KH_, KW_, 4, 1, 3, 2>), grid, block, 0, stream, a); break; \
    case 51: hipLaunchKernelGGL((conv::conv_v2_kernel<KH_, KW_, 4, 2, 2, 2>), grid, block, 0, stream, a); break; \
    case 52: hipLaunchKernelGGL((conv::conv_v2_kernel<KH_, KW_, 4, 2, (KH_ == 5 ? 2 : 3), 2>), grid, block, 0, stream, a); break; \
    case 53: hipLaunchKernelGGL((conv::conv_v2_kernel<KH_, KW_, 4, 2, 2, 1>), grid, block, 0, stream, a); break; \
    case 54: hipLaunchKernelGGL((conv::conv_v2_kernel<KH_, KW_, 3, 2, (KH_ == 5 ? 2 : 3), 2>), grid, block, 0, stream, a); break; \
    default: hipLaunchKernelGGL((conv::conv_v2_kernel<KH_, KW_, 2, 2, 3>), grid, block, 0, stream, a); break; \
  }
  if (a.KH == 3 && a.KW == 3) {
    RS_V2(3, 3);
  } else if (a.KH == 1 && a.KW == 5) {
    RS_V2(1, 5);
  } else if (a.KH == 5 && a.KW == 1) {
    RS_V2(5, 1);
  } else {
    return false;
  }
#undef RS_V2
  return true;
}

}  // namespace rs
