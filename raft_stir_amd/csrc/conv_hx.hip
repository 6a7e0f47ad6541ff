// Pipelined halo implicit-GEMM convolution (see the comment below); tiles
// 34-39 of conv_fused (ops/conv.py choose_tile).  Reference semantics:
// the update-block convolutions of core/update.py:6-136.
#include "conv_common.h"

namespace rs {
namespace conv {

// ------------------------------------------------------------------ pipelined halo variant
// The update-block convs are bound by the L2 -> LDS fill rate (~30 B/clk/CU
// for gathered rows, profiles/conv_tiles_r2.md), so the tile is chosen to
// minimise staged bytes per MAC rather than to maximise the MFMA tile:
//  * B (pixels) is a TH x 16 patch of one image whose (TH+KH-1) x (16+KW-1)
//    halo is staged ONCE per 64-channel chunk and read by every tap of that
//    chunk from LDS (B traffic / taps);
//  * A (weights) is the only per-step stream: BM x 64 bf16, MAC/B = BN / 2,
//    so a narrow Cout tile (BM = 64) with a wide pixel patch is the cheapest
//    tile per staged byte for the 1x5 / 5x1 / 3x3 convs.
// Pipeline: an S-slot weight ring with S-1 steps of lookahead, a 2-slot halo
// ring whose next-chunk pieces ride along with the weight groups of taps
// S-1 .. taps-1 of the current chunk (host: taps >= S), per-group DMA counts
// kept in a scalar shift register so each step waits (counted vmcnt) only for
// its own group, and register double-buffered fragments: the ds_reads of step
// k+1 are in flight while the MFMAs of step k run.
// LDS rows are 128 B (64 channels); logical 16-B chunk c of row r sits at slot
// c ^ (r & 7): conflict-free ds_read_b128 for 16 consecutive rows starting
// at ANY row (the tap shift makes halo reads start anywhere).
__device__ __forceinline__ void wait_vm_rt(int n) {
  switch (n) {
#define RS_W(N) \
  case N: wait_vmcnt<N>(); break;
    RS_W(1) RS_W(2) RS_W(3) RS_W(4) RS_W(5) RS_W(6) RS_W(7) RS_W(8) RS_W(9) RS_W(10) RS_W(11) RS_W(12)
    RS_W(13) RS_W(14) RS_W(15) RS_W(16) RS_W(17) RS_W(18) RS_W(19) RS_W(20) RS_W(21) RS_W(22) RS_W(23)
    RS_W(24) RS_W(25) RS_W(26) RS_W(27) RS_W(28) RS_W(29) RS_W(30) RS_W(31) RS_W(32) RS_W(33) RS_W(34)
    RS_W(35) RS_W(36) RS_W(37) RS_W(38) RS_W(39) RS_W(40) RS_W(41) RS_W(42) RS_W(43) RS_W(44) RS_W(45)
    RS_W(46) RS_W(47) RS_W(48)
#undef RS_W
    default:
      if (n > 48) wait_vmcnt<48>();
      else wait_vmcnt<0>();
      break;
  }
}

template <int BM, int TH, int WAVES_M, int WAVES_N, int S, int HCAP, int DBG = 0>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) void conv_hx_kernel(Args a) {
  constexpr int NT = 64 * WAVES_M * WAVES_N, TW = 16;
  constexpr int WM = BM / WAVES_M / 16, WN = TH / WAVES_N;
  static_assert(BM % (WAVES_M * 16) == 0 && TH % WAVES_N == 0, "wave tiles");
  static_assert((BM * 8) % NT == 0 && (HCAP * 8) % NT == 0, "staging");
  static_assert(S >= 2 && S <= 7, "ring depth");
  constexpr int NA = BM * 8 / NT, NH = HCAP * 8 / NT;
  constexpr int AST = BM * 8, HST = HCAP * 8;  // 16-B chunks per weight slot / halo slot
  constexpr int kFar = 0x7ffffff0;
  __shared__ uint4 lds[S * AST + 2 * HST];

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave % WAVES_M, wn = wave / WAVES_M;
  const int H = a.H, W = a.W, KW = a.KW, Ktot = a.Ktot;
  const int taps = a.KH * KW;
  const int hw = TW + KW - 1;
  const int hrows = (TH + a.KH - 1) * hw;
  const int ntx = cdiv(W, TW), npb = cdiv(H, TH) * ntx;
  const int nct = cdiv(a.Cout, BM);
  const int lid = a.xcd_remap ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int bm0 = (lid % nct) * BM;
  const int pt = lid / nct;
  const int img = pt / npb, pq = pt - img * npb;
  const int pty = pq / ntx;
  const int y0 = pty * TH, x0 = (pq - pty * ntx) * TW;
  const int m0 = bm0 + wm * WM * 16;

  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, a.w_bytes, 0x00020000);
  const Seg s0 = a.seg[0], s1 = a.seg[1], s2 = a.seg[2];
  const __amdgpu_buffer_rsrc_t rs0 =
      __builtin_amdgcn_make_buffer_rsrc((void*)s0.ptr, (short)0, a.seg_bytes[0], 0x00020000);
  const __amdgpu_buffer_rsrc_t rs1 =
      __builtin_amdgcn_make_buffer_rsrc((void*)s1.ptr, (short)0, a.seg_bytes[1], 0x00020000);
  const __amdgpu_buffer_rsrc_t rs2 =
      __builtin_amdgcn_make_buffer_rsrc((void*)s2.ptr, (short)0, a.seg_bytes[2], 0x00020000);

  // staging slot (thread t, instruction i) = chunk id t + NT i: row id / 8, physical
  // 16-B slot id % 8 holding logical chunk (id % 8) ^ (row & 7)
  int aoff[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int id = t + NT * i, r = id >> 3;
    aoff[i] = ((bm0 + r) * taps * Ktot + (((id & 7) ^ (r & 7)) * 8)) * 2;
  }
  int hpix[NH], hch[NH];
#pragma unroll
  for (int i = 0; i < NH; ++i) {
    const int id = t + NT * i, r = id >> 3;
    hch[i] = ((id & 7) ^ (r & 7)) * 8;
    hpix[i] = -1;
    if (r < hrows) {
      const int hy = r / hw, hx = r - hy * hw;
      const int y = y0 + hy - a.PH, x = x0 + hx - a.PW;
      if (y >= 0 && y < H && x >= 0 && x < W) hpix[i] = (img * H + y) * W + x;
    }
  }
  const int wbase = wave * 64;
  const int nchunks = (s0.C >> 6) + (a.nseg > 1 ? (s1.C >> 6) : 0) + (a.nseg > 2 ? (s2.C >> 6) : 0);
  const int nsteps = taps * nchunks;
  const int ntaph = taps - S + 1;  // taps carrying next-chunk halo pieces (host: >= 1)

  // halo pieces of one chunk: instruction i of every thread goes with tap S-1 + min(i, ntaph-1)
#define RS_HALO(SI, C0, SLOT, COND)                                                              \
  do {                                                                                           \
    const int sst_ = (SI) == 0 ? s0.stride : ((SI) == 1 ? s1.stride : s2.stride);                \
    const __amdgpu_buffer_rsrc_t rb_ = (SI) == 0 ? rs0 : ((SI) == 1 ? rs1 : rs2);                \
    uint4* hd_ = lds + S * AST + (SLOT) * HST;                                                   \
    _Pragma("unroll") for (int i = 0; i < NH; ++i) {                                             \
      if (COND) {                                                                                \
        const int v_ = hpix[i] >= 0 ? (hpix[i] * sst_ + hch[i]) * 2 : kFar;                     \
        bdma16(rb_, hd_ + wbase + NT * i, v_, (C0) * 2);                                         \
      }                                                                                          \
    }                                                                                            \
  } while (0)

  // issue-side scalar walk over groups j = (chunk ic, tap it); next chunk's (segment, c0)
  int it = 0, ic = 0, isi = 0, ic0 = 0, ikseg = 0;
  int nsi = 0, nc0 = 0;  // chunk ic + 1
  {
    nc0 = 64;
    if (nc0 == s0.C) { nc0 = 0; nsi = 1; }
  }
  unsigned long long hist = 0ull;  // DMA instructions per issued group, youngest in the low byte
#define RS_ISSUE()                                                                               \
  do {                                                                                           \
    uint4* ad_ = lds + (jslot) * AST;                                                            \
    const int asoff_ = (it * Ktot + ikseg + ic0) * 2;                                            \
    _Pragma("unroll") for (int i = 0; i < NA; ++i) bdma16(rw, ad_ + wbase + NT * i, aoff[i], asoff_); \
    int cnt_ = NA;                                                                               \
    if (it >= S - 1 && ic + 1 < nchunks) {                                                       \
      const int u_ = it - (S - 1);                                                               \
      RS_HALO(nsi, nc0, (ic + 1) & 1, i == u_ || (u_ == ntaph - 1 && i > u_));                   \
      cnt_ += u_ < ntaph - 1 ? (u_ < NH ? 1 : 0) : (NH > u_ ? NH - u_ : 0);                       \
    }                                                                                            \
    hist = (hist << 8) | (unsigned long long)cnt_;                                               \
    jslot = jslot == S - 1 ? 0 : jslot + 1;                                                      \
    if (++it == taps) {                                                                          \
      it = 0;                                                                                    \
      ++ic;                                                                                      \
      ic0 += 64;                                                                                 \
      const int sC_ = isi == 0 ? s0.C : (isi == 1 ? s1.C : s2.C);                                \
      if (ic0 == sC_) { ic0 = 0; ikseg += sC_; ++isi; }                                          \
      nc0 += 64;                                                                                 \
      const int nC_ = nsi == 0 ? s0.C : (nsi == 1 ? s1.C : s2.C);                                \
      if (nc0 == nC_) { nc0 = 0; ++nsi; }                                                        \
    }                                                                                            \
  } while (0)

  f32x4_t acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int lr = lane & 15, lc = lane >> 4;
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) uint4*)&lds[0];
  uint32_t abase[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
    abase[kk] = lds0 + (uint32_t)((wm * WM * 16 + lr) * 128 + (((kk * 4 + lc) ^ (lr & 7)) * 16));
  // weight rows start at multiples of 16, so (row & 7) == (lr & 7) for every m-tile
  int rbn[WN];
#pragma unroll
  for (int nt = 0; nt < WN; ++nt) rbn[nt] = (wn * WN + nt) * hw + lr;

  // compute-side walk (the step whose fragments are being READ): tap (cty, ctx), chunk parity
  int cty = 0, ctx = 0, ctap = 0, cpar = 0, cslot = 0;
#define RS_READ(F)                                                                               \
  do {                                                                                           \
    const uint32_t so_ = cslot * AST * 16;                                                       \
    const uint32_t hb_ = lds0 + (uint32_t)((S * AST + cpar * HST) * 16);                         \
    const int toff_ = cty * hw + ctx;                                                            \
    _Pragma("unroll") for (int kk = 0; kk < 2; ++kk) {                                           \
      _Pragma("unroll") for (int mt = 0; mt < WM; ++mt)                                          \
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(F[kk * (WM + WN) + mt])              \
                     : "v"(abase[kk] + so_), "i"(mt * 16 * 128) : "memory");                     \
      _Pragma("unroll") for (int nt = 0; nt < WN; ++nt) {                                        \
        const int row_ = rbn[nt] + toff_;                                                        \
        asm volatile("ds_read_b128 %0, %1" : "=v"(F[kk * (WM + WN) + WM + nt])                   \
                     : "v"(hb_ + (uint32_t)(row_ * 128) + ((((uint32_t)(kk * 4 + lc)) ^ (uint32_t)(row_ & 7)) << 4)) \
                     : "memory");                                                                \
      }                                                                                          \
    }                                                                                            \
    cslot = cslot == S - 1 ? 0 : cslot + 1;                                                      \
    if (++ctx == KW) { ctx = 0; ++cty; }                                                         \
    if (++ctap == taps) { ctap = 0; cty = 0; ctx = 0; cpar ^= 1; }                               \
  } while (0)
#define RS_FENCE(F)                                                                              \
  do {                                                                                           \
    _Pragma("unroll") for (int q = 0; q < 2 * (WM + WN); ++q) asm volatile("" : "+v"(F[q]));     \
  } while (0)
#define RS_MMA(F)                                                                                \
  do {                                                                                           \
    _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                             \
      _Pragma("unroll") for (int mt = 0; mt < WM; ++mt)                                          \
        _Pragma("unroll") for (int nt = 0; nt < WN; ++nt)                                        \
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(                                 \
              __builtin_bit_cast(bf16x8_t, F[kk * (WM + WN) + mt]),                              \
              __builtin_bit_cast(bf16x8_t, F[kk * (WM + WN) + WM + nt]), acc[mt][nt], 0, 0, 0);   \
  } while (0)
  // pending DMA instructions allowed while waiting for group k+1: groups k+2 .. k+S-1,
  // i.e. bytes 0 .. S-3 of hist (issued groups end at k+S-1 when the wait runs)
#define RS_PENDING(OUT)                                                                          \
  do {                                                                                           \
    int p_ = 0;                                                                                  \
    _Pragma("unroll") for (int q = 0; q < S - 2; ++q) p_ += (int)((hist >> (8 * q)) & 0xffull); \
    OUT = p_;                                                                                    \
  } while (0)

  int jslot = 0;
  // prologue: halo of chunk 0 (slot 0) + groups 0 .. S-1
  RS_HALO(0, 0, 0, true);
  const int hcnt0 = NH;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    if (j < nsteps) {
      RS_ISSUE();
      if (j == 0) hist += (unsigned long long)hcnt0;
    } else {
      hist <<= 8;
    }
  }
  u32x4_t F0[2 * (WM + WN)], F1[2 * (WM + WN)];
  {
    // group 0 (and the chunk-0 halo): groups 1 .. S-1 may stay in flight = bytes 0 .. S-2
    int p = 0;
#pragma unroll
    for (int q = 0; q < S - 1; ++q) p += (int)((hist >> (8 * q)) & 0xffull);
    wait_vm_rt(p);
    asm volatile("s_barrier" ::: "memory");
    RS_READ(F0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    RS_FENCE(F0);
  }
#define RS_ITER(FC, FN)                                                                          \
  do {                                                                                           \
    if (k + 1 < nsteps) {                                                                        \
      int pend_;                                                                                 \
      RS_PENDING(pend_);                                                                         \
      if (DBG != 1) wait_vm_rt(pend_);                                                           \
      if (DBG != 1) asm volatile("s_barrier" ::: "memory");                                      \
      if (k + S < nsteps && DBG != 2) RS_ISSUE(); else hist <<= 8;                               \
      RS_READ(FN);                                                                               \
    }                                                                                            \
    RS_MMA(FC);                                                                                  \
    __builtin_amdgcn_sched_barrier(0); /* keep every MFMA of step k ahead of the LDS wait */       \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                           \
    RS_FENCE(FN);                                                                                \
  } while (0)
  int k = 0;
  for (; k + 1 < nsteps; k += 2) {
    RS_ITER(F0, F1);
    ++k;
    RS_ITER(F1, F0);
    --k;
  }
  if (k < nsteps) RS_ITER(F0, F1);
#undef RS_ITER
#undef RS_PENDING
#undef RS_MMA
#undef RS_FENCE
#undef RS_READ
#undef RS_ISSUE
#undef RS_HALO

  int pp[WN], pb[WN], py[WN], px[WN];
#pragma unroll
  for (int nt = 0; nt < WN; ++nt) {
    const int y = y0 + wn * WN + nt, x = x0 + lr;
    if (y < H && x < W) {
      pb[nt] = img;
      py[nt] = y;
      px[nt] = x;
      pp[nt] = (img * H + y) * W + x;
    } else {
      pb[nt] = -1;
      py[nt] = px[nt] = pp[nt] = 0;
    }
  }
  epilogue_pix<WM, WN>(a, acc, m0, lane, pp, pb, py, px);
}

}  // namespace conv

void conv_hx_launch(const conv::Args& a, int tile, hipStream_t stream) {
  const int BM = (tile == 35 || tile == 37) ? 128 : tile == 39 ? 32 : 64;  // 40/41: debug forms of 34
  const int TH = (tile == 36 || tile == 37) ? 4 : 8;
  const dim3 grid(cdiv(a.Cout, BM) * a.B * cdiv(a.H, TH) * cdiv(a.W, 16));
  switch (tile) {
    case 34: hipLaunchKernelGGL((conv::conv_hx_kernel<64, 8, 1, 4, 4, 192>), grid, dim3(256), 0, stream, a); break;
    case 35: hipLaunchKernelGGL((conv::conv_hx_kernel<128, 8, 2, 2, 3, 192>), grid, dim3(256), 0, stream, a); break;
    case 36: hipLaunchKernelGGL((conv::conv_hx_kernel<64, 4, 1, 4, 4, 128>), grid, dim3(256), 0, stream, a); break;
    case 37: hipLaunchKernelGGL((conv::conv_hx_kernel<128, 4, 2, 2, 4, 128>), grid, dim3(256), 0, stream, a); break;
    case 38: hipLaunchKernelGGL((conv::conv_hx_kernel<64, 8, 1, 4, 3, 192>), grid, dim3(256), 0, stream, a); break;
    case 40: hipLaunchKernelGGL((conv::conv_hx_kernel<64, 8, 1, 4, 4, 192, 1>), grid, dim3(256), 0, stream, a); break;
    case 41: hipLaunchKernelGGL((conv::conv_hx_kernel<64, 8, 1, 4, 4, 192, 2>), grid, dim3(256), 0, stream, a); break;
    default: hipLaunchKernelGGL((conv::conv_hx_kernel<32, 8, 1, 4, 4, 192>), grid, dim3(256), 0, stream, a); break;
  }
}

}  // namespace rs
