// Weight / bias gradients of the fused update-block convolutions, batched over
// all refinement iterations (training).
//
// The 12 iterations of the refinement loop share every update-block weight,
// so instead of 12 small weight-gradient GEMMs per conv (and 12 gradient
// accumulations) the training engine stores each iteration's output gradient
// dY_i and input X_i in [iters * B, H, W, C] buffers and computes ONE
//
//   dW[co][tap][k] = sum_{p over iters*B*H*W} dY[p][co] * X[p + off(tap)][k]
//
// per conv: an MFMA GEMM with M = Cout, N = taps x Ktot, K = pixels (~270k at
// the Chairs crop, batch 8), split over blocks along K and accumulated into
// fp32 dW with atomics.  Both operands are channels-last (K = pixels is the
// strided dimension of both), so each 32-pixel K step is staged through LDS
// TRANSPOSED ([channel][pixel] rows, XOR-swizzled 16-B chunks) and the MFMA
// fragments are plain 16-byte ds_read_b128 K-runs.
//
// A segment may be broadcast over the iteration dimension (the context
// features `inp` are the same in every iteration): its row index is the
// pixel index modulo the segment's own pixel count.
//
//   colsum_kernel    : db[co] += sum_p dY[p][co]
//   flow_wgrad_kernel: convf1 (7x7, 2 -> Cout) weight/bias gradient from the
//                      flow (= coords - grid), VALU (K = 98 per output).
#include "common.h"

#include <stdlib.h>

#include <algorithm>

namespace rs {
namespace wgrad {

struct Seg {
  const bf16_t* ptr;
  int C, stride, period;  // period: pixel count of the segment (row = p % period)
};

struct Args {
  const bf16_t* dy;
  int ystr, yoff, Cout;
  Seg seg[3];
  int nseg;
  int Bp, H, W, P;
  int Hi, Wi, SY, SX;  // input grid / stride (wgrad_dma_kernel): X pixel = (y*SY + ky - PH, x*SX + kx - PW)
  int KH, KW, PH, PW;
  int Ktot, taps;
  float* dw;
  int kchunk;
  // deterministic mode: per-K-split partial tiles (plain stores) reduced in a
  // fixed order by det_reduce_kernel instead of fp32 atomics into dw / db
  float* part;    // [ksplit][Cout][taps][Ktot]
  float* dbpart;  // [ksplit][Cout]
  unsigned dy_bytes, seg_bytes[3];
};

typedef short v4s_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// Transposed 4x16 read (gfx950 ds_read_b64_tr_b16): lane 4q+p of each 16-lane
// group addresses row q, columns 4p..4p+3 of a 4-row x 16-column bf16 block;
// lane i of the group receives column i of the 4 rows.
__device__ __forceinline__ v4s_t tr16(const uint16_t* lds_base, int byte_off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) v4s_t*)((__attribute__((address_space(3))) char*)lds_base + byte_off));
}

constexpr int BK = 64;

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

// Block: BM output channels x 64 input channels (one tap) x K split over
// pixels; 4 waves (2 x 2), 64-pixel K steps staged in LDS in their natural
// [pixel][channel] layout (16-byte rows copied as loaded) and read back as
// MFMA fragments with the hardware transpose read.  Blocks of the first
// N tile also accumulate the bias gradient (column sums of dY) from the
// staging registers.
template <int BM, int BN>
__global__ __launch_bounds__(256) void wgrad_kernel(Args a, float* __restrict__ db) {
  constexpr int AROW = BM * 2 + 16, BROW = BN * 2 + 16;  // bytes per staged pixel row (+16 pad)
  constexpr int CA = BM / 8, CB = BN / 8;                // 16-B chunks per row
  constexpr int NA = BK * CA / 256, NB = BK * CB / 256;  // chunks per thread
  constexpr int WM = BM / 2 / 16, WN = BN / 2 / 16;      // MFMA tiles per wave
  __shared__ __attribute__((aligned(16))) uint8_t lds[2][BK * (AROW + BROW)];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int nkb = a.Ktot / BN;
  const int ntiles = a.taps * nkb, mtiles = cdiv(a.Cout, BM);
  // XCD-aware order: the (tap, K-chunk, Cout) tiles of one pixel range are
  // consecutive logical blocks, and each XCD walks a contiguous run of them,
  // so a range's dY / X rows are fetched into one L2 and shared there
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int ntile = lid % ntiles;
  const int m0 = (lid / ntiles % mtiles) * BM;
  const int pbeg = lid / (ntiles * mtiles) * a.kchunk;
  const int tap = ntile / nkb, kb = (ntile % nkb) * BN;
  const int pend = min(a.P, pbeg + a.kchunk);
  const int H = a.H, W = a.W, HW = H * W;
  const int dy_ = tap / a.KW - a.PH, dx_ = tap % a.KW - a.PW;
  const bool do_bias = db != nullptr && ntile == 0;

  const Seg s0 = a.seg[0], s1 = a.seg[1], s2 = a.seg[2];
  const int c01 = s0.C, c012 = s0.C + (a.nseg > 1 ? s1.C : 0);
  const int si = (kb >= c01) + (kb >= c012);
  const bf16_t* sp = si == 0 ? s0.ptr : (si == 1 ? s1.ptr : s2.ptr);
  const int sst = si == 0 ? s0.stride : (si == 1 ? s1.stride : s2.stride);
  const int sper = si == 0 ? s0.period : (si == 1 ? s1.period : s2.period);
  const int nbs = sper / HW;  // images in the segment (it repeats with that period)
  const int cbase = kb - (si == 0 ? 0 : (si == 1 ? c01 : c012));
  const bf16_t* ybase = a.dy + a.yoff + m0;
  const int ystr = a.ystr;
  const u32x4_t zero = {0u, 0u, 0u, 0u};
  // chunk slot i of thread t: A (pixel (t + 256 i) / CA, channel group t % CA);
  //                          B (pixel (t + 256 i) / CB, channel group t % CB)
  const int acg = t % CA, bcg = t % CB;
  u32x4_t ra[NA], rb[NB];
  // (image within the segment period, y, x) of each B staging row's current pixel
  int bb[NB], by[NB], bx[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int p = pbeg + (t + 256 * i) / CB;
    const int b = p / HW, q = p - b * HW;
    bb[i] = b % nbs;
    by[i] = q / W;
    bx[i] = q - by[i] * W;
  }
  float bsum[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bsum[j] = 0.f;

#define RS_WG_LOAD(P0)                                                                           \
  do {                                                                                           \
    _Pragma("unroll") for (int i = 0; i < NA; ++i) {                                             \
      const int p = (P0) + (t + 256 * i) / CA;                                                   \
      const int pc = p < pend ? p : pbeg;                                                        \
      const u32x4_t v = *reinterpret_cast<const u32x4_t*>(ybase + (size_t)pc * ystr + acg * 8);      \
      ra[i] = p < pend ? v : zero;                                                               \
    }                                                                                            \
    _Pragma("unroll") for (int i = 0; i < NB; ++i) {                                             \
      const int p = (P0) + (t + 256 * i) / CB;                                                   \
      const int y = by[i] + dy_, x = bx[i] + dx_;                                                \
      const bool ok = p < pend && y >= 0 && y < H && x >= 0 && x < W;                            \
      const int src = ok ? (bb[i] * H + y) * W + x : 0;                                          \
      const u32x4_t v = *reinterpret_cast<const u32x4_t*>(sp + (size_t)src * sst + cbase + bcg * 8); \
      rb[i] = ok ? v : zero;                                                                     \
      bx[i] += BK; /* advance this row's pixel by one K step */                                  \
      while (bx[i] >= W) { bx[i] -= W; ++by[i]; }                                                \
      while (by[i] >= H) { by[i] -= H; if (++bb[i] == nbs) bb[i] = 0; }                          \
    }                                                                                            \
  } while (0)
#define RS_WG_STORE(BUF)                                                                         \
  do {                                                                                           \
    _Pragma("unroll") for (int i = 0; i < NA; ++i) {                                             \
      const int row = (t + 256 * i) / CA;                                                        \
      *reinterpret_cast<u32x4_t*>(&lds[BUF][row * AROW + acg * 16]) = ra[i];                       \
    }                                                                                            \
    _Pragma("unroll") for (int i = 0; i < NB; ++i) {                                             \
      const int row = (t + 256 * i) / CB;                                                        \
      *reinterpret_cast<u32x4_t*>(&lds[BUF][BK * AROW + row * BROW + bcg * 16]) = rb[i];           \
    }                                                                                            \
  } while (0)
#define RS_WG_BIAS()                                                                             \
  do {                                                                                           \
    if (do_bias) {                                                                               \
      _Pragma("unroll") for (int i = 0; i < NA; ++i) {                                           \
        bsum[0] += __uint_as_float(ra[i].x << 16);                                               \
        bsum[1] += __uint_as_float(ra[i].x & 0xffff0000u);                                       \
        bsum[2] += __uint_as_float(ra[i].y << 16);                                               \
        bsum[3] += __uint_as_float(ra[i].y & 0xffff0000u);                                       \
        bsum[4] += __uint_as_float(ra[i].z << 16);                                               \
        bsum[5] += __uint_as_float(ra[i].z & 0xffff0000u);                                       \
        bsum[6] += __uint_as_float(ra[i].w << 16);                                               \
        bsum[7] += __uint_as_float(ra[i].w & 0xffff0000u);                                       \
      }                                                                                          \
    }                                                                                            \
  } while (0)

  f32x4_t acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int gi = lane & 15, g = lane >> 4;          // 16-lane group g, lane i in it
  const int tq = gi >> 2, tp = gi & 3;              // tr16 address roles: row q, columns 4p..4p+3
  const int nsteps = pend > pbeg ? (pend - pbeg + BK - 1) / BK : 0;
  if (nsteps > 0) {
    RS_WG_LOAD(pbeg);
    RS_WG_BIAS();
    RS_WG_STORE(0);
  }
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    if (s + 1 < nsteps) RS_WG_LOAD(pbeg + (s + 1) * BK);
    const uint16_t* base = reinterpret_cast<const uint16_t*>(&lds[buf][0]);
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      // rows (pixels) of this lane group's k-run: 32kk + 8g + {0..3} and + {4..7}
      const int r0 = kk * 32 + 8 * g + tq;
      bf16x8_t fa[WM], fb[WN];
#pragma unroll
      for (int mt = 0; mt < WM; ++mt) {
        const int col = wm * (BM / 2) + mt * 16 + 4 * tp;
        const v4s_t lo = tr16(base, r0 * AROW + col * 2);
        const v4s_t hi = tr16(base, (r0 + 4) * AROW + col * 2);
        fa[mt] = bf16x8_t{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      }
#pragma unroll
      for (int nt = 0; nt < WN; ++nt) {
        const int col = wn * (BN / 2) + nt * 16 + 4 * tp;
        const v4s_t lo = tr16(base, BK * AROW + r0 * BROW + col * 2);
        const v4s_t hi = tr16(base, BK * AROW + (r0 + 4) * BROW + col * 2);
        fb[nt] = bf16x8_t{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      }
#pragma unroll
      for (int mt = 0; mt < WM; ++mt)
#pragma unroll
        for (int nt = 0; nt < WN; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mt], fb[nt], acc[mt][nt], 0, 0, 0);
    }
    if (s + 1 < nsteps) {
      RS_WG_BIAS();
      RS_WG_STORE(buf ^ 1);
    }
    __syncthreads();
  }
#undef RS_WG_LOAD
#undef RS_WG_STORE
#undef RS_WG_BIAS
  if (nsteps == 0) return;
  if (do_bias) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int co = m0 + acg * 8 + j;
      if (co < a.Cout) {
        if (a.dbpart)
          a.dbpart[(size_t)(lid / (ntiles * mtiles)) * a.Cout + co] = bsum[j];
        else
          atomicAdd(db + co, bsum[j]);
      }
    }
  }
  // C[co][k]: row = 4*(lane>>4) + j (co), col = lane & 15 (k)
#pragma unroll
  for (int mt = 0; mt < WM; ++mt)
#pragma unroll
    for (int nt = 0; nt < WN; ++nt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int co = m0 + wm * (BM / 2) + mt * 16 + (lane >> 4) * 4 + j;
        const int k = kb + wn * (BN / 2) + nt * 16 + (lane & 15);
        if (co < a.Cout) {
          const size_t o = ((size_t)co * a.taps + tap) * a.Ktot + k;
          if (a.part)
            a.part[(size_t)(lid / (ntiles * mtiles)) * a.Cout * a.taps * a.Ktot + o] = acc[mt][nt][j];
          else
            atomicAdd(a.dw + o, acc[mt][nt][j]);
        }
      }
}

// ------------------------------------------------------------------ DMA variant
// Same block decomposition as wgrad_kernel, but both tiles are copied
// global -> LDS by buffer_load_dwordx4 ... lds (no VGPR staging, no
// ds_write) and the per-step address work is nearly all scalar:
//  * dY rows: fixed per-lane offset + the step's scalar SOFFSET;
//  * X rows: per-lane (image, y, x) advanced incrementally, one bounds test,
//    out-of-image taps read past the buffer end (zeros);
//  * LDS rows are unpadded (DMA writes lane-linear 1 KiB pieces), so the
//    bank spread the +16 B pad gave the transpose reads comes from an XOR of
//    the 32-B column block with (row & 3) instead, applied to the per-lane
//    SOURCE chunk and to the tr16 read address.
// The bias gradient of the first N tile is summed from the staged dY tile in
// LDS.
template <int BM, int BN, int WGM, int WGN>
__global__ __launch_bounds__(64 * WGM * WGN) void wgrad_dma_kernel(Args a, float* __restrict__ db) {
  constexpr int RA = BM * 2, RB_ = BN * 2;               // bytes per staged pixel row
  constexpr int CA = BM / 8, CB = BN / 8;                // 16-B chunks per row
  constexpr int NT = 64 * WGM * WGN;                     // threads
  constexpr int NA = BK * CA / NT, NB = BK * CB / NT;    // DMA instructions per thread
  constexpr int WM = BM / WGM / 16, WN = BN / WGN / 16;  // MFMA tiles per wave
  static_assert(NA * NT == BK * CA && NB * NT == BK * CB && NT % CA == 0, "tile / thread split");
  constexpr int kFar = 0x7ffffff0;
  constexpr int STAGE = BK * (RA + RB_);
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * STAGE];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave % WGM, wn = wave / WGM;
  const int nkb = a.Ktot / BN;
  const int ntiles = a.taps * nkb, mtiles = cdiv(a.Cout, BM);
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int ntile = lid % ntiles;
  const int m0 = (lid / ntiles % mtiles) * BM;
  const int pbeg = lid / (ntiles * mtiles) * a.kchunk;
  const int tap = ntile / nkb, kb = (ntile % nkb) * BN;
  const int pend = min(a.P, pbeg + a.kchunk);
  const int nsteps = pend > pbeg ? (pend - pbeg + BK - 1) / BK : 0;
  if (nsteps == 0) return;
  const int H = a.H, W = a.W, HW = H * W;
  const int Hi = a.Hi, Wi = a.Wi, SY = a.SY, SX = a.SX;  // X grid and stride
  const int dy_ = tap / a.KW - a.PH, dx_ = tap % a.KW - a.PW;
  const bool do_bias = db != nullptr && ntile == 0;

  const Seg s0 = a.seg[0], s1 = a.seg[1], s2 = a.seg[2];
  const int c01 = s0.C, c012 = s0.C + (a.nseg > 1 ? s1.C : 0);
  const int si = (kb >= c01) + (kb >= c012);
  const bf16_t* sp = si == 0 ? s0.ptr : (si == 1 ? s1.ptr : s2.ptr);
  const int sst = si == 0 ? s0.stride : (si == 1 ? s1.stride : s2.stride);
  const int sper = si == 0 ? s0.period : (si == 1 ? s1.period : s2.period);
  const unsigned sbytes = si == 0 ? a.seg_bytes[0] : (si == 1 ? a.seg_bytes[1] : a.seg_bytes[2]);
  const int nbs = sper / (Hi * Wi);
  const int cbase = kb - (si == 0 ? 0 : (si == 1 ? c01 : c012));
  const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc((void*)a.dy, (short)0, a.dy_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)sp, (short)0, sbytes, 0x00020000);

  // staging: thread t, instruction i -> LDS chunk t + NT i = (row, physical slot);
  // the slot holds logical chunk slot ^ ((row & 3) << 1)
  int arow[NA], aoff[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int id = t + NT * i, r = id / CA, pos = id % CA;
    arow[i] = r;
    aoff[i] = ((pbeg + r) * a.ystr + a.yoff + m0 + ((pos ^ ((r & 3) << 1)) * 8)) * 2;
  }
  int bb[NB], by[NB], bx[NB], brow[NB], bch[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int id = t + NT * i, r = id / CB, pos = id % CB;
    brow[i] = r;
    bch[i] = cbase + ((pos ^ ((r & 3) << 1)) * 8);
    const int p = pbeg + r;
    const int b = p / HW, q = p - b * HW;
    bb[i] = b % nbs;
    by[i] = q / W;
    bx[i] = q - by[i] * W;
  }
  const int wbase = wave * 64;
  const int ystep = BK * a.ystr * 2;  // dY bytes per K step

#define RS_WD_ISSUE(S, BUF)                                                                     \
  do {                                                                                          \
    uint8_t* st_ = lds + (BUF) * STAGE;                                                         \
    const int rem_ = pend - pbeg - (S) * BK;  /* valid rows in this step */                     \
    _Pragma("unroll") for (int i = 0; i < NA; ++i) {                                            \
      const int v = arow[i] < rem_ ? aoff[i] : kFar;                                            \
      __builtin_amdgcn_raw_ptr_buffer_load_lds(                                                 \
          ry, (__attribute__((address_space(3))) void*)(st_ + (wbase + NT * i) * 16), 16, v,   \
          (S) * ystep, 0, 0);                                                                   \
    }                                                                                           \
    _Pragma("unroll") for (int i = 0; i < NB; ++i) {                                            \
      const int y = by[i] * SY + dy_, x = bx[i] * SX + dx_;                                     \
      const bool ok = brow[i] < rem_ && (unsigned)y < (unsigned)Hi && (unsigned)x < (unsigned)Wi; \
      const int v = ok ? (((bb[i] * Hi + y) * Wi + x) * sst + bch[i]) * 2 : kFar;               \
      __builtin_amdgcn_raw_ptr_buffer_load_lds(                                                 \
          rx, (__attribute__((address_space(3))) void*)(st_ + BK * RA + (wbase + NT * i) * 16), \
          16, v, 0, 0, 0);                                                                      \
      bx[i] += BK;                                                                              \
      while (bx[i] >= W) { bx[i] -= W; ++by[i]; }                                               \
      while (by[i] >= H) { by[i] -= H; if (++bb[i] == nbs) bb[i] = 0; }                         \
    }                                                                                           \
  } while (0)

  f32x4_t acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float bsum[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bsum[j] = 0.f;
  // bias: thread t sums logical chunk t % CA of rows t / CA + (NT / CA) j
  const int bcol = t % CA;

  const int gi = lane & 15, g = lane >> 4;
  const int tq = gi >> 2, tp = gi & 3;
  const int swq = tq << 1;  // (row & 3) << 1 for every row this lane's tr16 reads touch
  // LDS reads are inline asm: the compiler cannot prove they miss the
  // in-flight DMA of the next tile and would drain vmcnt in front of them
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) uint8_t*)lds;
  uint32_t aaddr[WM], baddr[WN];
#pragma unroll
  for (int mt = 0; mt < WM; ++mt) {
    const int ch = ((wm * (BM / WGM) + mt * 16) / 8 + (tp >> 1)) ^ swq;  // 16-B chunk
    aaddr[mt] = lds0 + (8 * g + tq) * RA + ch * 16 + (tp & 1) * 8;
  }
#pragma unroll
  for (int nt = 0; nt < WN; ++nt) {
    const int ch = ((wn * (BN / WGN) + nt * 16) / 8 + (tp >> 1)) ^ swq;
    baddr[nt] = lds0 + BK * RA + (8 * g + tq) * RB_ + ch * 16 + (tp & 1) * 8;
  }
  RS_WD_ISSUE(0, 0);
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");  // tile s landed; buffer s-1 free
    if (s + 1 < nsteps) RS_WD_ISSUE(s + 1, buf ^ 1);
    const uint32_t so = buf * STAGE;
    if (do_bias) {
      u32x4_t bv[BK * CA / NT];
#pragma unroll
      for (int j = 0; j < BK * CA / NT; ++j) {
        const int r = t / CA + (NT / CA) * j;
        asm volatile("ds_read_b128 %0, %1" : "=v"(bv[j])
                     : "v"(lds0 + so + r * RA + ((bcol ^ ((r & 3) << 1)) * 16)) : "memory");
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int j = 0; j < BK * CA / NT; ++j) {
        asm volatile("" : "+v"(bv[j]));
        bsum[0] += __uint_as_float(bv[j].x << 16);
        bsum[1] += __uint_as_float(bv[j].x & 0xffff0000u);
        bsum[2] += __uint_as_float(bv[j].y << 16);
        bsum[3] += __uint_as_float(bv[j].y & 0xffff0000u);
        bsum[4] += __uint_as_float(bv[j].z << 16);
        bsum[5] += __uint_as_float(bv[j].z & 0xffff0000u);
        bsum[6] += __uint_as_float(bv[j].w << 16);
        bsum[7] += __uint_as_float(bv[j].w & 0xffff0000u);
      }
    }
    // fragments of both 32-pixel halves: rows 32kk + 8g + tq (lo) and + 4 (hi)
    v4s_t alo[2][WM], ahi[2][WM], blo[2][WN], bhi[2][WN];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int mt = 0; mt < WM; ++mt) {
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(alo[kk][mt]) : "v"(aaddr[mt] + so),
                     "i"(kk * 32 * RA) : "memory");
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(ahi[kk][mt]) : "v"(aaddr[mt] + so),
                     "i"((kk * 32 + 4) * RA) : "memory");
      }
#pragma unroll
      for (int nt = 0; nt < WN; ++nt) {
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(blo[kk][nt]) : "v"(baddr[nt] + so),
                     "i"(kk * 32 * RB_) : "memory");
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(bhi[kk][nt]) : "v"(baddr[nt] + so),
                     "i"((kk * 32 + 4) * RB_) : "memory");
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8_t fa[WM], fb[WN];
#pragma unroll
      for (int mt = 0; mt < WM; ++mt) {
        asm volatile("" : "+v"(alo[kk][mt]), "+v"(ahi[kk][mt]));
        fa[mt] = bf16x8_t{alo[kk][mt].x, alo[kk][mt].y, alo[kk][mt].z, alo[kk][mt].w,
                          ahi[kk][mt].x, ahi[kk][mt].y, ahi[kk][mt].z, ahi[kk][mt].w};
      }
#pragma unroll
      for (int nt = 0; nt < WN; ++nt) {
        asm volatile("" : "+v"(blo[kk][nt]), "+v"(bhi[kk][nt]));
        fb[nt] = bf16x8_t{blo[kk][nt].x, blo[kk][nt].y, blo[kk][nt].z, blo[kk][nt].w,
                          bhi[kk][nt].x, bhi[kk][nt].y, bhi[kk][nt].z, bhi[kk][nt].w};
      }
#pragma unroll
      for (int mt = 0; mt < WM; ++mt)
#pragma unroll
        for (int nt = 0; nt < WN; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mt], fb[nt], acc[mt][nt], 0, 0, 0);
    }
  }
#undef RS_WD_ISSUE
  if (do_bias) {
    // threads sharing a chunk column: reduce in LDS after the last use of the tiles
    __syncthreads();
    float* red = reinterpret_cast<float*>(lds);
#pragma unroll
    for (int j = 0; j < 8; ++j) red[t * 8 + j] = bsum[j];
    __syncthreads();
    if (t < CA) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float s = 0.f;
        for (int u = t; u < NT; u += CA) s += red[u * 8 + j];
        const int co = m0 + t * 8 + j;
        if (co < a.Cout) {
          if (a.dbpart)
            a.dbpart[(size_t)(lid / (ntiles * mtiles)) * a.Cout + co] = s;
          else
            atomicAdd(db + co, s);
        }
      }
    }
  }
#pragma unroll
  for (int mt = 0; mt < WM; ++mt)
#pragma unroll
    for (int nt = 0; nt < WN; ++nt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int co = m0 + wm * (BM / WGM) + mt * 16 + (lane >> 4) * 4 + j;
        const int k = kb + wn * (BN / WGN) + nt * 16 + (lane & 15);
        if (co < a.Cout) {
          const size_t o = ((size_t)co * a.taps + tap) * a.Ktot + k;
          if (a.part)
            a.part[(size_t)(lid / (ntiles * mtiles)) * a.Cout * a.taps * a.Ktot + o] = acc[mt][nt][j];
          else
            atomicAdd(a.dw + o, acc[mt][nt][j]);
        }
      }
}

// db[c] += sum_p dY[p][yoff + c]; block = 256 pixels, threads over channels.
__global__ __launch_bounds__(256) void colsum_kernel(const bf16_t* __restrict__ dy, int ystr, int yoff,
                                                     int C, int P, float* __restrict__ db,
                                                     float* __restrict__ part) {
  const int p0 = blockIdx.x * 256;
  const int p1 = min(P, p0 + 256);
  for (int c = threadIdx.x; c < C; c += 256) {
    float s = 0.f;
    for (int p = p0; p < p1; ++p) s += bf2f(dy[(size_t)p * ystr + yoff + c]);
    if (part)
      part[(size_t)blockIdx.x * C + c] = s;
    else
      atomicAdd(db + c, s);
  }
}

// convf1 weight gradient: dW[tap][ci][co] (the flow_encode layout [7][7][2][Cout])
// += sum_p dF[p][co] * flow[p + off(tap)][ci], flow = coords - grid (fp32 NCHW),
// and db[co] += sum_p dF[p][co].  K = 98 per output: a VALU kernel.
// Block = ROWS image rows of one image; the flow rows they touch (ROWS + 6,
// zero-padded by 3 columns) are staged in LDS; thread (co, ci) walks each
// row with a 7-wide sliding window in registers (7 LDS reads + 1 dF read per
// 49 FMAs) and keeps 49 tap accumulators; one atomic per output per block.
constexpr int FROWS = 8;
template <typename T>  // dF: bf16, or fp32 (the fp32 training engine)
__global__ __launch_bounds__(256) void flow_wgrad_kernel(const float* __restrict__ coords, int Bp, int H, int W,
                                                         const T* __restrict__ df, int fstr, int Cout,
                                                         float* __restrict__ dw, float* __restrict__ db,
                                                         float* __restrict__ part) {
  extern __shared__ float fl[];  // [2][FROWS + 6][W + 6]
  const int HW = H * W, WP = W + 6, RP = FROWS + 6;
  const int rblocks = cdiv(H, FROWS);
  const int b = blockIdx.x / rblocks, y0 = (blockIdx.x % rblocks) * FROWS;
  for (int i = threadIdx.x; i < 2 * RP * WP; i += blockDim.x) {
    const int ci = i / (RP * WP), rem = i % (RP * WP), ry = rem / WP, rx = rem % WP;
    const int y = y0 + ry - 3, x = rx - 3;
    float v = 0.f;
    if (y >= 0 && y < H && x >= 0 && x < W)
      v = coords[((size_t)b * 2 + ci) * HW + y * W + x] - (ci == 0 ? (float)x : (float)y);
    fl[i] = v;
  }
  __syncthreads();
  for (int pair = threadIdx.x; pair < Cout * 2; pair += blockDim.x) {
    const int co = pair % Cout, ci = pair / Cout;
    const float* F = fl + ci * RP * WP;
    float acc[49];
#pragma unroll
    for (int i = 0; i < 49; ++i) acc[i] = 0.f;
    float bsum = 0.f;
    for (int r = 0; r < FROWS && y0 + r < H; ++r) {
      const T* grow = df + ((size_t)b * HW + (size_t)(y0 + r) * W) * fstr + co;
      // x outer, taps inner: each dY value is loaded once and feeds 49 FMAs.
      // The 7 padded flow rows slide through a register ring: column c of the
      // window lives in slot c % 7, and x advances in chunks of 7 (fully
      // unrolled, so every slot index is a constant: no register shuffling,
      // and the chunk's 7 dF loads are issued together)
      float win[7][7];
#pragma unroll
      for (int ky = 0; ky < 7; ++ky)
#pragma unroll
        for (int kx = 0; kx < 6; ++kx) win[ky][kx] = F[(r + ky) * WP + kx];
      int x = 0;
      for (; x + 7 <= W; x += 7) {
        float g[7];
#pragma unroll
        for (int u = 0; u < 7; ++u) g[u] = io<T>::ld(grow + (size_t)(x + u) * fstr);
#pragma unroll
        for (int u = 0; u < 7; ++u) {
          bsum += g[u];
#pragma unroll
          for (int ky = 0; ky < 7; ++ky) win[ky][(u + 6) % 7] = F[(r + ky) * WP + x + u + 6];
#pragma unroll
          for (int ky = 0; ky < 7; ++ky)
#pragma unroll
            for (int kx = 0; kx < 7; ++kx) acc[ky * 7 + kx] += g[u] * win[ky][(kx + u) % 7];
        }
      }
      for (; x < W; ++x) {  // the last W % 7 columns: window straight from LDS
        const float g1 = io<T>::ld(grow + (size_t)x * fstr);
        bsum += g1;
#pragma unroll
        for (int ky = 0; ky < 7; ++ky)
#pragma unroll
          for (int kx = 0; kx < 7; ++kx) acc[ky * 7 + kx] += g1 * F[(r + ky) * WP + x + kx];
      }
    }
    if (part) {  // deterministic mode: this block's [98 * Cout | Cout] partial, reduced in order later
      float* pb = part + (size_t)blockIdx.x * 99 * Cout;
#pragma unroll
      for (int i = 0; i < 49; ++i) pb[(i * 2 + ci) * Cout + co] = acc[i];
      if (ci == 0) pb[98 * Cout + co] = bsum;
    } else {
#pragma unroll
      for (int i = 0; i < 49; ++i) atomicAdd(dw + ((size_t)i * 2 + ci) * Cout + co, acc[i]);
      if (ci == 0) atomicAdd(db + co, bsum);
    }
  }
}

// out[i] += sum_{s < nsplit} part[s * sstride + i], summed in split order
// (deterministic mode's replacement for the fp32 atomics above)
__global__ __launch_bounds__(256) void det_reduce_kernel(const float* __restrict__ part, int nsplit, long sstride,
                                                         long n, float* __restrict__ out) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < nsplit; ++k) s += part[(size_t)k * sstride + i];
    out[i] += s;
  }
}

}  // namespace wgrad

struct WgradLaunch {
  const void* dy;
  int ystr, yoff, Cout;
  const void* seg_ptr[3];
  int seg_C[3], seg_stride[3], seg_period[3];
  int nseg;
  int Bp, H, W, KH, KW, Ktot;
  float* dw;
  float* db;  // optional: bias gradient (column sums of dY) fused in
  int bn128;  // allow 128-wide N tiles
  unsigned dy_bytes, seg_bytes[3];  // buffer range checks
  int dma;  // 1: buffer-DMA kernel
  float* part;    // deterministic mode: >= wgrad_splits(L) * (Cout*taps*Ktot + Cout) floats, else null
  int Hi, Wi, SY, SX;  // strided conv (DMA kernel): X grid and stride; 0 = dY's grid, stride 1
};

namespace {
struct WgradPlan {
  int var, bm, bn, nthr, ntiles, mtiles, ksplit, kchunk;
};

// Tile variant and split-K of one weight-gradient GEMM.  ``det``: the
// deterministic mode's partial-tile buffers scale with the split count, so it
// is capped at 32 there.
WgradPlan wgrad_plan(const WgradLaunch& L, bool det) {
  WgradPlan pl{};
  // tile variant (L.bn128): 0 = 128x64 (64x64 for Cout <= 64), 1 = 128x128,
  // 8-wave DMA tiles: 2 = 128x128, 3 = 256x128, 4 = 256x64, 5 = 64x128 (4 waves)
  bool seg128 = true;  // a 128-wide N tile must stay inside one segment
  for (int s = 0; s < L.nseg; ++s) seg128 = seg128 && (L.seg_C[s] % 128 == 0);
  int var = L.bn128;
  if (var < 0 || var > 5 || (!L.dma && var > 1)) var = 0;
  if ((var == 1 || var == 2 || var == 3 || var == 5) && !seg128) var = 0;
  if (var == 1 && L.Cout <= 64) var = 0;
  pl.var = var;
  pl.bm = var == 3 || var == 4 ? 256 : (var == 5 ? 64 : (var == 0 && L.Cout <= 64 ? 64 : 128));
  pl.bn = var == 0 || var == 4 ? 64 : 128;
  pl.nthr = var >= 2 && var <= 4 ? 512 : 256;
  const int taps = L.KH * L.KW, P = L.Bp * L.H * L.W;
  pl.ntiles = taps * (L.Ktot / pl.bn);
  pl.mtiles = cdiv(L.Cout, pl.bm);
  // split-K over the pixels: more blocks hide latency, but every split adds a
  // full dW tile of fp32 atomics (~1.3 TB/s chip-wide, MI355X_MICROARCH.md)
  // and more blocks co-running with the main queue's kernels; in situ 1024
  // target blocks beat 2048 and 4096 (401.3 / 402.3 vs 397.8 / 399.3 vs
  // 390.6 / 392.0 pairs/s, profiles/r4/ab_knobs_s33.txt)
  constexpr int target_blocks = 1024;
  int ksplit = cdiv(target_blocks, pl.ntiles * pl.mtiles);
  ksplit = max(1, min(ksplit, cdiv(P, wgrad::BK * 8)));
  if (det) ksplit = min(ksplit, 32);
  pl.kchunk = round_up(cdiv(P, ksplit), wgrad::BK);
  pl.ksplit = cdiv(P, pl.kchunk);  // every split is non-empty (each writes its whole partial tile)
  return pl;
}
}  // namespace

int wgrad_splits(const WgradLaunch& L) { return wgrad_plan(L, true).ksplit; }

static void wgrad_kernels(const WgradLaunch& L, const wgrad::Args& a, int var, int bm, int bn, int nthr, dim3 grid,
                          hipStream_t stream);

void wgrad_launch(const WgradLaunch& L, hipStream_t stream) {
  wgrad::Args a{};
  a.dy = static_cast<const bf16_t*>(L.dy);
  a.ystr = L.ystr; a.yoff = L.yoff; a.Cout = L.Cout;
  for (int s = 0; s < 3; ++s) {
    a.seg[s].ptr = static_cast<const bf16_t*>(L.seg_ptr[s]);
    a.seg[s].C = L.seg_C[s];
    a.seg[s].stride = L.seg_stride[s];
    a.seg[s].period = L.seg_period[s];
  }
  a.nseg = L.nseg;
  a.Bp = L.Bp; a.H = L.H; a.W = L.W; a.P = L.Bp * L.H * L.W;
  a.Hi = L.Hi ? L.Hi : L.H; a.Wi = L.Wi ? L.Wi : L.W;
  a.SY = L.SY ? L.SY : 1; a.SX = L.SX ? L.SX : 1;
  a.KH = L.KH; a.KW = L.KW; a.PH = L.KH / 2; a.PW = L.KW / 2;
  a.Ktot = L.Ktot; a.taps = L.KH * L.KW;
  a.dw = L.dw;
  a.dy_bytes = L.dy_bytes;
  for (int s = 0; s < 3; ++s) a.seg_bytes[s] = L.seg_bytes[s];
  const bool det = L.part != nullptr;
  const WgradPlan pl = wgrad_plan(L, det);
  const int var = pl.var, bm = pl.bm, bn = pl.bn, nthr = pl.nthr;
  const int ksplit = pl.ksplit;
  a.kchunk = pl.kchunk;
  const long pstride = (long)a.Cout * a.taps * a.Ktot;
  if (det) {
    a.part = L.part;
    a.dbpart = L.db ? L.part + (size_t)ksplit * pstride : nullptr;
  }
  dim3 grid(pl.ntiles * pl.mtiles * ksplit);
  if (det) {
    wgrad_kernels(L, a, var, bm, bn, nthr, grid, stream);
    const int rb = (int)std::min<long>(4096, cdiv(pstride, 256));
    hipLaunchKernelGGL(wgrad::det_reduce_kernel, dim3(rb), dim3(256), 0, stream, a.part, ksplit, pstride, pstride,
                       a.dw);
    if (L.db)
      hipLaunchKernelGGL(wgrad::det_reduce_kernel, dim3(cdiv(a.Cout, 256)), dim3(256), 0, stream, a.dbpart, ksplit,
                         (long)a.Cout, (long)a.Cout, L.db);
    return;
  }
  wgrad_kernels(L, a, var, bm, bn, nthr, grid, stream);
}

static void wgrad_kernels(const WgradLaunch& L, const wgrad::Args& a, int var, int bm, int bn, int nthr, dim3 grid,
                          hipStream_t stream) {
  if (L.dma) {
    switch (var) {
      case 1: hipLaunchKernelGGL((wgrad::wgrad_dma_kernel<128, 128, 2, 2>), grid, dim3(nthr), 0, stream, a, L.db); break;
      case 2: hipLaunchKernelGGL((wgrad::wgrad_dma_kernel<128, 128, 2, 4>), grid, dim3(nthr), 0, stream, a, L.db); break;
      case 3: hipLaunchKernelGGL((wgrad::wgrad_dma_kernel<256, 128, 4, 2>), grid, dim3(nthr), 0, stream, a, L.db); break;
      case 4: hipLaunchKernelGGL((wgrad::wgrad_dma_kernel<256, 64, 4, 2>), grid, dim3(nthr), 0, stream, a, L.db); break;
      case 5: hipLaunchKernelGGL((wgrad::wgrad_dma_kernel<64, 128, 2, 2>), grid, dim3(nthr), 0, stream, a, L.db); break;
      default:
        if (bm == 128)
          hipLaunchKernelGGL((wgrad::wgrad_dma_kernel<128, 64, 2, 2>), grid, dim3(nthr), 0, stream, a, L.db);
        else
          hipLaunchKernelGGL((wgrad::wgrad_dma_kernel<64, 64, 2, 2>), grid, dim3(nthr), 0, stream, a, L.db);
    }
    return;
  }
  if (bn == 128)
    hipLaunchKernelGGL((wgrad::wgrad_kernel<128, 128>), grid, dim3(256), 0, stream, a, L.db);
  else if (bm == 128)
    hipLaunchKernelGGL((wgrad::wgrad_kernel<128, 64>), grid, dim3(256), 0, stream, a, L.db);
  else
    hipLaunchKernelGGL((wgrad::wgrad_kernel<64, 64>), grid, dim3(256), 0, stream, a, L.db);
}

int colsum_blocks(int P) { return cdiv(P, 256); }

void colsum_launch(const void* dy, int ystr, int yoff, int C, int P, float* db, float* part, hipStream_t stream) {
  const int blocks = colsum_blocks(P);
  hipLaunchKernelGGL(wgrad::colsum_kernel, dim3(blocks), dim3(256), 0, stream,
                     static_cast<const bf16_t*>(dy), ystr, yoff, C, P, db, part);
  if (part)
    hipLaunchKernelGGL(wgrad::det_reduce_kernel, dim3(cdiv(C, 256)), dim3(256), 0, stream, part, blocks, (long)C,
                       (long)C, db);
}

int flow_wgrad_blocks(int Bp, int H) { return Bp * cdiv(H, wgrad::FROWS); }

void flow_wgrad_launch(const float* coords, int Bp, int H, int W, const void* df, int fstr, int Cout, float* dw,
                       float* db, float* part, bool f32, hipStream_t stream) {
  const int blocks = flow_wgrad_blocks(Bp, H);
  const size_t lds = sizeof(float) * 2 * (wgrad::FROWS + 6) * (W + 6);
  if (f32)
    hipLaunchKernelGGL(wgrad::flow_wgrad_kernel<float>, dim3(blocks), dim3(256), lds, stream, coords, Bp, H, W,
                       static_cast<const float*>(df), fstr, Cout, dw, db, part);
  else
    hipLaunchKernelGGL(wgrad::flow_wgrad_kernel<bf16_t>, dim3(blocks), dim3(256), lds, stream, coords, Bp, H, W,
                       static_cast<const bf16_t*>(df), fstr, Cout, dw, db, part);
  if (part) {  // [blocks][98 * Cout | Cout] partials -> dw, db in block order
    const long st = 99L * Cout;
    hipLaunchKernelGGL(wgrad::det_reduce_kernel, dim3(cdiv(98 * Cout, 256)), dim3(256), 0, stream, part, blocks, st,
                       98L * Cout, dw);
    hipLaunchKernelGGL(wgrad::det_reduce_kernel, dim3(cdiv(Cout, 256)), dim3(256), 0, stream, part + 98 * Cout,
                       blocks, st, (long)Cout, db);
  }
}

}  // namespace rs
