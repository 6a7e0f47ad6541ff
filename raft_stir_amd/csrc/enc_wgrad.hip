// Halo-tile weight gradient of the encoders' stride-1 3x3 convolutions
// (reference core/extractor.py:6-56 ResidualBlock conv1 / conv2: layer1
// 64 -> 64 at 1/2 resolution, layer3 128 -> 128 at 1/8; the backward of
// reference train.py:173-181):
//
//   dW[co][ci][ky][kx] = sum_p dY[p][co] * X[p + (ky - 1, kx - 1)][ci]
//
// conv_wgrad.hip's wgrad_dma_kernel runs this as a GEMM whose N tile is one
// tap: every (tap, channel tile) block re-stages the same dY rows and a
// shifted copy of the X rows for its own 64-pixel K steps -- 9 x the dY and X
// traffic, with 64x64 output tiles (~380 TFLOP/s at the 1/2-res shape,
// profiles/r3).  Here a block owns a 64-output x 64-input channel slice of ALL
// NINE taps (a 64 x 576 fp32 tile in registers) and walks a contiguous range
// of 8 x 32-pixel image tiles:
//  * per tile the dY tile (256 pixels x 64 channels) and the 10 x 34 input
//    halo (64 channels) are copied global -> LDS once by buffer_load ... lds
//    DMA (double-buffered: the next tile is in flight during this tile's
//    MFMAs); halo pixels outside the image are read past the buffer end, i.e.
//    as zeros (the conv's zero padding);
//  * one K step = one 32-pixel tile row; every tap reads its shifted window
//    of the halo: the MFMA K operand is 8 consecutive pixels of one channel,
//    gathered from the pixel-major LDS rows by ds_read_b64_tr_b16;
//  * LDS rows are 128 B (64 channels) with 16-B chunks XOR-swizzled by
//    sw(row) = ((row & 3) ^ ((row >> 3) & 1)) << 1: the 32 lanes of each
//    transposed read hit 64 distinct banks for any row offset (halo shift);
//  * 8 waves: wave w owns input-channel tile w & 3 (16 channels) x all 9
//    taps x output-channel tiles 2 (w >> 2) .. +1: 18 v_mfma_f32_16x16x32_bf16
//    per K step against 4 + 18 transposed reads, two waves per SIMD.
// Each block writes its partial dW tile (plain stores); enc_wgrad_reduce sums
// the partials in block order into the weight's own [Cout][Cin][3][3] layout:
// deterministic, no atomics.  Channel counts that are an odd multiple of 32
// (layer2's 96) are covered by two OVERLAPPING 64-channel blocks, [0, 64) and
// [C - 64, C); the reduction takes each channel from the first block that
// holds it.
#include <stdlib.h>

#include <algorithm>

#include "common.h"

namespace rs {
namespace encw {

constexpr int TH = 8, TW = 32, HC = TW + 2, HR = TH + 2;  // output tile, input halo (10 x 34)
constexpr int NT = 512;                                   // 8 waves
constexpr int RB = 128;                                   // LDS bytes per row (64 bf16 channels)
constexpr int XCH = HR * HC * 8;                          // 2720 16-B halo chunks
constexpr int NX = (XCH + NT - 1) / NT;                   // 6 DMA instructions per thread
constexpr int XREAL = (XCH + 63) / 64 * 64;               // 2752: halo + the partial wave's lanes
constexpr int YCH = TH * TW * 8;                          // 2048 dY chunks
constexpr int NY = YCH / NT;                              // 4
constexpr int XOFF = 0, DUMMY = XREAL, YOFF = XREAL + 64; // chunk offsets within a stage
constexpr int STAGE = YOFF + YCH;                         // 4864 chunks = 76 KiB
constexpr int kFar = 0x7ffffff0;                          // past every buffer: reads as zero
static_assert(YCH % NT == 0 && 2 * STAGE * 16 <= 160 * 1024, "LDS");

struct WArgs {
  const bf16_t* x;   // NHWC input, xstr elements per pixel
  const bf16_t* dy;  // NHWC output gradient, ystr elements per pixel
  int xstr, ystr;
  unsigned x_bytes, dy_bytes;
  int B, H, W, Cin, Cout;
  int tiles_w, tiles_img, ntiles, tpb;  // tiles per block (contiguous range)
  int ncb, nib;                         // output / input channel blocks (64 each, last one at C - 64)
  float* part;                          // [nsplit][ncb][nib][64 co][9][64 ci]
};

__device__ __forceinline__ int swz(int row) { return ((row & 3) ^ ((row >> 3) & 1)) << 1; }

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, uint4* lds_base, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_base, 16, voff, 0, 0, 0);
}

typedef short v4s_t __attribute__((ext_vector_type(4)));

// B-operand rows: per-lane byte offset within the halo for a window whose
// first row has residue `res` (mod 16): row = base + 8g + tq, chunk
// (2 nw + (tp >> 1)) ^ swz(row), 8-byte half tp & 1.  The base itself is a
// compile-time immediate at the read.
__device__ __forceinline__ uint32_t boff(int res, int lane, int nw) {
  const int g = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  const int rr = res + 8 * g + tq;  // row - base + res: same residues mod 16 as the row
  return (uint32_t)((8 * g + tq) * RB + (((2 * nw + (tp >> 1)) ^ swz(rr)) * 16) + (tp & 1) * 8);
}

template <int OFF>
__device__ __forceinline__ void trd(v4s_t& d, uint32_t addr) {
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(OFF) : "memory");
}

// One K step (tile row R): 2 A (dY) and 9 B (halo) fragments, then 18 MFMAs.
template <int R>
__device__ __forceinline__ void kstep(f32x4_t (&acc)[2][9], uint32_t ya0, uint32_t ya1, const uint32_t (&xb)[16]) {
  v4s_t alo[2], ahi[2], blo[9], bhi[9];
  trd<R * 32 * RB>(alo[0], ya0);
  trd<(R * 32 + 4) * RB>(ahi[0], ya0);
  trd<R * 32 * RB>(alo[1], ya1);
  trd<(R * 32 + 4) * RB>(ahi[1], ya1);
#define RS_TAP(T)                                                              \
  {                                                                            \
    constexpr int ky = (T) / 3, kx = (T) % 3, base = (R + ky) * HC + kx;       \
    trd<base * RB>(blo[T], xb[base & 15]);                                     \
    trd<(base + 4) * RB>(bhi[T], xb[(base + 4) & 15]);                         \
  }
  RS_TAP(0) RS_TAP(1) RS_TAP(2) RS_TAP(3) RS_TAP(4) RS_TAP(5) RS_TAP(6) RS_TAP(7) RS_TAP(8)
#undef RS_TAP
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  bf16x8_t fa[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    asm volatile("" : "+v"(alo[m]), "+v"(ahi[m]));
    fa[m] = bf16x8_t{alo[m].x, alo[m].y, alo[m].z, alo[m].w, ahi[m].x, ahi[m].y, ahi[m].z, ahi[m].w};
  }
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    asm volatile("" : "+v"(blo[t]), "+v"(bhi[t]));
    const bf16x8_t fb = bf16x8_t{blo[t].x, blo[t].y, blo[t].z, blo[t].w, bhi[t].x, bhi[t].y, bhi[t].z, bhi[t].w};
#pragma unroll
    for (int m = 0; m < 2; ++m) acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[m], fb, acc[m][t], 0, 0, 0);
  }
}

__global__ __launch_bounds__(NT) void enc_wgrad_kernel(WArgs a) {
  __shared__ uint4 lds[2 * STAGE];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int nw = wave & 3, mh = wave >> 2;
  const int bid = blockIdx.x;
  const int cb = bid % a.ncb, ib = (bid / a.ncb) % a.nib, split = bid / (a.ncb * a.nib);
  const int co0 = min(cb * 64, a.Cout - 64), ci0 = min(ib * 64, a.Cin - 64);
  int tile = split * a.tpb;
  const int tend = min(a.ntiles, tile + a.tpb);  // host: every split has >= 1 tile

  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc((void*)a.dy, (short)0, a.dy_bytes, 0x00020000);

  // staging: thread t, instruction i -> stage chunk t + NT i (lane-linear 1 KiB per wave
  // instruction); the chunk at (row, pc) holds logical channel chunk pc ^ swz(row)
  int xhy[NX], xhx[NX], xch[NX];
  bool xdummy[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    const int q = t + NT * i, row = q >> 3, pc = q & 7;
    xhy[i] = row / HC;
    xhx[i] = row - xhy[i] * HC;
    xch[i] = ci0 + ((pc ^ swz(row)) * 8);
    xdummy[i] = (wave * 64 + NT * i) >= XREAL;  // the whole wave instruction is surplus
    if (q >= XCH) xhy[i] = -1000;               // pad lanes of the partial wave: zeros
  }
  int yr[NY], yc[NY], ych[NY];
#pragma unroll
  for (int i = 0; i < NY; ++i) {
    const int q = t + NT * i, row = q >> 3, pc = q & 7;
    yr[i] = row >> 5;
    yc[i] = row & 31;
    ych[i] = co0 + ((pc ^ swz(row)) * 8);
  }
  const int H = a.H, W = a.W;
  auto issue = [&](int tl, int buf) {
    const int b = tl / a.tiles_img, rem = tl - b * a.tiles_img;
    const int th = rem / a.tiles_w;
    const int ty0 = th * TH, tx0 = (rem - th * a.tiles_w) * TW;
    uint4* st = lds + buf * STAGE;
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const int iy = ty0 - 1 + xhy[i], ix = tx0 - 1 + xhx[i];
      const bool ok = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
      const int v = ok ? (((b * H + iy) * W + ix) * a.xstr + xch[i]) * 2 : kFar;
      dma16(rx, st + (xdummy[i] ? DUMMY : XOFF + wave * 64 + NT * i), v);
    }
#pragma unroll
    for (int i = 0; i < NY; ++i) {
      const int y = ty0 + yr[i], xx = tx0 + yc[i];
      const bool ok = y < H && xx < W;
      const int v = ok ? (((b * H + y) * W + xx) * a.ystr + ych[i]) * 2 : kFar;
      dma16(ry, st + YOFF + wave * 64 + NT * i, v);
    }
  };

  // fragment read offsets: A rows 8g + tq (+4), chunk 2 (2 mh + m) + (tp >> 1)
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) uint4*)&lds[0];
  const int g = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  uint32_t ya[2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
    ya[m] = lds0 + YOFF * 16 + (8 * g + tq) * RB + (((2 * (2 * mh + m) + (tp >> 1)) ^ swz(8 * g + tq)) * 16) +
            (tp & 1) * 8;
  uint32_t xb0[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) xb0[r] = lds0 + XOFF * 16 + boff(r, lane, nw);

  f32x4_t acc[2][9];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int k = 0; k < 9; ++k) acc[m][k] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  issue(tile, 0);
  int buf = 0;
  for (; tile < tend; ++tile) {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");  // this tile landed; the other buffer is free
    if (tile + 1 < tend) issue(tile + 1, buf ^ 1);
    const uint32_t so = buf * STAGE * 16;
    uint32_t xb[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) xb[r] = xb0[r] + so;
    const uint32_t y0 = ya[0] + so, y1 = ya[1] + so;
    kstep<0>(acc, y0, y1, xb);
    kstep<1>(acc, y0, y1, xb);
    kstep<2>(acc, y0, y1, xb);
    kstep<3>(acc, y0, y1, xb);
    kstep<4>(acc, y0, y1, xb);
    kstep<5>(acc, y0, y1, xb);
    kstep<6>(acc, y0, y1, xb);
    kstep<7>(acc, y0, y1, xb);
    buf ^= 1;
  }

  // partial tile: C[co][ci] of tap k, co = co0 + 16 (2 mh + m) + 4 g + j, ci = ci0 + 16 nw + (lane & 15)
  float* o = a.part + (size_t)((split * a.ncb + cb) * a.nib + ib) * (64 * 9 * 64);
  const int ci = 16 * nw + (lane & 15);
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int co = 16 * (2 * mh + m) + 4 * g + j;
#pragma unroll
      for (int k = 0; k < 9; ++k) o[(co * 9 + k) * 64 + ci] = acc[m][k][j];
    }
}

// dw[co][ci][ky][kx] = sum over splits of the partial of the block holding
// (co, ci).  A block = 64 consecutive outputs (walked as (co, tap, ci), ci
// fastest: coalesced partial rows) x 4 split slices; slice s sums splits
// s, s + 4, ... and the four slice sums are added in slice order through
// LDS: a fixed order (deterministic) with 4x the loads in flight of one
// thread per output (the split count is ~256).
__global__ __launch_bounds__(256) void enc_wgrad_reduce_kernel(const float* __restrict__ part, int nsplit, int Cout,
                                                               int Cin, float* __restrict__ dw) {
  __shared__ float red[4][64];
  const int o = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + o;  // dw element in channels_last order (co, tap, ci)
  const bool live = i < Cout * 9 * Cin;
  float s = 0.f;
  int co = 0, ci = 0, k = 0;
  if (live) {
    ci = i % Cin;
    const int r = i / Cin;
    k = r % 9;
    co = r / 9;
    const int ncb = (Cout + 63) / 64, nib = (Cin + 63) / 64;
    const int cb = min(co / 64, ncb - 1), ib = min(ci / 64, nib - 1);
    const int col = co - min(cb * 64, Cout - 64), cil = ci - min(ib * 64, Cin - 64);
    const size_t blk = (size_t)ncb * nib * (64 * 9 * 64);
    const float* p = part + (size_t)(cb * nib + ib) * (64 * 9 * 64) + (col * 9 + k) * 64 + cil;
#pragma unroll 8
    for (int sp = sl; sp < nsplit; sp += 4) s += p[sp * blk];
  }
  red[sl][o] = s;
  __syncthreads();
  // channels_last (the layout of the model's conv weights: the gradient is
  // stored as .grad without a layout copy), coalesced along ci
  if (sl == 0 && live) dw[i] = ((red[0][o] + red[1][o]) + red[2][o]) + red[3][o];
}

}  // namespace encw

// host launch (ops_conv.cpp enc_wgrad): shapes / alignment checked there
struct EncWgradLaunch {
  const void* x;
  const void* dy;
  int xstr, ystr;
  long x_bytes, dy_bytes;
  int B, H, W, Cin, Cout;
  float* part;
  float* dw;
  int nsplit, tpb;
};

int enc_wgrad_splits(int B, int H, int W, int Cin, int Cout, int* tpb) {
  const int ntiles = B * cdiv(H, encw::TH) * cdiv(W, encw::TW);
  const int chan = cdiv(Cout, 64) * cdiv(Cin, 64);
  int want = 256 / chan;  // ~one block per CU
  if (want < 1) want = 1;
  *tpb = cdiv(ntiles, want);
  return cdiv(ntiles, *tpb);
}

void enc_wgrad_launch(const EncWgradLaunch& L, hipStream_t stream) {
  encw::WArgs a{};
  a.x = static_cast<const bf16_t*>(L.x);
  a.dy = static_cast<const bf16_t*>(L.dy);
  a.xstr = L.xstr;
  a.ystr = L.ystr;
  a.x_bytes = (unsigned)L.x_bytes;
  a.dy_bytes = (unsigned)L.dy_bytes;
  a.B = L.B; a.H = L.H; a.W = L.W; a.Cin = L.Cin; a.Cout = L.Cout;
  a.tiles_w = cdiv(L.W, encw::TW);
  a.tiles_img = a.tiles_w * cdiv(L.H, encw::TH);
  a.ntiles = L.B * a.tiles_img;
  a.tpb = L.tpb;
  a.ncb = cdiv(L.Cout, 64);
  a.nib = cdiv(L.Cin, 64);
  a.part = L.part;
  hipLaunchKernelGGL(encw::enc_wgrad_kernel, dim3(L.nsplit * a.ncb * a.nib), dim3(encw::NT), 0, stream, a);
  const int n = L.Cout * 9 * L.Cin;
  hipLaunchKernelGGL(encw::enc_wgrad_reduce_kernel, dim3(cdiv(n, 64)), dim3(256), 0, stream, L.part, L.nsplit,
                     L.Cout, L.Cin, L.dw);
}

}  // namespace rs
