// All-taps weight gradient of the update-block convolutions, batched over the
// refinement iterations (training; reference core/update.py:6-136 backward):
//
//   dW[co][tap][k] = sum_p dY[p][co] * X[p + off(tap)][k]      (+ db[co] = sum_p dY[p][co])
//
// conv_wgrad.hip's wgrad_dma_kernel treats this as a GEMM whose N tile is ONE
// tap, so every (tap, channel tile) block re-stages the same dY rows and a
// shifted copy of the X rows: for the GRU z|r conv (1x5, 256 x 1920, 274k
// pixels) that is ~4 GB of L2 -> LDS traffic per call at ~540 TFLOP/s
// (profiles/r5/README.md).  Here a block owns BM output channels x one
// 64-channel input chunk x ALL T taps (a BM x T x 64 fp32 tile in AGPRs) and
// walks a contiguous range of TH x 32-pixel patches of the iterations x batch
// image stack:
//  * per patch, the dY rows (TH*32 pixels x BM channels) and the input halo
//    ((TH+KH-1) x (32+KW-1) pixels x 64 channels) are copied global -> LDS once
//    by buffer_load ... lds (double-buffered: the next patch is in flight during
//    this patch's MFMAs; out-of-image halo pixels and pixels past the range
//    read as zeros);
//  * one K step = 16 pixels of a patch row: the A operand (32 co x 16 px of
//    dY) and, per tap, the B operand (16 px x 32 k of the shifted halo window)
//    are K-major fragments gathered from the pixel-major LDS rows by
//    ds_read_b64_tr_b16; rows XOR-swizzle their 64-byte quarters so the 32
//    lanes of each transposed read hit 64 distinct banks for any row offset;
//  * 2 NWM waves: wave w owns output channels 32 (w % NWM) .. +32 and input
//    channels 32 (w / NWM) .. +32 of the chunk, all T taps: T
//    v_mfma_f32_32x32x16_bf16 per K step against 2 + 2T transposed reads;
//  * every block writes its partial tile to part[split] (plain stores) and
//    wg3_reduce_kernel adds the splits in order into dW: deterministic, no
//    atomics.  Blocks of the first input chunk also sum dY over their pixels
//    (the bias gradient) from the A fragments.
// A segment may repeat over the image stack (the context features `inp` are
// the same in every iteration): its image index is the stack index modulo
// the segment's own image count.
#include "common.h"

#include <stdlib.h>

#include <algorithm>
#include <type_traits>

namespace rs {
namespace wg3 {

typedef short v4s_t __attribute__((ext_vector_type(4)));
typedef short v8s_t __attribute__((ext_vector_type(8)));

struct Seg {
  const bf16_t* ptr;
  int C, stride, imgs;  // channels (multiple of 64), row stride, images (repeats with that period)
  unsigned bytes;
};

struct Args {
  const bf16_t* dy;
  int ystr, yoff, Cout;
  unsigned dy_bytes;
  Seg seg[3];
  int nseg;
  int NI, H, W;   // image stack and grid
  int Ktot;       // sum of the segments' channels
  int nsplit, ppb;  // pixel-range splits, patches per block
  float* part;    // [nsplit][Cpad][T][Ktot]
  float* bpart;   // [nsplit][Cpad] (null: no bias)
  int Cpad;
};

constexpr int kFar = 0x7ffffff0;

__device__ __forceinline__ v4s_t tr16(const uint8_t* lds, int byte_off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) v4s_t*)((__attribute__((address_space(3))) const uint8_t*)lds + byte_off));
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, const uint8_t* lds_base, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_base, 16, voff, 0, 0, 0);
}

template <int I, int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<I + 1, N>(f);
  }
}

// B fragments of every tap for the K step (patch row R, half KS): halo rows
// Ck + 8h + q (+4), Ck = (R + tap / KW) * HWD + 16 KS + tap % KW
template <int T0, int NT, int KW, int HWD, int R, int KS>
__device__ __forceinline__ void read_taps(v4s_t* blo, v4s_t* bhi, const uint32_t* baddr, uint32_t so) {
  if constexpr (T0 < NT) {
    constexpr int ck = (R + T0 / KW) * HWD + KS * 16 + T0 % KW;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(blo[T0]) : "v"(baddr[ck & 3] + so), "i"(ck * 128)
                 : "memory");
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(bhi[T0]) : "v"(baddr[ck & 3] + so),
                 "i"((ck + 4) * 128) : "memory");
    read_taps<T0 + 1, NT, KW, HWD, R, KS>(blo, bhi, baddr, so);
  }
}

template <int N>
__device__ __forceinline__ void wait_lgkm() {  // lgkmcnt is 4 bits: waiting for more is always safe
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N < 15 ? N : 15) : "memory");
}

// the MFMAs of one K step, tap by tap, each behind the wait for its own B fragment
template <int T0, int NT>
__device__ __forceinline__ void mfma_taps(f32x16_t* acc, const bf16x8_t& av, v4s_t* blo, v4s_t* bhi) {
  if constexpr (T0 < NT) {
    wait_lgkm<2 * (NT - 1 - T0)>();
    asm volatile("" : "+v"(blo[T0]), "+v"(bhi[T0]));
    __builtin_amdgcn_sched_barrier(0);
    const bf16x8_t bv = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(blo[T0], bhi[T0], 0, 1, 2, 3, 4, 5, 6, 7));
    acc[T0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc[T0], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    mfma_taps<T0 + 1, NT>(acc, av, blo, bhi);
  }
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

// swizzle of the 64-byte quarter (4 x 16-B chunks) of LDS row `row`:
// rows of 256 B (BM = 128 dY rows): quarter ^= row & 3; rows of 128 B: the
// quarter pair flips every second row
template <int ROWB>
__device__ __forceinline__ int swz(int row) {
  return ROWB == 256 ? (row & 3) : ((row >> 1) & 1);
}

template <int KH, int KW, int NWM, int TH>
struct G {
  static constexpr int T = KH * KW, BM = 32 * NWM, NW = 2 * NWM, NT = 64 * NW;
  static constexpr int HH = TH + KH - 1, HWD = 32 + KW - 1;
  static constexpr int YROWB = BM * 2, YCH = YROWB / 16;    // dY row bytes / chunks
  static constexpr int YSL = TH * 32 * YCH;                   // dY slots (16 B) per stage
  static constexpr int XSL = HH * HWD * 8;                    // halo slots per stage
  static constexpr int NYP = YSL / 64, NXP = (XSL + 63) / 64; // DMA pieces per stage
  static constexpr int NYW = NYP / NW, NXW = (NXP + NW - 1) / NW;  // ... per wave
  static constexpr int XOFF = YSL * 16;                       // halo bytes offset in a stage
  static constexpr int STAGE = (YSL + NXW * NW * 64) * 16;    // stage bytes (halo padded to whole pieces)
  static_assert(YROWB == 128 || YROWB == 256, "BM 64 or 128");
  static_assert(NYP % NW == 0, "dY pieces per wave");
  static_assert(2 * STAGE <= 160 * 1024, "LDS");
};

template <int KH, int KW, int NWM, int TH>
__global__ __launch_bounds__(128 * NWM) void wgrad3_kernel(Args a) {
  using C = G<KH, KW, NWM, TH>;
  constexpr int T = C::T, BM = C::BM, NW = C::NW, HWD = C::HWD, YCH = C::YCH;
  constexpr int NYW = C::NYW, NXW = C::NXW, STAGE = C::STAGE, XOFF = C::XOFF;
  constexpr int PH = KH / 2, PW = KW / 2;
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cw = wave % NWM, kh = wave / NWM;
  const int H = a.H, W = a.W;
  const int nty = cdiv(H, TH), ntx = cdiv(W, 32), npi = nty * ntx;
  const int npatch = a.NI * npi;
  const int nM = a.Cpad / BM, nC = a.Ktot / 64;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int c = lid % nC, m = lid / nC % nM, split = lid / (nC * nM);
  const int m0 = m * BM;
  const int p0 = split * a.ppb, p1 = min(npatch, p0 + a.ppb);

  // input chunk -> segment
  const int c01 = a.seg[0].C >> 6, c012 = c01 + (a.nseg > 1 ? (a.seg[1].C >> 6) : 0);
  const int si = (c >= c01) + (c >= c012);
  const Seg sg = si == 0 ? a.seg[0] : (si == 1 ? a.seg[1] : a.seg[2]);
  const int cb = (c - (si == 0 ? 0 : (si == 1 ? c01 : c012))) * 64;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)sg.ptr, (short)0, sg.bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc((void*)a.dy, (short)0, a.dy_bytes, 0x00020000);

  // ---- per-lane DMA roles (fixed): dY slot -> (patch pixel, logical chunk); halo slot -> (halo pixel, chunk)
  int ypix[NYW], ych[NYW], hy[NXW], hx[NXW], hch[NXW];
#pragma unroll
  for (int i = 0; i < NYW; ++i) {
    const int slot = (wave + NW * i) * 64 + lane, row = slot / YCH, pc = slot % YCH;
    ypix[i] = row;
    ych[i] = (pc ^ (swz<C::YROWB>(row) << 2)) * 8;
  }
#pragma unroll
  for (int i = 0; i < NXW; ++i) {
    const int slot = (wave + NW * i) * 64 + lane, row = slot >> 3, pc = slot & 7;
    hy[i] = row < C::HH * HWD ? row / HWD : -1000;
    hx[i] = row - (row / HWD) * HWD;
    hch[i] = (pc ^ (swz<128>(row) << 2)) * 8;
  }
  // issue the DMA of patch pi (or zeros past the range) into stage st
  auto issue = [&](int pi, int st) {
    const bool live = pi < p1;
    const int pp = live ? pi : p0;
    const int img = pp / npi, q = pp - img * npi, ty = q / ntx;
    const int y0 = ty * TH, x0 = (q - ty * ntx) * 32;
    const int simg = img % sg.imgs;
    const uint8_t* sb = lds + st * STAGE;
#pragma unroll
    for (int i = 0; i < NYW; ++i) {
      const int y = y0 + (ypix[i] >> 5), x = x0 + (ypix[i] & 31);
      const int v = (live && y < H && x < W) ? (((img * H + y) * W + x) * a.ystr + a.yoff + m0 + ych[i]) * 2 : kFar;
      dma16(ry, sb + (wave + NW * i) * 1024, v);
    }
#pragma unroll
    for (int i = 0; i < NXW; ++i) {
      const int y = y0 + hy[i] - PH, x = x0 + hx[i] - PW;
      const int v = (live && y >= 0 && y < H && x >= 0 && x < W)
                        ? (((simg * H + y) * W + x) * sg.stride + cb + hch[i]) * 2 : kFar;
      dma16(rx, sb + XOFF + (wave + NW * i) * 1024, v);
    }
  };

  // ---- fragment read roles: 16-lane group g, lane gi = 4q + p addresses row q, columns 4p..4p+3
  // (LDS reads are inline asm: the compiler cannot prove they miss the next
  // patch's in-flight DMA and would drain vmcnt in front of them)
  const int g = lane >> 4, gi = lane & 15, q4 = gi >> 2, p4 = gi & 3, h = lane >> 5;
  const int acb = (cw * 32 + 16 * (g & 1) + 4 * p4) * 2;  // dY column byte (output channel)
  const int bcb = (kh * 32 + 16 * (g & 1) + 4 * p4) * 2;  // halo column byte (input channel)
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) uint8_t*)lds;
  // A rows r*32 + ks*16 + 8h + q4 (+4): the quarter swizzle depends only on q4
  const uint32_t aaddr = lds0 + (8 * h + q4) * C::YROWB +
                         ((((acb >> 4) ^ (swz<C::YROWB>(q4) << 2)) << 4) | (acb & 15));
  // B halo rows Ck + 8h + q4 (+4) with Ck compile-time: the swizzle depends on (Ck + q4) & 3
  uint32_t baddr[4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
    baddr[m] = lds0 + XOFF + (8 * h + q4) * 128 + ((((bcb >> 4) ^ (swz<128>(m + q4) << 2)) << 4) | (bcb & 15));

  f32x16_t acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[t][j] = 0.f;
  float bsum = 0.f;
  const bool do_bias = a.bpart != nullptr && c == 0 && kh == 0;

  constexpr int PER = NYW + NXW;  // DMA instructions per wave per patch
  if (p0 < p1) issue(p0, 0);
  for (int pi = p0; pi < p1; ++pi) {
    const int st = (pi - p0) & 1;
    issue(pi + 1, st ^ 1);  // the next patch (zeros past the range): a static vmcnt count
    wait_vm<PER>();         // this patch's own pieces have landed
    asm volatile("s_barrier" ::: "memory");  // ... and every other wave's
    const uint32_t so = st * STAGE;
    // one K step = 16 pixels (patch row R, half KS); every LDS offset is an immediate
    sfor<0, 2 * TH>([&](auto step_) {
      constexpr int R = decltype(step_)::value / 2, KS = decltype(step_)::value % 2;
      v4s_t alo, ahi, blo[T], bhi[T];
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(alo)
                   : "v"(aaddr + so), "i"((R * 32 + KS * 16) * C::YROWB) : "memory");
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(ahi)
                   : "v"(aaddr + so), "i"((R * 32 + KS * 16 + 4) * C::YROWB) : "memory");
      read_taps<0, T, KW, HWD, R, KS>(blo, bhi, baddr, so);
      // LDS reads return in order: tap t's MFMA waits only for A and B[0..t]
      wait_lgkm<2 * (T - 1)>();
      asm volatile("" : "+v"(alo), "+v"(ahi));
      const bf16x8_t av = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(alo, ahi, 0, 1, 2, 3, 4, 5, 6, 7));
      __builtin_amdgcn_sched_barrier(0);
      mfma_taps<0, T>(acc, av, blo, bhi);
      if (do_bias) {
#pragma unroll
        for (int j = 0; j < 8; ++j) bsum += __uint_as_float((uint32_t)(uint16_t)av[j] << 16);  // raw bf16 bits
      }
    });
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // every wave done with this stage
  }
  wait_vm<0>();

  // ---- partial tile: acc[t] reg i -> co = m0 + cw*32 + (i&3) + 8(i>>2) + 4h, k = c*64 + kh*32 + lane&31
  float* out = a.part + (size_t)split * a.Cpad * T * a.Ktot;
  const int k = c * 64 + kh * 32 + (lane & 31);
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int co = m0 + cw * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
      out[((size_t)co * T + t) * a.Ktot + k] = acc[t][i];
    }
  if (do_bias) {
    bsum += __shfl_xor(bsum, 32);
    if (lane < 32) a.bpart[(size_t)split * a.Cpad + m0 + cw * 32 + lane] = bsum;
  }
}

// dW[co][t][k] += sum over splits (in order); db[co] += sum of the bias partials
__global__ __launch_bounds__(256) void wg3_reduce_kernel(const float* __restrict__ part, int nsplit, long n4,
                                                          int Cout, int rowlen, float* __restrict__ dw,
                                                          const float* __restrict__ bpart, int Cpad,
                                                          float* __restrict__ db) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n4) {
    if ((i * 4) / rowlen < Cout) {
      float4 s = reinterpret_cast<const float4*>(part)[i];
      for (int sp = 1; sp < nsplit; ++sp) {
        const float4 v = reinterpret_cast<const float4*>(part)[(long)sp * n4 + i];
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      }
      float4 o = reinterpret_cast<float4*>(dw)[i];
      o.x += s.x; o.y += s.y; o.z += s.z; o.w += s.w;
      reinterpret_cast<float4*>(dw)[i] = o;
    }
  }
  if (bpart != nullptr && i < Cout) {
    float s = 0.f;
    for (int sp = 0; sp < nsplit; ++sp) s += bpart[(long)sp * Cpad + i];
    db[i] += s;
  }
}

}  // namespace wg3

// host side ------------------------------------------------------------------
struct Wgrad3Launch {
  const void* dy;
  int ystr, yoff, Cout;
  unsigned dy_bytes;
  const void* seg_ptr[3];
  int seg_C[3], seg_stride[3], seg_imgs[3];
  unsigned seg_bytes[3];
  int nseg;
  int NI, H, W, KH, KW, Ktot;
  float* dw;  // [>= Cpad][T][Ktot] accumulated into (rows < Cout)
  float* db;  // [Cout] accumulated into, or null
  float* part;   // workspace: wgrad3_workspace() floats
  int bm;        // 64 or 128 output channels per block
  int nsplit;
};

static int wg3_th(int) { return 4; }  // patch rows (every instantiation below)

int wgrad3_splits(int NI, int H, int W, int KH, int Cout, int Ktot, int bm) {
  const int TH = wg3_th(KH);
  const int npatch = NI * cdiv(H, TH) * cdiv(W, 32);
  const int tiles = cdiv(Cout, bm) * (Ktot / 64);
  int ns = std::max(1, 512 / std::max(1, tiles));  // ~512 blocks: two rounds of one block per CU
  ns = std::min(ns, npatch);
  return ns;
}

long wgrad3_workspace(int Cout, int Ktot, int KH, int KW, int bm, int nsplit) {
  const int Cpad = cdiv(Cout, bm) * bm;
  return (long)nsplit * Cpad * KH * KW * Ktot + (long)nsplit * Cpad;
}

void wgrad3_launch(const Wgrad3Launch& L, hipStream_t stream) {
  wg3::Args a{};
  a.dy = static_cast<const bf16_t*>(L.dy);
  a.ystr = L.ystr; a.yoff = L.yoff; a.Cout = L.Cout; a.dy_bytes = L.dy_bytes;
  for (int s = 0; s < 3; ++s) {
    const int ss = s < L.nseg ? s : 0;
    a.seg[s].ptr = static_cast<const bf16_t*>(L.seg_ptr[ss]);
    a.seg[s].C = L.seg_C[ss];
    a.seg[s].stride = L.seg_stride[ss];
    a.seg[s].imgs = L.seg_imgs[ss];
    a.seg[s].bytes = L.seg_bytes[ss];
  }
  a.nseg = L.nseg;
  a.NI = L.NI; a.H = L.H; a.W = L.W; a.Ktot = L.Ktot;
  const int T = L.KH * L.KW;
  const int TH = wg3_th(L.KH);
  const int npatch = L.NI * cdiv(L.H, TH) * cdiv(L.W, 32);
  a.nsplit = L.nsplit;
  a.ppb = cdiv(npatch, L.nsplit);
  a.Cpad = cdiv(L.Cout, L.bm) * L.bm;
  a.part = L.part;
  a.bpart = L.db ? L.part + (long)L.nsplit * a.Cpad * T * L.Ktot : nullptr;
  const int nblk = L.nsplit * (a.Cpad / L.bm) * (L.Ktot / 64);
#define RS_WG3(KH_, KW_, NWM_)                                                                      \
  do {                                                                                              \
    using Gc = wg3::G<KH_, KW_, NWM_, 4>;                                                          \
    hipLaunchKernelGGL((wg3::wgrad3_kernel<KH_, KW_, NWM_, 4>), dim3(nblk), dim3(Gc::NT), 0, stream, a); \
  } while (0)
  if (L.bm == 128) {
    if (L.KH == 3) RS_WG3(3, 3, 4);
    else if (L.KH == 1) RS_WG3(1, 5, 4);
    else RS_WG3(5, 1, 4);
  } else {
    if (L.KH == 3) RS_WG3(3, 3, 2);
    else if (L.KH == 1) RS_WG3(1, 5, 2);
    else RS_WG3(5, 1, 2);
  }
#undef RS_WG3
  const long n4 = (long)a.Cpad * T * L.Ktot / 4;
  hipLaunchKernelGGL(wg3::wg3_reduce_kernel, dim3((unsigned)cdiv(std::max<long>(n4, a.Cpad), 256L)), dim3(256), 0,
                     stream, L.part, L.nsplit, n4, L.Cout, T * L.Ktot, L.dw, a.bpart, a.Cpad, L.db);
}

}  // namespace rs
