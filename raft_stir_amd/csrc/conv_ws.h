// Weight-stationary implicit-GEMM convolution for the RAFT update block
// (reference core/update.py:6-136: the motion encoder, SepConvGRU / ConvGRU,
// flow and mask heads, and their input-gradient convolutions in training).
//
// Why a third conv design (profiles/conv_tiles_r2.md): the tile kernels of
// conv.hip / conv_v2.hip re-stage a weight tile at EVERY (tap, 64-channel)
// K step.  At the update block's shapes (1 x 55 x 136 inference, 8 x 46 x 62
// training) that leaves one wave per SIMD doing ~100 SALU + ~60 VALU of
// staging bookkeeping, barriers and DMA issue around only 16 MFMA issue slots:
// ~10 % MFMA busy.  Here the weights are loaded ONCE per block, into VGPRs,
// and the loop is almost only `ds_read_b128` + `v_mfma_f32_32x32x16_bf16`:
//
// * Block = NCB co-blocks (32 output channels each) x NCS channel slices;
//   one wave per (co-block, slice).  A wave keeps the A fragments of ITS 32
//   output channels x (all taps x CPW = Ktot / NCS input channels) in
//   registers for the whole kernel: FR = taps * CPW / 16 fragments of 4 VGPRs
//   (FR <= 36, <= 144 VGPRs).  The host packs the weights in fragment order
//   (ops/conv.py frag_layout), so each fragment is one coalesced 1-KiB load.
// * Pixels: the block owns a 16-pixel-wide column strip of one image over a
//   range of rows, and walks down it TH = 2 rows (one 32 x 32 MFMA N-block =
//   2 rows x 16 columns) at a time.  The input rows live in an LDS ring of
//   2*TH + KH - 1 halo rows (16 + KW - 1 pixels, all Ktot channels): each
//   tile fetches only its TH new rows (global_load_lds, one step ahead), so a
//   3x3 / 5x1 conv reads every input row once per block, not KH times.
//   Pixel rows are CPW*2 + 16 bytes (an odd number of 16-B slots), so the 16
//   pixels of a ds_read_b128 lane group hit 16 distinct bank slots at every
//   tap shift; ring rows are whole 1-KiB pieces (256-B aligned), so the two
//   rows of an N-block never collide either.  Tap shifts are ds_read
//   immediates.
// * Per tile a wave issues FR MFMAs into one 32x32 accumulator (B fragments
//   read 4 ahead of the MFMAs); the NCS channel-slice partials are summed
//   through LDS and each wave of a co-block finishes a quarter of the
//   channels with the shared fused epilogues (conv_common.h: bias / ReLU /
//   scale / GRU gates / GRU update / dgrad epilogues).
// * Halo pixels outside the image read a zero page (zero padding); pixels of
//   the strip beyond W or rows beyond the chunk are computed and not stored.
//
// Template: (KH, KW) taps, G = CPW / 16 (fragments per tap), NB = N-blocks
// per tile.  NCS / NCB / the pixel chunking are launch arguments.
#pragma once
#include "conv_common.h"

namespace rs {
namespace conv {

static __device__ uint4 g_ws_zero[64];  // 1 KiB of zeros (one copy per translation unit)

// s_waitcnt through the builtin (the compiler's wait-insertion pass sees it and
// knows the counted operations completed; an inline-asm wait it does not see)
template <int N>
__device__ __forceinline__ void ws_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}
__device__ __forceinline__ void ws_wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }

constexpr int kWsLdsSlots = 10240;  // 160 KiB in 16-B slots: one block per CU
constexpr int kWsPieces = 10;       // halo-prefetch DMA pieces per MFMA wave per tile (host-checked)
constexpr int kWsSlices = 4;        // channel slices = MFMA waves per block (+ as many helper waves)

template <int KH, int KW, int G, int NB>
struct WsCfg {
  static constexpr int TAPS = KH * KW, PH = KH / 2, PW = KW / 2;
  static constexpr int CPW = 16 * G;          // input channels per wave slice
  static constexpr int FR = TAPS * G;         // A fragments per wave
  static constexpr int TW = 16, TH = 2 * NB;  // tile: TH rows x 16 columns
  static constexpr int HWD = TW + KW - 1;     // halo row width (pixels)
  static constexpr int CS = 2 * G + 1;        // 16-B slots per halo pixel (last = pad)
  static constexpr int RR = 2 * TH + KH - 1;  // ring rows (NCS >= 4 channel slices: host-checked)
  static constexpr int NF = NB * FR;          // MFMAs per wave per tile
  static constexpr int D = 4;                 // B-fragment read group
  static constexpr int NG = (NF + D - 1) / D;
  static_assert(FR <= 40, "weight fragments must fit the register file (and vmcnt counts < 64)");
};

// slot q (0 .. rsp-1) of a halo row -> this lane's DMA source column, packed
// in one register: bits 0-1 segment (3 = zero page: pad slots, columns outside
// the image), bits 2-31 element offset of (pixel x, channel) in row 0 of image 0
__device__ __forceinline__ int ws_col(const Args& a, int q, int x0, int hwd, int cs, int cpw, int pw) {
  const int per_slice = hwd * cs;
  if (q >= a.ws_ncs * per_slice) return 3;
  const int sl = q / per_slice, r2 = q - sl * per_slice;
  const int j = r2 / cs, c = r2 - j * cs;
  if (c == cs - 1) return 3;  // pad slot
  const int x = x0 + j - pw;
  if (x < 0 || x >= a.W) return 3;
  int kc = sl * cpw + c * 8;
  if (kc < a.seg[0].C) return ((x * a.seg[0].stride + kc) << 2) | 0;
  kc -= a.seg[0].C;
  if (kc < a.seg[1].C) return ((x * a.seg[1].stride + kc) << 2) | 1;
  kc -= a.seg[1].C;
  return ((x * a.seg[2].stride + kc) << 2) | 2;
}

// The segment base pointers / row strides, read once from the kernel
// arguments into SGPRs: a per-lane select among them must not become a
// VGPR-indexed load of the kernarg block (plus a vmcnt(0) that would drain
// the in-flight halo prefetch).
__device__ __forceinline__ uint64_t ws_sgpr64(const void* p) {
  const uint64_t v = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// global source of a packed column at image row (img, y) (y inside the image)
__device__ __forceinline__ const void* ws_src(uint64_t p0, uint64_t p1, uint64_t p2, int r0, int r1, int r2, int code,
                                              int rowidx) {
  // (by value: a select among fields of a struct in memory becomes a
  // select of ADDRESSES + a per-lane scratch load)
  const int sg = code & 3;
  uint64_t base = sg == 0 ? p0 : p1;
  base = sg == 2 ? p2 : base;
  int rs = sg == 0 ? r0 : r1;
  rs = sg == 2 ? r2 : rs;
  const uint64_t addr = base + ((uint64_t)((int64_t)rowidx * rs + (code >> 2)) << 1);
  return sg == 3 ? (const void*)g_ws_zero : (const void*)addr;
}

// ---- epilogues, split in two so that no global-load latency sits between
// a tile's barrier and its stores: ws_pre loads the operands of 4 output
// channels co..co+3 of pixel p (bias, or the fp32 accumulator being added to;
// h / z / r / the ReLU output) BEFORE the tile's MFMAs, ws_fin applies the
// epilogue after the channel-slice reduction.  Same math as conv_common.h
// epi_frag (host-checked: vector-aligned operands, no EPI_FLOW, no bias on
// the accumulating epilogues).
// epilogue classes (template parameter EK of the kernel): the kernel is
// compiled per class so that only the operands and fields it uses are live
enum WsEk : int { EK_PLAIN = 0, EK_ZR = 1, EK_Q = 2, EK_RELUBWD = 3, EK_ACC = 4, EK_QBWD = 5 };
__host__ __device__ constexpr int ws_class(int epi) {
  return epi == EPI_GRU_ZR ? EK_ZR : epi == EPI_GRU_Q ? EK_Q : epi == EPI_RELU_BWD ? EK_RELUBWD
       : epi == EPI_ACC_F32 ? EK_ACC : epi == EPI_GRU_QBWD ? EK_QBWD : EK_PLAIN;
}

struct WsPre {
  f32x4_t bo;  // bias, or the fp32 output being accumulated into
  uint2 a1, a2;
};

__device__ __forceinline__ uint2 ws_ld8(const bf16_t* p) { return *reinterpret_cast<const uint2*>(p); }
__device__ __forceinline__ float ws_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float ws_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ void ws_unpack(uint2 u, float (&f)[4]) {
  f[0] = ws_lo(u.x);
  f[1] = ws_hi(u.x);
  f[2] = ws_lo(u.y);
  f[3] = ws_hi(u.y);
}

template <int EK>
__device__ __forceinline__ void ws_pre(const Args& a, int co, int p, bool ok, WsPre& r) {
  // host-checked: the bias holds round_up(Cout, 4) values; every epilogue but
  // the plain one has Cout % 4 == 0 -- so all loads are whole 4-channel vectors
  r.bo = f32x4_t{0.f, 0.f, 0.f, 0.f};
  r.a1 = r.a2 = make_uint2(0u, 0u);
  if (!ok) return;
  if constexpr (EK == EK_ACC || EK == EK_QBWD) {
    r.bo = *reinterpret_cast<const f32x4_t*>(static_cast<const float*>(a.out) + (size_t)p * a.ostr + a.ooff + co);
  } else {
    if (a.bias) r.bo = *reinterpret_cast<const f32x4_t*>(a.bias + co);
  }
  if constexpr (EK == EK_ZR) {
    if (co >= a.hd) r.a1 = ws_ld8(a.aux1 + (size_t)p * a.a1str + a.a1off + co - a.hd);
  } else if constexpr (EK == EK_Q) {
    r.a1 = ws_ld8(a.aux1 + (size_t)p * a.a1str + a.a1off + co);
    r.a2 = ws_ld8(a.aux2 + (size_t)p * a.a2str + a.a2off + co);
  } else if constexpr (EK == EK_QBWD) {
    if (co < a.hd) {
      r.a1 = ws_ld8(a.aux1 + (size_t)p * a.a1str + a.a1off + co);
      r.a2 = ws_ld8(a.aux2 + (size_t)p * a.a2str + a.a2off + co);
    }
  } else if constexpr (EK == EK_RELUBWD) {
    r.a1 = ws_ld8(a.aux1 + (size_t)p * a.a1str + a.a1off + co);
  }
}

__device__ __forceinline__ void ws_st_bf16(bf16_t* o, const float (&f)[4], int n) {
  if (n == 4) {
    st4(o, f);
  } else {
    for (int j = 0; j < n; ++j) o[j] = f2bf(f[j]);
  }
}

template <int EK>
__device__ __forceinline__ void ws_fin(const Args& a, float (&v)[4], int co, int p, const WsPre& r) {
  const int n = min(4, a.Cout - co);
  if constexpr (EK == EK_ACC) {
    float* o = static_cast<float*>(a.out) + (size_t)p * a.ostr + a.ooff + co;
    *reinterpret_cast<f32x4_t*>(o) = f32x4_t{r.bo[0] + v[0], r.bo[1] + v[1], r.bo[2] + v[2], r.bo[3] + v[3]};
    return;
  }
  if constexpr (EK == EK_QBWD) {
    float* o = static_cast<float*>(a.out) + (size_t)p * a.ostr + a.ooff + co;
    if (co < a.hd) {
      float hv[4], rv[4], dv[4];
      ws_unpack(r.a1, hv);
      ws_unpack(r.a2, rv);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dv[j] = v[j] * hv[j] * rv[j] * (1.f - rv[j]);
        v[j] *= rv[j];
      }
      st4(static_cast<bf16_t*>(a.out2) + (size_t)p * a.o2str + a.o2off + co, dv);
    }
    *reinterpret_cast<f32x4_t*>(o) = f32x4_t{r.bo[0] + v[0], r.bo[1] + v[1], r.bo[2] + v[2], r.bo[3] + v[3]};
    return;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] += r.bo[j];
  if constexpr (EK == EK_ZR) {
    float g[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) g[j] = sigmoidf_(v[j]);
    if (co < a.hd) {
      st4(static_cast<bf16_t*>(a.out) + (size_t)p * a.ostr + a.ooff + co, g);
    } else {
      const int c = co - a.hd;
      float hv[4], rh[4];
      ws_unpack(r.a1, hv);
#pragma unroll
      for (int j = 0; j < 4; ++j) rh[j] = g[j] * hv[j];
      st4(static_cast<bf16_t*>(a.out2) + (size_t)p * a.o2str + a.o2off + c, rh);
      if (a.out3) st4(static_cast<bf16_t*>(a.out3) + (size_t)p * a.o3str + a.o3off + c, g);
    }
  } else if constexpr (EK == EK_Q) {
    float hv[4], zv[4], qv[4], nv[4];
    ws_unpack(r.a1, hv);
    ws_unpack(r.a2, zv);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      qv[j] = tanhf_(v[j]);
      nv[j] = (1.f - zv[j]) * hv[j] + zv[j] * qv[j];
    }
    st4(static_cast<bf16_t*>(a.out) + (size_t)p * a.ostr + a.ooff + co, nv);
    if (a.out2) st4(static_cast<bf16_t*>(a.out2) + (size_t)p * a.o2str + a.o2off + co, qv);
  } else if constexpr (EK == EK_RELUBWD) {
    float av[4];
    ws_unpack(r.a1, av);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = av[j] > 0.f ? v[j] : 0.f;
    st4(static_cast<bf16_t*>(a.out) + (size_t)p * a.ostr + a.ooff + co, v);
  } else {  // EK_PLAIN: bias / ReLU / scale
    const int e = a.epi;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (e == EPI_RELU) v[j] = fmaxf(v[j], 0.f);
      if (e == EPI_SCALE) v[j] *= a.scale;
    }
    ws_st_bf16(static_cast<bf16_t*>(a.out) + (size_t)p * a.ostr + a.ooff + co, v, n);
  }
}

// In-kernel timestamps (diagnostic builds with -DRS_WS_STAMPS only): per wave,
// stamp 0 at entry, 1 after the prologue barrier, then per tile t < 16:
// 2+4t tile start, 3+4t after the MFMAs, 4+4t after the first barrier,
// 5+4t after the epilogue.
constexpr int kWsStamps = 66;
#ifdef RS_WS_STAMPS
#define RS_WS_STAMP(I)                                                                            \
  do {                                                                                            \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                   \
    if (a.ws_stamps && (I) < kWsStamps && (threadIdx.x & 63) == 0)                                \
      a.ws_stamps[((size_t)blockIdx.x * 8 + (threadIdx.x >> 6)) * kWsStamps + (I)] = t_;          \
  } while (0)
#else
#define RS_WS_STAMP(I) \
  do {                 \
  } while (0)
#endif

template <int KH, int KW, int G, int EK>
__global__ __launch_bounds__(512) void conv_ws_kernel(Args a) {
  using C = WsCfg<KH, KW, G, 1>;
  constexpr int FR = C::FR, TH = C::TH, HWD = C::HWD, CS = C::CS, RR = C::RR, PH = C::PH, PW = C::PW;
  constexpr int CPW = C::CPW, NF = C::NF, D = C::D, NG = C::NG;
  constexpr int NCS = kWsSlices;  // MFMA waves = channel slices; waves NCS .. 2*NCS-1 are the helpers
  __shared__ uint4 lds[kWsLdsSlots];

  RS_WS_STAMP(0);
  const int lane_ = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool mfma_wave = wave < NCS;
  const int s = wave & (NCS - 1);  // MFMA wave: channel slice; helper: 8-channel output group
  const int RSP = a.ws_rsp;        // slots per ring row (multiple of 64)
  const int NPR = RSP >> 6;        // DMA pieces per ring row
  const int H = a.H, W = a.W;

  // ---- block -> (32-channel output block, image, column strip, row chunk)
  const int nstrips = a.ws_nstrips, nrch = a.ws_nrch;
  const int per_img = nstrips * nrch;
  const int nchunk = a.B * per_img;
  // chunk-major block order: with the XCD remap, each XCD (private L2) takes a
  // contiguous run of pixel chunks with ALL their output blocks, so its L2
  // holds ~1/8 of the input rows (+ all the weights) instead of every row
  const int ncob = gridDim.x / nchunk;
  const int lid = a.xcd_remap ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int chunk = lid / ncob;
  const int cob = lid - chunk * ncob;
  int rem = chunk;
  const int img = rem / per_img;
  rem -= img * per_img;
  const int strip = rem / nrch, rch = rem - strip * nrch;
  const int x0 = strip * C::TW, R0 = rch * a.ws_rpc;
  const int R1 = min(H, R0 + a.ws_rpc);
  const int ntiles = (R1 - R0 + TH - 1) / TH;
  // segment base pointers and row strides (elements), in SGPRs
  const uint64_t sp0 = ws_sgpr64(a.seg[0].ptr), sp1 = ws_sgpr64(a.seg[1].ptr), sp2 = ws_sgpr64(a.seg[2].ptr);
  const int sr0 = __builtin_amdgcn_readfirstlane(W * a.seg[0].stride);
  const int sr1 = __builtin_amdgcn_readfirstlane(W * a.seg[1].stride);
  const int sr2 = __builtin_amdgcn_readfirstlane(W * a.seg[2].stride);

  // ---- prologue: the tile-0 halo rows R0-PH .. R0+TH+PH-1 -> ring rows 0 .. TH+KH-2 (all waves)
  uint4* const ring = lds;
  {
    const int np0 = (TH + KH - 1) * NPR;
    for (int P = wave; P < np0; P += 2 * NCS) {
      const int rr = P / NPR, pc = P - rr * NPR;
      const int y = R0 - PH + rr;
      const int code = ws_col(a, pc * 64 + lane_, x0, HWD, CS, CPW, PW);
      const void* src =
          (y >= 0 && y < H) ? ws_src(sp0, sp1, sp2, sr0, sr1, sr2, code, img * H + y) : (const void*)g_ws_zero;
      glds16(src, ring + rr * RSP + pc * 64);
    }
  }
  const int l32 = lane_ & 31, nr_ = l32 >> 4, nc_ = l32 & 15, h_ = lane_ >> 5;
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) uint4*)&lds[0];
  const int red0 = RR * RSP;  // partial sums: 2 buffers x [NCS slices][4 groups][64 lanes] slots

  if (mfma_wave) {
    // ================= MFMA waves: weights in VGPRs, B fragments from the ring
    u32x4_t wr[FR];
    {
      const int KG = a.ws_kg;
      const u32x4_t* wp = reinterpret_cast<const u32x4_t*>(a.wf) + (size_t)cob * C::TAPS * KG * 64 + lane_;
#pragma unroll
      for (int t = 0; t < C::TAPS; ++t)
#pragma unroll
        for (int g = 0; g < G; ++g) wr[t * G + g] = wp[((size_t)t * KG + s * G + g) * 64];
    }
    const uint32_t lane_off = lds0 + (uint32_t)(((s * HWD + nc_) * CS + h_) * 16);
    const uint32_t row_bytes = (uint32_t)RSP * 16;
    // the tile-0 halo (issued before the weights) has landed once at most the FR
    // weight loads are outstanding; tile 0's MFMAs then wait for the weights
    // (compiler-inserted counted waits).  The empty memory-clobbering asm keeps
    // the weight loads above the counted wait.
    asm volatile("" ::: "memory");
    ws_wait_vm<FR>();
    asm volatile("s_barrier" ::: "memory");
    RS_WS_STAMP(1);
    // the MFMA waves win issue arbitration against the helper wave on their SIMD
    __builtin_amdgcn_s_setprio(1);

    int rb = 0;  // ring row of tile t's first (top-halo) row = (t * TH) % RR
    auto tile = [&](const int t) __attribute__((always_inline)) {
      RS_WS_STAMP(2 + 4 * t);
      // LDS base of this lane's B fragments per kernel row
      uint32_t bbase[KH];
#pragma unroll
      for (int ty = 0; ty < KH; ++ty) {
        int rr = rb + nr_ + ty;
        rr = rr >= RR ? rr - RR : rr;
        bbase[ty] = lane_off + (uint32_t)rr * row_bytes;
      }
      f32x16_t acc;
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[j] = 0.f;
      // MFMA i (0 .. NF-1): fragment i = (ty*KW + tx)*G + g.  B fragments are
      // read in groups of D, two groups ahead of their MFMAs (3 buffers)
      u32x4_t bf[3][D];
#define RS_WS_READ(GRP, BUF)                                                                     \
  _Pragma("unroll") for (int d = 0; d < D; ++d) {                                                \
    const int i_ = (GRP) * D + d;                                                                \
    if (i_ < NF) {                                                                               \
      const int tap_ = i_ / G, g_ = i_ % G;                                                      \
      const int ty_ = tap_ / KW, tx_ = tap_ % KW;                                                \
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(bf[BUF][d])                           \
                   : "v"(bbase[ty_]), "i"((tx_ * CS + 2 * g_) * 16) : "memory");                \
    }                                                                                            \
  }
      RS_WS_READ(0, 0);
      if (NG > 1) RS_WS_READ(1, 1);
#pragma unroll
      for (int k = 0; k < NG; ++k) {
        // reads still in flight after group k's: groups k+1 and k+2
        if (k + 2 < NG) RS_WS_READ(k + 2, (k + 2) % 3);
        const int after = (k + 1 < NG ? ((k + 2) * D <= NF ? D : NF - (k + 1) * D) : 0) +
                          (k + 2 < NG ? ((k + 3) * D <= NF ? D : NF - (k + 2) * D) : 0);
        if (after >= 8) asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
        else if (after == 7) asm volatile("s_waitcnt lgkmcnt(7)" ::: "memory");
        else if (after == 6) asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory");
        else if (after == 5) asm volatile("s_waitcnt lgkmcnt(5)" ::: "memory");
        else if (after == 4) asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
        else if (after == 3) asm volatile("s_waitcnt lgkmcnt(3)" ::: "memory");
        else if (after == 2) asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
        else if (after == 1) asm volatile("s_waitcnt lgkmcnt(1)" ::: "memory");
        else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int d = 0; d < D; ++d) asm volatile("" : "+v"(bf[k % 3][d]));
#pragma unroll
        for (int d = 0; d < D; ++d) {
          const int i = k * D + d;
          if (i < NF)
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, wr[i]),
                                                          __builtin_bit_cast(bf16x8_t, bf[k % 3][d]), acc, 0, 0, 0);
        }
      }
#undef RS_WS_READ
      RS_WS_STAMP(3 + 4 * t);
      // this slice's partial of the 4 output groups -> red[t & 1][s][g]; a
      // compiler-visible store (it pads the MFMA-result -> LDS-store hazard,
      // which an inline-asm ds_write right behind the last MFMA does not get)
      const uint32_t paddr = lds0 + (uint32_t)((red0 + ((t & 1) * NCS * 4 + s * 4) * 64 + lane_) * 16);
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<__attribute__((address_space(3))) f32x4_t*>(paddr + g * 1024) =
            f32x4_t{acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]};
      ws_wait_lgkm0();
      asm volatile("s_barrier" ::: "memory");
      RS_WS_STAMP(4 + 4 * t);
    };
    if (ntiles > 0) tile(0);
    // every weight load has retired: redefine the fragments so the compiler
    // inserts no vmcnt wait for them in the loop (it would drain the prefetch)
    ws_wait_vm<0>();
#pragma unroll
    for (int f = 0; f < FR; ++f) asm volatile("" : "+v"(wr[f]));
    for (int t = 1; t < ntiles; ++t) {
      rb += TH;
      rb = rb >= RR ? rb - RR : rb;
      tile(t);
    }
  } else {
    // ================= helper waves, while the MFMA waves compute tile t:
    // the halo rows tile t+1 adds (LDS-DMA), tile t-1's reduction + epilogue,
    // and tile t's epilogue operands (loaded a tile ahead)
    const int np = TH * NPR;
    int pcode[kWsPieces];  // per-lane DMA source columns of pieces s, s + NCS, ... (host-checked count)
#pragma unroll
    for (int i = 0; i < kWsPieces; ++i) {
      const int P = s + NCS * i;
      pcode[i] = 3;
      if (P < np) {
        const int rr = P / NPR, pc = P - rr * NPR;
        pcode[i] = ws_col(a, pc * 64 + lane_, x0, HWD, CS, CPW, PW);
      }
    }
    ws_wait_vm<0>();
    asm volatile("s_barrier" ::: "memory");
    const int g = s;
    WsPre preC, preN;
    preC.bo = preN.bo = f32x4_t{0.f, 0.f, 0.f, 0.f};
    preC.a1 = preC.a2 = preN.a1 = preN.a2 = make_uint2(0u, 0u);
    for (int t = 0; t <= ntiles; ++t) {
      if (t + 1 < ntiles) {
        // pieces of the TH rows tile t+1 adds; their ring rows were last read
        // by tile t-1, whose MFMAs finished before the previous barrier
        const int ybase = R0 + (t + 1) * TH + PH;
#pragma unroll
        for (int i = 0; i < kWsPieces; ++i) {
          const int P = s + NCS * i;  // wave-uniform
          if (P < np) {
            const int prow = P / NPR, pdst = (P - prow * NPR) * 64;
            const int y = ybase + prow;
            const int rr = ((t + 1) * TH + KH - 1 + prow) % RR;
            int code = pcode[i];
            asm volatile("" : "+v"(code));  // per-tile address math: nothing hoisted out of the loop
            const void* src =
                y < H ? ws_src(sp0, sp1, sp2, sr0, sr1, sr2, code, img * H + y) : (const void*)g_ws_zero;
            glds16(src, ring + rr * RSP + pdst);
          }
        }
      }
      int h = h_, nr = nr_, nc = nc_, lane = lane_;
      asm volatile("" : "+v"(h), "+v"(nr), "+v"(nc), "+v"(lane));  // no per-lane hoisting out of the loop
      const int co = cob * 32 + 8 * g + 4 * h;
      const int x = x0 + nc;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      if (t >= 1) {
        const uint32_t rbase = lds0 + (uint32_t)((red0 + (((t - 1) & 1) * NCS * 4 + g) * 64 + lane) * 16);
        f32x4_t r0, r1, r2, r3;
        asm volatile("ds_read_b128 %0, %1" : "=v"(r0) : "v"(rbase) : "memory");
        asm volatile("ds_read_b128 %0, %1 offset:4096" : "=v"(r1) : "v"(rbase) : "memory");
        asm volatile("ds_read_b128 %0, %1 offset:8192" : "=v"(r2) : "v"(rbase) : "memory");
        asm volatile("ds_read_b128 %0, %1 offset:12288" : "=v"(r3) : "v"(rbase) : "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        asm volatile("" : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3));
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = (r0[j] + r1[j]) + (r2[j] + r3[j]);
      }
      // the DMA pieces just issued (due before the barrier) and the operands
      // loaded in the previous phase; every store of this phase comes after
      // this wait, so it never waits for a store
      ws_wait_vm<0>();
      if (t >= 1) {
        const int y = R0 + (t - 1) * TH + nr;
        if (co < a.Cout && y < R1 && x < W) ws_fin<EK>(a, v, co, (img * H + y) * W + x, preC);
      }
      if (t < ntiles) {
        const int y = R0 + t * TH + nr;
        ws_pre<EK>(a, co, (img * H + y) * W + x, co < a.Cout && y < R1 && x < W, preN);
      }
      preC = preN;
      if (t < ntiles) asm volatile("s_barrier" ::: "memory");
    }
  }
}

// launch one instantiation (a == nullptr: only report whether it exists);
// each epilogue class's instantiations live in their own translation unit
// (conv_ws_<class>.hip) so they compile in parallel
#define RS_WS(KH_, KW_, G_)                                                                           \
  if (KH == KH_ && KW == KW_ && G == G_) {                                                            \
    if (a)                                                                                            \
      hipLaunchKernelGGL((conv::conv_ws_kernel<KH_, KW_, G_, EK_>), dim3(nblocks), dim3(64 * 2 * kWsSlices), \
                         0, stream, *a);                                                              \
    return true;                                                                                      \
  }
#define RS_WS_1X1 RS_WS(1, 1, 4) RS_WS(1, 1, 6) RS_WS(1, 1, 8) RS_WS(1, 1, 12) RS_WS(1, 1, 16) RS_WS(1, 1, 18) RS_WS(1, 1, 24)
#define RS_WS_3X3 RS_WS(3, 3, 1) RS_WS(3, 3, 2) RS_WS(3, 3, 3) RS_WS(3, 3, 4)
#define RS_WS_SEP RS_WS(1, 5, 2) RS_WS(1, 5, 4) RS_WS(1, 5, 6) RS_WS(5, 1, 2) RS_WS(5, 1, 4) RS_WS(5, 1, 6)
#define RS_WS_DISPATCH(NAME, EK, LIST)                                                              \
  bool NAME(const conv::Args* a, int KH, int KW, int G, int NB, int nblocks, hipStream_t stream) {  \
    constexpr int EK_ = EK;                                                                         \
    if (NB != 1) return false;                                                                      \
    LIST                                                                                            \
    return false;                                                                                   \
  }

}  // namespace conv
}  // namespace rs
