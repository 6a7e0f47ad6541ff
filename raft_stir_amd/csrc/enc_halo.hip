// Halo-tile 3x3 convolution for the encoder residual blocks
// (reference core/extractor.py:6-56: the stride-1 3x3 convs of layer1 (64 ch,
// 1/2 resolution) and layer2 (96 ch, 1/4)), forward and -- with the flipped,
// transposed packed weight -- input gradient.
//
// profiles/r2/enc_conv_tiles.txt: the implicit-GEMM tiles of conv.hip run the
// 1/2-res 64->64 conv at 125-140 us (53.8 GFLOP, 730k pixels): every block
// re-fetches the whole 64 x 576 weight matrix (73 KB) for its 64-128 pixels
// and every pixel row 9 times (once per tap), ~1.7 GB of L2->CU traffic for
// 186 MB of real HBM traffic.  Here
//  * the block's weights (COB output channels x 9 taps x CIN) are staged ONCE
//    in LDS and the block walks 12 consecutive tiles (~130 KB of LDS: one
//    block per CU at a time);
//  * a tile is 8 output rows x 32 pixels of one image; its 10 x 34 input
//    halo is loaded once (global -> registers, issued before the previous
//    tile's MFMAs, written to LDS after them between two barriers) and every
//    tap reads its shifted window from LDS;
//  * v_mfma_f32_32x32x16_bf16: wave w owns output rows 2w, 2w+1 of the tile
//    (2 x 32 pixels) x COB channels; per 16-deep K slice 2 pixel-operand and
//    COB/32 weight-operand ds_read_b128 feed 2 * COB/32 MFMAs, the reads of
//    slice s+3 issued before the MFMAs of slice s (explicit lgkmcnt waits);
//  * LDS rows (a halo pixel, a weight row) are CIN*2 + 16 bytes: an odd
//    number of 16-B bank slots, so the 16 lanes of a ds_read_b128 group
//    (consecutive pixels / consecutive output channels) hit 16 distinct slots
//    at any tap shift.
// Zero padding: halo pixels outside the image are written as zeros.
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "enc_epi.h"

namespace rs {
namespace ench {

struct HArgs {
  const bf16_t* x;  // NHWC input, xstr elements per pixel
  const bf16_t* w;  // packed [Cout_pad][9][Ktot]: (co, tap, ci) at co * 9 * Ktot + tap * Ktot + ci
  bf16_t* y;        // NHWC output, ystr elements per pixel
  int xstr, ystr, Ktot;
  int B, H, W, Cout;
  int tiles_w, tiles_img, ntiles;
  int tpb;  // consecutive tiles per block
  // optional epilogue extras (ops_conv.cpp conv3x3_halo):
  //   chs / shift: y = [relu](acc * chs + shift) [then relu(y + res)] (eval-mode BatchNorm)
  const float* chs;
  const float* shift;
  const bf16_t* res;
  int rstr, relu, res_relu;
};

template <int CIN, int COB>
struct Cfg {
  static constexpr int RPW = CIN >= 128 ? 1 : 2;  // output rows per wave (LDS: 128-ch halo rows are 272 B)
  static constexpr int TH = 4 * RPW, TW = 32;     // output tile
  static constexpr int HR = TH + 2, HC = TW + 2;  // input halo
  static constexpr int RB = CIN * 2 + 16;         // LDS bytes per halo pixel / weight row
  static constexpr int HALO_B = HR * HC * RB;
  static constexpr int W_B = 9 * COB * RB;
  static constexpr int LDS_B = W_B + HALO_B;      // one halo buffer: the next tile waits in registers
  static constexpr int CPP = CIN / 8;            // 16-B chunks per pixel
  static constexpr int NCH = HR * HC * CPP;      // chunks per halo
  static constexpr int NLD = (NCH + 255) / 256;  // per thread
  static constexpr int NMF = COB / 32;
  static_assert(CIN % 16 == 0 && COB % 32 == 0, "shape");
  static_assert(((RB / 16) & 1) == 1, "odd slot count per LDS row");
  static_assert(LDS_B <= 160 * 1024, "LDS");
};

typedef unsigned int v4u __attribute__((ext_vector_type(4)));  // 16-B fragment (register vector)

template <int N>
__device__ __forceinline__ void wait_lgkm() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}

// K slice S (16 deep) = tap S / (CIN/16), channels 16 * (S % (CIN/16)): one
// ds_read_b128 of the pixel operand and COB/32 of the weight operand into
// register slot S % 4 (prefetch distance 3: the reads of slice S + 3 are
// issued before the MFMAs of slice S).  Offsets are compile-time immediates.
// F[slot]: [0, RPW) pixel operands (one per output row of the wave), then NMF weight operands
template <int CIN, int COB, int S>
__device__ __forceinline__ void rd(v4u (&F)[4][4], uint32_t a0, uint32_t a1, uint32_t b) {
  using C = Cfg<CIN, COB>;
  constexpr int KS = CIN / 16, tap = S / KS, kk = S % KS, ky = tap / 3, kx = tap % 3;
  constexpr int boff = (ky * C::HC + kx) * C::RB + kk * 32;
  constexpr int aoff = (tap < 5 ? tap : tap - 5) * COB * C::RB + kk * 32;
  constexpr int sl = S % 4;
  const uint32_t ab = tap < 5 ? a0 : a1;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(F[sl][0]) : "v"(b), "i"(boff) : "memory");
  if constexpr (C::RPW == 2)
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(F[sl][1]) : "v"(b), "i"(boff + C::HC * C::RB) : "memory");
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(F[sl][C::RPW]) : "v"(ab), "i"(aoff) : "memory");
  if constexpr (C::NMF == 2)
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(F[sl][C::RPW + 1]) : "v"(ab), "i"(aoff + 32 * C::RB) : "memory");
}

template <int CIN, int COB, int S>
struct Steps {
  using C = Cfg<CIN, COB>;
  static constexpr int NS = 9 * (CIN / 16), R = C::RPW + C::NMF;
  static_assert(3 * R <= 15, "lgkmcnt range");
  __device__ __forceinline__ static void run(v4u (&F)[4][4], f32x16_t (&acc)[C::RPW][C::NMF], uint32_t a0,
                                             uint32_t a1, uint32_t b) {
    if constexpr (S < NS) {
      if constexpr (S + 3 < NS) rd<CIN, COB, S + 3>(F, a0, a1, b);
      constexpr int ahead = (NS - 1 - S) < 3 ? (NS - 1 - S) : 3;  // slices issued after S
      wait_lgkm<ahead * R>();
      constexpr int sl = S % 4;
      // fence: the operands are only valid after the wait (the reads are inline asm)
      v4u f0 = F[sl][0], f1 = F[sl][1], f2 = F[sl][2], f3 = F[sl][3];
      if constexpr (R == 4)
        asm volatile("" : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3));
      else if constexpr (R == 3)
        asm volatile("" : "+v"(f0), "+v"(f1), "+v"(f2));
      else
        asm volatile("" : "+v"(f0), "+v"(f1));
      const v4u fr[4] = {f0, f1, f2, f3};
#pragma unroll
      for (int r = 0; r < C::RPW; ++r)
#pragma unroll
        for (int mi = 0; mi < C::NMF; ++mi)
          acc[r][mi] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, fr[C::RPW + mi]),
                                                               __builtin_bit_cast(bf16x8_t, fr[r]), acc[r][mi], 0, 0, 0);
      Steps<CIN, COB, S + 1>::run(F, acc, a0, a1, b);
    }
  }
};

template <int CIN, int COB>
__global__ __launch_bounds__(256) void enc_halo_kernel(HArgs a) {
  using C = Cfg<CIN, COB>;
  __shared__ __attribute__((aligned(16))) uint8_t lds[C::LDS_B];
  uint8_t* wl = lds;            // [9][COB] rows
  uint8_t* hl = lds + C::W_B;   // [2][HR * HC] rows
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int co0 = blockIdx.y * COB;

  // weights of this block's output channels, all taps, once
  constexpr int WCH = 9 * COB * C::CPP;
  for (int q = t; q < WCH; q += 256) {
    const int kc = q % C::CPP, r = q / C::CPP;  // r = co_local * 9 + tap
    const int col = r / 9, tap = r - col * 9;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (co0 + col < a.Cout)
      v = *reinterpret_cast<const uint4*>(a.w + ((size_t)(co0 + col) * 9 + tap) * a.Ktot + kc * 8);
    *reinterpret_cast<uint4*>(wl + (tap * COB + col) * C::RB + kc * 16) = v;
  }

  uint4 pre[C::NLD];
  auto gload = [&](int tile) {
    const int b = tile / a.tiles_img, r = tile - b * a.tiles_img;
    const int th = r / a.tiles_w;
    const int ty0 = th * C::TH, tx0 = (r - th * a.tiles_w) * C::TW;
#pragma unroll
    for (int i = 0; i < C::NLD; ++i) {
      const int q = t + 256 * i;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (q < C::NCH) {
        const int kc = q % C::CPP, hp = q / C::CPP;
        const int hr = hp / C::HC, hc = hp - hr * C::HC;
        const int iy = ty0 - 1 + hr, ix = tx0 - 1 + hc;
        if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W)
          v = *reinterpret_cast<const uint4*>(a.x + ((size_t)(b * a.H + iy) * a.W + ix) * a.xstr + kc * 8);
      }
      pre[i] = v;
    }
  };
  auto lstore = [&]() {
    uint8_t* h = hl;
#pragma unroll
    for (int i = 0; i < C::NLD; ++i) {
      const int q = t + 256 * i;
      if (q < C::NCH) {
        const int kc = q % C::CPP, hp = q / C::CPP;
        *reinterpret_cast<uint4*>(h + hp * C::RB + kc * 16) = pre[i];
      }
    }
  };

  int tile = blockIdx.x * a.tpb;
  const int tend = min(a.ntiles, tile + a.tpb);
  if (tile < tend) {
    gload(tile);
    lstore();
  }
  __syncthreads();
  // LDS byte addresses of this lane's fragment rows: weights (taps 0-4 / 5-8, so
  // every ds_read offset fits the 16-bit immediate) and the halo
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) uint8_t*)&lds[0];
  const uint32_t a0 = lds0 + (lane & 31) * C::RB + (lane >> 5) * 16;
  const uint32_t a1 = a0 + 5 * COB * C::RB;
  const uint32_t hb0 = lds0 + C::W_B + (wave * C::RPW * C::HC + (lane & 31)) * C::RB + (lane >> 5) * 16;
  for (; tile < tend; ++tile) {
    const int nxt = tile + 1;
    if (nxt < tend) gload(nxt);  // in flight during this tile's MFMAs

    f32x16_t acc[C::RPW][C::NMF];
#pragma unroll
    for (int r = 0; r < C::RPW; ++r)
#pragma unroll
      for (int mi = 0; mi < C::NMF; ++mi)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[r][mi][j] = 0.f;
    const uint32_t b = hb0;
    v4u F[4][4];
    rd<CIN, COB, 0>(F, a0, a1, b);
    rd<CIN, COB, 1>(F, a0, a1, b);
    rd<CIN, COB, 2>(F, a0, a1, b);
    Steps<CIN, COB, 0>::run(F, acc, a0, a1, b);

    // the next tile's halo goes to LDS BEFORE this tile's output stores: the
    // vmcnt wait for the prefetched loads then never waits on fresh stores
    // (vmcnt counts both), and the stores drain during the next tile's MFMAs
    if (nxt < tend) {
      __syncthreads();  // every wave is done reading this tile's halo
      lstore();
    }
    // epilogue: lane holds pixel (lane & 31) of row wave*RPW + r, channels
    // mi*32 + 8g + 4*(lane>>5) + 0..3 in acc[r][mi][4g .. 4g+3]
    {
      const int bi = tile / a.tiles_img, rr = tile - bi * a.tiles_img;
      const int th = rr / a.tiles_w;
      const int ox = (rr - th * a.tiles_w) * C::TW + (lane & 31);
      if (a.chs) {  // eval-mode BatchNorm folded in: per-channel scale / shift (host-checked: padded, aligned)
#pragma unroll
        for (int mi = 0; mi < C::NMF; ++mi)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int c = co0 + mi * 32 + 8 * g + 4 * (lane >> 5);
            const float4 sv = *reinterpret_cast<const float4*>(a.chs + c);
            const float4 bv = *reinterpret_cast<const float4*>(a.shift + c);
            const float scv[4] = {sv.x, sv.y, sv.z, sv.w}, shv[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
            for (int r = 0; r < C::RPW; ++r)
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                float v = acc[r][mi][4 * g + j] * scv[j] + shv[j];
                acc[r][mi][4 * g + j] = a.relu ? fmaxf(v, 0.f) : v;
              }
          }
      }
#pragma unroll
      for (int r = 0; r < C::RPW; ++r) {
        const int oy = th * C::TH + wave * C::RPW + r;
        if (oy < a.H && ox < a.W) {
          const size_t pix = (size_t)(bi * a.H + oy) * a.W + ox;
          bf16_t* o = a.y + pix * a.ystr + co0;
          const bf16_t* rp = a.res ? a.res + pix * a.rstr + co0 : nullptr;
#pragma unroll
          for (int mi = 0; mi < C::NMF; ++mi)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const int cb = mi * 32 + 8 * g + 4 * (lane >> 5);
              if (co0 + cb < a.Cout) {
                float v[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = acc[r][mi][4 * g + j];
                if (rp) {
                  const uint2 u = *reinterpret_cast<const uint2*>(rp + cb);
                  v[0] += __uint_as_float(u.x << 16);
                  v[1] += __uint_as_float(u.x & 0xffff0000u);
                  v[2] += __uint_as_float(u.y << 16);
                  v[3] += __uint_as_float(u.y & 0xffff0000u);
                  if (a.res_relu) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
                  }
                }
                const uint2 pk = make_uint2(uint32_t(f2bf(v[0])) | (uint32_t(f2bf(v[1])) << 16),
                                            uint32_t(f2bf(v[2])) | (uint32_t(f2bf(v[3])) << 16));
                *reinterpret_cast<uint2*>(o + cb) = pk;
              }
            }
        }
      }
    }
    __syncthreads();
  }
}

}  // namespace ench

// Supported (cin, cout-block) instantiations; false = caller falls back.
bool enc_halo_supported(int cin, int cout) {
  return (cin == 64 && cout % 64 == 0) || (cin == 96 && cout % 32 == 0);
}

bool enc_halo_launch(const bf16_t* x, int xstr, const bf16_t* w, int Ktot, bf16_t* y, int ystr, int B, int H, int W,
                     int cin, int cout, int num_cus, const EncEpi& e, hipStream_t stream) {
  if (!enc_halo_supported(cin, cout)) return false;
  ench::HArgs a{};
  a.chs = e.chs; a.shift = e.shift; a.res = e.res; a.rstr = e.rstr; a.relu = e.relu; a.res_relu = e.res_relu;
  a.x = x; a.w = w; a.y = y;
  a.xstr = xstr; a.ystr = ystr; a.Ktot = Ktot;
  a.B = B; a.H = H; a.W = W; a.Cout = cout;
  a.tiles_w = cdiv(W, 32);
  static_assert(ench::Cfg<64, 64>::TH == ench::Cfg<96, 32>::TH, "one tile height for both channel counts");
  a.tiles_img = cdiv(H, ench::Cfg<64, 64>::TH) * a.tiles_w;
  a.ntiles = B * a.tiles_img;
  if (a.ntiles == 0) return true;
  const int cob = cin == 64 ? 64 : 32;
  const int gy = cdiv(cout, cob);
  // consecutive tiles per block (the LDS weights are loaded once per block),
  // picked by in-situ A/B (scripts/ab_halo_tpb.sh, ab_halo_tpb_infer.sh; paired
  // runs on one box): training (>= 1024 tile-blocks per conv) 12 tiles 383
  // pairs/s, 16: 380, 24: 374, 48 (~persistent): 350, 2-8: 368-379 -- the
  // encoders run these convs on two HIP streams at once and long-lived
  // CU-filling blocks of one stream serialise behind the other's; graphed
  // 1088x436 inference (< 1024) 4 tiles 286-289 FPS, 2: 278-281, 12: 266-268
  a.tpb = a.ntiles * gy >= 1024 ? 12 : 4;
  const int gx = cdiv(a.ntiles, a.tpb);
  if (cin == 64)
    hipLaunchKernelGGL((ench::enc_halo_kernel<64, 64>), dim3(gx, gy), dim3(256), 0, stream, a);
  else
    hipLaunchKernelGGL((ench::enc_halo_kernel<96, 32>), dim3(gx, gy), dim3(256), 0, stream, a);
  return true;
}

}  // namespace rs
