// Backward of the all-pairs correlation volume on MFMA, with the pyramid
// gradient folded into the operand load (reference: the autograd backward of
// core/corr.py:52-60 corr() = fmap1^T fmap2 / sqrt(C) and of the avg_pool2d
// pyramid, core/corr.py:24-27).
//
// The lookups' backward accumulated the gradient of every pyramid level
// g_l[b][p1][cell] (fp32, one row per query pixel p1).  The gradient of the
// level-0 volume is
//   G[b][p1][p2] = scale * sum_l 4^-l g_l[b][p1][(y2 >> l, x2 >> l)]     (p2 = (y2, x2);
//                  a level-l cell exists for floor-pooled sizes only)
// and the features' gradients are two GEMMs over it:
//   df1[b][p1][c] = sum_p2 G[b][p1][p2] f2[b][p2][c]        (TRANS = false, M = N1, K = N2)
//   df2[b][p2][c] = sum_p1 G[b][p1][p2] f1[b][p1][c]        (TRANS = true,  M = N2, K = N1)
// G is never materialised: each block folds its 64 x 32 tile of G per K step
// straight from the gradient pyramid into LDS (bf16), instead of a fold pass
// writing a 130 MB bf16 G and two library GEMMs reading it back.
//
// Block: 64 output rows x all 256 channels, 4 waves; wave w owns channels
// [64w, 64w+64): 4 x 4 mfma_f32_16x16x32_bf16 tiles with the MFMA's A = the
// features (16 channels x 32 K; from fT, the features transposed to
// [b][c][K] so a lane's 8 K values are one 16-byte load) and B = the G tile
// (32 K x 16 rows, ds_read_b128 from the LDS image [row][K], 80-byte pitch:
// conflict-free for 16 consecutive rows).  The accumulator then holds
// D[channel][row]: a lane's 4 values are 4 consecutive channels of one output
// row, one 8-byte (bf16) / 16-byte (fp32) store.
// G tile staging: TRANS = false, thread (row m = t/4, 8 consecutive p2) reads
// two float4 of g_0 plus the coarser levels' cells; TRANS = true, thread
// (p2 = t%64, 8 consecutive p1) reads one g_0 value per p1 row (coalesced
// across the wave) and the 3 coarser cells of the same (y2, x2).  Next step's
// g loads are in flight while this step's MFMAs run (register prefetch, LDS
// double buffer, one barrier per step).
#include "common.h"

namespace rs {
namespace corrbwd {

struct GArgs {
  const float* g[4];
  int H[4], W[4], S[4];
  int levels;
  int B, N1, N2;
  float scale;
  const bf16_t* fT;  // [B][256][NP] bf16, rows zero-padded to NP (a multiple of 32)
  int NP;
  void* out;         // [B][M][256]
  int M, K;          // output rows, reduction length
  int vec;           // g_0 rows 16-byte aligned (8-float loads) -- the non-transposed staging
  int ksplit, kchunk;  // K split over ksplit blocks of kchunk (a multiple of KS) each: fp32 atomics into out
};

constexpr int BMR = 64, KS = 32, GP = 40;  // G tile rows, K step, LDS pitch (bf16)

__device__ __forceinline__ uint32_t pk2(float a, float b) { return uint32_t(f2bf(a)) | (uint32_t(f2bf(b)) << 16); }

// C: feature channels (256: RAFT, 128: RAFT-small); a wave owns C/4 of them (NT 16-channel tiles)
// SPLIT: the K range is split over a.ksplit blocks (more blocks in flight for
// the latency-bound G staging); each adds its partial tile into the zeroed
// fp32 output with atomics (not used in deterministic mode).
template <bool TRANS, typename OT, int C, bool SPLIT>
__global__ __launch_bounds__(256) void corr_bwd_kernel(GArgs a_) {
  constexpr int NT = C / 64;
  static_assert(!SPLIT || sizeof(OT) == 4, "split-K accumulates in fp32");
  __shared__ __attribute__((aligned(16))) bf16_t gs[2][BMR * GP];
  const GArgs a = a_;  // a local copy: the staging lambdas capture it (not the kernarg segment)
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int mblocks = cdiv(a.M, BMR);
  const int ks = SPLIT ? (int)(blockIdx.x % a.ksplit) : 0;
  const int bid = SPLIT ? (int)(blockIdx.x / a.ksplit) : (int)blockIdx.x;
  const int b = bid / mblocks, m0 = (bid - b * mblocks) * BMR;
  const int W0 = a.W[0];
  const size_t rowbase = (size_t)b * a.N1;  // g rows of image b
  const int kbeg = SPLIT ? ks * a.kchunk : 0;
  const int kend = SPLIT ? min(a.K, kbeg + a.kchunk) : a.K;
  const int nsteps = kend > kbeg ? cdiv(kend - kbeg, KS) : 0;

  // ---- G-tile staging: this thread's 8 values of the 64 x 32 tile
  // !TRANS: row m = m0 + t/4 (p1), K = k0 + 8*(t&3) .. +7 (p2)
  //  TRANS: row m = m0 + t%64 (p2), K = k0 + 8*(t>>6) .. +7 (p1)
  const int sm = TRANS ? (t & 63) : (t >> 2);
  const int sk = TRANS ? 8 * (t >> 6) : 8 * (t & 3);
  const int mrow = m0 + sm;
  const bool mok = mrow < a.M;
  // TRANS: the fixed p2 of this thread -> its coarser-level cell offsets (-1: no cell)
  int cell[4] = {0, -1, -1, -1};
  if (TRANS && mok) {
    const int y2 = mrow / W0, x2 = mrow - y2 * W0;
    cell[0] = mrow;
#pragma unroll
    for (int l = 1; l < 4; ++l)
      if (l < a.levels && (y2 >> l) < a.H[l] && (x2 >> l) < a.W[l]) cell[l] = (y2 >> l) * a.W[l] + (x2 >> l);
  }
  float v[8];
  auto load = [&](int k0) {
    if constexpr (TRANS) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int p1 = k0 + sk + i;
        float s = 0.f;
        if (mok && p1 < a.K) {
          const size_t r = rowbase + p1;
          s = a.g[0][r * a.S[0] + cell[0]];
          float w = 1.f;
#pragma unroll
          for (int l = 1; l < 4; ++l) {
            w *= 0.25f;
            if (cell[l] >= 0) s += w * a.g[l][r * a.S[l] + cell[l]];
          }
        }
        v[i] = s * a.scale;
      }
    } else {
      const int p2 = k0 + sk;
      const size_t r = rowbase + (mok ? mrow : 0);
      const float* g0 = a.g[0] + r * a.S[0];
      if (mok && a.vec && p2 + 8 <= a.K) {
        const float4 x = *reinterpret_cast<const float4*>(g0 + p2);
        const float4 y = *reinterpret_cast<const float4*>(g0 + p2 + 4);
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w; v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = (mok && p2 + i < a.K) ? g0[p2 + i] : 0.f;
      }
      int y2 = p2 / W0, x2 = p2 - y2 * W0;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (mok && p2 + i < a.K) {
          float w = 1.f;
#pragma unroll
          for (int l = 1; l < 4; ++l) {
            w *= 0.25f;
            if (l < a.levels && (y2 >> l) < a.H[l] && (x2 >> l) < a.W[l])
              v[i] += w * a.g[l][r * a.S[l] + (y2 >> l) * a.W[l] + (x2 >> l)];
          }
        }
        v[i] *= a.scale;
        if (++x2 == W0) { x2 = 0; ++y2; }
      }
    }
  };
  auto store = [&](int buf) {
    *reinterpret_cast<uint4*>(&gs[buf][sm * GP + sk]) =
        make_uint4(pk2(v[0], v[1]), pk2(v[2], v[3]), pk2(v[4], v[5]), pk2(v[6], v[7]));
  };

  // ---- MFMA operands
  const int r16 = lane & 15, q = lane >> 4;
  const bf16_t* fT = a.fT + ((size_t)b * C + wave * (C / 4) + r16) * a.NP + 8 * q;  // + nt*16 rows, + k0
  f32x4_t acc[NT][4];  // [n-tile: 16 channels][m-tile: 16 rows]
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // the features' fragments of step s + 1 are loaded during step s (a dependent
  // global load per step otherwise exposes its full latency every K step)
  uint4 fa[NT], fn[NT];
  if (nsteps > 0) {
    load(kbeg);
    store(0);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) fa[nt] = *reinterpret_cast<const uint4*>(fT + (size_t)nt * 16 * a.NP + kbeg);
  }
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1, k0 = kbeg + s * KS;
    const bool more = s + 1 < nsteps;
    if (more) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) fn[nt] = *reinterpret_cast<const uint4*>(fT + (size_t)nt * 16 * a.NP + k0 + KS);
      load(k0 + KS);
    }
    uint4 gb[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) gb[mt] = *reinterpret_cast<const uint4*>(&gs[buf][(mt * 16 + r16) * GP + 8 * q]);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
        acc[nt][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[nt]),
                                                              __builtin_bit_cast(bf16x8_t, gb[mt]), acc[nt][mt], 0,
                                                              0, 0);
    if (more) {
      store(buf ^ 1);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) fa[nt] = fn[nt];
    }
    __syncthreads();
  }
  if (SPLIT && nsteps == 0) return;

  // ---- epilogue: D[channel = 4q + j][row = r16] of each tile -> out[b][row][channel]
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    const int row = m0 + mt * 16 + r16;
    if (row >= a.M) continue;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int c = wave * (C / 4) + nt * 16 + 4 * q;
      const size_t o = ((size_t)b * a.M + row) * C + c;
      if constexpr (SPLIT) {
        float* op = static_cast<float*>(a.out) + o;
#pragma unroll
        for (int j = 0; j < 4; ++j) atomicAdd(op + j, acc[nt][mt][j]);
      } else if constexpr (sizeof(OT) == 2) {
        *reinterpret_cast<uint2*>(static_cast<bf16_t*>(a.out) + o) =
            make_uint2(pk2(acc[nt][mt][0], acc[nt][mt][1]), pk2(acc[nt][mt][2], acc[nt][mt][3]));
      } else {
        *reinterpret_cast<float4*>(static_cast<float*>(a.out) + o) =
            make_float4(acc[nt][mt][0], acc[nt][mt][1], acc[nt][mt][2], acc[nt][mt][3]);
      }
    }
  }
}

// x [B][N][C] bf16 -> xT [B][C][NP] bf16, columns N .. NP-1 zero (64 x 64 tiles via LDS)
__global__ __launch_bounds__(256) void transpose_kernel(const bf16_t* __restrict__ x, int N, int NP, int C,
                                                        bf16_t* __restrict__ xT) {
  __shared__ bf16_t tile[64][66];
  const int nb = cdiv(NP, 64), cb = C / 64;
  const int b = blockIdx.x / (nb * cb), rem = blockIdx.x - b * nb * cb;
  const int n0 = (rem / cb) * 64, c0 = (rem % cb) * 64;
  const int t = threadIdx.x;
  for (int i = t; i < 64 * 64; i += 256) {
    const int n = i >> 6, c = i & 63;
    tile[n][c] = (n0 + n < N) ? x[((size_t)b * N + n0 + n) * C + c0 + c] : (bf16_t)0;
  }
  __syncthreads();
  for (int i = t; i < 64 * 64; i += 256) {
    const int c = i >> 6, n = i & 63;
    if (n0 + n < NP) xT[((size_t)b * C + c0 + c) * NP + n0 + n] = tile[n][c];
  }
}

}  // namespace corrbwd

// gpyr: levels of [B][N1][cells] fp32 (row pitch S[l]); f1 [B][N1][C], f2 [B][N2][C] bf16 (N2 = H0*W0 = N1)
// -> df1 [B][N1][C], df2 [B][N2][C] (bf16, or fp32: out_f32); scratch: xT [B][C][NP] bf16, NP = round_up(N, 32)
// ksplit > 1: df1 / df2 must be ZEROED fp32 (out_f32) -- the K-split blocks add into them
void corr_bwd_launch(float* const* g, const int* H, const int* W, const int* S, int levels, int B, int N1, int C,
                     const void* f1, const void* f2, float scale, void* df1, void* df2, bool out_f32, void* scratch,
                     int NP, int ksplit, hipStream_t stream) {
  corrbwd::GArgs a{};
  for (int l = 0; l < 4; ++l) {
    a.g[l] = l < levels ? g[l] : g[0];
    a.H[l] = l < levels ? H[l] : 1;
    a.W[l] = l < levels ? W[l] : 1;
    a.S[l] = l < levels ? S[l] : S[0];
  }
  a.levels = levels;
  a.B = B;
  a.N1 = N1;
  a.N2 = H[0] * W[0];
  a.scale = scale;
  a.NP = NP;
  a.vec = (S[0] % 4 == 0) && ((uintptr_t)g[0] % 16 == 0);
  bf16_t* xT = static_cast<bf16_t*>(scratch);
  const dim3 gt(B * cdiv(NP, 64) * (C / 64));
  a.ksplit = ksplit > 1 ? ksplit : 1;
#define RS_CB(TR, OT_)                                                                                   \
  do {                                                                                                  \
    a.kchunk = round_up(cdiv(a.K, a.ksplit), corrbwd::KS);                                              \
    const dim3 g_(B * cdiv(a.M, corrbwd::BMR) * a.ksplit);                                              \
    if (a.ksplit > 1) {                                                                                 \
      if (C == 256) hipLaunchKernelGGL((corrbwd::corr_bwd_kernel<TR, float, 256, true>), g_, dim3(256), 0, stream, a); \
      else hipLaunchKernelGGL((corrbwd::corr_bwd_kernel<TR, float, 128, true>), g_, dim3(256), 0, stream, a);     \
    } else {                                                                                            \
      if (C == 256) hipLaunchKernelGGL((corrbwd::corr_bwd_kernel<TR, OT_, 256, false>), g_, dim3(256), 0, stream, a); \
      else hipLaunchKernelGGL((corrbwd::corr_bwd_kernel<TR, OT_, 128, false>), g_, dim3(256), 0, stream, a);     \
    }                                                                                                   \
  } while (0)
  // df1 = G f2: fT = f2^T
  hipLaunchKernelGGL(corrbwd::transpose_kernel, gt, dim3(256), 0, stream, static_cast<const bf16_t*>(f2), a.N2, NP,
                     C, xT);
  a.fT = xT;
  a.out = df1;
  a.M = N1;
  a.K = a.N2;
  if (out_f32) RS_CB(false, float); else RS_CB(false, bf16_t);
  // df2 = G^T f1: fT = f1^T (the same scratch: stream-ordered after the first GEMM)
  hipLaunchKernelGGL(corrbwd::transpose_kernel, gt, dim3(256), 0, stream, static_cast<const bf16_t*>(f1), N1, NP, C,
                     xT);
  a.out = df2;
  a.M = a.N2;
  a.K = N1;
  if (out_f32) RS_CB(true, float); else RS_CB(true, bf16_t);
#undef RS_CB
}

}  // namespace rs
