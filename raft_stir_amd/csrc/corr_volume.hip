// All-pairs correlation volume + fused 4-level pyramid, CDNA4 MFMA.
//
// Replaces reference core/corr.py:13-27 + :52-60 (torch.matmul of fmap1^T and
// fmap2 / sqrt(C), then 3x avg_pool2d(2,2)) with ONE kernel:
//
//   out_l[b, i, y, x] = mean_{2^l x 2^l block}( <f1[b,i,:], f2[b,(y',x'),:]> ) / sqrt(C)
//
// Layout: f1 (B, N1, C) and f2 (B, H2, W2, C) are channels-last (K-contiguous)
// so both MFMA operands are read as 16-byte K-runs (the "TN" GEMM).
//
// Tiling (wave64, 256 threads = 4 waves):
//   * BM = 64 query pixels (rows of the volume) x BN = 256 target pixels that
//     form an 8 x 32 2-D block of the target image;
//   * wave w owns all 64 query rows x the 8 x 8 target sub-block
//     [rows 0..7] x [cols 8w .. 8w+7]: 4 x 4 tiles of mfma_f32_16x16x32_bf16;
//   * because each 8 x 8 pooling window lives inside one wave, levels 1..3 are
//     reduced in registers with lane shuffles (xor 1/8 -> 2x2, xor 2 -> 4x4,
//     xor 4 -> 8x8) -- no LDS round trip and no extra pass over the volume;
//   * operands staged global -> registers -> LDS (XOR-swizzled 128-B rows,
//     conflict-free ds_read_b128 fragment reads), K step 64, next K-step's
//     loads issued before the current step's MFMAs.
// The kernel is write-bound (1.33 x B x N1 x H2W2 x 4 bytes of output), so the
// epilogue's coalescing matters more than MFMA issue rate.  (This 2-D-block
// kernel now serves fp32 feature maps only; see the flat path below.)
//
// An exact-fp32 variant (mfma_f32_16x16x4f32, bit-identical to an fmaf chain)
// serves fp32 mode.
//
// bf16 feature maps (autocast encoder) take the FLAT path instead
// (corr_flat_kernel below): the epilogue above stores 8-float runs from a
// 2-D target block, so with W = 136 a 128-B line of the volume is shared by
// neighbouring blocks on different XCDs and the kernel ran at ~0.9 TB/s
// (profiles/infer_kernel_stats_r1_final.csv, ~320 us at 1088x440).  By
// linearity pyramid level l equals corr(f1, avgpool^l(f2)), so
// the flat path pools f2 first (pool_f2_kernel, fp32 sums, one bf16 rounding)
// and runs one grouped GEMM over all levels whose tiles are 128 CONSECUTIVE
// targets of a volume row: every wave store is 16 B per lane along the row,
// rows start at 128-B multiples (padded pitch), so each line is written by
// one block, in fp32 or bf16 (RAFTConfig.corr_dtype).  Plain (L2 write-
// combining) stores: with the nontemporal hint each lane's 16 B left L2 as its
// own 64-B DRAM write (3.3x the volume bytes, TCC_EA0_WRREQ_64B).

#include "common.h"

namespace rs {
namespace corrvol {

constexpr int BM = 64;
constexpr int TH = 8;
constexpr int TW = 32;
constexpr int BN = TH * TW;
constexpr int THREADS = 256;

struct PyrOut {
  float* p[4];
  int H[4];
  int W[4];
  int S[4];  // row pitch (elements) of one (b, i) row of level l: >= H*W, 128-B multiple
};

// chunk (16 B) index of chunk c of LDS row r, 8 chunks per 128-B row.
__device__ __forceinline__ int swz(int r, int c) { return r * 8 + (c ^ ((r >> 1) & 7)); }

// Row of the B tile (8 x 32 target block, row-major) for wave w, n-tile t, lane col lc.
__device__ __forceinline__ int brow(int w, int t, int lc) {
  return (2 * t + (lc >> 3)) * TW + 8 * w + (lc & 7);
}

__device__ __forceinline__ void epilogue(const f32x4_t (&acc)[4][4], int levels, float scale,
                                         const PyrOut& out, int b, int N1, int m0, int th0,
                                         int tw0, int wave, int lane) {
  const int lr = lane & 15, lg = lane >> 4;
  const int wx = tw0 + 8 * wave;  // first target column of this wave
  float s1[4][4][4];              // [mt][nt][j]
  // level 0
  {
    const int H = out.H[0], W = out.W[0];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int h = th0 + 2 * nt + (lr >> 3);
        const int w = wx + (lr & 7);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int i = m0 + mt * 16 + lg * 4 + j;
          const float v = acc[mt][nt][j] * scale;
          s1[mt][nt][j] = v;
          if (i < N1 && h < H && w < W)
            out.p[0][((size_t)b * N1 + i) * out.S[0] + (size_t)h * W + w] = v;
        }
      }
  }
  if (levels < 2) return;
  // level 1: 2x2 = lanes {lc, lc^1} x rows {lc, lc^8}
  {
    const int H = out.H[1], W = out.W[1];
    const bool st = (lr & 9) == 0;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float v = s1[mt][nt][j];
          v += __shfl_xor(v, 1, 64);
          v += __shfl_xor(v, 8, 64);
          v *= 0.25f;
          s1[mt][nt][j] = v;
          const int i = m0 + mt * 16 + lg * 4 + j;
          const int h = (th0 >> 1) + nt, w = (wx >> 1) + ((lr & 7) >> 1);
          if (st && i < N1 && h < H && w < W)
            out.p[1][((size_t)b * N1 + i) * out.S[1] + (size_t)h * W + w] = v;
        }
  }
  if (levels < 3) return;
  float s2[4][2][4];
  {
    const int H = out.H[2], W = out.W[2];
    const bool st = (lr & 11) == 0;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float v = s1[mt][2 * s][j] + s1[mt][2 * s + 1][j];
          v += __shfl_xor(v, 2, 64);
          v *= 0.25f;
          s2[mt][s][j] = v;
          const int i = m0 + mt * 16 + lg * 4 + j;
          const int h = (th0 >> 2) + s, w = (wx >> 2) + ((lr & 7) >> 2);
          if (st && i < N1 && h < H && w < W)
            out.p[2][((size_t)b * N1 + i) * out.S[2] + (size_t)h * W + w] = v;
        }
  }
  if (levels < 4) return;
  {
    const int H = out.H[3], W = out.W[3];
    const bool st = (lr & 15) == 0;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v = s2[mt][0][j] + s2[mt][1][j];
        v += __shfl_xor(v, 4, 64);
        v *= 0.25f;
        const int i = m0 + mt * 16 + lg * 4 + j;
        const int h = th0 >> 3, w = wx >> 3;
        if (st && i < N1 && h < H && w < W)
          out.p[3][((size_t)b * N1 + i) * out.S[3] + (size_t)h * W + w] = v;
      }
  }
}

// ---------------------------------------------------------- exact fp32 MFMA
__global__ __launch_bounds__(THREADS) void corr_volume_f32_kernel(
    const float* __restrict__ f1, const float* __restrict__ f2, int N1, int H2, int W2, int C,
    float scale, int levels, PyrOut out) {
  constexpr int BK = 32;
  constexpr int LD = BK + 1;  // pad: 16 lanes reading 16 rows at one k hit 16 banks
  __shared__ float As[BM * LD];
  __shared__ float Bs[BN * LD];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.z;
  const int m0 = blockIdx.y * BM;
  const int nTW = cdiv(W2, TW);
  const int th0 = (blockIdx.x / nTW) * TH;
  const int tw0 = (blockIdx.x % nTW) * TW;
  const float* f1b = f1 + (size_t)b * N1 * C;
  const float* f2b = f2 + (size_t)b * H2 * W2 * C;

  float4 ra[2], rb[8];
  auto gload = [&](int k0) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int idx = tid + THREADS * q, r = idx >> 3, c = idx & 7;
      const int m = m0 + r;
      const float4 v_ = *reinterpret_cast<const float4*>(f1b + (size_t)min(m, N1 - 1) * C + k0 + c * 4);
      ra[q] = (m < N1) ? v_ : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int idx = tid + THREADS * q, r = idx >> 3, c = idx & 7;
      const int h = th0 + r / TW, w = tw0 + r % TW;
      const float4 v_ = *reinterpret_cast<const float4*>(f2b + ((size_t)min(h, H2 - 1) * W2 + min(w, W2 - 1)) * C + k0 + c * 4);
      rb[q] = (h < H2 && w < W2) ? v_ : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int idx = tid + THREADS * q, r = idx >> 3, c = (idx & 7) * 4;
      float* d = As + r * LD + c;
      d[0] = ra[q].x; d[1] = ra[q].y; d[2] = ra[q].z; d[3] = ra[q].w;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int idx = tid + THREADS * q, r = idx >> 3, c = (idx & 7) * 4;
      float* d = Bs + r * LD + c;
      d[0] = rb[q].x; d[1] = rb[q].y; d[2] = rb[q].z; d[3] = rb[q].w;
    }
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[a][c] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int lr = lane & 15, lg = lane >> 4;
  const int nk = C / BK;
  gload(0);
  lstore();
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    if (ks + 1 < nk) gload((ks + 1) * BK);
#pragma unroll
    for (int s = 0; s < BK / 4; ++s) {
      float af[4], bfr[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) af[mt] = As[(mt * 16 + lr) * LD + 4 * s + lg];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) bfr[nt] = Bs[brow(wave, nt, lr) * LD + 4 * s + lg];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[mt], bfr[nt], acc[mt][nt], 0, 0, 0);
    }
    __syncthreads();
    if (ks + 1 < nk) {
      lstore();
      __syncthreads();
    }
  }
  epilogue(acc, levels, scale, out, b, N1, m0, th0, tw0, wave, lane);
}


// ------------------------------------------------------------- flat path (bf16)
// avg_pool2d(2^l) of f2 for l = 1..levels-1, from the level-0 map directly
// (fp32 sum of the 4^l bf16 values, one rounding): (B, H_l, W_l, C) bf16.
struct PoolArgs {
  const bf16_t* f2;
  bf16_t* o[4];
  int B, H, W, C, levels;
  long start[5];  // first thread of level l (l = 1..levels-1), start[levels] = total (levels <= 4)
};

__global__ __launch_bounds__(256) void pool_f2_kernel(PoolArgs a) {
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int cq = a.C >> 3;
  // constant indices only: a runtime index into the byval kernarg arrays would
  // copy the whole struct to scratch in every lane
#pragma unroll
  for (int l = 1; l < 4; ++l) {
    if (l >= a.levels) break;
    if (tid < a.start[l] || tid >= a.start[l + 1]) continue;
    const long q = tid - a.start[l];
    const int Hl = a.H >> l, Wl = a.W >> l, k = 1 << l;
    const int c8 = (int)(q % cq);
    const long pix = q / cq;
    const int x = (int)(pix % Wl), y = (int)((pix / Wl) % Hl), b = (int)(pix / ((long)Wl * Hl));
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int dy = 0; dy < k; ++dy)
      for (int dx = 0; dx < k; ++dx) {
        const uint4 v = *reinterpret_cast<const uint4*>(
            a.f2 + (((size_t)b * a.H + y * k + dy) * a.W + x * k + dx) * a.C + c8 * 8);
        const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[2 * j] += bf2f((bf16_t)(u[j] & 0xffffu));
          acc[2 * j + 1] += bf2f((bf16_t)(u[j] >> 16));
        }
      }
    const float inv = 1.f / (float)(k * k);
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      o[j] = uint32_t(f2bf(acc[2 * j] * inv)) | (uint32_t(f2bf(acc[2 * j + 1] * inv)) << 16);
    *reinterpret_cast<uint4*>(a.o[l] + (size_t)pix * a.C + c8 * 8) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

struct FlatArgs {
  const bf16_t* f1;     // (B, N1, C)
  const bf16_t* f2[4];  // level l targets (B, N2_l, C)
  void* out[4];         // (B, N1, S_l) fp32 or bf16
  int N2[4], S[4];
  int tstart[5];        // per-batch prefix of (target tile x query tile) counts over levels
  int N1, C, levels, nq;
  float scale;
};

constexpr int FB = 128;  // targets (M) and queries (N) per block tile

// vol_l[b, i, n] = scale * <f1[b, i, :], f2_l[b, n, :]>: M = targets, N = queries,
// so an MFMA accumulator lane holds 4 CONSECUTIVE targets of one query row.
template <bool OB>
__global__ __launch_bounds__(256) void corr_flat_kernel(FlatArgs a) {
  // A | B operand tiles (64-channel K step, 32 KiB), then reused by the epilogue
  // transpose: 4 wave-private 64 x (64+4) fp32 tiles (68 KiB)
  constexpr int OPND = 2 * FB * 8, EPI = 4 * 64 * 68 / 4;
  __shared__ __attribute__((aligned(16))) uint4 lds[OPND > EPI ? OPND : EPI];
  uint4* As = lds;
  uint4* Bs = lds + FB * 8;
  // level / tile decode with constant kernarg indices only (a runtime index
  // into FlatArgs' arrays copied the struct to scratch: 160 B per lane)
  const int per_b = a.levels == 1 ? a.tstart[1] : a.levels == 2 ? a.tstart[2] : a.levels == 3 ? a.tstart[3] : a.tstart[4];
  const int b = blockIdx.x / per_b;
  int t = blockIdx.x - b * per_b;
  const int l = (a.levels > 3 && t >= a.tstart[3]) ? 3 : (a.levels > 2 && t >= a.tstart[2]) ? 2
              : (a.levels > 1 && t >= a.tstart[1]) ? 1 : 0;
  t -= l == 0 ? a.tstart[0] : l == 1 ? a.tstart[1] : l == 2 ? a.tstart[2] : a.tstart[3];
  const int tn = t / a.nq, tq = t - tn * a.nq;
  const int n0 = tn * FB, q0 = tq * FB;
  const int N1 = a.N1, C = a.C;
  const int N2 = l == 0 ? a.N2[0] : l == 1 ? a.N2[1] : l == 2 ? a.N2[2] : a.N2[3];
  const bf16_t* f1b = a.f1 + (size_t)b * N1 * C;
  const bf16_t* f2b = (l == 0 ? a.f2[0] : l == 1 ? a.f2[1] : l == 2 ? a.f2[2] : a.f2[3]) + (size_t)b * N2 * C;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  uint4 ra[4], rb[4];
#define RS_FL_LOAD(K0)                                                                   \
  do {                                                                                   \
    _Pragma("unroll") for (int q = 0; q < 4; ++q) {                                      \
      const int idx = tid + 256 * q, r = idx >> 3, c = idx & 7;                         \
      /* clamped row + value select (a select between the load and a local   */ \
      /* zero takes the zero's address: the whole staging array to scratch)  */ \
      const uint4 va_ = *reinterpret_cast<const uint4*>(f2b + (size_t)min(n0 + r, N2 - 1) * C + (K0) + c * 8); \
      const uint4 vb_ = *reinterpret_cast<const uint4*>(f1b + (size_t)min(q0 + r, N1 - 1) * C + (K0) + c * 8); \
      ra[q] = n0 + r < N2 ? va_ : make_uint4(0, 0, 0, 0);                              \
      rb[q] = q0 + r < N1 ? vb_ : make_uint4(0, 0, 0, 0);                              \
    }                                                                                    \
  } while (0)
#define RS_FL_STORE()                                                                    \
  do {                                                                                   \
    _Pragma("unroll") for (int q = 0; q < 4; ++q) {                                      \
      const int idx = tid + 256 * q;                                                     \
      As[swz(idx >> 3, idx & 7)] = ra[q];                                                \
      Bs[swz(idx >> 3, idx & 7)] = rb[q];                                                \
    }                                                                                    \
  } while (0)

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int lr = lane & 15, lg = lane >> 4;
  const int nk = C / 64;
  RS_FL_LOAD(0);
  RS_FL_STORE();
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    if (ks + 1 < nk) RS_FL_LOAD((ks + 1) * 64);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8_t af[4], bfr[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        uint4 v = As[swz(wm * 64 + mt * 16 + lr, kk * 4 + lg)];
        af[mt] = *reinterpret_cast<bf16x8_t*>(&v);
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        uint4 v = Bs[swz(wn * 64 + nt * 16 + lr, kk * 4 + lg)];
        bfr[nt] = *reinterpret_cast<bf16x8_t*>(&v);
      }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], bfr[nt], acc[mt][nt], 0, 0, 0);
    }
    if (ks + 1 < nk) {
      __syncthreads();
      RS_FL_STORE();
      __syncthreads();
    }
  }
#undef RS_FL_LOAD
#undef RS_FL_STORE
  // epilogue: acc[mt][nt][j] = vol[query wn*64 + nt*16 + lr][target wm*64 + mt*16 + 4 lg + j].
  // Transposed through a wave-private LDS tile T[query][target] (row pitch 68
  // floats: conflict-free float4 writes and reads) so that 16 consecutive
  // lanes store 64 consecutive targets of ONE volume row: 256-B (fp32) /
  // 128-B (bf16) fully coalesced segments.  Storing the accumulator layout
  // directly (4 lanes 16 lanes apart per 64-B segment) reached DRAM as one
  // 64-B write per lane (TCC_EA0_WRREQ_64B = 3x the volume bytes).
  __syncthreads();  // every wave done with the operand tiles
  float* T = reinterpret_cast<float*>(lds) + wave * 64 * 68;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
      *reinterpret_cast<f32x4_t*>(T + (nt * 16 + lr) * 68 + mt * 16 + lg * 4) = acc[mt][nt] * a.scale;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  const int S = l == 0 ? a.S[0] : l == 1 ? a.S[1] : l == 2 ? a.S[2] : a.S[3];
  void* const ob = l == 0 ? a.out[0] : l == 1 ? a.out[1] : l == 2 ? a.out[2] : a.out[3];
  const int tl = (lane & 15) * 4;  // this lane's 4 targets within the wave's 64
  const int n = n0 + wm * 64 + tl;
#pragma unroll 4
  for (int rr = 0; rr < 64; rr += 4) {
    const int qr = rr + lg;  // query row within the wave tile
    const int i = q0 + wn * 64 + qr;
    const f32x4_t v = *reinterpret_cast<const f32x4_t*>(T + qr * 68 + tl);
    if (i >= N1) continue;
    const size_t o = ((size_t)b * N1 + i) * S + n;
    if constexpr (OB) {
      bf16_t* op = static_cast<bf16_t*>(ob) + o;
      if (n + 3 < N2) {
        *reinterpret_cast<uint2*>(op) = make_uint2(uint32_t(f2bf(v[0])) | (uint32_t(f2bf(v[1])) << 16),
                                                   uint32_t(f2bf(v[2])) | (uint32_t(f2bf(v[3])) << 16));
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (n + j < N2) op[j] = f2bf(v[j]);
      }
    } else {
      float* op = static_cast<float*>(ob) + o;
      if (n + 3 < N2) {
        *reinterpret_cast<f32x4_t*>(op) = v;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (n + j < N2) op[j] = v[j];
      }
    }
  }
}

// fp32 feature maps on the bf16 flat GEMM by operand splitting (as the F32
// conv tiles): x = xh + xl, xh = bf16(x), xl = bf16(x - xh), and
// <f1, f2> ~= <f1h, f2h> + <f1h, f2l> + <f1l, f2h> (relative error ~2^-17;
// the dropped <f1l, f2l> is ~2^-16 of a product) = ONE bf16 GEMM over K = 3C
// with f1x = [f1h | f1h | f1l] and f2x = [f2h | f2l | f2h].  This kernel
// writes those operands: level l of the source map averaged over 2^l x 2^l
// blocks in fp32 (the pyramid by linearity, as pool_f2_kernel), then split;
// pat 0: [h | h | l] (f1), pat 1: [h | l | h] (f2 levels).  One thread per
// 4 channels of one output pixel.
struct SplitArgs {
  const float* x;  // (B, H, W, C) fp32 (the level-0 map)
  bf16_t* o[5];    // o[0]: f1x (B, N1, 3C); o[1 + l]: f2x level l (B, H_l, W_l, 3C)
  int B, H, W, C, levels, N1;
  const float* f1;
  long start[6];   // first thread of each job: 0 = f1, 1 + l = f2 level l; start[levels + 1] = total
};

__global__ __launch_bounds__(256) void split3_kernel(SplitArgs a) {
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int cq = a.C >> 2;
#pragma unroll
  for (int j = 0; j < 5; ++j) {  // constant kernarg indices only (see pool_f2_kernel)
    if (j > a.levels) break;
    if (tid < a.start[j] || tid >= a.start[j + 1]) continue;
    const long q = tid - a.start[j];
    const int c4 = (int)(q % cq);
    const long pix = q / cq;
    float4 v;
    if (j == 0) {
      v = *reinterpret_cast<const float4*>(a.f1 + (size_t)pix * a.C + c4 * 4);
    } else {
      const int l = j - 1, k = 1 << l, Hl = a.H >> l, Wl = a.W >> l;
      const int x = (int)(pix % Wl), y = (int)((pix / Wl) % Hl), b = (int)(pix / ((long)Wl * Hl));
      v = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int dy = 0; dy < k; ++dy)
        for (int dx = 0; dx < k; ++dx) {
          const float4 u = *reinterpret_cast<const float4*>(
              a.x + (((size_t)b * a.H + y * k + dy) * a.W + x * k + dx) * a.C + c4 * 4);
          v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
        }
      const float inv = 1.f / (float)(k * k);
      v.x *= inv; v.y *= inv; v.z *= inv; v.w *= inv;
    }
    const float f[4] = {v.x, v.y, v.z, v.w};
    uint32_t hi[2], lo[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bf16_t h0 = f2bf(f[2 * i]), h1 = f2bf(f[2 * i + 1]);
      hi[i] = uint32_t(h0) | (uint32_t(h1) << 16);
      lo[i] = uint32_t(f2bf(f[2 * i] - bf2f(h0))) | (uint32_t(f2bf(f[2 * i + 1] - bf2f(h1))) << 16);
    }
    bf16_t* ob = (j == 0 ? a.o[0] : j == 1 ? a.o[1] : j == 2 ? a.o[2] : j == 3 ? a.o[3] : a.o[4]) +
                 (size_t)pix * 3 * a.C + c4 * 4;
    const uint2 H = make_uint2(hi[0], hi[1]), L = make_uint2(lo[0], lo[1]);
    *reinterpret_cast<uint2*>(ob) = H;
    *reinterpret_cast<uint2*>(ob + a.C) = j == 0 ? H : L;
    *reinterpret_cast<uint2*>(ob + 2 * a.C) = j == 0 ? L : H;
  }
}

}  // namespace corrvol

// Host launcher. f1: (B,N1,C), f2: (B,H2,W2,C), both channels-last.
// out[l]: (B, N1, S[l]) rows, level l element (h, w) at h*W[l] + w; fp32, or bf16
// when out_bf16 (bf16 inputs only).  bf16 inputs: pooled-f2 workspace `ws`
// (>= sum_{l>=1} B*H_l*W_l*C bf16) and the flat grouped GEMM; fp32 inputs: the
// exact fp32 2-D-block kernel.  C % 64 == 0 (bf16) / C % 32 == 0 (f32).
static void flat_launch(const bf16_t* f1, const bf16_t* const* f2l, int B, int N1, int C, int levels,
                        void* const* out, const int* Hs, const int* Ws, const int* Ss, bool out_bf16, float scale,
                        hipStream_t stream) {
  corrvol::FlatArgs fa{};
  fa.f1 = f1;
  fa.N1 = N1; fa.C = C; fa.levels = levels; fa.scale = scale;
  fa.nq = cdiv(N1, corrvol::FB);
  int acc_t = 0;
  for (int l = 0; l < 4; ++l) {
    fa.tstart[l] = acc_t;
    if (l < levels) {
      fa.f2[l] = f2l[l];
      fa.out[l] = out[l];
      fa.N2[l] = Hs[l] * Ws[l];
      fa.S[l] = Ss[l];
      acc_t += cdiv(fa.N2[l], corrvol::FB) * fa.nq;
    }
  }
  fa.tstart[levels] = acc_t;
  const dim3 grid((unsigned)(acc_t * B));
  if (out_bf16)
    hipLaunchKernelGGL(corrvol::corr_flat_kernel<true>, grid, dim3(256), 0, stream, fa);
  else
    hipLaunchKernelGGL(corrvol::corr_flat_kernel<false>, grid, dim3(256), 0, stream, fa);
}

// bytes of the fp32 split path's workspace (corr_volume_launch with bf16 = false, ws != null)
size_t corr_volume_split_ws(int B, int N1, int C, int levels, const int* Hs, const int* Ws) {
  size_t n = (size_t)B * N1 * 3 * C;
  for (int l = 0; l < levels; ++l) n += (size_t)B * Hs[l] * Ws[l] * 3 * C;
  return n * sizeof(bf16_t);
}

void corr_volume_launch(const void* f1, const void* f2, bool bf16, int B, int N1, int H2, int W2,
                        int C, int levels, void* const* out, const int* Hs, const int* Ws, const int* Ss,
                        bool out_bf16, void* ws, float scale, hipStream_t stream) {
  if (!bf16 && ws) {  // fp32 maps: split-bf16 operands + the flat GEMM over K = 3C
    corrvol::SplitArgs sa{};
    sa.x = static_cast<const float*>(f2);
    sa.f1 = static_cast<const float*>(f1);
    sa.B = B; sa.H = H2; sa.W = W2; sa.C = C; sa.levels = levels; sa.N1 = N1;
    bf16_t* w = static_cast<bf16_t*>(ws);
    long tot = 0;
    sa.start[0] = 0;
    sa.o[0] = w;
    w += (size_t)B * N1 * 3 * C;
    tot += (long)B * N1 * (C / 4);
    const bf16_t* f2l[4];
    for (int l = 0; l < 4; ++l) {
      sa.start[1 + l] = tot;
      if (l < levels) {
        sa.o[1 + l] = w;
        f2l[l] = w;
        w += (size_t)B * Hs[l] * Ws[l] * 3 * C;
        tot += (long)B * Hs[l] * Ws[l] * (C / 4);
      }
    }
    sa.start[levels + 1] = tot;
    hipLaunchKernelGGL(corrvol::split3_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, sa);
    flat_launch(sa.o[0], f2l, B, N1, 3 * C, levels, out, Hs, Ws, Ss, false, scale, stream);
    return;
  }
  if (bf16) {
    corrvol::PoolArgs pa{};
    pa.f2 = static_cast<const bf16_t*>(f2);
    pa.B = B; pa.H = H2; pa.W = W2; pa.C = C; pa.levels = levels;
    bf16_t* w = static_cast<bf16_t*>(ws);
    long tot = 0;
    for (int l = 1; l < 4; ++l) {
      pa.start[l] = tot;
      if (l < levels) {
        pa.o[l] = w;
        w += (size_t)B * Hs[l] * Ws[l] * C;
        tot += (long)B * Hs[l] * Ws[l] * (C / 8);
      }
    }
    pa.start[levels] = tot;
    if (levels > 1 && tot > 0)
      hipLaunchKernelGGL(corrvol::pool_f2_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, pa);
    corrvol::FlatArgs fa{};
    fa.f1 = static_cast<const bf16_t*>(f1);
    fa.N1 = N1; fa.C = C; fa.levels = levels; fa.scale = scale;
    fa.nq = cdiv(N1, corrvol::FB);
    int acc_t = 0;
    for (int l = 0; l < 4; ++l) {
      fa.tstart[l] = acc_t;
      if (l < levels) {
        fa.f2[l] = l == 0 ? static_cast<const bf16_t*>(f2) : pa.o[l];
        fa.out[l] = out[l];
        fa.N2[l] = Hs[l] * Ws[l];
        fa.S[l] = Ss[l];
        acc_t += cdiv(fa.N2[l], corrvol::FB) * fa.nq;
      }
    }
    fa.tstart[levels] = acc_t;
    const dim3 grid((unsigned)(acc_t * B));
    if (out_bf16)
      hipLaunchKernelGGL(corrvol::corr_flat_kernel<true>, grid, dim3(256), 0, stream, fa);
    else
      hipLaunchKernelGGL(corrvol::corr_flat_kernel<false>, grid, dim3(256), 0, stream, fa);
    return;
  }
  corrvol::PyrOut po;
  for (int l = 0; l < 4; ++l) {
    po.p[l] = l < levels ? static_cast<float*>(out[l]) : nullptr;
    po.H[l] = l < levels ? Hs[l] : 0;
    po.W[l] = l < levels ? Ws[l] : 0;
    po.S[l] = l < levels ? Ss[l] : 0;
  }
  dim3 grid(cdiv(H2, corrvol::TH) * cdiv(W2, corrvol::TW), cdiv(N1, corrvol::BM), B);
  hipLaunchKernelGGL(corrvol::corr_volume_f32_kernel, grid, dim3(corrvol::THREADS), 0, stream,
                     static_cast<const float*>(f1), static_cast<const float*>(f2), N1, H2, W2, C,
                     scale, levels, po);
}

}  // namespace rs
