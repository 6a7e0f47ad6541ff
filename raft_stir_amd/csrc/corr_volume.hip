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
// epilogue's coalescing matters more than MFMA issue rate.
//
// An exact-fp32 variant (mfma_f32_16x16x4f32, bit-identical to an fmaf chain)
// serves fp32 mode; the bf16 variant is used when the feature maps come from
// a bf16-autocast encoder (then the bf16 operands are exact).

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
            out.p[0][((size_t)b * N1 + i) * H * W + (size_t)h * W + w] = v;
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
            out.p[1][((size_t)b * N1 + i) * H * W + (size_t)h * W + w] = v;
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
            out.p[2][((size_t)b * N1 + i) * H * W + (size_t)h * W + w] = v;
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
          out.p[3][((size_t)b * N1 + i) * H * W + (size_t)h * W + w] = v;
      }
  }
}

// ---------------------------------------------------------------- bf16 MFMA
__global__ __launch_bounds__(THREADS) void corr_volume_bf16_kernel(
    const bf16_t* __restrict__ f1, const bf16_t* __restrict__ f2, int N1, int H2, int W2, int C,
    float scale, int levels, PyrOut out) {
  constexpr int BK = 64;  // 8 x 16-B chunks per row
  __shared__ __attribute__((aligned(16))) uint4 lds[(BM + BN) * 8];  // 40 KiB
  uint4* As = lds;
  uint4* Bs = lds + BM * 8;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.z;
  const int m0 = blockIdx.y * BM;
  const int nTW = cdiv(W2, TW);
  const int th0 = (blockIdx.x / nTW) * TH;
  const int tw0 = (blockIdx.x % nTW) * TW;
  const bf16_t* f1b = f1 + (size_t)b * N1 * C;
  const bf16_t* f2b = f2 + (size_t)b * H2 * W2 * C;
  const uint4 zero = make_uint4(0, 0, 0, 0);

  uint4 ra[2], rb[8];
  auto gload = [&](int k0) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int idx = tid + THREADS * q, r = idx >> 3, c = idx & 7;
      const int m = m0 + r;
      ra[q] = (m < N1) ? *reinterpret_cast<const uint4*>(f1b + (size_t)m * C + k0 + c * 8) : zero;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int idx = tid + THREADS * q, r = idx >> 3, c = idx & 7;
      const int h = th0 + r / TW, w = tw0 + r % TW;
      rb[q] = (h < H2 && w < W2)
                  ? *reinterpret_cast<const uint4*>(f2b + ((size_t)h * W2 + w) * C + k0 + c * 8)
                  : zero;
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int idx = tid + THREADS * q;
      As[swz(idx >> 3, idx & 7)] = ra[q];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int idx = tid + THREADS * q;
      Bs[swz(idx >> 3, idx & 7)] = rb[q];
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
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8_t af[4], bfr[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        uint4 v = As[swz(mt * 16 + lr, kk * 4 + lg)];
        af[mt] = *reinterpret_cast<bf16x8_t*>(&v);
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        uint4 v = Bs[swz(brow(wave, nt, lr), kk * 4 + lg)];
        bfr[nt] = *reinterpret_cast<bf16x8_t*>(&v);
      }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], bfr[nt], acc[mt][nt], 0, 0, 0);
    }
    __syncthreads();
    if (ks + 1 < nk) {
      lstore();
      __syncthreads();
    }
  }
  epilogue(acc, levels, scale, out, b, N1, m0, th0, tw0, wave, lane);
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
  const float4 zero = make_float4(0.f, 0.f, 0.f, 0.f);

  float4 ra[2], rb[8];
  auto gload = [&](int k0) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int idx = tid + THREADS * q, r = idx >> 3, c = idx & 7;
      const int m = m0 + r;
      ra[q] = (m < N1) ? *reinterpret_cast<const float4*>(f1b + (size_t)m * C + k0 + c * 4) : zero;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int idx = tid + THREADS * q, r = idx >> 3, c = idx & 7;
      const int h = th0 + r / TW, w = tw0 + r % TW;
      rb[q] = (h < H2 && w < W2)
                  ? *reinterpret_cast<const float4*>(f2b + ((size_t)h * W2 + w) * C + k0 + c * 4)
                  : zero;
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

}  // namespace corrvol

// Host launcher. f1: (B,N1,C), f2: (B,H2,W2,C), both channels-last.
// out[l]: (B, N1, H[l], W[l]) fp32.  C % 64 == 0 (bf16) / C % 32 == 0 (f32).
void corr_volume_launch(const void* f1, const void* f2, bool bf16, int B, int N1, int H2, int W2,
                        int C, int levels, float* const* out, const int* Hs, const int* Ws,
                        float scale, hipStream_t stream) {
  corrvol::PyrOut po;
  for (int l = 0; l < 4; ++l) {
    po.p[l] = l < levels ? out[l] : nullptr;
    po.H[l] = l < levels ? Hs[l] : 0;
    po.W[l] = l < levels ? Ws[l] : 0;
  }
  dim3 grid(cdiv(H2, corrvol::TH) * cdiv(W2, corrvol::TW), cdiv(N1, corrvol::BM), B);
  if (bf16) {
    hipLaunchKernelGGL(corrvol::corr_volume_bf16_kernel, grid, dim3(corrvol::THREADS), 0, stream,
                       static_cast<const bf16_t*>(f1), static_cast<const bf16_t*>(f2), N1, H2, W2,
                       C, scale, levels, po);
  } else {
    hipLaunchKernelGGL(corrvol::corr_volume_f32_kernel, grid, dim3(corrvol::THREADS), 0, stream,
                       static_cast<const float*>(f1), static_cast<const float*>(f2), N1, H2, W2, C,
                       scale, levels, po);
  }
}

}  // namespace rs
