// Backward of the all-pairs correlation volume: the two feature-gradient GEMMs
// on MFMA (reference: the autograd backward of core/corr.py:52-60,
// corr() = fmap1^T fmap2 / sqrt(C), and of the avg_pool2d pyramid,
// core/corr.py:24-27).
//
// The lookups' backward accumulated the gradient of every pyramid level; one
// fold pass (corr_lookup.hip pyr_fold_rows_kernel) turns it into the bf16
// level-0 volume gradient G[b][p1][p2] (scale and every level's avg-pool
// adjoint applied), rows padded with zeros to a multiple of 64 (pitch Ep).
// The features' gradients are then, per batch image b,
//   df1[b] = G[b]   f2[b]     (M = N1, K = N2)   "NN": A = rows of G (K-contiguous)
//   df2[b] = G[b]^T f1[b]     (M = N2, K = N1)   "TN": A = columns of G
// with f1 / f2 pixel-major [p][C] (the B operand is K-major rows).
//
// One launch runs both GEMMs (the two sets of output tiles are independent;
// together ~740 blocks of 4 waves at the training shape, two blocks per CU).
// Block = 128 output rows x 128 channels, K step 64, 4 waves in 2 x 2, each a
// 64 x 64 tile of four v_mfma_f32_32x32x16_bf16 accumulators:
//  * A and B K-step tiles are copied global -> LDS by buffer_load ... lds
//    (double-buffered: the next K step is in flight during this step's MFMAs;
//    rows past M / K come back as zeros from the buffer range check);
//  * NN A tile: 128 rows x 128 B, the 16-B chunk index XOR ((row >> 1) & 7)
//    so a ds_read_b128 of 16 consecutive rows hits all 64 banks;
//  * K-major tiles (B, and the TN A tile): 64 K rows x 256 B; fragments are
//    gathered by ds_read_b64_tr_b16 (4 K values of one column per lane), rows
//    XOR-swizzle their 64-B quarters by (row & 3) so the 32 lanes of a
//    transposed read cover all 64 banks;
//  * the next sub-step's fragments are read while this sub-step's MFMAs run
//    (counted lgkmcnt waits; the LDS reads are inline asm so the compiler does
//    not drain the in-flight DMA in front of them);
//  * fp32 accumulation, bf16 output rows written once: no atomics, no
//    split-K -- deterministic by construction;
//  * fp32 training: the operands as bf16 hi / lo pairs and three K passes
//    (hi.hi + hi.lo + lo.hi, ~2^-16 relative error), fp32 output.
#include "common.h"

#include <algorithm>
#include <type_traits>

namespace rs {
namespace cgemm {

typedef short v4s_t __attribute__((ext_vector_type(4)));

struct Args {
  const bf16_t* G;   // [B][N1][Ep]
  const bf16_t* f1;  // [B][N1][C]
  const bf16_t* f2;  // [B][N2][C]
  void* d1;          // [B][N1][C] bf16 (fp32: split mode)
  void* d2;          // [B][N2][C]
  // split mode (fp32 operands as bf16 hi + lo pairs): x.y ~= xh.yh + xh.yl + xl.yh,
  // three K passes over (G hi, f hi), (G hi, f lo), (G lo, f hi), fp32 output
  const bf16_t* Gl;
  const bf16_t* f1l;
  const bf16_t* f2l;
  unsigned g_bytes, f1_bytes, f2_bytes;
  int B, N1, N2, C, Ep;
  int nm1, nm2, nn;  // M tiles of each GEMM, channel tiles
};

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int TILE = BK * 256;     // bytes of one operand tile (128 x 64 or 64 x 128 bf16)
constexpr int STAGE = 2 * TILE;    // A + B
constexpr int kFar = 0x7ffffff0;   // buffer offset past every range: reads zeros

template <int I, int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<I + 1, N>(f);
  }
}

template <int N>
__device__ __forceinline__ void wait_lgkm() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N < 15 ? N : 15) : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, const uint8_t* lds_base, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_base, 16, voff, 0, 0, 0);
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

// logical 16-B chunk held by LDS slot (row r, physical chunk pc) of a tile
__device__ __forceinline__ int chunk_rowmajor(int r, int pc) { return pc ^ ((r >> 1) & 7); }        // 8 chunks / row
__device__ __forceinline__ int chunk_kmajor(int r, int pc) { return pc ^ ((r & 3) << 2); }          // 16 chunks / row

// One K-step's fragments for sub-step KK: A (2 x 32 rows), B (2 x 32 columns).
// TA: A from a K-major tile (transposed reads) instead of the row-major one.
template <bool TA>
struct Frags {
  v4s_t a[2][2], b[2][2];  // [fragment][lo / hi 4 K values]
};

template <bool TA, int KK>
__device__ __forceinline__ void read_frags(Frags<TA>& f, const uint32_t (&aaddr)[2][4], const uint32_t (&baddr)[2],
                                           uint32_t so) {
  if constexpr (TA) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(f.a[i][0]) : "v"(aaddr[i][0] + so),
                   "i"((16 * KK) * 256) : "memory");
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(f.a[i][1]) : "v"(aaddr[i][0] + so),
                   "i"((16 * KK + 4) * 256) : "memory");
    }
  } else {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      // one 16-B read = both 4-value halves
      typedef short v8s_t __attribute__((ext_vector_type(8)));
      v8s_t v;
      asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(aaddr[i][KK] + so) : "memory");
      f.a[i][0] = __builtin_shufflevector(v, v, 0, 1, 2, 3);
      f.a[i][1] = __builtin_shufflevector(v, v, 4, 5, 6, 7);
    }
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(f.b[j][0]) : "v"(baddr[j] + so),
                 "i"(TILE + (16 * KK) * 256) : "memory");
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(f.b[j][1]) : "v"(baddr[j] + so),
                 "i"(TILE + (16 * KK + 4) * 256) : "memory");
  }
}

template <bool TA>
__device__ __forceinline__ void mfma4(f32x16_t (&acc)[2][2], Frags<TA>& f) {
  asm volatile("" : "+v"(f.a[0][0]), "+v"(f.a[0][1]), "+v"(f.a[1][0]), "+v"(f.a[1][1]));
  asm volatile("" : "+v"(f.b[0][0]), "+v"(f.b[0][1]), "+v"(f.b[1][0]), "+v"(f.b[1][1]));
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const bf16x8_t av = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(f.a[i][0], f.a[i][1], 0, 1, 2, 3, 4, 5, 6, 7));
      const bf16x8_t bv = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(f.b[j][0], f.b[j][1], 0, 1, 2, 3, 4, 5, 6, 7));
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc[i][j], 0, 0, 0);
    }
  __builtin_amdgcn_sched_barrier(0);
}

// TA = false: D1 = G F2 (A rows = G rows); TA = true: D2 = G^T F1 (A = G columns).
// NP = 3: split mode (hi / lo K passes, fp32 output).
template <bool TA, int NP>
__device__ __forceinline__ void gemm_tile(const Args& a, uint8_t* lds, int b, int mt, int nt) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1;
  const int M = TA ? a.N2 : a.N1, K = TA ? a.N1 : a.N2;
  const int m0 = mt * BM, n0 = nt * BN, C = a.C, Ep = a.Ep;
  const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc((void*)a.G, (short)0, a.g_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rf = TA ? __builtin_amdgcn_make_buffer_rsrc((void*)a.f1, (short)0, a.f1_bytes, 0x00020000)
                                       : __builtin_amdgcn_make_buffer_rsrc((void*)a.f2, (short)0, a.f2_bytes, 0x00020000);
  // split mode: the lo halves (same shapes and byte counts)
  const __amdgpu_buffer_rsrc_t rgl =
      __builtin_amdgcn_make_buffer_rsrc((void*)(NP == 3 ? a.Gl : a.G), (short)0, a.g_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rfl =
      TA ? __builtin_amdgcn_make_buffer_rsrc((void*)(NP == 3 ? a.f1l : a.f1), (short)0, a.f1_bytes, 0x00020000)
         : __builtin_amdgcn_make_buffer_rsrc((void*)(NP == 3 ? a.f2l : a.f2), (short)0, a.f2_bytes, 0x00020000);
  const long gbase = (long)b * a.N1;   // first G row of this image
  const long fbase = (long)b * K;      // first feature row (the K rows)

  // ---- per-lane DMA roles: 4 A slots + 4 B slots (16 B each) per K step
  // A: (row, element) of this lane's slots -- NN: G row m0+r, column k0+8c; TA: G row k0+r, column m0+8c
  int aro[4], aco[4], bro[4], bco[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int s = (wave + 4 * i) * 64 + lane;
    if constexpr (TA) {
      const int r = s >> 4;
      aro[i] = r;
      aco[i] = 8 * chunk_kmajor(r, s & 15);
    } else {
      const int r = s >> 3;
      aro[i] = r;
      aco[i] = 8 * chunk_rowmajor(r, s & 7);
    }
    const int r = s >> 4;
    bro[i] = r;
    bco[i] = 8 * chunk_kmajor(r, s & 15);
  }
  const int nk1 = cdiv(K, BK), nk = NP * nk1;  // K steps of one pass, of all passes
  auto issue = [&](int kt, int st) {
    const uint8_t* sb = lds + st * STAGE;
    const bool live = kt < nk;
    const int pass = NP == 1 ? 0 : kt / nk1;  // 0: (hi, hi), 1: (hi, lo), 2: (lo, hi)
    const int k0 = (kt - pass * nk1) * BK;
    const __amdgpu_buffer_rsrc_t ra = pass == 2 ? rgl : rg;
    const __amdgpu_buffer_rsrc_t rb = pass == 1 ? rfl : rf;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int v;
      if constexpr (TA) {
        v = (live && k0 + aro[i] < K) ? (int)(((gbase + k0 + aro[i]) * Ep + m0 + aco[i]) * 2) : kFar;
      } else {
        // columns k0 .. k0+63 < Ep always (Ep = round_up(N2, 64), zero pad)
        v = (live && m0 + aro[i] < M) ? (int)(((gbase + m0 + aro[i]) * Ep + k0 + aco[i]) * 2) : kFar;
      }
      dma16(ra, sb + (wave + 4 * i) * 1024, v);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int v = (live && k0 + bro[i] < K) ? (int)(((fbase + k0 + bro[i]) * C + n0 + bco[i]) * 2) : kFar;
      dma16(rb, sb + TILE + (wave + 4 * i) * 1024, v);
    }
  };

  // ---- fragment read addresses (bytes, LDS)
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) uint8_t*)lds;
  const int g = lane >> 4, gi = lane & 15, q = gi >> 2, p = gi & 3, h = lane >> 5;
  // K-major tile, columns col0 .. col0+31 (col0 % 32 == 0): lane (g, 4q+p) reads row 8(g>>1) + q (+4, + 16 KK),
  // columns col0 + 16(g&1) + 4p .. +3; quarter (col0 / 32) ^ q
  auto kmaj = [&](int col0) -> uint32_t {
    return (uint32_t)((8 * (g >> 1) + q) * 256 + (((col0 >> 5) ^ q) << 6) + (16 * (g & 1) + 4 * p) * 2);
  };
  uint32_t aaddr[2][4], baddr[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    if constexpr (TA) {
      aaddr[i][0] = lds0 + kmaj(wm * 64 + 32 * i);
      aaddr[i][1] = aaddr[i][2] = aaddr[i][3] = 0;
    } else {
      // row-major tile: row wm*64 + 32i + (lane & 31), logical chunk 2 KK + h
      const int r = wm * 64 + 32 * i + (lane & 31);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) aaddr[i][kk] = lds0 + r * 128 + (chunk_rowmajor(r, 2 * kk + h) << 4);
    }
    baddr[i] = lds0 + kmaj(wn * 64 + 32 * i);
  }

  f32x16_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  constexpr int RPS = (TA ? 4 : 2) + 4;  // LDS reads per sub-step
  issue(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    const int st = kt & 1;
    issue(kt + 1, st ^ 1);   // zeros past the end: a static vmcnt count
    wait_vm<8>();            // this step's own pieces have landed
    asm volatile("s_barrier" ::: "memory");  // ... and every other wave's
    const uint32_t so = st * STAGE;
    Frags<TA> f0, f1;
    read_frags<TA, 0>(f0, aaddr, baddr, so);
    read_frags<TA, 1>(f1, aaddr, baddr, so);
    wait_lgkm<RPS>();
    mfma4<TA>(acc, f0);
    read_frags<TA, 2>(f0, aaddr, baddr, so);
    wait_lgkm<RPS>();
    mfma4<TA>(acc, f1);
    read_frags<TA, 3>(f1, aaddr, baddr, so);
    wait_lgkm<RPS>();
    mfma4<TA>(acc, f0);
    wait_lgkm<0>();
    mfma4<TA>(acc, f1);
    asm volatile("s_barrier" ::: "memory");  // every wave done reading this stage
  }
  wait_vm<0>();

  // ---- epilogue: acc[i][j] reg r -> row m0 + wm*64 + 32i + (r&3) + 8(r>>2) + 4h, channel n0 + wn*64 + 32j + lane&31
  const long obase = (long)b * M;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (m < M) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const long o = (obase + m) * C + n0 + wn * 64 + 32 * j + (lane & 31);
          if constexpr (NP == 3)
            static_cast<float*>(TA ? a.d2 : a.d1)[o] = acc[i][j][r];
          else
            static_cast<bf16_t*>(TA ? a.d2 : a.d1)[o] = f2bf(acc[i][j][r]);
        }
      }
    }
}

template <int NP>
__global__ __launch_bounds__(256) void corr_bwd_gemm_kernel(Args a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * STAGE];
  const int nblk1 = a.B * a.nm1 * a.nn;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  if (lid < nblk1) {
    const int nt = lid % a.nn, r = lid / a.nn;
    gemm_tile<false, NP>(a, lds, r / a.nm1, r % a.nm1, nt);
  } else {
    const int l2 = lid - nblk1;
    const int nt = l2 % a.nn, r = l2 / a.nn;
    gemm_tile<true, NP>(a, lds, r / a.nm2, r % a.nm2, nt);
  }
}

}  // namespace cgemm

int corr_bwd_pitch(int N2) { return round_up(N2, cgemm::BK); }

// G [B][N1][Ep] bf16 (Ep = corr_bwd_pitch(N2), zero columns past N2); f1 [B][N1][C], f2 [B][N2][C] bf16,
// C % 128 == 0 -> df1 [B][N1][C], df2 [B][N2][C] bf16.  Gl / f1l / f2l non-null: split mode, the lo
// halves of fp32 operands (same layouts) -> fp32 df1 / df2.
void corr_bwd_gemm_launch(const void* G, const void* Gl, int Ep, const void* f1, const void* f1l, const void* f2,
                          const void* f2l, int B, int N1, int N2, int C, void* df1, void* df2, hipStream_t stream) {
  cgemm::Args a{};
  a.G = static_cast<const bf16_t*>(G);
  a.f1 = static_cast<const bf16_t*>(f1);
  a.f2 = static_cast<const bf16_t*>(f2);
  a.Gl = static_cast<const bf16_t*>(Gl);
  a.f1l = static_cast<const bf16_t*>(f1l);
  a.f2l = static_cast<const bf16_t*>(f2l);
  a.d1 = df1;
  a.d2 = df2;
  a.g_bytes = (unsigned)((long)B * N1 * Ep * 2);
  a.f1_bytes = (unsigned)((long)B * N1 * C * 2);
  a.f2_bytes = (unsigned)((long)B * N2 * C * 2);
  a.B = B; a.N1 = N1; a.N2 = N2; a.C = C; a.Ep = Ep;
  a.nm1 = cdiv(N1, cgemm::BM);
  a.nm2 = cdiv(N2, cgemm::BM);
  a.nn = C / cgemm::BN;
  const int nblk = B * (a.nm1 + a.nm2) * a.nn;
  if (nblk == 0) return;
  if (Gl != nullptr)
    hipLaunchKernelGGL(cgemm::corr_bwd_gemm_kernel<3>, dim3(nblk), dim3(256), 0, stream, a);
  else
    hipLaunchKernelGGL(cgemm::corr_bwd_gemm_kernel<1>, dim3(nblk), dim3(256), 0, stream, a);
}

}  // namespace rs
