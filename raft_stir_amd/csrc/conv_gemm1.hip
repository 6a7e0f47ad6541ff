// 1x1 convolutions of the update block as plain MFMA GEMMs (tile 70 of
// conv_fused; reference core/update.py:64 BasicMotionEncoder.convc1 and
// :116 the mask head's 1x1, forward and input gradient):
//
//   D[co][p] = sum_k W[co][k] X[p][k]      (X = the concatenated input segments, NHWC)
//
// Both operands are K-contiguous rows (packed weights [Cout_pad][1][Ktot],
// activations [pixel][channels]), so neither needs a transpose: the generic
// implicit-GEMM tiles spend their K loop on per-pixel tap bookkeeping a 1x1
// conv does not have (~180 TFLOP/s on these shapes, profiles/r5/README.md).
// Block = 128 output channels x 128 pixels, K step = one 64-channel chunk of
// one segment, 4 waves in 2 x 2, each a 64 x 64 tile of four
// v_mfma_f32_32x32x16_bf16 accumulators:
//  * weight and activation K-step tiles copied global -> LDS by
//    buffer_load ... lds, double-buffered (the next K step in flight during
//    this step's MFMAs); pixels past P read zeros from the range check;
//  * 128-B tile rows, the 16-B chunk index XOR ((row >> 1) & 7): a
//    ds_read_b128 of 16 consecutive rows covers all 64 banks;
//  * the next 16-deep sub-step's fragments are read while this one's MFMAs
//    run (inline-asm LDS reads + counted lgkmcnt waits: the compiler would
//    otherwise drain the in-flight DMA in front of every read);
//  * the accumulators go through the shared 32 x 32 epilogue of the conv
//    tiles (bias, ReLU, scale, ReLU backward, GRU gates, fp32 accumulation).
#include "conv_common.h"

namespace rs {
namespace conv1 {

using conv::Args;

constexpr int BM = 128, BN = 128;
constexpr int TILE = 128 * 128;    // bytes of one operand tile (128 rows x 64 bf16)
constexpr int STAGE = 2 * TILE;    // weights + activations
constexpr int kFar = 0x7ffffff0;   // buffer offset past every range: reads zeros

__device__ __forceinline__ int chunk_of(int r, int pc) { return pc ^ ((r >> 1) & 7); }

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, const uint8_t* lds_base, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_base, 16, voff, 0, 0, 0);
}

typedef short v8s_t __attribute__((ext_vector_type(8)));

// the fragments of one 16-deep sub-step: 2 weight (co) x 2 activation (pixel) blocks
struct Frags {
  v8s_t a[2], b[2];
};

template <int KK>
__device__ __forceinline__ void read_frags(Frags& f, const uint32_t (&aaddr)[2][4], const uint32_t (&baddr)[2][4],
                                           uint32_t so) {
#pragma unroll
  for (int i = 0; i < 2; ++i)
    asm volatile("ds_read_b128 %0, %1" : "=v"(f.a[i]) : "v"(aaddr[i][KK] + so) : "memory");
#pragma unroll
  for (int j = 0; j < 2; ++j)
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f.b[j]) : "v"(baddr[j][KK] + so), "i"(TILE) : "memory");
}

__device__ __forceinline__ void mfma4(f32x16_t (&acc)[2][2], Frags& f) {
  asm volatile("" : "+v"(f.a[0]), "+v"(f.a[1]), "+v"(f.b[0]), "+v"(f.b[1]));
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, f.a[i]),
                                                          __builtin_bit_cast(bf16x8_t, f.b[j]), acc[i][j], 0, 0, 0);
  __builtin_amdgcn_sched_barrier(0);
}

__global__ __launch_bounds__(256) void conv1x1_kernel(Args a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1;
  const int nm = cdiv(a.Cout, BM);
  const int lid = conv::xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (lid % nm) * BM, n0 = (lid / nm) * BN;  // the Cout tiles of one pixel tile run together
  const int P = a.P;

  // K chunks (64 channels) of the concatenated segments
  const int e1 = a.seg[0].C >> 6;
  const int e2 = e1 + (a.nseg > 1 ? (a.seg[1].C >> 6) : 0);
  const int nk = e2 + (a.nseg > 2 ? (a.seg[2].C >> 6) : 0);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, a.w_bytes, 0x00020000);

  // per-lane DMA roles: 4 weight + 4 activation slots of 16 B per K step
  int ro[4], co8[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int s = (wave + 4 * i) * 64 + lane, r = s >> 3;
    ro[i] = r;
    co8[i] = 8 * chunk_of(r, s & 7);
  }
  auto issue = [&](int kt, int st) {
    const uint8_t* sb = lds + st * STAGE;
    const bool live = kt < nk;
    const int si = live ? (kt >= e1) + (kt >= e2) : 0;
    const int c0 = (kt - (si == 0 ? 0 : (si == 1 ? e1 : e2))) * 64;
    const conv::Seg sg = si == 0 ? a.seg[0] : (si == 1 ? a.seg[1] : a.seg[2]);
    const unsigned sbytes = si == 0 ? a.seg_bytes[0] : (si == 1 ? a.seg_bytes[1] : a.seg_bytes[2]);
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)sg.ptr, (short)0, sbytes, 0x00020000);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      // weight row m0 + r, columns kt*64 + chunk (rows past Cout are the packed zero padding)
      const int v = live ? ((m0 + ro[i]) * a.Ktot + kt * 64 + co8[i]) * 2 : kFar;
      dma16(rw, sb + (wave + 4 * i) * 1024, v);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = n0 + ro[i];
      const int v = (live && p < P) ? (p * sg.stride + c0 + co8[i]) * 2 : kFar;
      dma16(rx, sb + TILE + (wave + 4 * i) * 1024, v);
    }
  };

  // fragment read addresses: row (wm*64 + 32 i + lane & 31), logical chunk 2 KK + h
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) uint8_t*)lds;
  const int h = lane >> 5;
  uint32_t aaddr[2][4], baddr[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ra = wm * 64 + 32 * i + (lane & 31), rb = wn * 64 + 32 * i + (lane & 31);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      aaddr[i][kk] = lds0 + ra * 128 + (chunk_of(ra, 2 * kk + h) << 4);
      baddr[i][kk] = lds0 + rb * 128 + (chunk_of(rb, 2 * kk + h) << 4);
    }
  }

  f32x16_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  issue(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    const int st = kt & 1;
    issue(kt + 1, st ^ 1);            // zeros past the end: a static vmcnt count
    conv::wait_vmcnt<8>();            // this step's own pieces have landed
    asm volatile("s_barrier" ::: "memory");  // ... and every other wave's
    const uint32_t so = st * STAGE;
    Frags f0, f1;
    read_frags<0>(f0, aaddr, baddr, so);
    read_frags<1>(f1, aaddr, baddr, so);
    conv::wait_lgkm<4>();
    mfma4(acc, f0);
    read_frags<2>(f0, aaddr, baddr, so);
    conv::wait_lgkm<4>();
    mfma4(acc, f1);
    read_frags<3>(f1, aaddr, baddr, so);
    conv::wait_lgkm<4>();
    mfma4(acc, f0);
    conv::wait_lgkm<0>();
    mfma4(acc, f1);
    asm volatile("s_barrier" ::: "memory");  // every wave done reading this stage
  }
  conv::wait_vmcnt<0>();  // the trailing zero DMA lands before the LDS is released

  // epilogue: acc[i][j] = channels m0 + wm*64 + 32 i (+ reg rows) x pixels n0 + wn*64 + 32 j + lane & 31
  const int HW = a.H * a.W;
  int pp[2], pb[2], py[2], px[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int p = n0 + wn * 64 + 32 * j + (lane & 31);
    if (p < P) {
      pb[j] = p / HW;
      const int q = p - pb[j] * HW;
      py[j] = q / a.W;
      px[j] = q - py[j] * a.W;
      pp[j] = p;
    } else {
      pb[j] = -1;
      py[j] = px[j] = pp[j] = 0;
    }
  }
  // (two explicit calls: a runtime-indexed acc[i] would go through scratch)
  conv::epilogue32<2>(a, acc[0], m0 + wm * 64, lane, pp, pb, py, px);
  conv::epilogue32<2>(a, acc[1], m0 + wm * 64 + 32, lane, pp, pb, py, px);
}

}  // namespace conv1

// tile 70: 1x1, bf16, every segment's channels a multiple of 64, weights with
// round_up(Cout, 128) rows (host-checked in ops_conv.cpp)
bool conv_1x1_launch(const conv::Args& a, int tile, hipStream_t stream) {
  if (tile != 70 || a.KH != 1 || a.KW != 1) return false;
  const int nblk = cdiv(a.Cout, conv1::BM) * cdiv(a.P, conv1::BN);
  if (nblk > 0) hipLaunchKernelGGL(conv1::conv1x1_kernel, dim3(nblk), dim3(256), 0, stream, a);
  return true;
}

}  // namespace rs
