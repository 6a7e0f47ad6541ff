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
  int KH, KW, PH, PW;
  int Ktot, taps;
  float* dw;
  int kchunk;
};

__device__ __forceinline__ int tswz(int row, int chunk) { return row * 4 + (chunk ^ ((row >> 2) & 3)); }

constexpr int BM = 64, BN = 64, BK = 32;

__global__ __launch_bounds__(256) void wgrad_kernel(Args a) {
  __shared__ uint4 lds[2][(BM + BN) * 4];  // rows of 32 pixels (4 x 16 B)
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int ntile = blockIdx.x;
  const int nkb = a.Ktot / BN;
  const int tap = ntile / nkb, kb = (ntile % nkb) * BN;
  const int m0 = blockIdx.y * BM;
  const int pbeg = blockIdx.z * a.kchunk;
  const int pend = min(a.P, pbeg + a.kchunk);
  const int H = a.H, W = a.W, HW = H * W;
  const int dy_ = tap / a.KW - a.PH, dx_ = tap % a.KW - a.PW;

  // segment holding channels [kb, kb + 64) of the concatenated input
  const Seg s0 = a.seg[0], s1 = a.seg[1], s2 = a.seg[2];
  const int c01 = s0.C, c012 = s0.C + (a.nseg > 1 ? s1.C : 0);
  const int si = (kb >= c01) + (kb >= c012);
  const bf16_t* sp = si == 0 ? s0.ptr : (si == 1 ? s1.ptr : s2.ptr);
  const int sst = si == 0 ? s0.stride : (si == 1 ? s1.stride : s2.stride);
  const int sper = si == 0 ? s0.period : (si == 1 ? s1.period : s2.period);
  const int cbase = kb - (si == 0 ? 0 : (si == 1 ? c01 : c012));

  // staging assignment: thread -> (pixel row px = t / 8, channel group cg = t % 8).
  // (macros, not lambdas: a lambda capturing the kernarg struct spills it to scratch)
  const int spx = t >> 3, scg = t & 7;
  const bf16_t* ybase = a.dy + a.yoff + m0 + scg * 8;
  const int ystr = a.ystr;
  const uint4 zero = make_uint4(0, 0, 0, 0);
  uint4 ry, rx;
#define RS_WG_LOAD(P0)                                                                          \
  do {                                                                                          \
    const int p = (P0) + spx;                                                                   \
    ry = zero;                                                                                  \
    rx = zero;                                                                                  \
    if (p < pend) {                                                                             \
      ry = *reinterpret_cast<const uint4*>(ybase + (size_t)p * ystr);                           \
      const int q = p % HW, y = q / W + dy_, x = q % W + dx_;                                   \
      if (y >= 0 && y < H && x >= 0 && x < W) {                                                 \
        const int src = (p - q) + y * W + x;                                                    \
        rx = *reinterpret_cast<const uint4*>(sp + (size_t)(src % sper) * sst + cbase + scg * 8); \
      }                                                                                         \
    }                                                                                           \
  } while (0)
  // transposed store: element j of the chunk -> row (cg*8 + j), pixel spx
#define RS_WG_STORE(BUF)                                                                        \
  do {                                                                                          \
    uint16_t* A_ = reinterpret_cast<uint16_t*>(&lds[BUF][0]);                                   \
    uint16_t* B_ = reinterpret_cast<uint16_t*>(&lds[BUF][BM * 4]);                              \
    const uint32_t wy[4] = {ry.x, ry.y, ry.z, ry.w};                                            \
    const uint32_t wx[4] = {rx.x, rx.y, rx.z, rx.w};                                            \
    const int ch = spx >> 3, e = spx & 7;                                                       \
    _Pragma("unroll") for (int j = 0; j < 8; ++j) {                                             \
      const int row = scg * 8 + j;                                                              \
      A_[tswz(row, ch) * 8 + e] = (uint16_t)(j & 1 ? wy[j >> 1] >> 16 : wy[j >> 1] & 0xffff);   \
      B_[tswz(row, ch) * 8 + e] = (uint16_t)(j & 1 ? wx[j >> 1] >> 16 : wx[j >> 1] & 0xffff);   \
    }                                                                                           \
  } while (0)

  f32x4_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int lr = lane & 15, lc = lane >> 4;
  const int nsteps = pend > pbeg ? (pend - pbeg + BK - 1) / BK : 0;
  if (nsteps > 0) {
    RS_WG_LOAD(pbeg);
    RS_WG_STORE(0);
  }
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    if (s + 1 < nsteps) RS_WG_LOAD(pbeg + (s + 1) * BK);
    uint4 fa[2], fb[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) fa[mt] = lds[buf][tswz(wm * 32 + mt * 16 + lr, lc)];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) fb[nt] = lds[buf][BM * 4 + tswz(wn * 32 + nt * 16 + lr, lc)];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fa[mt]),
                                                              __builtin_bit_cast(bf16x8_t, fb[nt]),
                                                              acc[mt][nt], 0, 0, 0);
    if (s + 1 < nsteps) RS_WG_STORE(buf ^ 1);
    __syncthreads();
  }
#undef RS_WG_LOAD
#undef RS_WG_STORE
  if (nsteps == 0) return;
  // C[co][k]: row = 4*(lane>>4) + j (co), col = lane & 15 (k)
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int co = m0 + wm * 32 + mt * 16 + (lane >> 4) * 4 + j;
        const int k = kb + wn * 32 + nt * 16 + (lane & 15);
        if (co < a.Cout) atomicAdd(a.dw + ((size_t)co * a.taps + tap) * a.Ktot + k, acc[mt][nt][j]);
      }
}

// db[c] += sum_p dY[p][yoff + c]; block = 256 pixels, threads over channels.
__global__ __launch_bounds__(256) void colsum_kernel(const bf16_t* __restrict__ dy, int ystr, int yoff,
                                                     int C, int P, float* __restrict__ db) {
  const int p0 = blockIdx.x * 256;
  const int p1 = min(P, p0 + 256);
  for (int c = threadIdx.x; c < C; c += 256) {
    float s = 0.f;
    for (int p = p0; p < p1; ++p) s += bf2f(dy[(size_t)p * ystr + yoff + c]);
    atomicAdd(db + c, s);
  }
}

// convf1 weight gradient: dW[tap][ci][co] (the flow_encode layout [7][7][2][Cout])
// += sum_p dF[p][co] * flow[p + off(tap)][ci], flow = coords - grid (fp32 NCHW),
// and db[co] += sum_p dF[p][co].  Block = 64 pixels; thread (co, ci) keeps
// 49 tap accumulators; per-block partials go out with atomics.
__global__ __launch_bounds__(256) void flow_wgrad_kernel(const float* __restrict__ coords, int Bp, int H, int W,
                                                         const bf16_t* __restrict__ df,
                                                         int fstr, int Cout, float* __restrict__ dw,
                                                         float* __restrict__ db) {
  const int HW = H * W;
  const int P = Bp * HW;
  const int p0 = blockIdx.x * 64, p1 = min(P, p0 + 64);
  for (int pair = threadIdx.x; pair < Cout * 2; pair += 256) {
    const int co = pair % Cout, ci = pair / Cout;
    float acc[49];
#pragma unroll
    for (int i = 0; i < 49; ++i) acc[i] = 0.f;
    float bsum = 0.f;
    for (int p = p0; p < p1; ++p) {
      const float g = bf2f(df[(size_t)p * fstr + co]);
      if (ci == 0) bsum += g;
      if (g == 0.f) continue;
      const int q = p % HW, y = q / W, x = q % W;
      const float* cp = coords + ((size_t)(p / HW) * 2 + ci) * HW;
#pragma unroll
      for (int ky = 0; ky < 7; ++ky) {
        const int yy = y + ky - 3;
        if (yy < 0 || yy >= H) continue;
#pragma unroll
        for (int kx = 0; kx < 7; ++kx) {
          const int xx = x + kx - 3;
          if (xx < 0 || xx >= W) continue;
          const float f = cp[yy * W + xx] - (ci == 0 ? (float)xx : (float)yy);
          acc[ky * 7 + kx] += g * f;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 49; ++i) atomicAdd(dw + ((size_t)i * 2 + ci) * Cout + co, acc[i]);
    if (ci == 0) atomicAdd(db + co, bsum);
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
};

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
  a.KH = L.KH; a.KW = L.KW; a.PH = L.KH / 2; a.PW = L.KW / 2;
  a.Ktot = L.Ktot; a.taps = L.KH * L.KW;
  a.dw = L.dw;
  const int ntiles = a.taps * (a.Ktot / wgrad::BN);
  const int mtiles = cdiv(a.Cout, wgrad::BM);
  int ksplit = cdiv(2048, ntiles * mtiles);
  ksplit = max(1, min(ksplit, cdiv(a.P, 32 * 16)));
  a.kchunk = round_up(cdiv(a.P, ksplit), 32);
  ksplit = cdiv(a.P, a.kchunk);
  dim3 grid(ntiles, mtiles, ksplit);
  hipLaunchKernelGGL(wgrad::wgrad_kernel, grid, dim3(256), 0, stream, a);
}

void colsum_launch(const void* dy, int ystr, int yoff, int C, int P, float* db, hipStream_t stream) {
  hipLaunchKernelGGL(wgrad::colsum_kernel, dim3(cdiv(P, 256)), dim3(256), 0, stream,
                     static_cast<const bf16_t*>(dy), ystr, yoff, C, P, db);
}

void flow_wgrad_launch(const float* coords, int Bp, int H, int W, const void* df, int fstr, int Cout, float* dw,
                       float* db, hipStream_t stream) {
  const int P = Bp * H * W;
  hipLaunchKernelGGL(wgrad::flow_wgrad_kernel, dim3(cdiv(P, 64)), dim3(256), 0, stream, coords, Bp, H, W,
                     static_cast<const bf16_t*>(df), fstr, Cout, dw, db);
}

}  // namespace rs
