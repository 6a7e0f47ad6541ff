// Flow encoder of the motion encoder (convf1, 7x7, 2 -> Cout, ReLU) on the
// matrix cores; see the kernel comment.  Launched through
// torch.ops.raft_stir.flow_encode (csrc/ops_conv.cpp).
#include "common.h"

namespace rs {
namespace fe {

// ------------------------------------------------------------------ flow encoder
// convf1 of the motion encoder (reference core/update.py:67,84): a 7x7 conv
// of the 2-channel flow (= coords1 - coords0, computed here from coords1)
// with ReLU, written as bf16 NHWC; it also writes the flow itself (bf16)
// into its slot of the GRU input buffer (reference: cat([out, flow])).
//
// MFMA with split-bf16 operands: the flow can be ~100 px at 1/8 resolution
// (plain bf16 would quantise it to 0.5 px), so both operands are split as
// x = hi + lo (two bf16, ~16 mantissa bits) and each K step issues
// Whi*Fhi + Whi*Flo + Wlo*Fhi -- fp32-level accuracy on the matrix cores.
// GEMM per 7x7 tap ROW: K = 16 = 8 columns x 2 channels (column 7 has zero
// weight), M = output channels, N = pixels.  Block = an 8 x 8 pixel tile x
// 64 channels; wave w: channels 32*(w&1).., pixel rows 4*(w>>1)..+3 (one
// 32x32x16 tile, 7 rows x 3 MFMAs).  The flow patch (14 x 15, hi and lo) is
// staged in LDS as one uint32 (2 bf16 channels) per pixel, the block's 64
// channels of split weights as [co][ky][16] bf16 (one 16-B read per operand).
// (Previous VALU versions were bound by scalar weight loads / LDS weight
// broadcasts: 34.5 -> 18.1 us at the training shape.)
constexpr int FE_T = 8;                 // tile edge (pixels)
constexpr int FE_PH = FE_T + 6;         // patch rows
constexpr int FE_PW = FE_T + 7;         // patch columns (+1: the zero-weight 8th column)

__device__ __forceinline__ void split_bf16(float x, uint32_t& hi, uint32_t& lo) {
  const bf16_t h = f2bf(x);
  hi = h;
  lo = f2bf(x - bf2f(h));
}

// OT: output activation type (bf16_t, or float for the fp32 inference engine)
template <typename OT>
__global__ __launch_bounds__(256) void flow_enc_kernel(const float* __restrict__ coords, int B, int H,
                                                       int W, const float* __restrict__ w,  // [49][2][Cout]
                                                       const float* __restrict__ bias, int Cout,
                                                       OT* __restrict__ out, int ostr, int ooff,
                                                       OT* __restrict__ fout, int fstr, int foff) {
  __shared__ uint32_t fh[FE_PH * FE_PW], flo[FE_PH * FE_PW];  // (u | v << 16) bf16 pairs
  // the block's 64 channels of split weights, [co][ky][16 = kx * 2 + ci] (kx = 7: zero)
  __shared__ __attribute__((aligned(16))) bf16_t wh[64 * 7 * 16], wlo[64 * 7 * 16];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int tx_n = cdiv(W, FE_T), ty_n = cdiv(H, FE_T);
  const int tile = blockIdx.x;
  const int b = tile / (tx_n * ty_n), rem = tile - b * tx_n * ty_n;
  const int y0 = (rem / tx_n) * FE_T, x0 = (rem % tx_n) * FE_T;
  const int HW = H * W;
  const float* cx = coords + (size_t)b * 2 * HW;
  const float* cy = cx + HW;
  for (int i = t; i < FE_PH * FE_PW; i += 256) {
    const int yy = y0 + i / FE_PW - 3, xx = x0 + i % FE_PW - 3;
    const bool in = yy >= 0 && yy < H && xx >= 0 && xx < W;
    const int o = in ? yy * W + xx : 0;
    const float u = in ? cx[o] - (float)xx : 0.f, v = in ? cy[o] - (float)yy : 0.f;
    uint32_t uh, ul, vh, vl;
    split_bf16(u, uh, ul);
    split_bf16(v, vh, vl);
    fh[i] = uh | (vh << 16);
    flo[i] = ul | (vl << 16);
  }
  const int cb0 = blockIdx.y * 64;
  // all 25 loads per thread in flight at once (a rolled loop waits on each)
  float wv[(98 * 64 + 255) / 256];
#pragma unroll
  for (int j = 0; j < (98 * 64 + 255) / 256; ++j) {  // coalesced over channels
    const int i = t + 256 * j, tc = i >> 6, cl = i & 63;
    wv[j] = (i < 98 * 64 && cb0 + cl < Cout) ? w[(size_t)tc * Cout + cb0 + cl] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < (98 * 64 + 255) / 256; ++j) {
    const int i = t + 256 * j, tc = i >> 6, cl = i & 63, tap = tc >> 1, ci = tc & 1;
    if (i >= 98 * 64) break;
    const float v = wv[j];
    const int o = (cl * 7 + tap / 7) * 16 + (tap % 7) * 2 + ci;
    const bf16_t h = f2bf(v);
    wh[o] = h;
    wlo[o] = f2bf(v - bf2f(h));
  }
  for (int i = t; i < 64 * 7 * 2; i += 256) {  // the zero 8th column
    const int o = (i >> 1) * 16 + 14 + (i & 1);
    wh[o] = 0;
    wlo[o] = 0;
  }
  // A fragments (weights) for this wave: co = cb + (lane & 31), k = 8*(lane>>5) .. +7
  const int cb = cb0 + 32 * (wave & 1);
  const int kh = lane >> 5;  // columns 4*kh .. 4*kh+3
  const int arow = (32 * (wave & 1) + (lane & 31)) * 7 * 16 + 8 * kh;
  __syncthreads();
  const int n = lane & 31;                       // pixel of the 32-pixel N tile
  const int pr = 4 * (wave >> 1) + (n >> 3), pc = n & 7;
  f32x16_t acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
  for (int ky = 0; ky < 7; ++ky) {
    const uint4 ah4 = *reinterpret_cast<const uint4*>(wh + arow + ky * 16);
    const uint4 al4 = *reinterpret_cast<const uint4*>(wlo + arow + ky * 16);
    const int pi = (pr + ky) * FE_PW + pc + 4 * kh;
    uint32_t bh[4], bl[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bh[j] = fh[pi + j];
      bl[j] = flo[pi + j];
    }
    const bf16x8_t Ah = __builtin_bit_cast(bf16x8_t, ah4);
    const bf16x8_t Al = __builtin_bit_cast(bf16x8_t, al4);
    const bf16x8_t Bh = __builtin_bit_cast(bf16x8_t, make_uint4(bh[0], bh[1], bh[2], bh[3]));
    const bf16x8_t Bl = __builtin_bit_cast(bf16x8_t, make_uint4(bl[0], bl[1], bl[2], bl[3]));
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Ah, Bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Ah, Bl, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Al, Bh, acc, 0, 0, 0);
  }
  // C[co][px]: px = lane & 31, co = cb + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)
  const int y = y0 + pr, x = x0 + pc;
  if (y >= H || x >= W) return;
  const size_t p = (size_t)b * HW + (size_t)y * W + x;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int c = cb + 8 * g + 4 * (lane >> 5);
    if (c >= Cout) continue;
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = fmaxf(acc[4 * g + j] + bias[c + j], 0.f);
    if constexpr (sizeof(OT) == 4) {
      *reinterpret_cast<float4*>(out + p * ostr + ooff + c) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
      uint2 u;
      u.x = uint32_t(f2bf(v[0])) | (uint32_t(f2bf(v[1])) << 16);
      u.y = uint32_t(f2bf(v[2])) | (uint32_t(f2bf(v[3])) << 16);
      *reinterpret_cast<uint2*>(out + p * ostr + ooff + c) = u;
    }
  }
  if (cb == 0 && lane < 32 && fout) {
    if constexpr (sizeof(OT) == 4) {  // the exact fp32 flow
      fout[p * fstr + foff] = cx[(size_t)y * W + x] - (float)x;
      fout[p * fstr + foff + 1] = cy[(size_t)y * W + x] - (float)y;
    } else {
      const int pi = (pr + 3) * FE_PW + pc + 3;
      const uint32_t h = fh[pi], l = flo[pi];
      fout[p * fstr + foff] = f2bf(bf2f((bf16_t)(h & 0xffffu)) + bf2f((bf16_t)(l & 0xffffu)));
      fout[p * fstr + foff + 1] = f2bf(bf2f((bf16_t)(h >> 16)) + bf2f((bf16_t)(l >> 16)));
    }
  }
}

}  // namespace fe

void flow_enc_launch(const float* coords, int B, int H, int W, const float* w, const float* bias,
                     int Cout, void* out, int ostr, int ooff, void* fout, int fstr, int foff, bool f32,
                     hipStream_t stream) {
  const dim3 grid((unsigned)(B * cdiv(H, fe::FE_T) * cdiv(W, fe::FE_T)), (unsigned)cdiv(Cout, 64));
  if (f32)
    hipLaunchKernelGGL(fe::flow_enc_kernel<float>, grid, dim3(256), 0, stream, coords, B, H, W, w, bias, Cout,
                       static_cast<float*>(out), ostr, ooff, static_cast<float*>(fout), fstr, foff);
  else
    hipLaunchKernelGGL(fe::flow_enc_kernel<bf16_t>, grid, dim3(256), 0, stream, coords, B, H, W, w, bias, Cout,
                       static_cast<bf16_t*>(out), ostr, ooff, static_cast<bf16_t*>(fout), fstr, foff);
}

}  // namespace rs
