// Packed-weight gather (ops/wpack.py, models/fused_train.py pack): every
// packed layout element is a static code into the layout's SOURCE parameters,
// read in place with the parameters' own strides (channels_last conv weights
// included) and cast to the packed dtype:
//
//   out[i] = scale(i) * src_s[unravel(li)],   code[i] = (lo << 30) | (s << 24) | li,  code < 0 -> 0
//   (lo: the split-weight low part src - bf16(src) of the F32 conv tiles)
//
// One launch per chunk replaces flatten-copies of every channels_last source,
// a cat of all sources, an index_select and a cast (4 + #sources launches and
// two full copies of the parameters).
#include "common.h"

namespace rs {
namespace wpack {

// source table row (int64): ptr, is_bf16, size[4] (leading dims padded with 1), stride[4]
constexpr int kTabCols = 10;
constexpr int kMaxRanges = 4;

struct Ranges {
  long long lo[kMaxRanges], hi[kMaxRanges];
  float s[kMaxRanges];
  int n;
};

template <bool OUT_BF16>
__global__ __launch_bounds__(256) void gather_kernel(const int* __restrict__ code, long long n,
                                                     const long long* __restrict__ tab, void* __restrict__ out,
                                                     Ranges rg) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int c = code[i];
    float v = 0.f;
    if (c >= 0) {
      const long long* t = tab + (long long)((c >> 24) & 63) * kTabCols;
      const long long ptr = t[0];
      if (ptr != 0) {
        // 32-bit unravel (li < 2^24, every dim < 2^24): 64-bit division is a
        // long software sequence on CDNA
        unsigned li = (unsigned)(c & 0xffffff);
        const unsigned s3 = (unsigned)t[5], s2 = (unsigned)t[4], s1 = (unsigned)t[3];
        const unsigned q3 = li / s3, i3 = li - q3 * s3;
        const unsigned q2 = q3 / s2, i2 = q3 - q2 * s2;
        const unsigned i0 = q2 / s1, i1 = q2 - i0 * s1;
        const long long off = (long long)i0 * t[6] + (long long)i1 * t[7] + (long long)i2 * t[8] + (long long)i3 * t[9];
        v = t[1] ? bf2f(reinterpret_cast<const bf16_t*>(ptr)[off]) : reinterpret_cast<const float*>(ptr)[off];
        if (c & (1 << 30)) v -= bf2f(f2bf(v));  // the lo half of a split (F32-tile) weight
      }
    }
    for (int r = 0; r < rg.n; ++r)
      if (i >= rg.lo[r] && i < rg.hi[r]) v *= rg.s[r];
    if constexpr (OUT_BF16)
      static_cast<bf16_t*>(out)[i] = f2bf(v);
    else
      static_cast<float*>(out)[i] = v;
  }
}

}  // namespace wpack

void wpack_gather_launch(const int* code, long long n, const long long* tab, void* out, bool out_bf16,
                         const long long* lo, const long long* hi, const float* s, int nr, hipStream_t stream) {
  wpack::Ranges rg{};
  rg.n = nr;
  for (int r = 0; r < nr; ++r) {
    rg.lo[r] = lo[r];
    rg.hi[r] = hi[r];
    rg.s[r] = s[r];
  }
  const long long blocks = (n + 255) / 256;
  const int grid = (int)(blocks < 8192 ? (blocks > 0 ? blocks : 1) : 8192);
  if (out_bf16)
    hipLaunchKernelGGL(wpack::gather_kernel<true>, dim3(grid), dim3(256), 0, stream, code, n, tab, out, rg);
  else
    hipLaunchKernelGGL(wpack::gather_kernel<false>, dim3(grid), dim3(256), 0, stream, code, n, tab, out, rg);
}

}  // namespace rs
