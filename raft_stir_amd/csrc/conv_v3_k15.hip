// conv_v3.h instantiated for the 1x5 kernel (one translation unit per shape).
#include "conv_v3.h"

namespace rs {
// timing experiments (RS_V3_EXP builds only): tiles 70-76 run tile 60's geometry with
// 70: no A wait, 71: no halo refill, 72: no barrier, 73: every A load from slice 0,
// 74: ring 20 deep, 75: 74 on tile 61's geometry, 76: no A wait + no halo + no barrier,
// 77: MFMAs only (no loads, LDS reads or waits in the loop), 78: no main loop, 79: 77 on tile 61's geometry
#ifdef RS_V3_EXP
bool conv_v3_exp_k15(const conv::Args& a, int tile, hipStream_t stream) {
  const dim3 g6(cdiv(a.Cout, 128) * a.B * cdiv(a.H, 6) * cdiv(a.W, 32)), g3(cdiv(a.Cout, 128) * a.B * cdiv(a.H, 3) * cdiv(a.W, 32));
  switch (tile) {
    case 70: hipLaunchKernelGGL((conv::conv_v3_kernel<1, 5, 4, 1, 6, 10, 1>), g6, dim3(256), 0, stream, a); return true;
    case 71: hipLaunchKernelGGL((conv::conv_v3_kernel<1, 5, 4, 1, 6, 10, 2>), g6, dim3(256), 0, stream, a); return true;
    case 72: hipLaunchKernelGGL((conv::conv_v3_kernel<1, 5, 4, 1, 6, 10, 4>), g6, dim3(256), 0, stream, a); return true;
    case 73: hipLaunchKernelGGL((conv::conv_v3_kernel<1, 5, 4, 1, 6, 10, 8>), g6, dim3(256), 0, stream, a); return true;
    case 74: hipLaunchKernelGGL((conv::conv_v3_kernel<1, 5, 4, 1, 6, 20, 0>), g6, dim3(256), 0, stream, a); return true;
    case 75: hipLaunchKernelGGL((conv::conv_v3_kernel<1, 5, 4, 1, 3, 20, 0>), g3, dim3(256), 0, stream, a); return true;
    case 76: hipLaunchKernelGGL((conv::conv_v3_kernel<1, 5, 4, 1, 6, 10, 7>), g6, dim3(256), 0, stream, a); return true;
    case 77: hipLaunchKernelGGL((conv::conv_v3_kernel<1, 5, 4, 1, 6, 10, 16 | 4>), g6, dim3(256), 0, stream, a); return true;
    case 78: hipLaunchKernelGGL((conv::conv_v3_kernel<1, 5, 4, 1, 6, 10, 32>), g6, dim3(256), 0, stream, a); return true;
    case 79: hipLaunchKernelGGL((conv::conv_v3_kernel<1, 5, 4, 1, 3, 10, 16 | 4>), g3, dim3(256), 0, stream, a); return true;
    default: return false;
  }
}
#endif
RS_V3_LAUNCHER(conv_v3_launch_k15, 1, 5)
}  // namespace rs
