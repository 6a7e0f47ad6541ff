// Weight-stationary implicit-GEMM convolution (the kernel: conv_ws.h):
// the zero page, the per-epilogue-class dispatch and the host-side launcher.
#include "conv_ws.h"

namespace rs {
namespace conv {

bool ws_plain(const Args* a, int KH, int KW, int G, int NB, int nblocks, hipStream_t stream);
bool ws_zr(const Args* a, int KH, int KW, int G, int NB, int nblocks, hipStream_t stream);
bool ws_q(const Args* a, int KH, int KW, int G, int NB, int nblocks, hipStream_t stream);
bool ws_relubwd(const Args* a, int KH, int KW, int G, int NB, int nblocks, hipStream_t stream);
bool ws_acc(const Args* a, int KH, int KW, int G, int NB, int nblocks, hipStream_t stream);
bool ws_qbwd(const Args* a, int KH, int KW, int G, int NB, int nblocks, hipStream_t stream);

static bool ws_dispatch(const Args* a, int epi, int KH, int KW, int G, int NB, int nblocks, hipStream_t stream) {
  switch (ws_class(epi)) {
    case EK_ZR: return ws_zr(a, KH, KW, G, NB, nblocks, stream);
    case EK_Q: return ws_q(a, KH, KW, G, NB, nblocks, stream);
    case EK_RELUBWD: return ws_relubwd(a, KH, KW, G, NB, nblocks, stream);
    case EK_ACC: return ws_acc(a, KH, KW, G, NB, nblocks, stream);
    case EK_QBWD: return ws_qbwd(a, KH, KW, G, NB, nblocks, stream);
    default: return (epi == EPI_FLOW || epi == EPI_NORM) ? false : ws_plain(a, KH, KW, G, NB, nblocks, stream);
  }
}

}  // namespace conv

bool conv_ws_launch(const conv::Args& a, int G, int NB, int nblocks, hipStream_t stream) {
  return conv::ws_dispatch(&a, a.epi, a.KH, a.KW, G, NB, nblocks, stream);
}

bool conv_ws_instantiated(int KH, int KW, int G, int NB, int epi) {
  return conv::ws_dispatch(nullptr, epi, KH, KW, G, NB, 0, 0);
}

}  // namespace rs
