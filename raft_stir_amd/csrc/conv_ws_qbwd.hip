// conv_ws.h instantiations for the EK_QBWD epilogue class.
#include "conv_ws.h"

namespace rs {
namespace conv {
#ifdef RS_WS_LIST  // (kernel experiments: build a subset)
RS_WS_DISPATCH(ws_qbwd, EK_QBWD, RS_WS_LIST)
#else
RS_WS_DISPATCH(ws_qbwd, EK_QBWD, RS_WS_SEP RS_WS_3X3)
#endif
}  // namespace conv
}  // namespace rs
