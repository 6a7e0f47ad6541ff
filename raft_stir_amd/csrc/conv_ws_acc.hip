// conv_ws.h instantiations for the EK_ACC epilogue class.
#include "conv_ws.h"

namespace rs {
namespace conv {
#ifdef RS_WS_LIST  // (kernel experiments: build a subset)
RS_WS_DISPATCH(ws_acc, EK_ACC, RS_WS_LIST)
#else
RS_WS_DISPATCH(ws_acc, EK_ACC, RS_WS_1X1 RS_WS_3X3 RS_WS_SEP)
#endif
}  // namespace conv
}  // namespace rs
