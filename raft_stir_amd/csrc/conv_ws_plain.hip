// conv_ws.h instantiations for the EK_PLAIN epilogue class.
#include "conv_ws.h"

namespace rs {
namespace conv {
#ifdef RS_WS_LIST  // (kernel experiments: build a subset)
RS_WS_DISPATCH(ws_plain, EK_PLAIN, RS_WS_LIST)
#else
RS_WS_DISPATCH(ws_plain, EK_PLAIN, RS_WS_1X1 RS_WS_3X3)
#endif
}  // namespace conv
}  // namespace rs
