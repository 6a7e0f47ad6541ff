// conv_v3.h instantiated for the 1x5 kernel (one translation unit per shape).
#include "conv_v3.h"

namespace rs {
RS_V3_LAUNCHER(conv_v3_launch_k15, 1, 5)
}  // namespace rs
