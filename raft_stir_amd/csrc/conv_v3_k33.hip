// conv_v3.h instantiated for the 3x3 kernel (one translation unit per shape).
#include "conv_v3.h"

namespace rs {
RS_V3_LAUNCHER(conv_v3_launch_k33, 3, 3)
}  // namespace rs
