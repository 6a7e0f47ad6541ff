// conv_v3.h instantiated for the 5x1 kernel (one translation unit per shape).
#include "conv_v3.h"

namespace rs {
RS_V3_LAUNCHER(conv_v3_launch_k51, 5, 1)
}  // namespace rs
