// Launch-group table of the fused clip + AdamW kernels (optim.hip), shared
// with its host op (ops_optim.cpp): passed by value as a kernel argument.
#pragma once

namespace rs {
namespace optim {

constexpr int MAXT = 96;   // tensors per launch group (the table stays under the 4 KiB argument limit)
constexpr int CH = 8192;   // elements per block

struct TList {
  float* p[MAXT];
  float* g[MAXT];
  long long off[MAXT + 1];  // prefix offsets (elements) of the group's tensors in its own element space
  long long moff[MAXT];     // each tensor's offset in the flat moment buffers
  int n;                    // tensors in the group
  int pbase;                // the group's first block partial
};

}  // namespace optim
}  // namespace rs
