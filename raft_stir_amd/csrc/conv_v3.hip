// Dispatch of the weight-streaming conv tiles 60-65 (conv_v3.h) by kernel shape.
#include "conv_v3.h"

namespace rs {

int conv_v3_block_m(int tile) {
  int nwm, mw, thw, nwp;
  return v3_geom(tile, &nwm, &mw, &thw, &nwp) ? 32 * nwm * mw : 0;
}

bool conv_v3_launch(const conv::Args& a, int tile, hipStream_t stream) {
  if (a.KH == 3 && a.KW == 3) return conv_v3_launch_k33(a, tile, stream);
  if (a.KH == 1 && a.KW == 5) return conv_v3_launch_k15(a, tile, stream);
  if (a.KH == 5 && a.KW == 1) return conv_v3_launch_k51(a, tile, stream);
  return false;
}

}  // namespace rs
