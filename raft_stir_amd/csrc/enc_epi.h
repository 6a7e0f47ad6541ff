// Epilogue extras of the encoder halo conv (enc_halo.hip HArgs), shared by
// the kernel TU and its host launcher (ops_conv.cpp conv3x3_halo).
#pragma once
#include <stdint.h>

namespace rs {
struct EncEpi {
  const float* chs = nullptr;    // eval-mode BatchNorm: y = [relu](acc * chs + shift) ...
  const float* shift = nullptr;
  const uint16_t* res = nullptr;  // ... then relu(y + res)  (bf16 NHWC, rstr elements per pixel)
  int rstr = 0, relu = 0;
  int res_relu = 1;               // 0: plain y + res (res may alias y: in-place accumulation)
};
}  // namespace rs
