// Host-side helpers shared by the TORCH_LIBRARY op files (ops*.cpp).
//
// * current_stream(): the caller's current HIP stream, straight from c10's
//   HIP stream API (no CUDA-named compatibility layer), so every launch is
//   ordered with the surrounding PyTorch work and is graph-capturable.
// * RS_CHECK_LAUNCH(): a kernel launch reports a bad configuration (grid,
//   block, LDS size, missing code object) only through hipGetLastError; every
//   launcher call site is followed by this check, which turns such an error
//   into a Python RuntimeError naming the op instead of a silent no-op.
#pragma once

#include <c10/hip/HIPStream.h>
#include <c10/util/Exception.h>
#include <hip/hip_runtime.h>

namespace rs {
inline hipStream_t current_stream() { return c10::hip::getCurrentHIPStream().stream(); }
}  // namespace rs

#define RS_CHECK_LAUNCH()                                                                         \
  do {                                                                                            \
    const hipError_t rs_e_ = hipGetLastError();                                                   \
    TORCH_CHECK(rs_e_ == hipSuccess, "raft_stir: kernel launch failed in ", __func__, ": ",       \
                hipGetErrorString(rs_e_));                                                        \
  } while (0)
