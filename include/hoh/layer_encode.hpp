// Drop-in for layer_encode (layer_encode.hpp:11-20) at cruncher_mode 0 (-s0: fast-path MED,
// no predictor search).  LEMPEL_NUKE (may be null) marks pixels covered by LZ copies, which are
// left out of the residual stream.  compressed must hold (depth*size + depth*size % 8 + 1024)/8
// bytes, the reference's own bound (layer_encode.hpp:22).  Returns bytes written, 0 on error
// (cruncher_mode > 0 is reported as unsupported).
#pragma once
#include <cstddef>
#include <cstdint>
#include "hoh_gpu.hpp"

inline size_t layer_encode(uint16_t* data, size_t size, int width, int height, int depth, size_t cruncher_mode,
                           uint8_t* LEMPEL_NUKE, uint8_t* compressed) {
  const size_t cap = ((size_t)depth * size + (size_t)depth * size % 8 + 1024) / 8;
  size_t n = 0;
  if (!hoh_gpu::ok(hoh_layer_encode(hoh_gpu::ctx(), data, size, width, height, depth, cruncher_mode, LEMPEL_NUKE,
                                    compressed, cap, &n),
                   "layer_encode"))
    return 0;
  return n;
}
