// Drop-in for layer_encode (layer_encode.hpp:11-20), cruncher_mode 0..4: -s0 is the fast-path
// MED; 1..4 add the 40-px grid predictor search, the predictor map and the prob_bits ladder with
// the reference's stale-prefix output.  LEMPEL_NUKE (may be null) marks pixels
// covered by LZ copies, which are left out of the residual stream.  compressed must hold the
// reference's bound (depth*size + depth*size % 8 + 1024)/8 (layer_encode.hpp:22) plus the
// predictor header (callers in the reference allocate 3*size + 256).  Returns bytes written, 0
// on error.
#pragma once
#include <cstddef>
#include <cstdint>
#include <cmath>
#include "entropy_encoding.hpp"   // the reference header includes these (layer_encode.hpp:4-9)
#include "entropy_decoding.hpp"
#include "prediction.hpp"
#include "hoh_gpu.hpp"

inline size_t layer_encode(uint16_t* data, size_t size, int width, int height, int depth, size_t cruncher_mode,
                           uint8_t* LEMPEL_NUKE, uint8_t* compressed) {
  const size_t cap = ((size_t)depth * size + (size_t)depth * size % 8 + 1024) / 8 + 512;
  size_t n = 0;
  if (!hoh_gpu::ok(hoh_layer_encode(hoh_gpu::ctx(), data, size, width, height, depth, cruncher_mode, LEMPEL_NUKE,
                                    compressed, cap, &n),
                   "layer_encode"))
    return 0;
  return n;
}
