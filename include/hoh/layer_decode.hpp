// Drop-in for decode_layer (layer_decode.hpp:128-136): returns a new[]'d width*height plane as
// uint8_t like the reference (9-bit planes are truncated to 8 bits there too; the caller's
// inverse subtract-green works modulo 256).  Predictor-map layers are inverted by
// unpredict_all; the -s0 MED layer with MED on every row (SURVEY Q9 fixed).  nullptr on error.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>
#include "hoh_gpu.hpp"

inline uint8_t* decode_layer(uint8_t* in_bytes, size_t in_size, size_t byte_pointer, size_t width, size_t height,
                             uint8_t bit_depth, uint16_t* LEMPEL_BACKREF) {
  std::vector<uint16_t> plane(width * height ? width * height : 1);
  if (!hoh_gpu::ok(hoh_layer_decode(hoh_gpu::ctx(), in_bytes, in_size, byte_pointer, (int)width, (int)height,
                                    bit_depth, LEMPEL_BACKREF, plane.data()),
                   "decode_layer"))
    return nullptr;
  uint8_t* out = new uint8_t[width * height ? width * height : 1];
  for (size_t i = 0; i < width * height; i++) out[i] = (uint8_t)plane[i];
  return out;
}
