// Drop-in for the reference's layer_decode.hpp: decode_layer (:128-136) and its diagnostic walk
// decode_layer_simple (:7-126).
//
// decode_layer returns a new[]'d width*height plane as uint8_t like the reference (9-bit planes
// are truncated to 8 bits there too; the caller's inverse subtract-green works modulo 256).
// Predictor-map layers are inverted by unpredict_all; the -s0 MED layer with MED on every row
// (SURVEY Q9 fixed).  nullptr on error.  decode_layer_simple prints the layer's framing the way
// the reference does and walks its streams with decode_entropy_simple.
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <vector>
#include "entropy_decoding.hpp"   // the reference header includes both (layer_decode.hpp:4-5)
#include "unprediction.hpp"
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

inline void decode_layer_simple(uint8_t* in_bytes, size_t in_size, size_t byte_pointer, size_t /*width*/,
                                size_t /*height*/, uint8_t bit_depth) {
  const uint8_t tr = in_bytes[byte_pointer++];
  const int compaction = (tr & 0xe0) >> 5, prediction = (tr & 0x10) >> 4;
  switch (compaction) {                                           // :19-72 (bytes skipped only)
    case 1:
      std::printf("[SIMPLE]     clamped channel\n");
      if (bit_depth == 8) byte_pointer += 2;
      else std::printf("[SIMPLE] unimplemented bit depth!\n");
      break;
    case 2:
      std::printf("[SIMPLE]     bitmasked channel\n");
      byte_pointer += (size_t(1) << bit_depth) / 8;
      break;
    case 4: byte_pointer += 1 + in_bytes[byte_pointer]; break;
    case 5: {
      const int c1 = in_bytes[byte_pointer], c2 = in_bytes[byte_pointer + 1];
      byte_pointer += 2 + (c2 - c1 + 8) / 8;
      break;
    }
    default: break;
  }
  std::printf("[SIMPLE] prediction mode: %d\n", prediction);
  size_t symbol_size = 0;
  if (prediction) {                                               // :76-114
    const size_t xt = in_bytes[byte_pointer] + 1u, yt = in_bytes[byte_pointer + 1] + 1u;
    byte_pointer += 2;
    if (xt == 1 && yt == 1) {
      byte_pointer += 2;
    } else {
      std::printf("[SIMPLE]     unimplemented prediction mode!\n");
      byte_pointer += 1 + 2 * (size_t)in_bytes[byte_pointer];
      decode_entropy_simple(in_bytes, in_size, &byte_pointer, &symbol_size, 1);
    }
  }
  decode_entropy_simple(in_bytes, in_size, &byte_pointer, &symbol_size, 0);
  std::printf("[SIMPLE] layer completed\n");
}
