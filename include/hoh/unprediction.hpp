// Drop-in for unpredict_all (unprediction.hpp:6-16): size residuals (pixels not covered by
// LEMPEL_BACKREF copies) -> a new[]'d width*height plane.  Any predictor map: the exact inverse
// of channelpredict_all.  The 1x1 {0x0010} map written by -s0 (whose encoder uses MED on every
// row) is inverted with MED on every row (SURVEY Q9 fixed).  nullptr on error.
#pragma once
#include <cstddef>
#include <cstdint>
#include "hoh_gpu.hpp"
#if __has_include("predictor_operations.hpp")   // included by the reference header (:4)
#include "predictor_operations.hpp"
#endif

inline uint16_t* unpredict_all(uint16_t* data, size_t size, int width, int height, int depth, int x_tiles,
                               int y_tiles, uint16_t* tile_map, uint16_t* LEMPEL_BACKREF) {
  uint16_t* out = new uint16_t[(size_t)width * height ? (size_t)width * height : 1];
  if (!hoh_gpu::ok(hoh_unpredict_all(hoh_gpu::ctx(), data, size, LEMPEL_BACKREF, width, height, depth, x_tiles, y_tiles,
                                     tile_map, out),
                   "unpredict_all")) {
    delete[] out;
    return nullptr;
  }
  return out;
}
