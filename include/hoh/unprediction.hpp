// Drop-in for unpredict_all (unprediction.hpp:6-16) with the fast-path predictor map
// (x_tiles = y_tiles = 1, tile_map = {0x0010}, what -s0 writes); other predictor maps (-s>=1)
// return nullptr.  size residuals (pixels not covered by LEMPEL_BACKREF copies); returns a
// new[]'d width*height plane, MED inverted on every row (SURVEY Q9 fixed).
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include "hoh_gpu.hpp"

inline uint16_t* unpredict_all(uint16_t* data, size_t size, int width, int height, int depth, int x_tiles,
                               int y_tiles, uint16_t* tile_map, uint16_t* LEMPEL_BACKREF) {
  if (x_tiles != 1 || y_tiles != 1 || !tile_map || tile_map[0] != 0x0010) {
    std::fprintf(stderr, "hoh-ans: unpredict_all: only the -s0 fast-path predictor is implemented\n");
    return nullptr;
  }
  uint16_t* out = new uint16_t[(size_t)width * height ? (size_t)width * height : 1];
  if (!hoh_gpu::ok(hoh_unpredict_fastpath(hoh_gpu::ctx(), data, size, LEMPEL_BACKREF, width, height, depth, out),
                   "unpredict_all")) {
    delete[] out;
    return nullptr;
  }
  return out;
}
