// Drop-ins for the predictors of prediction.hpp: channelpredict_fastpath (:6-44),
// channelpredict_section (:46-151, the -s>=1 cost-search predictor of one grid cell) and
// channelpredict_all (:153-229, one predictor mask per cell).  Each returns a new[]'d array
// (the caller delete[]s it, as with the reference); nullptr on error.
#pragma once
#include <cstddef>
#include <cstdint>
#include "hoh_gpu.hpp"
#if __has_include("predictor_operations.hpp")   // included by the reference header (:4)
#include "predictor_operations.hpp"
#endif

inline uint16_t* channelpredict_fastpath(uint16_t* data, size_t size, int width, int height, int depth,
                                         size_t* buffer_size) {
  uint16_t* out = new uint16_t[size ? size : 1];
  if (!hoh_gpu::ok(hoh_predict_fastpath(hoh_gpu::ctx(), data, width, height, depth, out), "channelpredict_fastpath")) {
    delete[] out;
    return nullptr;
  }
  *buffer_size = size;
  return out;
}

inline uint16_t* channelpredict_section(uint16_t* data, size_t size, int width, int height, int depth,
                                        size_t x_tiles, size_t y_tiles, int x, int y, uint16_t predictor,
                                        size_t* buffer_size) {
  (void)size;
  const size_t tw = (width + x_tiles - 1) / x_tiles, th = (height + y_tiles - 1) / y_tiles;
  uint16_t* out = new uint16_t[tw * th ? tw * th : 1];
  if (!hoh_gpu::ok(hoh_predict_section(hoh_gpu::ctx(), data, width, height, depth, (int)x_tiles, (int)y_tiles, x, y,
                                       predictor, out, buffer_size),
                   "channelpredict_section")) {
    delete[] out;
    return nullptr;
  }
  return out;
}

inline uint16_t* channelpredict_all(uint16_t* data, size_t size, int width, int height, int depth, int x_tiles,
                                    int y_tiles, uint16_t* tile_map) {
  uint16_t* out = new uint16_t[size ? size : 1];
  if (!hoh_gpu::ok(hoh_predict_all(hoh_gpu::ctx(), data, width, height, depth, x_tiles, y_tiles, tile_map, out),
                   "channelpredict_all")) {
    delete[] out;
    return nullptr;
  }
  return out;
}
