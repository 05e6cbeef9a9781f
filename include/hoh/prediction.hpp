// Drop-in for channelpredict_fastpath (prediction.hpp:6-13): returns a new[]'d array of size
// MED residuals, *buffer_size = size.  nullptr on error.
#pragma once
#include <cstddef>
#include <cstdint>
#include "hoh_gpu.hpp"

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
