// Drop-in for the reference's decode_entropy (entropy_decoding.hpp:134-140): returns a new[]'d
// array of *symbol_size symbols (caller delete[]s it) and advances *byte_pointer past the whole
// stream (the reference leaves it after the frequency table; every caller in the
// reference that reads a second stream relies on the corrected behaviour).  Returns nullptr on a
// malformed / undecodable stream (the reference crashes or returns garbage there).
#pragma once
#include <cstddef>
#include <cstdint>
#include "hoh_gpu.hpp"

inline uint16_t* decode_entropy(uint8_t* in_bytes, size_t in_size, size_t* byte_pointer, size_t* symbol_size,
                                uint8_t /*diagnostics*/) {
  size_t n = 0;
  if (!hoh_gpu::ok(hoh_entropy_count(in_bytes, in_size, *byte_pointer, &n), "decode_entropy")) return nullptr;
  uint16_t* out = new uint16_t[n ? n : 1];
  size_t got = 0;
  if (!hoh_gpu::ok(hoh_decode_entropy(hoh_gpu::ctx(), in_bytes, in_size, byte_pointer, out, n ? n : 1, &got),
                   "decode_entropy")) {
    delete[] out;
    return nullptr;
  }
  *symbol_size = got;
  return out;
}
