// Drop-in for the reference's entropy_encoding.hpp: same signatures, computed on the GPU through
// libhohgpu (bit-identical output).  Replaces entropy_encoding.hpp:8-15 (uint16_t symbols) and
// :283-290 (uint8_t symbols).  output_bytes must hold hoh_entropy_bound(symbol_size, range,
// prob_bits) bytes (the reference writes unchecked into a caller buffer of similar size).
// Returns the stream size in bytes, 0 on error (message on stderr).  diagnostics is ignored.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>
#include "hoh_gpu.hpp"
// The reference header brings these in for its callers (entropy_encoding.hpp:4-6); keep that
// when this header stands in the reference tree.
#if __has_include("rans64.hpp") && __has_include("varint.hpp") && __has_include("stattools.hpp")
#include "rans64.hpp"
#include "varint.hpp"
#include "stattools.hpp"
#endif

inline size_t encode_entropy(uint16_t* symbols, size_t symbol_size, size_t range, uint8_t* output_bytes,
                             uint32_t prob_bits, uint8_t /*diagnostics*/) {
  size_t n = 0;
  const size_t cap = hoh_entropy_bound(symbol_size, range, prob_bits);
  if (!hoh_gpu::ok(hoh_encode_entropy(hoh_gpu::ctx(), symbols, symbol_size, range, prob_bits, output_bytes, cap, &n),
                   "encode_entropy"))
    return 0;
  return n;
}

inline size_t encode_entropy(uint8_t* symbols, size_t symbol_size, size_t range, uint8_t* output_bytes,
                             uint32_t prob_bits, uint8_t diagnostics) {
  std::vector<uint16_t> s(symbols, symbols + symbol_size);
  return encode_entropy(s.data(), symbol_size, range, output_bytes, prob_bits, diagnostics);
}
