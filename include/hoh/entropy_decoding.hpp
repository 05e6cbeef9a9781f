// Drop-in for the reference's entropy_decoding.hpp: decode_entropy_simple (:8-132),
// decode_entropy (:134-292) and decode_entropy_8bit (:294-314), same signatures, the symbols
// decoded on the GPU through libhohgpu.
//
// decode_entropy returns a new[]'d array of *symbol_size symbols (caller delete[]s it) and
// advances *byte_pointer past the whole stream (the reference leaves it after the frequency
// table; every caller in the reference that reads a second stream relies on the
// corrected behaviour).  Returns nullptr on a malformed / undecodable stream (the reference
// crashes or returns garbage there).  decode_entropy_8bit is the same with each symbol truncated
// to 8 bits (entropy_decoding.hpp:308-311).  decode_entropy_simple is the reference's diagnostic
// walk: it prints the stream header when `diagnostics` is set, sets *symbol_size and advances
// *byte_pointer past the stream (Q1 fixed as above), returning nothing.
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include "hoh_gpu.hpp"
// The reference header brings these in for its callers (entropy_decoding.hpp:4-6); keep that
// when this header stands in the reference tree.
#if __has_include("rans64.hpp") && __has_include("varint.hpp") && __has_include("stattools.hpp")
#include "rans64.hpp"
#include "varint.hpp"
#include "stattools.hpp"
#endif

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

inline uint8_t* decode_entropy_8bit(uint8_t* in_bytes, size_t in_size, size_t* byte_pointer, size_t* symbol_size,
                                    uint8_t diagnostics) {
  uint16_t* wide = decode_entropy(in_bytes, in_size, byte_pointer, symbol_size, diagnostics);
  if (!wide) return nullptr;
  uint8_t* out = new uint8_t[*symbol_size ? *symbol_size : 1];
  for (size_t i = 0; i < *symbol_size; i++) out[i] = (uint8_t)wide[i];
  delete[] wide;
  return out;
}

inline void decode_entropy_simple(uint8_t* in_bytes, size_t in_size, size_t* byte_pointer, size_t* symbol_size,
                                  uint8_t diagnostics) {
  hoh_entropy_header h{};
  if (!hoh_gpu::ok(hoh_entropy_parse(in_bytes, in_size, *byte_pointer, &h), "decode_entropy_simple")) {
    *symbol_size = 0;
    return;
  }
  *symbol_size = (size_t)h.count;
  if (diagnostics) {                                              // entropy_decoding.hpp:30-37
    std::printf("[SIMPLE]     entropy_mode       : %d\n", (int)h.entropy_mode);
    std::printf("[SIMPLE]     prob_bits          : %d\n", (int)h.prob_bits);
    std::printf("[SIMPLE]     table_storage_mode : %d\n", (int)h.table_mode);
    std::printf("[SIMPLE]     range              : %d\n", (int)h.range);
    std::printf("[SIMPLE]     bits per symbol    : %d\n", (int)h.symbol_bits);
    std::printf("[SIMPLE]     symbols            : %d\n\n", (int)h.count);
    if (h.entropy_mode) std::printf("[SIMPLE] entropy_size %d\n", (int)(h.table_end - *byte_pointer));
  }
  if (h.entropy_mode) std::printf("[SIMPLE] ---rANS size: %d\n", (int)h.payload_bytes);  // :117
  *byte_pointer = (size_t)h.stream_end;
}
