// Compile check + GPU round trip of the drop-in headers: the reference's call surface
// (encode_entropy / decode_entropy / layer_encode / decode_layer / channelpredict_fastpath /
// unpredict_all) exactly as its callers spell it, here served by libhohgpu.
#include <cstdio>
#include <cstring>
#include <vector>
#include "../../include/hoh/entropy_encoding.hpp"
#include "../../include/hoh/entropy_decoding.hpp"
#include "../../include/hoh/layer_encode.hpp"
#include "../../include/hoh/layer_decode.hpp"
#include "../../include/hoh/prediction.hpp"
#include "../../include/hoh/unprediction.hpp"

int main() {
  const int w = 300, h = 200;
  std::vector<uint16_t> plane((size_t)w * h);
  uint32_t s = 12345;
  for (size_t i = 0; i < plane.size(); i++) {
    s = s * 1103515245u + 12345u;
    plane[i] = (uint16_t)(((i % w) + (i / w) / 3 + ((s >> 16) & 3)) & 255);
  }
  // entropy stream round trip
  std::vector<uint16_t> sym(plane.begin(), plane.begin() + 5000);
  std::vector<uint8_t> buf(hoh_entropy_bound(sym.size(), 256, 15));
  const size_t n = encode_entropy(sym.data(), sym.size(), 256, buf.data(), 15, 0);
  size_t bp = 0, cnt = 0;
  uint16_t* back = decode_entropy(buf.data(), n, &bp, &cnt, 0);
  if (!n || !back || cnt != sym.size() || bp != n || std::memcmp(back, sym.data(), cnt * 2)) {
    std::printf("entropy round trip FAILED\n");
    return 1;
  }
  delete[] back;
  // two streams back to back through decode_entropy_8bit / decode_entropy_simple
  // (simple_entropy_decoder.cpp:28, un_lz.hpp:30-139: each call must leave *byte_pointer at the next stream)
  std::vector<uint8_t> sym8(3000);
  for (size_t i = 0; i < sym8.size(); i++) sym8[i] = (uint8_t)((i * 7 + (i >> 4)) % 40);
  std::vector<uint8_t> two(2 * hoh_entropy_bound(sym8.size(), 256, 15));
  const size_t n1 = encode_entropy(sym8.data(), sym8.size(), 256, two.data(), 15, 0);
  const size_t n2 = encode_entropy(sym.data(), 700, 256, two.data() + n1, 15, 0);
  bp = 0;
  uint8_t* b8 = decode_entropy_8bit(two.data(), n1 + n2, &bp, &cnt, 0);
  if (!n1 || !n2 || !b8 || cnt != sym8.size() || bp != n1 || std::memcmp(b8, sym8.data(), cnt)) {
    std::printf("decode_entropy_8bit FAILED\n");
    return 1;
  }
  delete[] b8;
  size_t c2 = 0;
  decode_entropy_simple(two.data(), n1 + n2, &bp, &c2, 1);
  if (bp != n1 + n2 || c2 != 700) { std::printf("decode_entropy_simple FAILED (%zu %zu)\n", bp, c2); return 1; }
  bp = 0;
  decode_entropy_simple(two.data(), n1 + n2, &bp, &c2, 0);
  if (bp != n1 || c2 != sym8.size()) { std::printf("decode_entropy_simple FAILED\n"); return 1; }
  // predictor round trip
  size_t bs = 0;
  uint16_t* res = channelpredict_fastpath(plane.data(), plane.size(), w, h, 8, &bs);
  uint16_t tmap[1] = {0x0010};
  uint16_t* un = unpredict_all(res, bs, w, h, 8, 1, 1, tmap, nullptr);
  if (!res || !un || std::memcmp(un, plane.data(), plane.size() * 2)) { std::printf("predictor round trip FAILED\n"); return 1; }
  delete[] res;
  delete[] un;
  // layer round trip
  std::vector<uint8_t> lay(((size_t)8 * plane.size() + 8 * plane.size() % 8 + 1024) / 8 + 4096);
  const size_t ln = layer_encode(plane.data(), plane.size(), w, h, 8, 0, nullptr, lay.data());
  uint8_t* dec = decode_layer(lay.data(), ln, 0, w, h, 8, nullptr);
  if (!ln || !dec) { std::printf("layer round trip FAILED\n"); return 1; }
  for (size_t i = 0; i < plane.size(); i++)
    if (dec[i] != (uint8_t)plane[i]) { std::printf("layer round trip FAILED at %zu\n", i); return 1; }
  delete[] dec;
  decode_layer_simple(lay.data(), ln, 0, w, h, 8);
  std::printf("drop-in headers ok: stream %zu B, layer %zu B\n", n, ln);
  return 0;
}
