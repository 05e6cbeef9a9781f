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
  std::printf("drop-in headers ok: stream %zu B, layer %zu B\n", n, ln);
  return 0;
}
