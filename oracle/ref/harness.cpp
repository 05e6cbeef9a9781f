// TEST INFRASTRUCTURE ONLY.  Compiles the reference's own headers, in place under
// $(REF) (= /root/reference), into oracle/_ref/libref.so so tests can call the reference
// functions directly and generate golden vectors.  No reference source is copied here:
// this file only #includes it.  Built by oracle/ref/Makefile.
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <unistd.h>
#include <fcntl.h>

#define main choh_main
#include "choh.cpp"            // encode_tile, count_colours, palette_encode (+ all encoder headers)
#undef main
#include "entropy_decoding.hpp"
#include "unprediction.hpp"

// silence the reference's unconditional printf()s (entropy_decoding.hpp:257, lz, ...)
struct Quiet {
  int saved;
  Quiet() { fflush(stdout); saved = dup(1); int dn = open("/dev/null", O_WRONLY); dup2(dn, 1); close(dn); }
  ~Quiet() { fflush(stdout); dup2(saved, 1); close(saved); }
};

extern "C" {

size_t ref_encode_entropy(const uint16_t* sym, size_t n, size_t range, uint32_t pb, uint8_t* out) {
  uint16_t* s = new uint16_t[n ? n : 1];
  memcpy(s, sym, n * 2);
  size_t r = encode_entropy(s, n, range, out, pb, 0);            // entropy_encoding.hpp:8
  delete[] s;
  return r;
}

void ref_normalize_freqs(uint32_t* freqs, uint32_t* cum, size_t size, uint32_t target) {
  normalize_freqs(freqs, cum, size, target);                      // stattools.hpp:13
}

void ref_esym_init(uint32_t start, uint32_t freq, uint32_t pb, uint64_t* rcp, uint32_t* bias,
                   uint32_t* cmpl, uint32_t* shift) {
  Rans64EncSymbol s;
  Rans64EncSymbolInit(&s, start, freq, pb);                        // rans64.hpp:167
  *rcp = s.rcp_freq; *bias = s.bias; *cmpl = s.cmpl_freq; *shift = s.rcp_shift;
}

// one Rans64EncPutSymbol step (rans64.hpp:262): returns the new state, *emitted = word or -1
uint64_t ref_enc_put(uint64_t x, uint32_t start, uint32_t freq, uint32_t pb, int64_t* emitted) {
  Rans64EncSymbol s;
  Rans64EncSymbolInit(&s, start, freq, pb);
  uint32_t buf[2];
  uint32_t* p = buf + 1;
  Rans64State r = x;
  Rans64EncPutSymbol(&r, &p, &s, pb);
  *emitted = (p == buf + 1) ? -1 : (int64_t)buf[0];
  return r;
}

// decode_entropy (entropy_decoding.hpp:134); returns the count, symbols into out (cap)
size_t ref_decode_entropy(const uint8_t* in, size_t in_size, size_t bp, uint16_t* out, size_t cap) {
  Quiet q;
  size_t n = 0;
  uint16_t* d = decode_entropy((uint8_t*)in, in_size, &bp, &n, 0);
  if (n <= cap) memcpy(out, d, n * 2);
  delete[] d;
  return n;
}

void ref_channelpredict_fastpath(const uint16_t* data, int w, int h, int depth, uint16_t* out) {
  size_t bs;
  uint16_t* r = channelpredict_fastpath((uint16_t*)data, (size_t)w * h, w, h, depth, &bs);  // prediction.hpp:6
  memcpy(out, r, (size_t)w * h * 2);
  delete[] r;
}

void ref_unpredict_all(const uint16_t* res, int w, int h, int depth, uint16_t predictor,
                       const uint16_t* backref, uint16_t* out) {
  uint16_t tm = predictor;
  uint16_t* r = unpredict_all((uint16_t*)res, (size_t)w * h, w, h, depth, 1, 1, &tm,
                              (uint16_t*)backref);                // unprediction.hpp:6
  memcpy(out, r, (size_t)w * h * 2);
  delete[] r;
}

size_t ref_channelpredict_section(const uint16_t* data, int w, int h, int depth, int xt, int yt, int cx,
                                  int cy, uint16_t mask, uint16_t* out) {
  size_t bs = 0;
  uint16_t* r = channelpredict_section((uint16_t*)data, (size_t)w * h, w, h, depth, xt, yt, cx, cy, mask,
                                       &bs);                     // prediction.hpp:46
  memcpy(out, r, bs * 2);
  delete[] r;
  return bs;
}

void ref_channelpredict_all(const uint16_t* data, int w, int h, int depth, int xt, int yt,
                            const uint16_t* tile_map, uint16_t* out) {
  uint16_t* r = channelpredict_all((uint16_t*)data, (size_t)w * h, w, h, depth, xt, yt,
                                   (uint16_t*)tile_map);          // prediction.hpp:153
  memcpy(out, r, (size_t)w * h * 2);
  delete[] r;
}

void ref_unpredict_map(const uint16_t* res, int w, int h, int depth, int xt, int yt, const uint16_t* tile_map,
                       const uint16_t* backref, uint16_t* out) {
  uint16_t* r = unpredict_all((uint16_t*)res, (size_t)w * h, w, h, depth, xt, yt, (uint16_t*)tile_map,
                              (uint16_t*)backref);                // unprediction.hpp:6
  memcpy(out, r, (size_t)w * h * 2);
  delete[] r;
}

void ref_subtract_green(const uint8_t* rgb, size_t npix, uint16_t* G, uint16_t* R, uint16_t* B) {
  subtract_green((uint8_t*)rgb, npix * 3, G, R, B);                // channel.hpp:73
}

int ref_count_colours(const uint8_t* rgb, size_t size) { return count_colours((uint8_t*)rgb, size); }

size_t ref_find_lz_rgb(const uint8_t* rgb, size_t size, int w, int h, uint8_t* lz, uint8_t* nuke,
                       int distance, int bonus) {
  return find_lz_rgb((uint8_t*)rgb, size, w, h, lz, nuke, distance, bonus);   // lz.hpp:6
}

size_t ref_layer_encode(const uint16_t* data, size_t n, int w, int h, int depth, size_t cruncher,
                        const uint8_t* nuke, uint8_t* out) {
  uint16_t* d = new uint16_t[n];
  memcpy(d, data, n * 2);
  size_t r = layer_encode(d, n, w, h, depth, cruncher, (uint8_t*)nuke, out);   // layer_encode.hpp:11
  delete[] d;
  return r;
}

size_t ref_encode_tile(const uint8_t* rgb, int w, int h, size_t cruncher, uint8_t* out) {
  size_t n = (size_t)w * h * 3;
  uint8_t* in = new uint8_t[n];
  memcpy(in, rgb, n);
  size_t r = encode_tile(in, n, out, w, h, cruncher);              // choh.cpp:104
  delete[] in;
  return r;
}

}  // extern "C"
