// TEST/BENCH INFRASTRUCTURE ONLY: times the reference's own CPU functions, compiled in place
// from /root/reference, on a bounded sample of bench.py's workload (256x256 tiles of a raw
// RGB file).  Encode = encode_tile(-s0) per tile (the whole of choh's per-tile work,
// choh.cpp:104-383); decode = decode_entropy + unpredict_all per plane + inverse subtract-green
// (entropy_decoding.hpp:134, unprediction.hpp:6) -- dhoh itself cannot be timed: it crashes on
// every tiled file.  Prints one JSON line.  Single thread, like the reference; the
// optional 5th argument (first tile) lets bench.py run one process per core on disjoint tile
// ranges for the all-cores leg.  The decode gets each tile's real back-reference map (lz_backref
// below), so copied pixels decode as in dhoh.cpp:143-266 and the output is checked against the
// input (mismatch_excl_last_row: the reference's unpredict_all decodes the last row with the
// non-MED edge rule).  t_enc / t_dec cover encode_tile and the decode calls only: the
// LZ locate below (find_lz_rgb, which finds where the planes start because the reference's
// decode_entropy cannot skip a stream) is outside both clocks.  Only tiles whose
// encode AND decode were timed (sub-green tiles) count in raw_bytes / t_enc / t_dec.
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
#include <time.h>
#include <unistd.h>
#include <fcntl.h>
#define main choh_main
#include "choh.cpp"
#undef main
#include "entropy_decoding.hpp"
#include "unprediction.hpp"

static double now() { timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec + t.tv_nsec * 1e-9; }

// The per-pixel back distance map the reference's decoder feeds unpredict_all (LEMPEL_BACKREF,
// un_lz.hpp:150-170: 0 for predicted pixels, the copy's back distance for copied ones), rebuilt
// from the same greedy walk as find_lz_rgb (lz.hpp:32-95 at seek distance 6: backs 1..64, no
// vertical search), because the reference's own un_lz cannot read a tile's LZ streams back
// (SURVEY Q1).  Outside the clocks, like the plane locate.
static void lz_backref(const uint8_t* s, size_t size, int distance, int bonus, uint16_t* br) {
  const int lim = 1 << distance;
  for (size_t i = 0; i < size; i += 3) {
    int longest = 0, best = -1;
    for (int back = 1; back <= lim && (long)i - back * 3 >= 0; back++) {
      int off = 0;
      while (i + off * 3 + 2 < size && s[i + off * 3] == s[i - back * 3 + off * 3] &&
             s[i + off * 3 + 1] == s[i - back * 3 + off * 3 + 1] && s[i + off * 3 + 2] == s[i - back * 3 + off * 3 + 2] &&
             off < 259)
        off++;
      if (off > longest) { longest = off; best = back; if (off == 259) back = lim; }
    }
    if (longest < 4 + bonus) { br[i / 3] = 0; continue; }
    for (int k = 0; k < longest; k++) br[i / 3 + k] = (uint16_t)best;
    i += (size_t)(longest - 1) * 3;
  }
}

int main(int argc, char** argv) {
  if (argc < 5) { fprintf(stderr, "usage: ref_bench in.rgb W H max_tiles [first_tile]\n"); return 1; }
  int W = atoi(argv[2]), H = atoi(argv[3]), maxt = atoi(argv[4]);
  const int first = argc > 5 ? atoi(argv[5]) : 0;
  int xt = W / 256, yt = H / 256, tw = (W + xt - 1) / xt, th = (H + yt - 1) / yt;
  int nt = xt * yt - first < maxt ? xt * yt - first : maxt;
  if (nt < 0) nt = 0;
  // only the rows of this process's tiles are read (one process per core holds a band, not the
  // whole image)
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  const int r0 = nt ? (first / xt) * th : 0;
  const int r1 = nt ? ((first + nt - 1) / xt + 1) * th < H ? ((first + nt - 1) / xt + 1) * th : H : 0;
  const size_t rowb = (size_t)W * 3;
  uint8_t* band = new uint8_t[(size_t)(r1 - r0) * rowb + 1];
  if (fseek(f, (long)((size_t)r0 * rowb), SEEK_SET) != 0) return 2;
  if (fread(band, 1, (size_t)(r1 - r0) * rowb, f) != (size_t)(r1 - r0) * rowb) return 2;
  fclose(f);
  uint8_t* img = band - (size_t)r0 * rowb;          // indexed by absolute row below
  int saved = dup(1); int dn = open("/dev/null", O_WRONLY);
  double tenc = 0, tdec = 0;
  size_t raw = 0, comp = 0;
  long bad = 0;
  int ntimed = 0, skipped = 0;       // tiles not sub-green (grey / palette) have no timed decode
  for (int i = first; i < first + nt; i++) {
    int xo = (i % xt) * tw, yo = (i / xt) * th, nw = tw, nh = th;
    if (W - xo < nw) nw = W - xo;
    if (H - yo < nh) nh = H - yo;
    size_t np = (size_t)nw * nh;
    uint8_t* t = new uint8_t[np * 3];
    for (int y = 0; y < nh; y++) memcpy(t + (size_t)y * nw * 3, img + ((size_t)(y + yo) * W + xo) * 3, (size_t)nw * 3);
    uint8_t* out = new uint8_t[np * 6 + 4096];
    fflush(stdout); dup2(dn, 1);
    double a = now();
    size_t n = encode_tile(t, np * 3, out, nw, nh, 0);
    double b = now();
    // decode: locate the three planes (G, R-G, B-G) behind the LZ bytes and the varint offsets
    uint8_t* lzb = new uint8_t[np * 4 + 64];
    uint8_t* nuke = new uint8_t[np]; memset(nuke, 0, np);
    int cc = count_colours(t, np * 3), bonus = 0;
    if (cc != -1) { if (cc <= 4) bonus = 32; else if (cc <= 8) bonus = 20; else if (cc <= 16) bonus = 10; else if (cc <= 32) bonus = 2; }
    size_t lzn = find_lz_rgb(t, np * 3, nw, nh, lzb, nuke, 6, bonus);
    size_t q = 2 + 1 + lzn;
    bool timed = false;
    double c = now();
    if (out[2] == 128 && out[q] == 0x24) {
      q++;
      size_t o1 = read_varint(out, &q), o2 = read_varint(out, &q);
      size_t starts[3] = {q, q + o1, q + o1 + o2};
      int depth[3] = {8, 9, 9};
      uint16_t* planes[3];
      uint16_t* br = new uint16_t[np]; memset(br, 0, np * 2);
      const double c0 = now();
      lz_backref(t, np * 3, 6, bonus, br);
      c += now() - c0;                 // (kept out of the decode clock)
      for (int k = 0; k < 3; k++) {
        size_t bp = starts[k] + 5, cnt = 0;
        uint16_t* sym = decode_entropy(out, n, &bp, &cnt, 0);
        uint16_t tm = 0x0010;
        planes[k] = unpredict_all(sym, cnt, nw, nh, depth[k], 1, 1, &tm, br);
        delete[] sym;
      }
      uint8_t* rgb = new uint8_t[np * 3];
      for (size_t j = 0; j < np; j++) {
        rgb[3 * j + 1] = (uint8_t)planes[0][j];
        rgb[3 * j] = (uint8_t)(planes[1][j] + planes[0][j] - 256);
        rgb[3 * j + 2] = (uint8_t)(planes[2][j] + planes[0][j] - 256);
      }
      double d = now();
      tdec += d - c;
      timed = true;
      // the reference decoder mis-decodes the last row; count the rest
      for (size_t j = 0; j < (size_t)nw * (nh - 1) * 3; j++) bad += rgb[j] != t[j];
      delete[] rgb; delete[] br;
      for (int k = 0; k < 3; k++) delete[] planes[k];
    }
    fflush(stdout); dup2(saved, 1);
    if (timed) {                 // a tile counts only when both its encode and its decode were timed
      tenc += b - a;
      raw += np * 3; comp += n;
      ntimed++;
    } else {
      skipped++;
    }
    delete[] t; delete[] out; delete[] lzb; delete[] nuke;
  }
  printf("{\"tiles\": %d, \"tiles_skipped\": %d, \"raw_bytes\": %zu, \"comp_bytes\": %zu, \"t_enc\": %.6f, \"t_dec\": %.6f, "
         "\"enc_MBps\": %.3f, \"dec_MBps\": %.3f, \"encdec_MBps\": %.3f, \"mismatch_excl_last_row\": %ld}\n",
         ntimed, skipped, raw, comp, tenc, tdec, raw / tenc / 1e6, raw / tdec / 1e6, raw / (tenc + tdec) / 1e6, bad);
  return 0;
}
