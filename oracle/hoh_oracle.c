/*
 * hoh_oracle.c -- TEST INFRASTRUCTURE ONLY (see hoh_oracle.h).
 *
 * CPU restatement of the hoh-ANS encode path (-s0 and the -s1..-s4 predictor search) and a
 * corrected decoder.  Written from the
 * reference's documented behaviour -- the reference's integer promotion
 * rules are reproduced explicitly where they change bytes (entropy_encoding.hpp:48,121).
 * Build: gcc -O2 -shared -fPIC -o oracle/liboracle.so oracle/hoh_oracle.c -lm
 * (glibc log2 and IEEE double sums in the reference's order: the -s>=1 cost estimate matches the
 * reference's selection bit for bit)
 */
#include "hoh_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ varint / bit stuffer */

/* varint.hpp:29-45: 1..3 bytes, high bit = continuation; values >= 2^21 write NOTHING (Q2) */
size_t or_write_varint(uint8_t* b, size_t loc, size_t v) {
  if (v < (1u << 7)) {
    b[loc++] = (uint8_t)v;
  } else if (v < (1u << 14)) {
    b[loc++] = (uint8_t)((v >> 7) + 128);
    b[loc++] = (uint8_t)(v % 128);
  } else if (v < (1u << 21)) {
    b[loc++] = (uint8_t)((v >> 14) + 128);
    b[loc++] = (uint8_t)(((v >> 7) % 128) + 128);
    b[loc++] = (uint8_t)(v % 128);
  }
  return loc;
}

/* varint.hpp:6-27: at most three bytes; the third byte is taken whole */
size_t or_read_varint(const uint8_t* b, size_t* loc) {
  size_t b0 = b[(*loc)++];
  if (!(b0 & 0x80)) return b0;
  size_t b1 = b[(*loc)++];
  if (!(b1 & 0x80)) return ((b0 & 0x7f) << 7) + b1;
  size_t b2 = b[(*loc)++];
  return ((b0 & 0x7f) << 14) + ((b1 & 0x7f) << 7) + b2;
}

typedef struct { uint8_t rem; uint8_t br; } bitsink;

/* varint.hpp:47-77 (stuffer).  MSB-first packer; a value wider than `bits` is NOT masked: its
 * excess bits are added into the pending byte, exactly as the uint8 arithmetic
 * of the reference does. */
static void stuff(uint8_t* b, size_t* loc, bitsink* s, uint32_t value, unsigned bits) {
  if (bits < s->br) {
    s->rem = (uint8_t)(s->rem + (uint8_t)(value << (s->br - bits)));
    s->br = (uint8_t)(s->br - bits);
  } else if (bits == s->br) {
    b[(*loc)++] = (uint8_t)(s->rem + (uint8_t)value);
    s->rem = 0;
    s->br = 8;
  } else {
    if (bits > 8) {
      uint32_t top = value >> 8, bottom = value % 256;
      stuff(b, loc, s, top, bits - 8);
      stuff(b, loc, s, bottom, 8);
    } else {
      b[(*loc)++] = (uint8_t)(s->rem + (uint8_t)(value >> (bits - s->br)));
      s->br = (uint8_t)(8 - (bits - s->br));
      s->rem = (uint8_t)((value << s->br) % 256);
    }
  }
}

typedef struct { uint8_t slag; uint8_t bits; } bitsrc;

/* varint.hpp:79-106 (unstuffer) */
static uint32_t unstuff(const uint8_t* b, size_t* loc, bitsrc* s, unsigned bits) {
  uint32_t value = 0;
  while (bits > s->bits) {
    bits -= s->bits;
    value += (uint32_t)s->slag << bits;
    s->slag = b[(*loc)++];
    s->bits = 8;
  }
  s->bits = (uint8_t)(s->bits - bits);
  value += (uint32_t)(s->slag >> s->bits);
  s->slag = (uint8_t)(s->slag % (1u << s->bits));
  return value;
}

/* ------------------------------------------------------------------ stattools */

/* stattools.hpp:13-70.  The two live assert()s of the reference become OR_E_ASSERT. */
int or_normalize_freqs(uint32_t* freqs, uint32_t* cum, size_t size, uint32_t target) {
  if (target < size) return OR_E_ASSERT;                       /* :14 */
  cum[0] = 0;
  for (size_t i = 0; i < size; i++) cum[i + 1] = cum[i] + freqs[i];   /* :6-11 */
  uint32_t total = cum[size];
  if (total == 0) return OR_E_ASSERT;                          /* division by zero */
  for (size_t i = 1; i <= size; i++) cum[i] = (uint32_t)(((uint64_t)target * cum[i]) / total);
  for (size_t i = 0; i < size; i++) {
    if (freqs[i] && cum[i + 1] == cum[i]) {
      /* steal from the first strictly-smallest frequency > 1 (:33-40) */
      uint32_t best_freq = ~0u;
      long best = -1;
      for (size_t j = 0; j < size; j++) {
        uint32_t f = cum[j + 1] - cum[j];
        if (f > 1 && f < best_freq) { best_freq = f; best = (long)j; }
      }
      if (best < 0) return OR_E_ASSERT;                        /* :42 */
      if (best < (long)i) {
        for (size_t j = (size_t)best + 1; j <= i; j++) cum[j]--;
      } else {
        for (size_t j = i + 1; j <= (size_t)best; j++) cum[j]++;
      }
    }
  }
  for (size_t i = 0; i < size; i++) freqs[i] = cum[i + 1] - cum[i];
  return OR_OK;
}

/* ------------------------------------------------------------------ rans64 */

/* rans64.hpp:167-247: Alverson reciprocal, freq < 2 special case */
void or_esym_init(or_esym* s, uint32_t start, uint32_t freq, uint32_t sb) {
  s->freq = freq;
  s->cmpl_freq = (uint32_t)((1u << sb) - freq);
  if (freq < 2) {
    s->rcp_freq = ~0ull;
    s->rcp_shift = 0;
    s->bias = start + (1u << sb) - 1;
  } else {
    uint32_t shift = 0;
    while (freq > (1u << shift)) shift++;
    uint64_t x0 = freq - 1, x1 = 1ull << (shift + 31);
    uint64_t t1 = x1 / freq;
    x0 += (x1 % freq) << 32;
    uint64_t t0 = x0 / freq;
    s->rcp_freq = t0 + (t1 << 32);
    s->rcp_shift = shift - 1;
    s->bias = start;
  }
}

/* rans64.hpp:262-278 */
static inline void esym_put(uint64_t* r, uint32_t** pp, const or_esym* s, uint32_t sb) {
  uint64_t x = *r;
  uint64_t x_max = ((((uint64_t)1 << 31) >> sb) << 32) * s->freq;
  if (x >= x_max) {
    *pp -= 1;
    **pp = (uint32_t)x;
    x >>= 32;
  }
  uint64_t q = (uint64_t)(((unsigned __int128)x * s->rcp_freq) >> 64) >> s->rcp_shift;
  *r = x + s->bias + q * s->cmpl_freq;
}

/* ------------------------------------------------------------------ entropy stream */

static unsigned bitlen(size_t v) { unsigned b = 0; for (; v; v >>= 1) b++; return b; }

size_t or_entropy_bound(size_t n, size_t range, uint32_t pb) {
  size_t table = (2 * 8 * 17 + (size_t)range * (pb > 16 ? pb : 16) + 7) / 8 + 16;
  return 16 + table + 4 * (n + 2) + (bitlen(range) * n + 7) / 8;
}

/* entropy_encoding.hpp:8-280 */
long or_encode_entropy(const uint16_t* sym, size_t n, size_t range, uint32_t pb, uint8_t* out) {
  size_t es = 0;
  if (range == 0) return OR_E_ARG;
  if (n == 0) {                                                     /* :19-23 */
    es = or_write_varint(out, es, range - 1);
    es = or_write_varint(out, es, n);
    return (long)es;
  }
  if (pb == 0 || pb > 31) return OR_E_ARG;
  unsigned maxbits = bitlen(range - 1);                             /* :24-27 */
  uint32_t* freqs = (uint32_t*)calloc(range, 4);
  uint32_t* cum = (uint32_t*)calloc(range + 1, 4);
  long ret = OR_OK;
  for (size_t i = 0; i < n; i++) {
    if (sym[i] >= range) { ret = OR_E_ARG; goto done; }          /* out-of-bounds in the reference */
    freqs[sym[i]]++;
  }
  if ((ret = or_normalize_freqs(freqs, cum, range, 1u << pb)) != OR_OK) goto done;
  es = or_write_varint(out, es, range - 1);                         /* :43-44 */
  es = or_write_varint(out, es, n);
  size_t expected_stored = es + 1 + (maxbits * n + 8 - 1) / 8;     /* :45 */
  size_t expected_raw = (pb * range + 8 - 1) / 8;                  /* :47 */
  /* :48 -- int * unsigned int, i.e. 32-bit unsigned arithmetic, then widened */
  uint32_t cn32 = (pb - 1) / 4 + 2;
  size_t expected_clamped = (size_t)(uint32_t)((uint32_t)(2 * ((int)maxbits - 1)) * cn32);
  expected_clamped += (size_t)(pb * 2);                            /* :49 */
  unsigned clamp_number = (uint8_t)cn32;                            /* :51 */
  uint16_t lower[40], upper[40];
  if (clamp_number > 40) { ret = OR_E_ARG; goto done; }
  size_t size_bits = 0, climb = 0, lci = 0;
  for (; climb < range; climb++) {                                  /* :59-83 */
    while (freqs[climb] >= (size_t)(1u << size_bits)) {
      size_t idx;
      if (size_bits == 0) { size_bits = 1; idx = 0; lci = 1; }
      else if (size_bits == 1) { size_bits = 4; idx = 1; lci = 2; }
      else { idx = size_bits / 4 + 1; size_bits += 4; lci++; }
      /* single-symbol streams at prob_bits 8/12/16 write one element past the clamp array
       * (:72); that element is never read again -- checked against the compiled reference
       * (tests/test_oracle_vs_reference.py::test_single_symbol_overrun) -- so it is dropped */
      if (idx < clamp_number) lower[idx] = (uint16_t)climb;
    }
    if (size_bits >= pb) { size_bits = pb; expected_clamped += size_bits; break; }
    expected_clamped += size_bits;
  }
  while (lci < clamp_number) lower[lci++] = (uint16_t)(range - 1);  /* :84-86 */
  size_bits = 0;
  size_t climb2 = range - 1, uci = 0;
  for (;; climb2--) {                                               /* :90-117 */
    while (freqs[climb2] >= (size_t)(1u << size_bits)) {
      size_t idx;
      if (size_bits == 0) { size_bits = 1; idx = 0; uci = 1; }
      else if (size_bits == 1) { size_bits = 4; idx = 1; uci = 2; }
      else { idx = size_bits / 4 + 1; size_bits += 4; uci++; }
      if (idx < clamp_number) upper[idx] = (uint16_t)climb2;         /* (:103, as above) */
    }
    if (size_bits >= pb) { size_bits = pb; expected_clamped += size_bits; break; }
    expected_clamped += size_bits;
    if (climb2 == 0) break;
  }
  while (uci < clamp_number) upper[uci++] = 0;                      /* :118-120 */
  expected_clamped += size_bits * (climb2 - climb - 1);             /* :121 -- size_t wrap (Q5) */
  expected_clamped = (expected_clamped + 8 - 1) / 8;

  if (expected_raw < expected_clamped) {                            /* :135-147 raw table */
    out[es++] = (uint8_t)((1u << 7) + (pb << 2) + 1);
    bitsink s = {0, 8};
    for (size_t i = 0; i < range; i++) stuff(out, &es, &s, freqs[i], maxbits);
    if (s.br != 8) out[es++] = s.rem;
  } else {                                                          /* :148-200 clamped table */
    out[es++] = (uint8_t)((1u << 7) + (pb << 2) + 2);
    bitsink s = {0, 8};
    for (unsigned i = 0; i < clamp_number; i++) {
      stuff(out, &es, &s, lower[i], maxbits);
      stuff(out, &es, &s, upper[i], maxbits);
    }
    for (size_t i = 0; i < range; i++) {
      unsigned sbits = 0;
      if (lower[0] <= i && upper[0] >= i) sbits = 1;
      if (lower[1] <= i && upper[1] >= i) sbits = 4;
      for (unsigned j = 2; j < clamp_number; j++)
        if (lower[j] <= i && upper[j] >= i) sbits = 4 * j;
      if (sbits > pb) sbits = pb;
      stuff(out, &es, &s, freqs[i], sbits);
    }
    if (s.br != 8) out[es++] = s.rem;
  }
  {                                                                 /* :206-238 rANS */
    or_esym* es_tab = (or_esym*)malloc(range * sizeof(or_esym));
    for (size_t i = 0; i < range; i++) or_esym_init(&es_tab[i], cum[i], freqs[i], pb);
    uint32_t* buf = (uint32_t*)malloc((n + 2) * 4);
    uint32_t* end = buf + n + 2;
    uint32_t* p = end;
    uint64_t x = 1ull << 31;                                        /* Rans64EncInit */
    for (size_t i = n; i > 0; i--) esym_put(&x, &p, &es_tab[sym[i - 1]], pb);
    p -= 2;                                                         /* Rans64EncFlush */
    p[0] = (uint32_t)x;
    p[1] = (uint32_t)(x >> 32);
    size_t words = (size_t)(end - p);
    es = or_write_varint(out, es, words * 4);
    for (size_t k = 0; k < words; k++) {                           /* little-endian words */
      uint32_t w = p[k];
      out[es++] = (uint8_t)w; out[es++] = (uint8_t)(w >> 8);
      out[es++] = (uint8_t)(w >> 16); out[es++] = (uint8_t)(w >> 24);
    }
    free(buf);
    free(es_tab);
  }
  if (expected_stored < es) {                                       /* :244-267 stored */
    es = 0;
    es = or_write_varint(out, es, range - 1);
    es = or_write_varint(out, es, n);
    out[es++] = 0;
    bitsink s = {0, 8};
    for (size_t i = 0; i < n; i++) stuff(out, &es, &s, sym[i], maxbits);
    if (s.br != 8) out[es++] = s.rem;
  }
  ret = (long)es;
done:
  free(freqs);
  free(cum);
  return ret;
}

long or_peek_count(const uint8_t* in, size_t in_size, size_t bp) {
  if (bp + 2 > in_size) return OR_E_CORRUPT;
  (void)or_read_varint(in, &bp);
  return (long)or_read_varint(in, &bp);
}

/* Inverse of or_encode_entropy (entropy_decoding.hpp:134-292 semantics, with the payload skip
 * of Q1 fixed and the single-symbol table of Q6 recognised: lower[0] == upper[0]). */
long or_decode_entropy(const uint8_t* in, size_t in_size, size_t* bp, uint16_t* out, size_t cap) {
  size_t p = *bp;
  if (p + 2 > in_size) return OR_E_CORRUPT;
  size_t range = or_read_varint(in, &p) + 1;
  size_t n = or_read_varint(in, &p);
  if (n > cap) return OR_E_CAP;
  if (n == 0) { *bp = p; return 0; }
  if (p >= in_size) return OR_E_CORRUPT;
  unsigned maxbits = bitlen(range - 1);
  uint8_t meta = in[p++];
  unsigned mode = meta >> 7, pb = (meta & 0x3c) >> 2, tsm = meta & 3;
  if (!mode) {                                                      /* stored */
    bitsrc s = {0, 0};
    if (p + (maxbits * n + 7) / 8 > in_size) return OR_E_CORRUPT;
    for (size_t i = 0; i < n; i++) out[i] = (uint16_t)unstuff(in, &p, &s, maxbits);
    *bp = p;
    return (long)n;
  }
  if (pb == 0 || range > (1u << 20)) return OR_E_CORRUPT;
  uint32_t* freqs = (uint32_t*)calloc(range, 4);
  uint32_t* cum = (uint32_t*)calloc(range + 1, 4);
  long ret = OR_E_CORRUPT;
  bitsrc s = {0, 0};
  if (tsm == 1) {
    for (size_t i = 0; i < range; i++) freqs[i] = unstuff(in, &p, &s, maxbits);
  } else if (tsm == 2) {
    unsigned cn = (pb - 1) / 4 + 2;
    uint32_t lower[8], upper[8];
    for (unsigned i = 0; i < cn; i++) {
      lower[i] = unstuff(in, &p, &s, maxbits);
      upper[i] = unstuff(in, &p, &s, maxbits);
    }
    if (lower[0] == upper[0] && lower[0] < range) {
      /* single-symbol stream: freq = 2^pb overflowed its field (Q6); skip the field the
       * encoder wrote and restore the frequency */
      size_t sym0 = lower[0];
      unsigned sbits = cn >= 3 ? 4 * (cn - 1) : 4;
      if (sbits > pb) sbits = pb;
      (void)unstuff(in, &p, &s, sbits);
      freqs[sym0] = 1u << pb;
    } else {
      for (size_t i = 0; i < range; i++) {
        unsigned sbits = 0;
        if (lower[0] <= i && upper[0] >= i) sbits = 1;
        if (lower[1] <= i && upper[1] >= i) sbits = 4;
        for (unsigned j = 2; j < cn; j++)
          if (lower[j] <= i && upper[j] >= i) sbits = 4 * j;
        if (sbits > pb) sbits = pb;
        freqs[i] = unstuff(in, &p, &s, sbits);
      }
    }
  } else {
    ret = OR_E_UNSUPPORTED;
    goto done;
  }
  cum[0] = 0;
  for (size_t i = 0; i < range; i++) cum[i + 1] = cum[i] + freqs[i];
  if (cum[range] != (1u << pb)) goto done;                          /* undecodable table (Q4) */
  {
    size_t data = or_read_varint(in, &p);
    if (data < 8 || (data & 3) || p + data > in_size) goto done;
    const uint8_t* w = in + p;
    size_t nw = data / 4, wi = 0;
#define RDW(k) ((uint32_t)w[4 * (k)] | ((uint32_t)w[4 * (k) + 1] << 8) | ((uint32_t)w[4 * (k) + 2] << 16) | ((uint32_t)w[4 * (k) + 3] << 24))
    uint64_t x = (uint64_t)RDW(0) | ((uint64_t)RDW(1) << 32);      /* Rans64DecInit */
    wi = 2;
    uint32_t mask = (1u << pb) - 1;
    for (size_t i = 0; i < n; i++) {
      uint32_t slot = (uint32_t)(x & mask);
      size_t lo = 0, hi = range;                                    /* cum[lo] <= slot < cum[hi] */
      while (hi - lo > 1) { size_t mid = (lo + hi) / 2; if (cum[mid] <= slot) lo = mid; else hi = mid; }
      out[i] = (uint16_t)lo;
      x = (uint64_t)freqs[lo] * (x >> pb) + slot - cum[lo];         /* Rans64DecAdvance */
      if (x < (1ull << 31)) {
        if (wi >= nw) goto done;
        x = (x << 32) | RDW(wi);
        wi++;
      }
    }
#undef RDW
    if (x != (1ull << 31) || wi != nw) goto done;                   /* must end at EncInit state */
    p += data;                                                      /* Q1 fix */
  }
  *bp = p;
  ret = (long)n;
done:
  free(freqs);
  free(cum);
  return ret;
}

/* ------------------------------------------------------------------ predictor */

/* predictor_operations.hpp:37-60 (the uint16_t overload is the one selected, Q8) */
static inline uint16_t med16(uint16_t a, uint16_t b, uint16_t c) {
  if (a > b) {
    if (b > c) return b;
    else if (c > a) return a;
    else return c;
  } else {
    if (b < c) return b;
    else if (c > a) return c;
    else return a;
  }
}

/* prediction.hpp:6-44 */
void or_predict_fastpath(const uint16_t* d, int w, int h, int depth, uint16_t* res) {
  int c = 1 << depth, half = c / 2;
  for (int y = 0; y < h; y++) {
    for (int x = 0; x < w; x++) {
      uint16_t L = x ? d[y * w + x - 1] : (uint16_t)half;
      uint16_t T = y ? d[(y - 1) * w + x] : (uint16_t)half;
      uint16_t TL = (x && y) ? d[(y - 1) * w + x - 1] : (uint16_t)half;
      uint16_t p = med16(T, L, (uint16_t)(T + L - TL));
      res[y * w + x] = (uint16_t)(((int)d[y * w + x] - (int)p + half + c) % c);
    }
  }
}

long or_unpredict_fastpath(const uint16_t* res, size_t nres, const uint16_t* backref, int w, int h,
                           int depth, uint16_t* o) {
  int c = 1 << depth, half = c / 2;
  size_t k = 0;
  for (int y = 0; y < h; y++) {
    for (int x = 0; x < w; x++) {
      size_t i = (size_t)y * w + x;
      if (backref && backref[i]) {
        if (backref[i] > i) return OR_E_CORRUPT;
        o[i] = o[i - backref[i]];
        continue;
      }
      if (k >= nres) return OR_E_CORRUPT;
      uint16_t L = x ? o[i - 1] : (uint16_t)half;
      uint16_t T = y ? o[i - w] : (uint16_t)half;
      uint16_t TL = (x && y) ? o[i - w - 1] : (uint16_t)half;
      uint16_t p = med16(T, L, (uint16_t)(T + L - TL));
      o[i] = (uint16_t)(((int)res[k++] + (int)p - half + c) % c);
    }
  }
  return (long)k;
}

/* predictor_operations.hpp:8-10, 66-68, 89-106 (uint16_t overloads) */
static inline uint16_t midp16(uint16_t a, uint16_t b) { return (uint16_t)((int)a + ((int)b - (int)a) / 2); }
static inline uint16_t avg3(uint16_t a, uint16_t b, uint16_t c) { return (uint16_t)(((int)a + (int)b + (int)c) / 3); }
static inline uint16_t paeth16(uint16_t A, uint16_t B, uint16_t C) {
  int p = (int)A + (int)B - (int)C;
  int Ap = abs((int)A - p), Bp = abs((int)B - p), Cp = abs((int)C - p);
  if (Ap < Bp) return Ap < Cp ? A : C;
  return Bp < Cp ? B : C;
}

/* the 16 stock predictions (prediction.hpp:116-133 / :190-207; `all` passes paeth(L, TL, T)) */
static void preds16(uint16_t L, uint16_t T, uint16_t TL, uint16_t TR, int all, uint16_t* p) {
  p[0] = L; p[1] = T; p[2] = TL; p[3] = TR;
  p[4] = med16(T, L, (uint16_t)(T + L - TL));
  p[5] = midp16(L, T); p[6] = midp16(L, TL); p[7] = midp16(TL, T); p[8] = midp16(T, TR);
  p[9] = all ? paeth16(L, TL, T) : paeth16(L, T, TL);
  p[10] = avg3(L, L, TL); p[11] = avg3(L, TL, TL); p[12] = avg3(TL, TL, T);
  p[13] = avg3(TL, T, T); p[14] = avg3(T, T, TR); p[15] = avg3(T, TR, TR);
}

/* argmin_j |v - p[j]| over the masked predictors, first minimum (prediction.hpp:138-146) */
static inline int best_pred(uint16_t v, const uint16_t* p, uint16_t mask, int c) {
  int bv = 2 * c, b = 0;
  for (int j = 0; j < 16; j++) {
    int d = abs((int)v - (int)p[j]);
    if (d < bv && (mask & (1u << j))) { bv = d; b = j; }
  }
  return b;
}

/* prediction.hpp:46-151 (channelpredict_section): residuals of cell (cx, cy) of an xt x yt grid in
 * raster order within the cell; returns the count.  Reproduces the cell-local top row (read from
 * the row above the cell, wrapping into the cell's own row past the right edge), the TR wrap to
 * top_row[0] and best_pred reset to 4 per cell. */
size_t or_predict_section(const uint16_t* d, int w, int h, int depth, int xt, int yt, int cx, int cy,
                          uint16_t mask, uint16_t* out) {
  if (mask == 0x0010 && xt == 1 && yt == 1 && cx == 0 && cy == 0) {
    or_predict_fastpath(d, w, h, depth, out);
    return (size_t)w * h;
  }
  int c = 1 << depth, half = c / 2;
  int tw = (w + xt - 1) / xt, th = (h + yt - 1) / yt;
  int x0 = cx * tw, y0 = cy * th;
  int* bp = (int*)malloc(sizeof(int) * tw);
  uint16_t* top = (uint16_t*)malloc(2 * (size_t)tw);
  for (int i = 0; i < tw; i++) {
    bp[i] = 4;
    top[i] = cy ? d[(long)y0 * w + x0 + i - w] : (uint16_t)half;
  }
  size_t k = 0;
  for (int ym = 0; ym < th && y0 + ym < h; ym++) {
    uint16_t L, TL;
    if (cx) {
      L = d[(long)(y0 + ym) * w + x0 - 1];
      TL = (ym || cy) ? d[(long)(y0 + ym - 1) * w + x0 - 1] : (uint16_t)half;
    } else {
      L = TL = (uint16_t)half;
    }
    for (int xm = 0; xm < tw && x0 + xm < w; xm++) {
      long loc = (long)(y0 + ym) * w + x0 + xm;
      uint16_t T = top[xm], TR = top[(xm + tw + 1) % tw], p[16];
      preds16(L, T, TL, TR, 0, p);
      out[k++] = (uint16_t)(((int)d[loc] - (int)midp16(p[bp[xm]], p[bp[(xm + tw - 1) % tw]]) + half + c) % c);
      TL = top[xm];
      top[xm] = d[loc];
      L = d[loc];
      bp[xm] = best_pred(d[loc], p, mask, c);
    }
  }
  free(bp);
  free(top);
  return k;
}

/* prediction.hpp:153-229 (channelpredict_all): whole plane with a predictor mask per cell; the
 * best predictor of row y+1 is chosen with row y+1's cell mask, and the last row keeps 0. */
void or_predict_all(const uint16_t* d, int w, int h, int depth, int xt, int yt, const uint16_t* map,
                    uint16_t* out) {
  int c = 1 << depth, half = c / 2;
  int tw = (w + xt - 1) / xt, th = (h + yt - 1) / yt;
  int* bp = (int*)malloc(sizeof(int) * w);
  uint16_t* top = (uint16_t*)malloc(2 * (size_t)w);
  for (int i = 0; i < w; i++) { bp[i] = 4; top[i] = (uint16_t)half; }
  for (int y = 0; y < h; y++) {
    uint16_t L = (uint16_t)half, TL = (uint16_t)half;
    for (int x = 0; x < w; x++) {
      long loc = (long)y * w + x;
      uint16_t T = top[x], TR = top[(x + w + 1) % w], p[16];
      preds16(L, T, TL, TR, 1, p);
      out[loc] = (uint16_t)(((int)d[loc] - (int)midp16(p[bp[x]], p[bp[(x + w - 1) % w]]) + half + c) % c);
      TL = top[x];
      top[x] = d[loc];
      L = d[loc];
      bp[x] = 0;
      if (y + 1 < h) bp[x] = best_pred(d[loc], p, map[((y + 1) / th) * xt + x / tw], c);
    }
  }
  free(bp);
  free(top);
}

/* unprediction.hpp:6-91 (unpredict_all) for any predictor map: the inverse of or_predict_all,
 * LZ copies from backref (may be NULL).  Returns residuals consumed or OR_E_CORRUPT. */
long or_unpredict_all(const uint16_t* res, size_t nres, const uint16_t* backref, int w, int h, int depth, int xt,
                      int yt, const uint16_t* map, uint16_t* o) {
  int c = 1 << depth, half = c / 2;
  int tw = (w + xt - 1) / xt, th = (h + yt - 1) / yt;
  int* bp = (int*)malloc(sizeof(int) * w);
  uint16_t* top = (uint16_t*)malloc(2 * (size_t)w);
  for (int i = 0; i < w; i++) { bp[i] = 4; top[i] = (uint16_t)half; }
  size_t k = 0;
  long ret = 0;
  for (int y = 0; y < h && ret == 0; y++) {
    uint16_t L = (uint16_t)half, TL = (uint16_t)half;
    for (int x = 0; x < w; x++) {
      size_t loc = (size_t)y * w + x;
      uint16_t T = top[x], TR = top[(x + w + 1) % w], p[16];
      preds16(L, T, TL, TR, 1, p);
      if (backref && backref[loc]) {
        if (backref[loc] > loc) { ret = OR_E_CORRUPT; break; }
        o[loc] = o[loc - backref[loc]];
      } else {
        if (k >= nres) { ret = OR_E_CORRUPT; break; }
        uint16_t v = (uint16_t)(res[k++] - c - half + midp16(p[bp[x]], p[bp[(x + w - 1) % w]]));
        o[loc] = (uint16_t)(v % c);
      }
      TL = top[x];
      top[x] = o[loc];
      L = o[loc];
      bp[x] = 0;
      if (y + 1 < h) bp[x] = best_pred(o[loc], p, map[((y + 1) / th) * xt + x / tw], c);
    }
  }
  free(bp);
  free(top);
  return ret ? ret : (long)k;
}

/* ------------------------------------------------------------------ colour */

void or_subtract_green(const uint8_t* s, size_t npix, uint16_t* G, uint16_t* R, uint16_t* B) {
  for (size_t i = 0; i < npix; i++) {                               /* channel.hpp:73-79 */
    G[i] = s[3 * i + 1];
    R[i] = (uint16_t)((int)s[3 * i] - (int)s[3 * i + 1] + 256);
    B[i] = (uint16_t)((int)s[3 * i + 2] - (int)s[3 * i + 1] + 256);
  }
}

void or_add_green(const uint16_t* G, const uint16_t* R, const uint16_t* B, size_t npix, uint8_t* o) {
  for (size_t i = 0; i < npix; i++) {
    o[3 * i + 1] = (uint8_t)G[i];
    o[3 * i] = (uint8_t)(R[i] + G[i] - 256);
    o[3 * i + 2] = (uint8_t)(B[i] + G[i] - 256);
  }
}

/* choh.cpp:17-46: distinct colours in first-seen order, -1 at the 257th */
int or_count_colours(const uint8_t* s, size_t size) {
  uint32_t pal[257];
  int k = 0;
  for (size_t i = 0; i + 2 < size; i += 3) {
    uint32_t v = (uint32_t)s[i] | ((uint32_t)s[i + 1] << 8) | ((uint32_t)s[i + 2] << 16);
    int found = 0;
    for (int j = 0; j < k; j++) if (pal[j] == v) { found = 1; break; }
    if (!found) {
      pal[k++] = v;
      if (k == 257) return -1;
    }
  }
  return k;
}

/* ------------------------------------------------------------------ LZ */

static inline int pix_eq(const uint8_t* s, size_t a, size_t b) {
  return s[3 * a] == s[3 * b] && s[3 * a + 1] == s[3 * b + 1] && s[3 * a + 2] == s[3 * b + 2];
}

static long encode_u8(const uint8_t* v, size_t n, uint8_t* out) {
  uint16_t* t = (uint16_t*)malloc((n ? n : 1) * 2);
  for (size_t i = 0; i < n; i++) t[i] = v[i];
  long r = or_encode_entropy(t, n, 256, 10, out);                   /* lz.hpp:100-142 */
  free(t);
  return r;
}

/* lz.hpp:6-170 */
long or_find_lz_rgb(const uint8_t* s, size_t size, int w, int h, uint8_t* lz_out, uint8_t* nuke,
                    int distance, int bonus) {
  (void)h;
  size_t npix = size / 3;
  int limit = 1 << distance;
  size_t cap = npix + 16;
  uint8_t* fut = (uint8_t*)malloc(cap);
  uint8_t* len = (uint8_t*)malloc(cap);
  uint8_t* bb = (uint8_t*)malloc(cap);
  uint8_t* bb2 = (uint8_t*)malloc(cap);
  size_t nf = 0, nl = 0, nb = 0, nb2 = 0;
  int since = 0;
  for (size_t p = 0; p < npix; p++) {
    int longest = 0, best = -1;
    for (int back = 1; back <= limit && (long)p - back >= 0; back++) {
      int off = 0;
      while (p + off < npix && pix_eq(s, p + off, p + off - back) && off < 259) off++;
      if (off > longest) {
        longest = off;
        best = back;
        if (off == 259) break;
      }
    }
    if (longest < 259 && distance > 8) {                            /* lz.hpp:54-74 */
      for (int back = w; back <= (1 << 16) && (long)p - back >= 0; back += w) {
        int off = 0;
        while (p + off < npix && pix_eq(s, p + off, p + off - back) && off < 259) off++;
        if (off > longest) {
          longest = off;
          best = back;
          if (off == 259) back = limit;   /* the reference resets the loop variable only */
        }
      }
    }
    if (longest < 4 + bonus) {
      since++;
      if (since == 255) { since = 0; fut[nf++] = 255; }
    } else {
      fut[nf++] = (uint8_t)since;
      if (distance > 8) bb2[nb2++] = (uint8_t)(best / 256);
      bb[nb++] = (uint8_t)(best % 256);
      len[nl++] = (uint8_t)(longest - 4);
      since = 0;
      for (int o = 0; o < longest; o++) nuke[p + o] = 1;
      p += longest - 1;
    }
  }
  size_t bp = 0;
  long r;
  lz_out[bp++] = 0x03;
  if ((r = encode_u8(fut, nf, lz_out + bp)) < 0) goto out;
  bp += r;
  if ((r = encode_u8(len, nl, lz_out + bp)) < 0) goto out;
  bp += r;
  if ((r = encode_u8(bb, nb, lz_out + bp)) < 0) goto out;
  bp += r;
  if (distance > 8) {
    if ((r = encode_u8(bb2, nb2, lz_out + bp)) < 0) goto out;
    bp += r;
  }
  r = (long)bp;
out:
  free(fut); free(len); free(bb); free(bb2);
  return r;
}

/* ------------------------------------------------------------------ layer / tile / file */

/* stock predictor masks of the -s>=1 search (layer_encode.hpp:159-175) */
static const uint16_t kMasks[14] = {0x0001, 0x0002, 0x0020, 0x0010, 0xffbf, 0x0003, 0xfffd,
                                    0xfffb, 0xfff7, 0xffef, 0xffdf, 0xff7f, 0xfdff, 0xffff};

/* layer_encode.hpp:133-147: -log2((1 + count) / n) per symbol, counts over all n residuals */
static void entropy_table(const uint16_t* res, size_t n, int range, double* ent) {
  int* fr = (int*)malloc(sizeof(int) * range);
  for (int i = 0; i < range; i++) fr[i] = 1;
  for (size_t i = 0; i < n; i++) fr[res[i]]++;
  for (int i = 0; i < range; i++) ent[i] = -log2((double)fr[i] / (double)n);
  free(fr);
}

/* layer_encode.hpp:176-203: per cell, the first stock mask of least estimated cost */
static void search_cells(const uint16_t* d, int w, int h, int depth, int xt, int yt, int npred,
                         const double* ent, uint16_t* plist, uint8_t* pidx, uint16_t* scratch) {
  for (int i = 0; i < xt * yt; i++) {
    double best = 99999999999.0;
    for (int pr = 0; pr < npred; pr++) {
      size_t k = or_predict_section(d, w, h, depth, xt, yt, i % xt, i / xt, kMasks[pr], scratch);
      double cost = 0;
      for (size_t v = 0; v < k; v++) cost += ent[scratch[v]];
      if (cost < best) { best = cost; plist[i] = kMasks[pr]; pidx[i] = (uint8_t)pr; }
    }
  }
}

/* layer_encode.hpp:11-412.  cruncher 0: MED fast path, prob_bits 15.  cruncher >= 1: 40-px grid
 * predictor search (5 / 10 / 14 masks), refined once at cruncher > 2, predictor map stream, then
 * prob_bits 16 vs 15 and three more prob_bits in that direction; the output is `possible_size`
 * bytes of the `permanent` buffer, which is not swapped for the 16/15 pair (Q14), so it may be a
 * prefix of an older stream. */
long or_layer_encode(const uint16_t* data, size_t n, int w, int h, int depth, int cruncher,
                     const uint8_t* nuke, uint8_t* out) {
  size_t oi = 0;
  size_t possible = ((size_t)depth * n + ((size_t)depth * n) % 8 + 1024) / 8;   /* :22 */
  const int range = 1 << depth;
  out[oi++] = 0x10;                                                 /* :57 */
  uint16_t* res = (uint16_t*)malloc((n ? n : 1) * 2);
  uint16_t* clean = (uint16_t*)malloc((n ? n : 1) * 2);
  or_predict_fastpath(data, w, h, depth, res);                      /* :63-75 */
  size_t nc = 0;
  for (size_t i = 0; i < n; i++) if (!nuke || !nuke[i]) clean[nc++] = res[i];   /* :93-99 */
  const size_t cap = or_entropy_bound(nc, (size_t)range, 31);
  uint8_t* bufa = (uint8_t*)malloc(cap);
  uint8_t* bufb = (uint8_t*)malloc(cap);
  uint8_t* dummy = bufa;                                            /* dummyrand (:103) */
  uint8_t* perm = bufb;                                             /* permanent (:104) */
  int valid = 0;                                                    /* perm holds a stream */
  long r = or_encode_entropy(clean, nc, (size_t)range, 15, dummy);  /* :106-113 */
  if (r < 0) goto fail;
  if ((size_t)r < possible) {                                       /* :115-120 */
    possible = (size_t)r;
    uint8_t* x = perm; perm = dummy; dummy = x;
    valid = 1;
  }
  if (cruncher && ((w + 39) / 40 > 1 || (h + 39) / 40 > 1)) {       /* :124-132 */
    int xt = (w + 39) / 40, yt = (h + 39) / 40, T = xt * yt;
    int npred = cruncher * 5 < 14 ? (int)cruncher * 5 : 14;
    double* ent = (double*)malloc(sizeof(double) * range);
    uint16_t* plist = (uint16_t*)malloc(2 * (size_t)T);
    uint8_t* pidx = (uint8_t*)malloc((size_t)T);
    uint16_t* scratch = (uint16_t*)malloc((n ? n : 1) * 2);
    entropy_table(res, n, range, ent);
    search_cells(data, w, h, depth, xt, yt, npred, ent, plist, pidx, scratch);
    or_predict_all(data, w, h, depth, xt, yt, plist, res);          /* :205-214 */
    if (cruncher > 2) {                                             /* :215-272 */
      entropy_table(res, n, range, ent);
      search_cells(data, w, h, depth, xt, yt, npred, ent, plist, pidx, scratch);
      or_predict_all(data, w, h, depth, xt, yt, plist, res);
    }
    out[oi++] = (uint8_t)(xt - 1);                                  /* :276-277 */
    out[oi++] = (uint8_t)(yt - 1);
    int used[14] = {0}, nused = 0, map[14];
    for (int i = 0; i < T; i++) used[pidx[i]] = 1;
    for (int j = 0; j < 14; j++) nused += used[j];
    out[oi++] = (uint8_t)nused;                                     /* :291-297 */
    for (int j = 0, k = 0; j < 14; j++) {
      if (!used[j]) continue;
      out[oi++] = (uint8_t)(kMasks[j] >> 8);
      out[oi++] = (uint8_t)(kMasks[j] % 256);
      map[j] = k++;
    }
    for (int i = 0; i < T; i++) scratch[i] = (uint16_t)map[pidx[i]];
    long m = or_encode_entropy(scratch, (size_t)T, (size_t)nused, 8, out + oi);   /* :308-317 */
    free(ent); free(plist); free(pidx); free(scratch);
    if (m < 0) { r = m; goto fail; }
    oi += (size_t)m;
  } else {
    out[oi++] = 0; out[oi++] = 0; out[oi++] = 0x00; out[oi++] = 0x10;   /* :320-325 */
  }
  if (cruncher) {                                                   /* :326-392 */
    nc = 0;
    for (size_t i = 0; i < n; i++) if (!nuke || !nuke[i]) clean[nc++] = res[i];
    long t1 = or_encode_entropy(clean, nc, (size_t)range, 16, dummy);
    long t2 = t1 < 0 ? t1 : or_encode_entropy(clean, nc, (size_t)range, 15, dummy);
    if (t2 < 0) { r = t2; goto fail; }
    int pb0 = t1 < t2 ? 17 : 14, step = t1 < t2 ? 1 : -1;
    long t12 = t1 < t2 ? t1 : t2;
    if ((size_t)t12 < possible) possible = (size_t)t12;            /* no swap (Q14) */
    for (int k = 0; k < 3; k++) {
      long t = or_encode_entropy(clean, nc, (size_t)range, (uint32_t)(pb0 + step * k), dummy);
      if (t < 0) { r = t; goto fail; }
      if ((size_t)t < possible) {
        possible = (size_t)t;
        uint8_t* x = perm; perm = dummy; dummy = x;
        valid = 1;
      }
    }
  }
  if (!valid) { r = OR_E_UNREPRODUCIBLE; goto fail; }               /* copies garbage */
  memcpy(out + oi, perm, possible);                                 /* :396-398 */
  oi += possible;
  r = (long)oi;
fail:
  free(res); free(clean); free(bufa); free(bufb);
  return r;
}

long or_layer_encode_s0(const uint16_t* data, size_t n, int w, int h, int depth, const uint8_t* nuke,
                        uint8_t* out) {
  return or_layer_encode(data, n, w, h, depth, 0, nuke, out);
}

/* bytes a layer can take: the larger of the -s0 bound and the -s>=1 header + table + payload */
static size_t layer_bound(size_t n, int depth) {
  return or_entropy_bound(n, (size_t)1 << depth, 31) + 2 * 14 + 3 + or_entropy_bound(256, 14, 8) + 16;
}

/* worst case of one tile: stored planes (<= 9/8 B per pixel each, five planes at -s>=3) and the
 * LZ streams */
size_t or_tile_bound(int w, int h) {
  size_t npix = (size_t)w * h;
  return 8 * npix + 16384;
}

/* choh.cpp:125-137 */
static int seek_distance(int cruncher) {
  return cruncher == 1 ? 10 : cruncher == 2 ? 11 : cruncher == 3 ? 12 : cruncher == 4 ? 14 : 6;
}

/* choh.cpp:104-383 */
long or_encode_tile(const uint8_t* s, int w, int h, int cruncher, uint8_t* out, size_t cap) {
  size_t npix = (size_t)w * h, size = npix * 3, o = 0;
  if (cap < or_tile_bound(w, h)) return OR_E_CAP;
  out[o++] = 0; out[o++] = 0;                                       /* :115-116 */
  uint8_t* nuke = (uint8_t*)calloc(npix ? npix : 1, 1);
  uint8_t* lz = (uint8_t*)malloc(or_entropy_bound(npix, 256, 10) * 4 + 16);
  long ret;
  int bonus = 0;
  int cc = or_count_colours(s, size);                               /* :139-154 */
  if (cc != -1) {
    if (cc <= 4) bonus = 32;
    else if (cc <= 8) bonus = 20;
    else if (cc <= 16) bonus = 10;
    else if (cc <= 32) bonus = 2;
  }
  long lzn = or_find_lz_rgb(s, size, w, h, lz, nuke, seek_distance(cruncher), bonus);   /* :156-165 */
  if (lzn < 0) { ret = lzn; goto done; }
  int grey = 1;
  for (size_t i = 0; i < size; i += 3)                              /* channel.hpp:21-31 */
    if (s[i] != s[i + 1] || s[i] != s[i + 2]) { grey = 0; break; }
  if (grey) {
    int c1 = s[0], c2 = s[0], binary = 1;                           /* channel.hpp:33-49 */
    for (size_t i = 0; i < npix; i++) {
      int v = s[3 * i];
      if (v != c1) {
        if (c1 == c2) c2 = v;
        else if (v != c2) { binary = 0; break; }
      }
    }
    if (!binary) { ret = OR_E_UNREPRODUCIBLE; goto done; }          /* :196-205 copies garbage */
    out[o++] = 0;                                                   /* bitimage: no plane data */
    memcpy(out + o, lz, (size_t)lzn);
    o += (size_t)lzn;
    ret = (long)o;
    goto done;
  }
  {
    uint16_t* G = (uint16_t*)malloc(npix * 2);
    uint16_t* R = (uint16_t*)malloc(npix * 2);
    uint16_t* B = (uint16_t*)malloc(npix * 2);
    size_t pb_ = layer_bound(npix, 9);
    uint8_t* c1 = (uint8_t*)malloc(pb_);
    uint8_t* c2 = (uint8_t*)malloc(pb_);
    uint8_t* c3 = (uint8_t*)malloc(pb_);
    uint8_t* a2 = (uint8_t*)malloc(pb_);
    uint8_t* a3 = (uint8_t*)malloc(pb_);
    uint8_t* ci = (uint8_t*)malloc(pb_);
    or_subtract_green(s, npix, G, R, B);                            /* :215-219 */
    long s1 = or_layer_encode(G, npix, w, h, 8, cruncher, nuke, c1);
    long s2 = s1 < 0 ? s1 : or_layer_encode(R, npix, w, h, 9, cruncher, nuke, c2);
    long s3 = s2 < 0 ? s2 : or_layer_encode(B, npix, w, h, 9, cruncher, nuke, c3);
    long sr = -1, sb = -1;
    if (s3 >= 0 && cruncher > 2) {                                  /* :265-293 plain R and B */
      for (size_t i = 0; i < npix; i++) { R[i] = s[3 * i]; B[i] = s[3 * i + 2]; }
      sr = or_layer_encode(R, npix, w, h, 8, cruncher, nuke, a2);
      sb = sr < 0 ? sr : or_layer_encode(B, npix, w, h, 8, cruncher, nuke, a3);
      if (sb < 0) s3 = sb;
    }
    if (s3 < 0) { ret = s3; }
    else {
      long best = s1 + s2 + s3 + lzn;                               /* :295 */
      int mode = 128, chn = 3, ch1_indexed = 0;
      long si = -1;
      size_t z2 = (size_t)s2, z3 = (size_t)s3;
      const uint8_t *p2 = c2, *p3 = c3;
      ret = 0;
      if (cc != -1) {                                               /* :298-308 palette_encode */
        uint16_t* idx = (uint16_t*)malloc(npix * 2);
        uint32_t pal[256];
        int k = 0;
        for (size_t i = 0; i < npix; i++) {
          uint32_t v = (uint32_t)s[3 * i] | ((uint32_t)s[3 * i + 1] << 8) | ((uint32_t)s[3 * i + 2] << 16);
          int j;
          for (j = 0; j < k; j++) if (pal[j] == v) break;
          if (j == k) pal[k++] = v;
          idx[i] = (uint16_t)j;
        }
        si = or_layer_encode(idx, npix, w, h, 8, cruncher, nuke, ci);
        free(idx);
        if (si < 0) ret = si;
        else if (si + 3 * k + 1 + lzn < best) {
          best = si + 3 * k + 1 + lzn;
          mode = 127; chn = 1; ch1_indexed = 1;
        }
      }
      if (ret == 0 && sr >= 0 && sr + s1 + sb + lzn < best) {       /* :309-325 */
        mode = 2; chn = 3;
        z2 = (size_t)sr; z3 = (size_t)sb; p2 = a2; p3 = a3;
      }
      /* channel_compressed1 is the indexed layer once the palette has won (:305-307), but its
       * size stays the GREEN layer's (Q15): reproducible only as a prefix */
      if (ret == 0 && ch1_indexed && s1 > si) ret = OR_E_UNREPRODUCIBLE;
      if (ret == 0) {
        const uint8_t* p1 = ch1_indexed ? ci : c1;
        out[o++] = (uint8_t)mode;                                   /* :328 */
        memcpy(out + o, lz, (size_t)lzn); o += (size_t)lzn;         /* :329-331 */
        if (chn == 1) {
          memcpy(out + o, p1, (size_t)s1); o += (size_t)s1;         /* :335-338 */
        } else {
          out[o++] = 0x24;                                          /* :351-363 */
          o = or_write_varint(out, o, (size_t)s1);
          o = or_write_varint(out, o, z2);
          memcpy(out + o, p1, (size_t)s1); o += (size_t)s1;
          memcpy(out + o, p2, z2); o += z2;
          memcpy(out + o, p3, z3); o += z3;
        }
        ret = (long)o;
      }
    }
    free(G); free(R); free(B); free(c1); free(c2); free(c3); free(a2); free(a3); free(ci);
  }
done:
  free(nuke);
  free(lz);
  return ret;
}

long or_encode_tile_s0(const uint8_t* s, int w, int h, uint8_t* out, size_t cap) {
  return or_encode_tile(s, w, h, 0, out, cap);
}

int or_tiling(int W, int H, int* xt, int* yt, int* tw, int* th) {
  if ((W >= 512 || H >= 512) && W >= 256 && H >= 256) {            /* choh.cpp:454 */
    *xt = W / 256;
    *yt = H / 256;
    *tw = (W + *xt - 1) / *xt;
    *th = (H + *yt - 1) / *yt;
    return 1;
  }
  *xt = *yt = 1;
  *tw = W;
  *th = H;
  return 0;
}

size_t or_choh_bound(int W, int H) {
  int xt, yt, tw, th;
  or_tiling(W, H, &xt, &yt, &tw, &th);
  return 64 + (size_t)xt * yt * 3 + 5 * (size_t)W * H + (size_t)xt * yt * 4096;
}

/* choh.cpp:394-527 (speed = the -sN argument) */
long or_choh(const uint8_t* rgb, int W, int H, int speed, uint8_t* out, size_t cap, size_t* printed) {
  if (W <= 0 || H <= 0) return OR_E_ARG;
  if (cap < 64) return OR_E_CAP;
  size_t o = 0;
  out[o++] = 153; out[o++] = 72; out[o++] = 79; out[o++] = 72;      /* :437-440 */
  out[o++] = 2;                                                     /* :443 */
  out[o++] = 8;                                                     /* :446 */
  o = or_write_varint(out, o, (size_t)W - 1);                       /* :449-450 */
  o = or_write_varint(out, o, (size_t)H - 1);
  int xt, yt, tw, th;
  size_t tile_size = 0;
  if (or_tiling(W, H, &xt, &yt, &tw, &th)) {
    out[o++] = (uint8_t)(xt - 1);                                   /* :457-458 */
    out[o++] = (uint8_t)(yt - 1);
    int nt = xt * yt;
    size_t tcap = or_tile_bound(tw, th);
    uint8_t* tbuf = (uint8_t*)malloc(tcap);
    uint8_t** tiles = (uint8_t**)calloc((size_t)nt, sizeof(uint8_t*));
    size_t* sizes = (size_t*)malloc(sizeof(size_t) * nt);
    uint8_t* trgb = (uint8_t*)malloc((size_t)tw * th * 3);
    long ret = 0;
    for (int i = 0; i < nt; i++) {                                  /* :464-500 */
      int xo = (i % xt) * tw, yo = (i / xt) * th;
      int nw = tw, nh = th;
      if (W - xo < nw) nw = W - xo;
      if (H - yo < nh) nh = H - yo;
      for (int y = 0; y < nh; y++)
        memcpy(trgb + (size_t)y * nw * 3, rgb + ((size_t)(y + yo) * W + xo) * 3, (size_t)nw * 3);
      long r = or_encode_tile(trgb, nw, nh, speed, tbuf, tcap);
      if (r < 0) { ret = r; break; }
      sizes[i] = (size_t)r;
      tiles[i] = (uint8_t*)malloc((size_t)r);
      memcpy(tiles[i], tbuf, (size_t)r);
      if (i + 1 != nt) o = or_write_varint(out, o, sizes[i]);       /* :496-498 */
    }
    if (ret == 0) {
      for (int i = 0; i < nt; i++) {
        if (o + sizes[i] > cap) { ret = OR_E_CAP; break; }
        memcpy(out + o, tiles[i], sizes[i]);
        o += sizes[i];
      }
    }
    for (int i = 0; i < nt; i++) free(tiles[i]);
    free(tiles); free(tbuf); free(sizes); free(trgb);
    if (ret < 0) return ret;
  } else {
    /* :508-520 -- the tile is encoded and discarded (Q13) */
    size_t tcap = or_tile_bound(W, H);
    uint8_t* t = (uint8_t*)malloc(tcap);
    long r = or_encode_tile(rgb, W, H, speed, t, tcap);
    free(t);
    if (r < 0) return r;
    tile_size = (size_t)r;
  }
  if (printed) *printed = o + tile_size;                            /* :522 */
  return (long)o;
}

long or_choh_s0(const uint8_t* rgb, int W, int H, uint8_t* out, size_t cap, size_t* printed) {
  return or_choh(rgb, W, H, 0, out, cap, printed);
}

/* ------------------------------------------------------------------ decoder (corrected) */

static long dec_stream_alloc(const uint8_t* in, size_t size, size_t* p, uint16_t** out, size_t* n) {
  long c = or_peek_count(in, size, *p);
  if (c < 0) return c;
  *out = (uint16_t*)malloc(((size_t)c ? (size_t)c : 1) * 2);
  long r = or_decode_entropy(in, size, p, *out, (size_t)c);
  if (r < 0) { free(*out); *out = NULL; return r; }
  *n = (size_t)r;
  return r;
}

/* un_lz.hpp:68-180 with Q11 (3 vs 4 streams) and Q12 (trailing runs) handled */
static long dec_lz(const uint8_t* in, size_t size, size_t* p, size_t npix, uint16_t* backref) {
  memset(backref, 0, npix * 2);
  if (*p >= size) return OR_E_CORRUPT;
  uint8_t t = in[(*p)++];
  if (!(t & 1)) return 0;
  if (!(t & 2) || (t & 4)) return OR_E_UNSUPPORTED;
  uint16_t *fut = NULL, *len = NULL, *bb = NULL, *bb2 = NULL;
  size_t nf, nl, nb, nb2 = 0;
  long r;
  if ((r = dec_stream_alloc(in, size, p, &fut, &nf)) < 0) return r;
  if ((r = dec_stream_alloc(in, size, p, &len, &nl)) < 0) { free(fut); return r; }
  if ((r = dec_stream_alloc(in, size, p, &bb, &nb)) < 0) { free(fut); free(len); return r; }
  /* a 4th (backby2) stream exists only when the encoder searched > 256 back (-s>=1); its
   * header is varint(255) = 81 7f, which no layer or channel-order byte can start with */
  if (*p + 1 < size && in[*p] == 0x81 && in[*p + 1] == 0x7f) {
    if ((r = dec_stream_alloc(in, size, p, &bb2, &nb2)) < 0) { free(fut); free(len); free(bb); return r; }
  }
  size_t idx = 0, g = 0;
  r = 0;
  for (size_t i = 0; i < nf; i++) {
    size_t cnt = fut[i];
    if (fut[i] == 255) { idx += 255; continue; }
    idx += cnt;
    if (g >= nl || g >= nb) { r = OR_E_CORRUPT; break; }
    size_t L = (size_t)len[g] + 4;
    uint16_t back = (uint16_t)(((bb2 && g < nb2 ? bb2[g] : 0) << 8) + bb[g]);
    g++;
    if (back == 0 || idx + L > npix || back > idx) { r = OR_E_CORRUPT; break; }
    for (size_t j = 0; j < L; j++) backref[idx++] = back;
  }
  free(fut); free(len); free(bb); free(bb2);
  return r;
}

static long dec_layer(const uint8_t* in, size_t size, size_t p, int w, int h, int depth,
                      const uint16_t* backref, uint16_t* plane) {
  if (p + 5 > size) return OR_E_CORRUPT;
  uint8_t tr = in[p++];
  if (tr != 0x10) return OR_E_UNSUPPORTED;                          /* -s0: prediction only */
  uint8_t xt = in[p++], yt = in[p++];
  if (xt != 0 || yt != 0) return OR_E_UNSUPPORTED;                  /* -s>=1 predictor tiles */
  uint16_t pred = (uint16_t)((in[p] << 8) | in[p + 1]);
  p += 2;
  if (pred != 0x0010) return OR_E_UNSUPPORTED;
  uint16_t* res;
  size_t nres;
  long r = dec_stream_alloc(in, size, &p, &res, &nres);
  if (r < 0) return r;
  r = or_unpredict_fastpath(res, nres, backref, w, h, depth, plane);
  free(res);
  if (r < 0) return r;
  if ((size_t)r != nres) return OR_E_CORRUPT;
  return OR_OK;
}

long or_decode_tile(const uint8_t* in, size_t size, size_t p, int w, int h, uint8_t* rgb) {
  size_t npix = (size_t)w * h;
  if (p + 3 > size) return OR_E_CORRUPT;
  if (in[p] != 0 || in[p + 1] != 0) return OR_E_UNSUPPORTED;        /* inner tiling */
  p += 2;
  uint8_t mode = in[p++];
  uint16_t* backref = (uint16_t*)malloc(npix * 2 + 2);
  long r = dec_lz(in, size, &p, npix, backref);
  if (r < 0) { free(backref); return r; }
  if (mode == 0) {                                                  /* binary grey: not coded */
    free(backref);
    return OR_E_UNSUPPORTED;
  }
  if (mode != 128) { free(backref); return OR_E_UNSUPPORTED; }
  if (p >= size || in[p] != 0x24) { free(backref); return OR_E_CORRUPT; }
  p++;
  size_t o1 = or_read_varint(in, &p), o2 = or_read_varint(in, &p);
  uint16_t* G = (uint16_t*)malloc(npix * 2);
  uint16_t* R = (uint16_t*)malloc(npix * 2);
  uint16_t* B = (uint16_t*)malloc(npix * 2);
  r = dec_layer(in, size, p, w, h, 8, backref, G);
  if (r >= 0) r = dec_layer(in, size, p + o1, w, h, 9, backref, R);
  if (r >= 0) r = dec_layer(in, size, p + o1 + o2, w, h, 9, backref, B);
  if (r >= 0) or_add_green(G, R, B, npix, rgb);
  free(G); free(R); free(B); free(backref);
  return r < 0 ? r : OR_OK;
}

long or_dhoh(const uint8_t* in, size_t size, uint8_t* rgb, size_t cap, int* Wp, int* Hp) {
  size_t p = 0;
  if (size < 8 || in[0] != 153 || in[1] != 72 || in[2] != 79 || in[3] != 72) return OR_E_CORRUPT;
  if (in[4] != 2 || in[5] != 8) return OR_E_UNSUPPORTED;
  p = 6;
  int W = (int)or_read_varint(in, &p) + 1, H = (int)or_read_varint(in, &p) + 1;
  *Wp = W; *Hp = H;
  if ((size_t)W * H * 3 > cap) return OR_E_CAP;
  int xt, yt, tw, th;
  if (!or_tiling(W, H, &xt, &yt, &tw, &th)) return OR_E_UNSUPPORTED;   /* header-only file */
  if (p + 2 > size) return OR_E_CORRUPT;
  if (in[p] != (uint8_t)(xt - 1) || in[p + 1] != (uint8_t)(yt - 1)) return OR_E_CORRUPT;
  p += 2;
  int nt = xt * yt;
  size_t* off = (size_t*)malloc(sizeof(size_t) * (nt + 1));
  off[0] = 0;
  for (int i = 1; i < nt; i++) off[i] = off[i - 1] + or_read_varint(in, &p);
  uint8_t* trgb = (uint8_t*)malloc((size_t)tw * th * 3);
  long r = 0;
  for (int i = 0; i < nt && r >= 0; i++) {
    int xo = (i % xt) * tw, yo = (i / xt) * th;
    int nw = tw, nh = th;
    if (W - xo < nw) nw = W - xo;
    if (H - yo < nh) nh = H - yo;
    r = or_decode_tile(in, size, p + off[i], nw, nh, trgb);
    if (r < 0) break;
    for (int y = 0; y < nh; y++)
      memcpy(rgb + ((size_t)(y + yo) * W + xo) * 3, trgb + (size_t)y * nw * 3, (size_t)nw * 3);
  }
  free(off); free(trgb);
  return r < 0 ? r : OR_OK;
}
