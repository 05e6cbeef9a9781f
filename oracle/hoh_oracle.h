/*
 * hoh_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the hoh-ANS reference CPU path (rans64 + entropy stream codec +
 * MED predictor + subtract-green + greedy RGB LZ + layer/tile/container framing at -s0), plus
 * a corrected decoder.  It is the parity checker for the HIP path: only tests/, the
 * __graft_entry__.smoke() check and bench.py's cpu_baseline leg may load it.  The product
 * library (hoh-ans_amd/, libhohgpu.so) never links or calls it.
 *
 * Pinning: every encoder function here is checked byte-for-byte against the reference itself,
 * compiled in place from /root/reference by oracle/ref/Makefile into oracle/_ref/, and against
 * the committed fixtures in tests/golden/ (tests/test_oracle_golden.py).
 *
 * Citations are file:line into the reference (hohMiyazawa/hoh-ANS @ v1).
 */
#ifndef HOH_ORACLE_H
#define HOH_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* error codes (negative returns) */
#define OR_OK 0
#define OR_E_ARG (-1)           /* invalid argument (symbol >= range, pb out of range...)  */
#define OR_E_ASSERT (-2)        /* a live assert() in the reference would abort here      */
#define OR_E_UB (-3)            /* (reserved) undefined behaviour in the reference          */
#define OR_E_UNREPRODUCIBLE (-4)/* the reference emits uninitialised bytes here            */
#define OR_E_CORRUPT (-5)       /* decoder: malformed stream                               */
#define OR_E_CAP (-6)           /* caller buffer too small                                 */
#define OR_E_UNSUPPORTED (-7)   /* decoder: format feature not produced by -s0             */

/* varint.hpp:29-45 / :6-27 */
size_t or_write_varint(uint8_t* b, size_t loc, size_t v);
size_t or_read_varint(const uint8_t* b, size_t* loc);

/* stattools.hpp:13-70; returns OR_OK or OR_E_ASSERT */
int or_normalize_freqs(uint32_t* freqs, uint32_t* cum, size_t size, uint32_t target);

/* rans64.hpp:167-247 (Rans64EncSymbolInit) */
typedef struct { uint64_t rcp_freq; uint32_t freq, bias, cmpl_freq, rcp_shift; } or_esym;
void or_esym_init(or_esym* s, uint32_t start, uint32_t freq, uint32_t scale_bits);

/* entropy_encoding.hpp:8-280.  Returns bytes written (>= 0) or a negative error.
 * `out` must hold or_entropy_bound(n, range, pb) bytes. */
long or_encode_entropy(const uint16_t* sym, size_t n, size_t range, uint32_t prob_bits, uint8_t* out);
size_t or_entropy_bound(size_t n, size_t range, uint32_t prob_bits);

/* Corrected inverse of or_encode_entropy (advances *bp past the payload, handles the
 * single-symbol table of SURVEY Q6).  out must hold the symbol count (use or_peek_count). */
long or_decode_entropy(const uint8_t* in, size_t in_size, size_t* bp, uint16_t* out, size_t cap);
long or_peek_count(const uint8_t* in, size_t in_size, size_t bp);

/* prediction.hpp:6-44 (channelpredict_fastpath): MED residuals */
void or_predict_fastpath(const uint16_t* data, int w, int h, int depth, uint16_t* res);
/* inverse of the fast path (MED on every row; SURVEY Q9 fixed) with LZ back-references:
 * backref[i] != 0 copies out[i - backref[i]] and consumes no residual (unprediction.hpp:35-41). */
long or_unpredict_fastpath(const uint16_t* res, size_t nres, const uint16_t* backref, int w, int h,
                           int depth, uint16_t* out);

/* channel.hpp:73-79 and its inverse */
void or_subtract_green(const uint8_t* rgb, size_t npix, uint16_t* G, uint16_t* R, uint16_t* B);
void or_add_green(const uint16_t* G, const uint16_t* R, const uint16_t* B, size_t npix, uint8_t* rgb);

/* choh.cpp:17-46 */
int or_count_colours(const uint8_t* rgb, size_t size);

/* lz.hpp:6-170.  lz_out gets 0x03 + 3 (or 4 if distance > 8) entropy streams.  Returns bytes or
 * negative error.  nuke (npix bytes) must be zeroed by the caller. */
long or_find_lz_rgb(const uint8_t* rgb, size_t size, int w, int h, uint8_t* lz_out, uint8_t* nuke,
                    int distance, int bonus);

/* prediction.hpp:46-151 / :153-229 (the -s>=1 predictors); section returns the cell's count */
size_t or_predict_section(const uint16_t* data, int w, int h, int depth, int xt, int yt, int cx, int cy,
                          uint16_t mask, uint16_t* out);
void or_predict_all(const uint16_t* data, int w, int h, int depth, int xt, int yt, const uint16_t* map,
                    uint16_t* out);
long or_unpredict_all(const uint16_t* res, size_t nres, const uint16_t* backref, int w, int h, int depth, int xt,
                      int yt, const uint16_t* map, uint16_t* out);

/* layer_encode.hpp:11-412 / choh.cpp:104-383 / choh.cpp:394-527 at any cruncher_mode (-sN) */
long or_layer_encode(const uint16_t* data, size_t n, int w, int h, int depth, int cruncher,
                     const uint8_t* nuke, uint8_t* out);
long or_encode_tile(const uint8_t* rgb, int w, int h, int cruncher, uint8_t* out, size_t cap);
long or_choh(const uint8_t* rgb, int W, int H, int speed, uint8_t* out, size_t cap, size_t* printed);

/* layer_encode.hpp:11-412, cruncher_mode 0 */
long or_layer_encode_s0(const uint16_t* data, size_t n, int w, int h, int depth, const uint8_t* nuke,
                        uint8_t* out);

/* choh.cpp:104-383, cruncher_mode 0.  Returns tile bytes or negative error. */
long or_encode_tile_s0(const uint8_t* rgb, int w, int h, uint8_t* out, size_t cap);
size_t or_tile_bound(int w, int h);

/* choh.cpp:394-527 at -s0: the .hoh bytes the reference writes (header only for images that
 * are not tiled).  *printed = the number choh prints.  Returns bytes or error. */
long or_choh_s0(const uint8_t* rgb, int W, int H, uint8_t* out, size_t cap, size_t* printed);
size_t or_choh_bound(int W, int H);
/* tile geometry of choh.cpp:454-476 */
int or_tiling(int W, int H, int* x_tiles, int* y_tiles, int* tile_w, int* tile_h);

/* corrected decoder (dhoh.cpp:22-396 semantics with Q1, Q9-Q12 fixed) */
long or_decode_tile(const uint8_t* in, size_t size, size_t pos, int w, int h, uint8_t* rgb);
long or_dhoh(const uint8_t* in, size_t size, uint8_t* rgb, size_t cap, int* W, int* H);

#ifdef __cplusplus
}
#endif
#endif
