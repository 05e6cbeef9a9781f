/*
 * hoh_ans.h -- C ABI of libhohgpu.so, the MI355X (gfx950) implementation of the hoh-ANS hot path:
 * subtract-green colour transform, MED predictor / unpredictor, greedy RGB LZ, rans64 entropy
 * stream coding and the .hoh tile container of `choh -s0` / `dhoh`.
 *
 * Conventions: plain pointers and sizes, integer status codes (HOH_OK == 0), no exceptions or
 * C++ types across the boundary.  "d_" pointers are device (HBM) buffers; the others are host
 * buffers.  `stream` is a hipStream_t passed as void* (NULL = the context's own stream).
 * One context per host thread per device; contexts own grow-only device workspaces.
 *
 * Each entry point names the reference interface it replaces (hohMiyazawa/hoh-ANS @ v1,
 * file:line).  The reference has no FFI of its own: its API is the set of free functions in
 * the headers below, compiled into the choh / dhoh drivers.  include/hoh/ headers re-expose those
 * exact C++ signatures on top of this ABI.
 */
#ifndef HOH_ANS_H
#define HOH_ANS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------------------------- */
#define HOH_OK 0
#define HOH_E_ARG 1             /* invalid argument                                            */
#define HOH_E_CAP 2             /* output capacity too small (*written / *out_size = needed)   */
#define HOH_E_HIP 3             /* a HIP runtime call failed                                   */
#define HOH_E_RANGE 4           /* symbol >= range, or range / prob_bits outside the supported
                                   set (normalize_freqs assert, stattools.hpp:14)               */
#define HOH_E_UNREPRODUCIBLE 5  /* the reference writes uninitialised bytes for this input
                                   (grey non-binary tiles, choh.cpp:196-205; palette prefix
                                   longer than the indexed layer, choh.cpp:301-308)             */
#define HOH_E_UNSUPPORTED 6     /* valid but not implemented on this path (4-channel formats);
                                   decoder: indexed (mode 127) tiles, which carry no palette
                                   (SURVEY Q15), and -s>=1 layers (Q14)                         */
#define HOH_E_CORRUPT 7         /* decoder: malformed or undecodable bitstream (incl. the
                                   reference's lossy raw tables)                     */
#define HOH_E_NODEV 8           /* no GPU / HIP device unavailable                              */

typedef struct hoh_ctx hoh_ctx;

int hoh_ctx_create(hoh_ctx** ctx, int device);
void hoh_ctx_destroy(hoh_ctx* ctx);
const char* hoh_strerror(int code);
/* The context's own HIP stream (what a NULL `stream` argument means), as void*: callers that
 * order their own streams against it with events (the Python mirror fences torch's default
 * stream this way). */
void* hoh_ctx_stream(hoh_ctx* ctx);
const char* hoh_version(void);
/* Number of device allocations (hipMalloc) the library has made so far, process-wide.  Contexts
 * keep grow-only workspaces, so repeated calls of one shape allocate nothing after the first. */
uint64_t hoh_device_alloc_count(void);
/* per-kernel device time of the last call, for measurement (ms); enable with hoh_set_profiling */
void hoh_set_profiling(hoh_ctx* ctx, int on);
int hoh_get_kernel_ms(hoh_ctx* ctx, const char** names, float* ms, int max);
/* Per-kernel totals accumulated over every profiled call since the last reset (names are the
 * kernel stages; total_ms / count give the average launch duration on the call's stream). */
int hoh_get_kernel_stats(hoh_ctx* ctx, const char** names, double* total_ms, uint64_t* count, int max);
void hoh_reset_kernel_stats(hoh_ctx* ctx);

/* Per-context options (HOH_E_ARG for an unknown option or value).
 * HOH_OPT_NOIX_DECODER picks the rANS chain kernel of decodes WITHOUT a side index (any foreign
 * .hoh, dhoh.cpp:297-396; every stream one serial chain): HOH_NOIX_ADAPTIVE (default: one lane per
 * chain with full tables while the decode has the device to itself, compact-table lanes beside
 * other no-index decodes), HOH_NOIX_LANES (compact tables, up to 64 chains per workgroup),
 * HOH_NOIX_MULTI (full tables, 12 chains per CU) or HOH_NOIX_WAVE (one wave per stream).  Every
 * choice gives the same bytes; the library reads no environment variables for it. */
#define HOH_OPT_NOIX_DECODER 1
#define HOH_NOIX_ADAPTIVE (-1)
#define HOH_NOIX_LANES 0
#define HOH_NOIX_MULTI 1
#define HOH_NOIX_WAVE 2
int hoh_ctx_set_option(hoh_ctx* ctx, int option, int64_t value);

/* ---- image level: `choh in out W H -sN` / `dhoh in out` -------------------------------- */

/* Worst-case .hoh size for a W x H image (stored planes + LZ streams + framing). */
size_t hoh_encode_bound(int W, int H);

/* Replaces choh.cpp:394-527.  speed = cruncher_mode (-s0 .. -s4; choh.cpp:408-427).  Reads
 * W*H*3 interleaved RGB bytes from d_rgb, writes the exact bytes choh writes (header-only for
 * untiled images) to d_out.  *out_size = bytes written; *printed (optional) = the
 * number choh prints (choh.cpp:522).  -s1..-s4 run the predictor search, seek-distance LZ and
 * prob_bits ladder (layer_encode.hpp:122-392); their files are undecodable by construction
 * (SURVEY Q14), so they get no side index. */
int hoh_encode_image(hoh_ctx* ctx, const uint8_t* d_rgb, int W, int H, int speed,
                     uint8_t* d_out, size_t cap, size_t* out_size, size_t* printed, void* stream);

/* Decode side index: the encoder's coder state every 256 symbols of each plane stream (a
 * Recoil-style checkpoint list kept BESIDE the .hoh, never inside it -- the file bytes are
 * identical with or without it).  With an index the decoder splits every stream into
 * independent segments; without one (any foreign .hoh) it decodes each stream serially.  A
 * segment whose end state disagrees with the next checkpoint fails the decode (HOH_E_CORRUPT). */
typedef struct hoh_index hoh_index;
int hoh_index_create(hoh_index** idx);
void hoh_index_destroy(hoh_index* idx);
size_t hoh_index_bytes(const hoh_index* idx);
int hoh_encode_image_ix(hoh_ctx* ctx, const uint8_t* d_rgb, int W, int H, int speed,
                        uint8_t* d_out, size_t cap, size_t* out_size, size_t* printed,
                        hoh_index* idx, void* stream);

/* Replaces dhoh.cpp:297-396 (with the decoder defects of SURVEY Q1, Q9-Q12 fixed).  d_hoh holds
 * `size` bytes of a .hoh file (as written by choh -s0); writes W*H*3 RGB bytes to d_rgb. */
int hoh_decode_image(hoh_ctx* ctx, const uint8_t* d_hoh, size_t size, uint8_t* d_rgb, size_t cap,
                     int* W, int* H, void* stream);
int hoh_decode_image_ix(hoh_ctx* ctx, const uint8_t* d_hoh, size_t size, uint8_t* d_rgb, size_t cap,
                        int* W, int* H, const hoh_index* idx, void* stream);

/* ---- enqueue-only image path (no host synchronisation) ----------------------------------
 * The work of hoh_encode_image_ix / hoh_decode_image_ix for tiled images, enqueued on `stream`
 * with no host round trip, so one host thread keeps many images in flight on many streams (the
 * reference's choh/dhoh loop over files, choh.cpp:464-500 / dhoh.cpp:297-396, without the
 * per-file wait).  Results are written by the stream to d_status (device or pinned host memory,
 * two u64): d_status[0] = HOH_OK or an HOH_E_* code, d_status[1] = the .hoh size (encode) or
 * W*H*3 (decode).  Read it after synchronising the stream.  Calls on one stream run in order, so
 * a context's workspaces, the index and the caller's buffers may be reused by the next call on
 * the same stream.  The decoder takes W and H from the caller (the file header is checked on the
 * device: a mismatch gives HOH_E_CORRUPT) and reads at most `size` bytes (a bound suffices, e.g.
 * the encoder's cap).  Header-only (untiled) images return HOH_E_UNSUPPORTED here:
 * use the synchronous calls. */
int hoh_encode_image_async(hoh_ctx* ctx, const uint8_t* d_rgb, int W, int H, int speed, uint8_t* d_out,
                           size_t cap, hoh_index* idx, uint64_t* d_status, void* stream);
int hoh_decode_image_async(hoh_ctx* ctx, const uint8_t* d_hoh, size_t size, int W, int H, uint8_t* d_rgb,
                           size_t cap, const hoh_index* idx, uint64_t* d_status, void* stream);

/* ---- batched enqueue-only image path ------------------------------------------------------
 * n images of one shape per call: each kernel of the image path covers the tiles of all n images
 * in one launch (choh.cpp:464-500's tile loop, run over the batch), so a few streams -- and the
 * few hardware queues HIP gives a process by default -- keep the device busy.  Images are
 * contiguous (image i at d_rgb + i*W*H*3); file i is written at / read from d_hoh + i*stride
 * (stride >= each file's size, e.g. hoh_encode_bound(W, H)).  d_status holds 2n u64, {status,
 * size} per image as in the single-image calls: an image's own failures (HOH_E_CAP past its
 * stride, HOH_E_UNREPRODUCIBLE, ...) mark only its slot; a failure of the job marks every slot.
 * Files are byte-identical to the single-image calls'.  One side index serves the whole batch
 * (payload positions are absolute in the batch buffer), so a decode with it needs the same n and
 * stride (else HOH_E_ARG).  The batch runs as one job when its tiles stack -- H a multiple of 256,
 * so the n images are the 256-row tile grid of one n*H image; at -s1..-s4 (whose workspace is ~8 MB
 * per tile) as stacks of up to 1024 tiles (one 8192^2 image, or 64 of 1024^2) one after another,
 * and no side index (idx, if given, is emptied as in the single-image calls); otherwise tiled
 * images run one after another on the stream (without a side index when n > 1 at -s0:
 * HOH_E_UNSUPPORTED).  Untiled shapes (header-only files) return HOH_E_UNSUPPORTED for
 * any n, as in the single-image async calls: use hoh_encode_image / hoh_decode_image.  The decoder
 * bounds every parse of file i by [i*stride, (i+1)*stride) (a truncated file reads as corrupt) and
 * reads n*stride bytes of d_hoh at most; in a one-job batch an error in any file marks every
 * image's status. */
int hoh_encode_images_async(hoh_ctx* ctx, int n, const uint8_t* d_rgb, int W, int H, int speed, uint8_t* d_out,
                            size_t stride, hoh_index* idx, uint64_t* d_status, void* stream);
int hoh_decode_images_async(hoh_ctx* ctx, int n, const uint8_t* d_hoh, size_t stride, int W, int H, uint8_t* d_rgb,
                            const hoh_index* idx, uint64_t* d_status, void* stream);

/* Host-side header parse: W, H and tiling of a .hoh (dhoh.cpp:320-366). */
int hoh_peek_header(const uint8_t* hoh, size_t size, int* W, int* H, int* x_tiles, int* y_tiles);

/* ---- sharded image encode (multi-GPU: one process per GPU) ------------------------------ */

/* Encodes tiles [t0, t0+ntiles) (row-major tile index, choh.cpp:464-500) of the W x H image into
 * a blob of concatenated tile byte strings at d_out; d_tile_sizes (device, ntiles u32) receives
 * each tile's size.  A rank's blob plus everyone's sizes are what the gather exchanges.
 * d_rgb is the base of the whole image: a rank holding only rows [y0, y1) passes
 * (its buffer - y0*W*3); only the pixels of the named tiles are read. */
int hoh_encode_tiles(hoh_ctx* ctx, const uint8_t* d_rgb, int W, int H, int t0, int ntiles,
                     uint8_t* d_out, size_t cap, uint32_t* d_tile_sizes, size_t* out_size,
                     void* stream);
int hoh_encode_tiles_ix(hoh_ctx* ctx, const uint8_t* d_rgb, int W, int H, int t0, int ntiles,
                        uint8_t* d_out, size_t cap, uint32_t* d_tile_sizes, size_t* out_size,
                        hoh_index* idx, void* stream);
/* The same at any speed (-s0..-s4; -s>=1 tiles get no side index). */
int hoh_encode_tiles_speed(hoh_ctx* ctx, const uint8_t* d_rgb, int W, int H, int speed, int t0, int ntiles,
                           uint8_t* d_out, size_t cap, uint32_t* d_tile_sizes, size_t* out_size,
                           hoh_index* idx, void* stream);
/* Decodes tiles [t0, t0+ntiles) from d_blob (their byte strings concatenated, sizes in
 * h_tile_sizes) into the W x H image at d_rgb (only those tiles' pixels are written; d_rgb is
 * the base of the whole image).  idx may be the index hoh_encode_tiles_ix recorded. */
int hoh_decode_tiles(hoh_ctx* ctx, const uint8_t* d_blob, size_t size, int W, int H, int t0, int ntiles,
                     const uint32_t* h_tile_sizes, uint8_t* d_rgb, const hoh_index* idx, void* stream);
/* Enqueue-only forms of the two calls above (no host round trip; see the image-level async
 * calls for the d_status convention).  Encode: d_status[1] = the blob size.  Decode: the tile
 * sizes are read from DEVICE memory (d_tile_sizes, e.g. as the encoder wrote them), so a shard can
 * be decoded before its sizes ever reach the host; d_status[1] = the shard's RGB bytes. */
int hoh_encode_tiles_async(hoh_ctx* ctx, const uint8_t* d_rgb, int W, int H, int speed, int t0, int ntiles,
                           uint8_t* d_out, size_t cap, uint32_t* d_tile_sizes, hoh_index* idx, uint64_t* d_status,
                           void* stream);
int hoh_decode_tiles_async(hoh_ctx* ctx, const uint8_t* d_blob, size_t size, int W, int H, int t0, int ntiles,
                           const uint32_t* d_tile_sizes, uint8_t* d_rgb, const hoh_index* idx, uint64_t* d_status,
                           void* stream);
/* Batched shards (multi-GPU with several images in flight per GPU): the same tile band
 * [t0, t0+ntiles) of n W x H images per call.  The band must be whole tile rows (t0 and ntiles
 * multiples of x_tiles, else HOH_E_ARG).  d_rgb holds the n bands back to back (band i = rows
 * [y0, y1) of image i at d_rgb + i*W*(y1-y0)*3 -- NOT the image base as in the single-shard
 * calls); blob i is written at / read from d_blob + i*stride, its tile sizes at
 * d_tile_sizes + i*ntiles (device u32); d_status holds {status, blob size} (encode) or {status,
 * band RGB bytes} (decode) per shard.  When H is a multiple of 256 the n bands stack into one
 * tile grid and every kernel covers all n shards per launch (as hoh_encode_images_async does for
 * whole images); otherwise the shards run one after another on the stream.  Blobs are
 * byte-identical to n single-shard calls'.  -s1..-s4 stack up to 1024 tiles per job.  A side
 * index serves the batch it was recorded for (same n and stride).  The decoder bounds every parse
 * of blob i by [i*stride, (i+1)*stride) and reads n*stride bytes of d_blob at most; in a one-job
 * batch an error in any blob marks every shard's status. */
int hoh_encode_tiles_images_async(hoh_ctx* ctx, int n, const uint8_t* d_rgb, int W, int H, int speed, int t0,
                                  int ntiles, uint8_t* d_blob, size_t stride, uint32_t* d_tile_sizes, hoh_index* idx,
                                  uint64_t* d_status, void* stream);
int hoh_decode_tiles_images_async(hoh_ctx* ctx, int n, const uint8_t* d_blob, size_t stride, int W, int H, int t0,
                                  int ntiles, const uint32_t* d_tile_sizes, uint8_t* d_rgb, const hoh_index* idx,
                                  uint64_t* d_status, void* stream);
/* Host: the .hoh prefix for a tiled image given every tile's size (choh.cpp:437-498):
 * magic, format, depth, varint W-1, H-1, x_tiles-1, y_tiles-1, n-1 varint sizes.  Returns the
 * prefix length, or 0 if cap is too small. */
size_t hoh_file_prefix(int W, int H, const uint32_t* tile_sizes, int ntiles, uint8_t* out, size_t cap);
/* tiling of choh.cpp:454-461: returns 1 if tiled */
int hoh_tiling(int W, int H, int* x_tiles, int* y_tiles, int* tile_w, int* tile_h);

/* ---- multi-GPU in one process (choh / dhoh over several devices) ----------------------- */

/* One process drives ndev GPUs: a context and a HIP stream per device and, when the devices are
 * distinct, one RCCL communicator each (ncclCommInitAll; librccl.so is loaded here, not at link
 * time).  A device may be listed more than once (several shards on one GPU): the blobs then move
 * by device copies instead of RCCL (hoh_mgpu_transport returns 0; 1 = RCCL).  Distinct devices
 * fall back to the same peer copies when librccl cannot be loaded or ncclCommInitAll fails. */
typedef struct hoh_mgpu hoh_mgpu;
int hoh_mgpu_create(hoh_mgpu** m, int ndev, const int* devices);
void hoh_mgpu_destroy(hoh_mgpu* m);
int hoh_mgpu_transport(const hoh_mgpu* m);
/* choh.cpp:394-527 over all devices: device r encodes a band of tile rows (choh.cpp:464-500) of
 * the host image h_rgb; one RCCL group gathers the blobs over xGMI behind hoh_file_prefix into
 * the file d_out on the first device.  Same bytes and printed size as hoh_encode_image. */
int hoh_mgpu_encode_image(hoh_mgpu* m, const uint8_t* h_rgb, int W, int H, int speed, uint8_t* d_out, size_t cap,
                          size_t* out_size, size_t* printed);
/* dhoh.cpp:297-396 over all devices: the file d_hoh (size bytes, on the first device) -> the host
 * image h_rgb (W*H*3 bytes, cap at least that).  The tile table is parsed on the host, one RCCL
 * group sends each device its tiles' bytes, each decodes its band. */
int hoh_mgpu_decode_image(hoh_mgpu* m, const uint8_t* d_hoh, size_t size, uint8_t* h_rgb, size_t cap, int* W,
                          int* H);

/* ---- entropy stream level (host buffers; one call = one stream, batched inside) --------- */

/* Replaces encode_entropy(uint16_t*, size_t, size_t, uint8_t*, uint32_t, uint8_t)
 * (entropy_encoding.hpp:8-15; u8 overload :283-290).  Same bytes; *written = stream bytes. */
int hoh_encode_entropy(hoh_ctx* ctx, const uint16_t* symbols, size_t n, size_t range,
                       uint32_t prob_bits, uint8_t* out, size_t cap, size_t* written);
size_t hoh_entropy_bound(size_t n, size_t range, uint32_t prob_bits);

/* Replaces decode_entropy(uint8_t*, size_t, size_t*, size_t*, uint8_t)
 * (entropy_decoding.hpp:134-140).  Advances *byte_pointer past the whole stream (Q1 fix);
 * *n = symbol count; out must hold cap symbols (hoh_entropy_count tells the count). */
int hoh_decode_entropy(hoh_ctx* ctx, const uint8_t* in, size_t in_size, size_t* byte_pointer,
                       uint16_t* out, size_t cap, size_t* n);
int hoh_entropy_count(const uint8_t* in, size_t in_size, size_t byte_pointer, size_t* n);

/* Framing of the stream at byte_pointer without decoding it (decode_entropy_simple,
 * entropy_decoding.hpp:8-132): header fields, where the frequency table ends, the rANS payload
 * size and where the whole stream ends (the Q1-corrected *byte_pointer).  Host only. */
typedef struct hoh_entropy_header {
  uint64_t range, count;               /* symbol range, symbol count (:143-144)               */
  uint32_t entropy_mode, prob_bits;    /* metadata byte (:151-154): 1 = rANS, 0 = stored       */
  uint32_t table_mode, symbol_bits;    /* table storage mode; bits per stored symbol (:146-149) */
  uint64_t table_end;                  /* offset after the frequency table (rANS streams)      */
  uint64_t payload_bytes;              /* rANS payload size (:256) or stored bytes             */
  uint64_t stream_end;                 /* offset after the whole stream                        */
} hoh_entropy_header;
int hoh_entropy_parse(const uint8_t* in, size_t in_size, size_t byte_pointer, hoh_entropy_header* h);

/* Batched device form: nstreams streams, stream i = d_syms[h_offsets[i] .. + h_counts[i]]
 * (h_offsets multiples of 8), all with the same range and prob_bits; stream i is written to
 * d_out + h_out_offsets[i] (caller-chosen, each with hoh_entropy_bound room); h_sizes[i]
 * receives its size. */
int hoh_encode_entropy_batch(hoh_ctx* ctx, const uint16_t* d_syms, const uint64_t* h_offsets,
                             const uint32_t* h_counts, int nstreams, uint32_t range,
                             uint32_t prob_bits, uint8_t* d_out, const uint64_t* h_out_offsets,
                             uint32_t* h_sizes, void* stream);

/* ---- plane level ------------------------------------------------------------------------ */

/* Replaces layer_encode(uint16_t*, size_t, int, int, int, size_t, uint8_t*, uint8_t*)
 * (layer_encode.hpp:11-20), cruncher_mode 0..4 (1..4: grid predictor search and prob_bits ladder,
 * with the reference's stale-prefix output).  nuke may be NULL (no LZ). */
int hoh_layer_encode(hoh_ctx* ctx, const uint16_t* data, size_t size, int width, int height,
                     int depth, size_t cruncher_mode, const uint8_t* nuke, uint8_t* out,
                     size_t cap, size_t* written);
/* Replaces decode_layer (layer_decode.hpp:128-136), returning the full-depth plane (u16: the
 * reference truncates 9-bit planes to u8).  Predictor-map layers use unpredict_all;
 * the -s0 MED layer uses MED on every row (Q9 fixed).  backref may be NULL. */
int hoh_layer_decode(hoh_ctx* ctx, const uint8_t* in, size_t in_size, size_t byte_pointer,
                     int width, int height, int depth, const uint16_t* backref, uint16_t* out);
/* Replaces channelpredict_fastpath (prediction.hpp:6-13; reached via channelpredict_section
 * :59-68): MED residuals. */
int hoh_predict_fastpath(hoh_ctx* ctx, const uint16_t* data, int width, int height, int depth,
                         uint16_t* out);
/* Replaces unpredict_all (unprediction.hpp:6-16) for the fast-path predictor (tile_map =
 * {0x0010}) with MED on every row (SURVEY Q9 fixed).  res holds nres residuals; backref may be
 * NULL. */
int hoh_unpredict_fastpath(hoh_ctx* ctx, const uint16_t* res, size_t nres, const uint16_t* backref,
                           int width, int height, int depth, uint16_t* out);
/* Replaces channelpredict_section (prediction.hpp:46-151): residuals of cell (cx, cy) of an
 * xt x yt grid with one predictor mask, in the cell's raster order; *count = residuals written
 * (out must hold the cell's pixel count). */
int hoh_predict_section(hoh_ctx* ctx, const uint16_t* data, int width, int height, int depth, int x_tiles,
                        int y_tiles, int x, int y, uint16_t predictor, uint16_t* out, size_t* count);
/* Replaces channelpredict_all (prediction.hpp:153-229): whole plane, one mask per grid cell. */
int hoh_predict_all(hoh_ctx* ctx, const uint16_t* data, int width, int height, int depth, int x_tiles,
                    int y_tiles, const uint16_t* tile_map, uint16_t* out);
/* Replaces unpredict_all (unprediction.hpp:6-91) for any predictor map: the exact inverse of
 * channelpredict_all with LZ copies (backref may be NULL).  A 1x1 {0x0010} map is the -s0 layer
 * and is inverted with MED on every row (SURVEY Q9 fixed), as hoh_unpredict_fastpath. */
int hoh_unpredict_all(hoh_ctx* ctx, const uint16_t* res, size_t nres, const uint16_t* backref, int width,
                      int height, int depth, int x_tiles, int y_tiles, const uint16_t* tile_map, uint16_t* out);
/* Replaces subtract_green (channel.hpp:73-79) and provides its inverse. */
int hoh_subtract_green(hoh_ctx* ctx, const uint8_t* rgb, size_t npix, uint16_t* G, uint16_t* R, uint16_t* B);
int hoh_add_green(hoh_ctx* ctx, const uint16_t* G, const uint16_t* R, const uint16_t* B, size_t npix, uint8_t* rgb);

/* ---- utilities ---------------------------------------------------------------------------- */

/* Deterministic synthetic RGB (hoh_ans/synth.py formula) written to d_rgb; _rows writes only
 * rows [y0, y0+rows) of a width-W image (a shard). */
int hoh_synth_rgb(hoh_ctx* ctx, uint8_t* d_rgb, int W, int H, uint64_t seed, int noise, void* stream);
int hoh_synth_rgb_rows(hoh_ctx* ctx, uint8_t* d_rgb, int W, int y0, int rows, uint64_t seed, int noise,
                       void* stream);
/* Natural-statistic synthetic RGB (hoh_ans/natural.py formula: piecewise-smooth regions, hard
 * edges, textures, flat runs, short repeats), rows [y0, y0+rows) of a width-W image. */
int hoh_natural_rgb_rows(hoh_ctx* ctx, uint8_t* d_rgb, int W, int y0, int rows, uint64_t seed, void* stream);

#ifdef __cplusplus
}
#endif
#endif
