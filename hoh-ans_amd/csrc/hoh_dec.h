// Decoder-side internal definitions (k_decode.hip, hoh_decode.cpp).
#pragma once
#include "hoh_internal.h"

struct hoh_index;
struct hoh_ctx;

struct IndexStream {      // one stream of an encoded image, as recorded by the encoder
  uint64_t payload_off;   // byte offset (in the .hoh) of the first rANS payload word
  uint32_t n;             // symbols
  uint32_t mode;          // SM_*
  uint32_t widx_end;      // slab index of the first payload word (checkpoint widx base)
  uint32_t ckpt_off;      // first checkpoint of the stream in the index
  uint32_t words;
  uint32_t pad;
};

struct DecStream {        // one stream of a .hoh, as parsed by the decoder
  uint64_t table_off;     // where the frequency table bits start (byte), for the table kernel
  uint64_t payload_off;   // first payload byte (rANS words or stored bits)
  uint64_t out_off;       // element offset of the decoded symbols in the decode arena
  uint32_t n, range, pb, mode, tsm, maxbits;
  uint32_t words;         // rANS payload words
  uint32_t err;
  int32_t ix;             // matching index stream, -1 if none
  uint32_t blk;           // 1: decoded into the blocked plane layout (blk_pos, k_decode.hip)
};

struct DecTile {
  int32_t x0, y0, w, h;
  uint64_t off;           // byte offset of the tile in the file
  uint32_t mode, nmatch;
  uint32_t err, pad;
};

struct DecWork {
  void* bufs[16] = {nullptr};
  size_t sizes[16] = {0};
  hipEvent_t noix_ev = nullptr;   // recorded after this context's last no-index chain kernel
  int noix_dev = -1;              // device it is registered on (k_decode.hip, noix_busy)
  int64_t noix_t = 0;             // host time (steady clock, us) of its last no-index decode
};

void dec_free(DecWork& w);
void noix_release(DecWork& w);
int index_capture(hoh_index* idx, const EncodeJob& j, hipStream_t s);
int index_reserve(hoh_index* idx, size_t nstreams, size_t nck);
Checkpoint* index_ckpt_buf(hoh_index* idx);
void launch_index_capture(const EncodeJob& j, IndexStream* is, size_t per, hipStream_t s);
const IndexStream* index_streams(const hoh_index* idx);
const Checkpoint* index_ckpts(const hoh_index* idx);
int index_nstreams(const hoh_index* idx);
int index_batch(const hoh_index* idx, uint64_t* stride);    // images and file stride the index was recorded for
DecWork& ctx_dec(hoh_ctx* c);
hipStream_t ctx_stream(hoh_ctx* c, void* s);
uint64_t* ctx_pinned(hoh_ctx* c);
int ctx_device(hoh_ctx* c);
int ctx_cus(hoh_ctx* c);
int ctx_noix(hoh_ctx* c);                  // HOH_OPT_NOIX_DECODER (include/hoh_ans.h)
void ctx_mark(hoh_ctx* c, hipStream_t s, const char* name, bool reset);

// Per-context device scratch for the host-buffer entry points (encode_entropy, decode_entropy,
// layer_*, the predictor/unpredictor drop-ins): a grow-only chunk list used as a stack.  A frame
// releases everything allocated after it was opened; after the first call of a given shape no
// call allocates device memory.  alloc() returns nullptr on failure.
struct ScratchFrame {
  hoh_ctx* c;
  size_t cur, used;
  explicit ScratchFrame(hoh_ctx* ctx);
  ~ScratchFrame();
  void* alloc(size_t n);
  template <class T> T* get(size_t n) { return (T*)alloc(n); }
};
