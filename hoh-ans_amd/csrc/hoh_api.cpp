// Host orchestration and C ABI of libhohgpu (include/hoh_ans.h).  All compute runs in the HIP
// kernels of this directory; this file only sizes workspaces, launches, and moves the few bytes
// the host must see (sizes, status words).  There is no CPU fallback: without a HIP device every
// entry point returns HOH_E_NODEV.
#include "hoh_internal.h"
#include "hoh_dec.h"
#include "../../include/hoh_ans.h"

#include <math.h>
#include <string.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
#include <stdio.h>
#include <string>
#include <atomic>

void launch_synth(uint8_t* rgb, int W, int H, int y0, uint64_t seed, int noise, hipStream_t s);
void launch_natural(uint8_t* rgb, int W, int rows, int y0, uint64_t seed, hipStream_t s);
void launch_put_bytes(uint8_t* dst, const uint8_t* b, int n, hipStream_t s, int copies = 1, uint64_t stride = 0);
void launch_status_enc(const uint32_t* gerr, const uint64_t* total, uint64_t cap, uint64_t* out, hipStream_t s);
void launch_status_enc_batch(const uint32_t* gerr, const uint64_t* img_total, const uint32_t* img_err,
                             uint64_t stride, uint64_t* out, int n, hipStream_t s);

std::atomic<uint64_t> g_device_allocs{0};     // every hipMalloc this library makes

namespace {

struct Buf {
  void* p = nullptr;
  size_t n = 0;
};

int ensure(Buf& b, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (b.n >= bytes) return HOH_OK;
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.n = 0;
  if (hipMalloc(&b.p, bytes) != hipSuccess) return HOH_E_HIP;
  g_device_allocs.fetch_add(1, std::memory_order_relaxed);
  b.n = bytes;
  return HOH_OK;
}

size_t rup(size_t v, size_t a) { return (v + a - 1) / a * a; }

}  // namespace

struct hoh_index {
  Buf ck;                       // Checkpoint[]
  Buf streams;                  // IndexStream[]
  int nstreams = 0;
  size_t ck_count = 0;
  int nimg = 1;                 // a batch's index: its image count and file stride (payload
  uint64_t stride = 0;          //   offsets are absolute in the batch buffer)
};

struct Scratch {                // see ScratchFrame (hoh_dec.h)
  std::vector<Buf> chunks;
  size_t cur = 0, used = 0;
};

struct hoh_ctx {
  int device = 0;
  int cus = 256;                // compute units of the device
  Scratch scr;
  hipStream_t own = nullptr;
  SideStream side;              // -s>=1: the LZ screen beside the predictor search (created on first use)
  Buf dbg;                      // measurement builds (HOH_DEBUG_READ): per-tile kernel counters
  Buf idx8, fpb, pinfo, lg;     // -s>=1 workspaces (fpb: fingerprints, then the tile-major pixels)
  Buf lzs;                      // -s>=2: LZ posting lists (k_lzsort): sorted positions + ping-pong (then the sorted fingerprints) + ranks
  uint32_t lg_key[4] = {0, 0, 0, 0};
  uint64_t lg_off[4] = {0, 0, 0, 0};
  Buf sym, hist, candbits, matches, lzspec, pal, streams, tiles, hdr, tab_fast, tab_gen, slabs, ckpt, misc, tsizes;
  DecWork dec;                  // decoder workspaces (k_decode.hip)
  uint64_t* pinned = nullptr;   // small host staging (status words, sizes)
  int profiling = 0;
  int noix = HOH_NOIX_ADAPTIVE;  // HOH_OPT_NOIX_DECODER
  std::vector<std::string> knames;      // names of the marks recorded by the current call
  std::vector<hipEvent_t> kev;          // event pool, kev[0..nmark) recorded by the current call
  size_t nmark = 0;
  std::vector<std::string> snames;      // accumulated per-kernel totals since the last reset
  std::vector<double> sms;
  std::vector<uint64_t> scount;
  std::vector<float> kms;
};

static hipStream_t pick(hoh_ctx* c, void* s) { return s ? (hipStream_t)s : c->own; }

// ---------------------------------------------------------------- profiling helpers

// Events are recorded between consecutive launches on the call's stream (no host sync); at the
// start of the next call, or when stats are read, the previous call's intervals are folded into
// per-name totals.  Every API call ends with a stream sync, so the fold never waits.
static void prof_fold(hoh_ctx* c) {
  if (c->nmark >= 2) {
    (void)hipEventSynchronize(c->kev[c->nmark - 1]);
    for (size_t i = 1; i < c->nmark; i++) {
      if (c->knames[i] == "start") continue;
      float v = 0;
      (void)hipEventElapsedTime(&v, c->kev[i - 1], c->kev[i]);
      size_t k = 0;
      while (k < c->snames.size() && c->snames[k] != c->knames[i]) k++;
      if (k == c->snames.size()) { c->snames.push_back(c->knames[i]); c->sms.push_back(0); c->scount.push_back(0); }
      c->sms[k] += v;
      c->scount[k] += 1;
    }
  }
  c->nmark = 0;
  c->knames.clear();
}

static void prof_mark(hoh_ctx* c, hipStream_t s, const char* name, bool reset) {
  if (!c->profiling) return;
  if (reset) prof_fold(c);
  if (c->nmark == c->kev.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return;
    c->kev.push_back(e);
  }
  (void)hipEventRecord(c->kev[c->nmark++], s);
  c->knames.push_back(name);
}

struct Prof {
  hoh_ctx* c;
  hipStream_t s;
  // an enqueue-only call must not wait for the previous call's events: it appends its marks
  // (the interval ending at its "start" mark spans the gap between calls and is not counted)
  Prof(hoh_ctx* c_, hipStream_t s_, bool async = false) : c(c_), s(s_) { prof_mark(c, s, "start", !async); }
  void mark(const char* name) { prof_mark(c, s, name, false); }
};

extern "C" {

const char* hoh_version(void) { return "hoh-ans_amd 0.2 (gfx950)"; }

uint64_t hoh_device_alloc_count(void) { return g_device_allocs.load(std::memory_order_relaxed); }

const char* hoh_strerror(int code) {
  switch (code) {
    case HOH_OK: return "ok";
    case HOH_E_ARG: return "invalid argument";
    case HOH_E_CAP: return "output capacity too small";
    case HOH_E_HIP: return "HIP runtime error";
    case HOH_E_RANGE: return "symbol / range / prob_bits outside the supported set";
    case HOH_E_UNREPRODUCIBLE: return "the reference emits uninitialised bytes for this input";
    case HOH_E_UNSUPPORTED: return "not implemented on this path";
    case HOH_E_CORRUPT: return "malformed or undecodable bitstream";
    case HOH_E_NODEV: return "no HIP device";
  }
  return "unknown error";
}

int hoh_ctx_create(hoh_ctx** out, int device) {
  if (!out) return HOH_E_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0) return HOH_E_NODEV;
  if (hipSetDevice(device) != hipSuccess) return HOH_E_NODEV;
  {
    // More hardware queues than ~20 per process oversubscribe the device's queue slots: measured
    // -15% at 24 and -28% at 28 images in flight, each on its own queue (docs/EXPERIMENTS.md, in-flight
    // sweep).  HIP reads the variable once, before this library can act on it, so say it once.
    static std::atomic<int> warned{0};
    const char* q = getenv("GPU_MAX_HW_QUEUES");
    if (q && atoi(q) > 20 && !getenv("HOH_QUIET") && !warned.exchange(1))
      fprintf(stderr, "hoh: GPU_MAX_HW_QUEUES=%s: more than 20 hardware queues per process cost 15-30%% "
                      "throughput on MI355X; share queues between streams instead\n", q);
  }
  hoh_ctx* c = new hoh_ctx();
  c->device = device;
  if (hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || c->cus <= 0)
    c->cus = 256;
  if (hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) { delete c; return HOH_E_HIP; }
  if (hipHostMalloc((void**)&c->pinned, 4096) != hipSuccess) { delete c; return HOH_E_HIP; }
  *out = c;
  return HOH_OK;
}

// knob LZ_POSTING=0: -s1..-s4 LZ scans walk every back distance (the round-3 scan, for comparison)
static int lz_posting() { return HOH_KNOB(LZ_POSTING, 1); }

static void freebuf(Buf& b) { if (b.p) (void)hipFree(b.p); b.p = nullptr; b.n = 0; }

void hoh_ctx_destroy(hoh_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  Buf* all[] = {&c->dbg, &c->idx8, &c->fpb, &c->lzs, &c->pinfo, &c->lg, &c->sym, &c->hist, &c->candbits, &c->matches, &c->lzspec, &c->pal, &c->streams, &c->tiles, &c->hdr,
                &c->tab_fast, &c->tab_gen, &c->slabs, &c->ckpt, &c->misc, &c->tsizes};
  for (Buf* b : all) freebuf(*b);
  for (Buf& b : c->scr.chunks) freebuf(b);
  dec_free(c->dec);
  for (auto e : c->kev) (void)hipEventDestroy(e);
  if (c->pinned) (void)hipHostFree(c->pinned);
  if (c->own) (void)hipStreamDestroy(c->own);
  if (c->side.s) (void)hipStreamDestroy(c->side.s);
  if (c->side.fork) (void)hipEventDestroy(c->side.fork);
  if (c->side.join) (void)hipEventDestroy(c->side.join);
  delete c;
}

void hoh_set_profiling(hoh_ctx* c, int on) { if (c) c->profiling = on; }

void* hoh_ctx_stream(hoh_ctx* c) { return c ? (void*)c->own : nullptr; }

int hoh_ctx_set_option(hoh_ctx* c, int option, int64_t value) {
  if (!c) return HOH_E_ARG;
  switch (option) {
    case HOH_OPT_NOIX_DECODER:
      if (value < HOH_NOIX_ADAPTIVE || value > HOH_NOIX_WAVE) return HOH_E_ARG;
      c->noix = (int)value;
      return HOH_OK;
  }
  return HOH_E_ARG;
}

int hoh_get_kernel_ms(hoh_ctx* c, const char** names, float* ms, int max) {
  if (!c || c->nmark < 2) return 0;
  int k = 0;
  (void)hipEventSynchronize(c->kev[c->nmark - 1]);
  for (size_t i = 1; i < c->nmark && k < max; i++, k++) {
    float v = 0;
    (void)hipEventElapsedTime(&v, c->kev[i - 1], c->kev[i]);
    if (names) names[k] = c->knames[i].c_str();
    if (ms) ms[k] = v;
  }
  return k;
}

int hoh_get_kernel_stats(hoh_ctx* c, const char** names, double* total_ms, uint64_t* count, int max) {
  if (!c) return 0;
  prof_fold(c);
  int k = 0;
  for (; k < (int)c->snames.size() && k < max; k++) {
    if (names) names[k] = c->snames[k].c_str();
    if (total_ms) total_ms[k] = c->sms[k];
    if (count) count[k] = c->scount[k];
  }
  return k;
}

#ifdef HOH_DEBUG_READ
// debug builds only (make DEBUG_READ=1; not in include/, not in the product library): copy a
// workspace of the last encode to the host (0: the LZ match lists, 1: k_lz's segment walks)
extern "C" int hoh_debug_read(hoh_ctx* c, int which, void* dst, size_t bytes) {
  if (!c || !dst) return HOH_E_ARG;
  if (which == 2) {                    // the tail of the decoder's back-distance map buffer
    if (!c->dec.bufs[15] || bytes > c->dec.sizes[15]) return HOH_E_ARG;
    return hipMemcpy(dst, (const uint8_t*)c->dec.bufs[15] + c->dec.sizes[15] - bytes, bytes, hipMemcpyDeviceToHost) == hipSuccess
               ? HOH_OK : HOH_E_HIP;
  }
  // 3: k_lzsort's posting lists of the last -s1..-s4 encode (per entry key | fingerprint << 32, first-pass entries,
  // u16 ranks: tools/scripts/lzsort_check.py); 4: the fingerprints + tile pixel words (k_lzfp)
  // 5: the per-tile kernel counters of the last encode (EncodeJob::dbg, [tile][64] u32)
  // 6: the StreamInfo records of the last encode (tests/test_gpu_check_build.py: ladder bounds)
  const Buf& b = which == 0 ? c->matches : which == 3 ? c->lzs : which == 4 ? c->fpb : which == 5 ? c->dbg
               : which == 6 ? c->streams : c->lzspec;
  if (bytes > b.n || !b.p) return HOH_E_ARG;
  return hipMemcpy(dst, b.p, bytes, hipMemcpyDeviceToHost) == hipSuccess ? HOH_OK : HOH_E_HIP;
}
#endif

void hoh_reset_kernel_stats(hoh_ctx* c) {
  if (!c) return;
  prof_fold(c);
  c->snames.clear();
  c->sms.clear();
  c->scount.clear();
}

int hoh_tiling(int W, int H, int* xt, int* yt, int* tw, int* th) {
  if ((W >= 512 || H >= 512) && W >= 256 && H >= 256) {                 // choh.cpp:454-461
    *xt = W / 256; *yt = H / 256;
    *tw = (W + *xt - 1) / *xt; *th = (H + *yt - 1) / *yt;
    return 1;
  }
  *xt = *yt = 1; *tw = W; *th = H;
  return 0;
}

size_t hoh_encode_bound(int W, int H) {
  int xt, yt, tw, th;
  hoh_tiling(W, H, &xt, &yt, &tw, &th);
  return 64 + (size_t)xt * yt * 3 + 5 * (size_t)W * H + (size_t)xt * yt * 4096;
}

static size_t header_fixed(int W, int H, uint8_t* o) {
  size_t p = 0;
  o[p++] = 153; o[p++] = 72; o[p++] = 79; o[p++] = 72;                   // choh.cpp:437-440
  o[p++] = 2;                                                           // :443 rgb
  o[p++] = 8;                                                           // :446 depth
  p = hoh_write_varint(o, (uint32_t)p, (uint64_t)W - 1);                // :449-450
  p = hoh_write_varint(o, (uint32_t)p, (uint64_t)H - 1);
  return p;
}

size_t hoh_file_prefix(int W, int H, const uint32_t* ts, int nt, uint8_t* out, size_t cap) {
  int xt, yt, tw, th;
  if (!hoh_tiling(W, H, &xt, &yt, &tw, &th) || nt != xt * yt) return 0;
  std::vector<uint8_t> b(32 + 3 * (size_t)nt);
  size_t p = header_fixed(W, H, b.data());
  b[p++] = (uint8_t)(xt - 1);                                           // :457-458
  b[p++] = (uint8_t)(yt - 1);
  for (int i = 0; i + 1 < nt; i++) p = hoh_write_varint(b.data(), (uint32_t)p, ts[i]);   // :496-498
  if (p > cap) return 0;
  memcpy(out, b.data(), p);
  return p;
}

int hoh_peek_header(const uint8_t* h, size_t size, int* W, int* H, int* xt, int* yt) {
  if (!h || size < 8 || h[0] != 153 || h[1] != 72 || h[2] != 79 || h[3] != 72) return HOH_E_CORRUPT;
  if (h[4] != 2 || h[5] != 8) return HOH_E_UNSUPPORTED;
  size_t p = 6;
  auto rv = [&](uint64_t& v) -> bool {                                  // varint.hpp:6-27
    if (p >= size) return false;
    uint64_t b0 = h[p++];
    if (!(b0 & 0x80)) { v = b0; return true; }
    if (p >= size) return false;
    uint64_t b1 = h[p++];
    if (!(b1 & 0x80)) { v = ((b0 & 0x7f) << 7) + b1; return true; }
    if (p >= size) return false;
    uint64_t b2 = h[p++];
    v = ((b0 & 0x7f) << 14) + ((b1 & 0x7f) << 7) + b2;
    return true;
  };
  uint64_t w, hh;
  if (!rv(w) || !rv(hh)) return HOH_E_CORRUPT;
  *W = (int)w + 1; *H = (int)hh + 1;
  int tw, th, x, y;
  hoh_tiling(*W, *H, &x, &y, &tw, &th);
  if (xt) *xt = x;
  if (yt) *yt = y;
  return HOH_OK;
}

// ---------------------------------------------------------------- image encode

static void prof_cb(void* p, const char* name) { ((Prof*)p)->mark(name); }

// -log2(k / n) for k = 0..n+1 and every tile pixel count n of the image (layer_encode.hpp:143),
// computed once per image shape with the host's log2 so the -s>=1 search sees the reference's
// exact doubles
static int ensure_log2_tables(hoh_ctx* c, int W, int H, EncodeJob& j) {
  const int rw = W - (j.xt - 1) * j.tw, bh = H - (j.yt - 1) * j.th;
  uint32_t ns[4] = {(uint32_t)(j.tw * j.th), (uint32_t)(rw * j.th), (uint32_t)(j.tw * bh), (uint32_t)(rw * bh)};
  uint32_t un[4] = {0, 0, 0, 0};
  int nu = 0;
  for (int i = 0; i < 4; i++) {
    bool dup = false;
    for (int k = 0; k < nu; k++) dup |= un[k] == ns[i];
    if (!dup && ns[i]) un[nu++] = ns[i];
  }
  if (!(c->lg_key[0] == un[0] && c->lg_key[1] == un[1] && c->lg_key[2] == un[2] && c->lg_key[3] == un[3])) {
    std::vector<double> tab;
    for (int k = 0; k < nu; k++) {
      c->lg_off[k] = tab.size();
      for (uint32_t f = 0; f <= un[k] + 1; f++) tab.push_back(f ? -log2((double)f / (double)un[k]) : 0.0);
    }
    int e = ensure(c->lg, tab.size() * sizeof(double));
    if (e) return e;
    if (hipMemcpy(c->lg.p, tab.data(), tab.size() * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) return HOH_E_HIP;
    for (int k = 0; k < 4; k++) c->lg_key[k] = un[k];
  }
  j.lg = (const double*)c->lg.p;
  for (int k = 0; k < 4; k++) { j.lg_n[k] = c->lg_key[k]; j.lg_off[k] = c->lg_off[k]; }
  return HOH_OK;
}

// d_status == nullptr: synchronous (the host waits and maps the status word).  Otherwise
// enqueue-only: {status code, total bytes} are written to d_status by the stream.
static int encode_tiles_impl(hoh_ctx* c, const uint8_t* d_rgb, int W, int H, int t0, int ntiles,
                             uint8_t* d_out, size_t cap, uint64_t prefix, int write_table,
                             uint32_t* d_tile_sizes, uint64_t* total_out, hoh_index* idx,
                             hipStream_t s, int speed = 0, uint64_t* d_status = nullptr, int nimg = 1,
                             uint64_t out_stride = 0) {
  const bool async = d_status != nullptr;
  int xt, yt, tw, th;
  hoh_tiling(W, H, &xt, &yt, &tw, &th);
  if (tw > HOH_MAX_TILE_W || (size_t)tw * th > (1u << 24)) return HOH_E_UNSUPPORTED;
  // -s>=1: k_search keeps a tile's 40-px predictor grid (HOH_MAPCAP cells) in LDS and writes a
  // row's residuals four per thread; tiles are < 512 on a side, so only untiled images (one side
  // under 256, the other wider than ~1000) exceed either
  if (speed && ((size_t)((tw + 39) / 40) * ((th + 39) / 40) > HOH_MAPCAP || tw > 1024)) return HOH_E_UNSUPPORTED;
  if (t0 < 0 || ntiles <= 0 || t0 + ntiles > xt * yt) return HOH_E_ARG;
  Prof prof(c, s, async);
  EncodeJob j{};
  memset(&j, 0, sizeof(j));
  j.speed = speed;
  j.spt = speed ? SPT_S : SK_PER_TILE;
  j.rgb = d_rgb; j.W = W; j.H = H;
  j.xt = xt; j.yt = yt; j.tw = tw; j.th = th;
  j.t0 = t0; j.ntiles = ntiles;
  j.npix_cap = (uint32_t)rup((size_t)tw * th, HOH_SEG > 64 ? 64 : 64);
  j.lz_cap = (uint32_t)rup(j.npix_cap / 4 + j.npix_cap / 255 + 16, 8);
  j.gen_stride = 512;
  j.hdr_cap = HOH_HDR_CAP;
  const size_t S = (size_t)ntiles * j.spt;
  // the -s0 chains address every stream's table by a 32-bit offset from one base (k_rans_enc.hip;
  // the -s>=1 ones by 64-bit addresses)
  if (!speed && S * HOH_FAST_STRIDE * sizeof(EncFast) > 0xffffffffull) return HOH_E_UNSUPPORTED;
  // arenas: [tile][3] planes, [tile][3] LZ streams, [tile] indexed plane (hoh_internal.h); the
  // -s>=1 layout is in hoh_internal.h too
  size_t nsym = (size_t)ntiles * 3 * (j.npix_cap + j.lz_cap) + (size_t)ntiles * j.npix_cap;
  size_t nslab = (size_t)ntiles * 3 * (j.npix_cap + 8 + j.lz_cap + 8) + (size_t)ntiles * (j.npix_cap + 8);
  if (speed) {
    nsym = sym_total_s(ntiles, j.npix_cap, j.lz_cap);
    nslab = slab_total_s(ntiles, j.npix_cap, j.lz_cap);
    // the trial pool (EncodeJob::tpool_*): half a plane's words per plane -- a kept trial takes
    // its word bound (k_tables' whi), a compressed plane ~1/4 of that; when it runs out the
    // remaining trials count only and their winners are encoded again (same bytes)
    j.tpool_off = nslab;
    j.tpool_words = HOH_KNOB(TRIAL_POOL, 1) ? (size_t)ntiles * HOH_NPLANE_S * (j.npix_cap / 2) : 0;
    nslab += j.tpool_words;
  }
  const size_t nck = speed ? 1 : S * (j.npix_cap / HOH_SEG + 2);
  int e = HOH_OK;
  if (speed) {
    if ((e = ensure(c->idx8, (size_t)ntiles * j.npix_cap))) return e;
    if ((e = ensure(c->fpb, (size_t)ntiles * j.npix_cap * 13))) return e;   // fingerprints + pixels + transposed + runs
    if ((e = ensure(c->pinfo, (size_t)ntiles * HOH_NPLANE_S * (sizeof(PlaneInfo) + 8 * 4)))) return e;   // + trial list
    if ((e = ensure_log2_tables(c, W, H, j))) return e;
    j.idx8 = (uint8_t*)c->idx8.p;
    j.fpb = (uint32_t*)c->fpb.p;
    j.tpx = j.fpb + (size_t)ntiles * j.npix_cap;
    j.fpt = j.fpb + 2 * (size_t)ntiles * j.npix_cap;
    j.run8 = (uint8_t*)(j.fpb + 3 * (size_t)ntiles * j.npix_cap);
    j.lzs = nullptr;
    j.lzrank = nullptr;
    // posting lists for the LZ windows (-s1..-s4) of tiles whose positions fit 16 bits
    if (speed >= 1 && j.npix_cap <= 65536 && lz_posting()) {
      const size_t per = (size_t)ntiles * j.npix_cap;
      // [entries: 8 B][first-pass entries: 8 B][ranks: 2 B][run ends: 2 B] per position
      if ((e = ensure(c->lzs, per * 20))) return e;
      j.lzsf = (uint64_t*)c->lzs.p;
      j.lzs = (uint32_t*)(j.lzsf + per);
      j.lzrank = (uint16_t*)(j.lzsf + 2 * per);
      j.lzend = j.lzrank + per;
      j.lzs_hmask = (uint32_t)HOH_KNOB(LZS_HMASK, 0xffff);
      j.cus = c->cus;
    }
    j.pinfo = (PlaneInfo*)c->pinfo.p;
    j.trials = (uint32_t*)(j.pinfo + (size_t)ntiles * HOH_NPLANE_S);
  }
  if ((e = ensure(c->sym, nsym * 2 + 64))) return e;
  if ((e = ensure(c->hist, S * 512 * 4))) return e;
  if ((e = ensure(c->candbits, (size_t)ntiles * (j.npix_cap / 64) * 8))) return e;
  if ((e = ensure(c->matches, (size_t)ntiles * 3 * (j.lz_cap + 1) * 4))) return e;
  if ((e = ensure(c->lzspec, (size_t)ntiles * j.lz_cap * (speed ? 8 : 4)))) return e;   // k_lz / k_lzscan segments
  if ((e = ensure(c->pal, (size_t)ntiles * 257 * 4))) return e;   // palettes, then colour counts
  if ((e = ensure(c->streams, S * sizeof(StreamInfo)))) return e;
  if ((e = ensure(c->tiles, (size_t)ntiles * sizeof(TileInfo)))) return e;
  if ((e = ensure(c->hdr, S * HOH_HDR_CAP))) return e;
  if ((e = ensure(c->tab_fast, S * HOH_FAST_STRIDE * sizeof(EncFast)))) return e;
  if ((e = ensure(c->tab_gen, S * 512 * sizeof(EncGen)))) return e;
  if ((e = ensure(c->slabs, nslab * 4))) return e;
  if ((e = ensure(c->misc, 64 + (size_t)nimg * 16))) return e;   // gerr, total | batch: img_total[n], img_err[n]
  j.cus = c->cus;                 // grids that stride over the tiles (k_lzsort, k_nuke)
  j.sym = (uint16_t*)c->sym.p;
  j.hist = (uint32_t*)c->hist.p;
  j.candbits = (uint64_t*)c->candbits.p;
  j.matches = (uint32_t*)c->matches.p;
  j.lzspec = (uint32_t*)c->lzspec.p;
  j.palette = (uint32_t*)c->pal.p;
  j.ncol = (int32_t*)c->pal.p + (size_t)ntiles * 256;
  j.streams = (StreamInfo*)c->streams.p;
  j.tiles = (TileInfo*)c->tiles.p;
  j.hdr = (uint8_t*)c->hdr.p;
  j.tab_fast = (EncFast*)c->tab_fast.p;
  j.tab_wide = (size_t)S * HOH_FAST_STRIDE * sizeof(EncFast) > 0xffffffffull;
  j.tab_gen = (EncGen*)c->tab_gen.p;
  j.slabs = (uint32_t*)c->slabs.p;
  j.slab_words = nslab;
  // checkpoints are only kept for a side index, and the encoder writes them straight into it
  // (its layout is the index's: stream s at s * (npix_cap / HOH_SEG + 2)); -s>=1 files get none
  j.ckpt = nullptr;
  if (!speed && idx) {
    if ((e = index_reserve(idx, S, nck))) return e;
    j.ckpt = index_ckpt_buf(idx);
  }
#ifdef HOH_DEBUG_READ
  if ((e = ensure(c->dbg, (size_t)ntiles * 64 * 4))) return e;
  j.dbg = (uint32_t*)c->dbg.p;
  if (hipMemsetAsync(j.dbg, 0, (size_t)ntiles * 64 * 4, s) != hipSuccess) return HOH_E_HIP;
#endif
  j.exp = (uint32_t)HOH_KNOB(EXP, 0);   // measurement what-ifs (tools/scripts): 0 in the product
  j.gerr = (uint32_t*)c->misc.p;
  j.total = (uint64_t*)((uint8_t*)c->misc.p + 8);
  j.ntrial = (uint32_t*)((uint8_t*)c->misc.p + 16);
  j.tpool_head = (unsigned long long*)((uint8_t*)c->misc.p + 24);
  j.tile_sizes = d_tile_sizes;
  j.out = d_out;
  j.cap = cap;
  j.prefix = prefix;
  j.write_table = write_table;
  j.nimg = nimg;
  j.img_tiles = ntiles / nimg;
  j.out_stride = out_stride;
  j.img_total = (uint64_t*)((uint8_t*)c->misc.p + 64);
  j.img_err = (uint32_t*)(j.img_total + nimg);
  // at -s0 k_front writes every candidate word of every tile (k_lz reads no others)
  if (speed &&
      hipMemsetAsync(j.candbits, 0, (size_t)ntiles * (j.npix_cap / 64) * 8, s) != hipSuccess) return HOH_E_HIP;
  if (hipMemsetAsync(c->misc.p, 0, 64 + (size_t)nimg * 16, s) != hipSuccess) return HOH_E_HIP;
  prof.mark("memset");
  // knob ENC_STOP = k (measurement, -s0): the encode stops after stage k (1 front, 2 palette, 3 LZ
  // + nuke, 4 tables, 5 chains, 6 rANS generic + finalize, 7 layout + assembly); output invalid
  const int stop = HOH_KNOB(ENC_STOP, 0);
  launch_front(j, s);            prof.mark("front");
  if (stop != 1) launch_palette(j, s);
  prof.mark("palette");
  if (speed) {
    if (!c->side.s) {           // all three or none: a partial set is destroyed, never kept
      SideStream t;
      if (hipStreamCreateWithFlags(&t.s, hipStreamNonBlocking) != hipSuccess ||
          hipEventCreateWithFlags(&t.fork, hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&t.join, hipEventDisableTiming) != hipSuccess) {
        if (t.s) (void)hipStreamDestroy(t.s);
        if (t.fork) (void)hipEventDestroy(t.fork);
        if (t.join) (void)hipEventDestroy(t.join);
        return HOH_E_HIP;
      }
      c->side = t;
    }
    encode_speed_s(j, s, c->side, prof_cb, &prof);
    if (hipGetLastError() != hipSuccess) return HOH_E_HIP;
    idx = nullptr;
  } else {
    if (!stop || stop > 2) { launch_lz(j, s); launch_nuke(j, s); }
    prof.mark("lz");
    if (!stop || stop > 3) launch_tables(j, (int)S, s);
    prof.mark("tables");
    // the plane chains and the LZ streams (prob_bits 10) in one launch
    if (!stop || stop > 4)
      launch_rans_fast01(j, s, ntiles * 4, SidMap{3, SK_G}, ntiles * 3, SidMap{1, SK_I}, ntiles * 3, SidMap{3, 0},
                         ntiles * 3, SidMap{0, 0});
    prof.mark("rans_enc_fast");
    if (!stop || stop > 5) { launch_rans_gen(j, (int)S, s); launch_finalize(j, (int)S, s); }
    prof.mark("rans_enc_gen");
    prof.mark("finalize");
    if (!stop || stop > 6) { launch_layout(j, s); launch_assemble(j, (int)S, s); }
    prof.mark("layout");
    prof.mark("assemble");
    if (stop) idx = nullptr;
  }
  if (hipGetLastError() != hipSuccess) return HOH_E_HIP;
  if (idx) {
    int r = index_capture(idx, j, s);
    if (r) return r;
    prof.mark("index");
  }
  if (async) {
    if (nimg > 1) launch_status_enc_batch(j.gerr, j.img_total, j.img_err, out_stride, d_status, nimg, s);
    else launch_status_enc(j.gerr, j.total, cap, d_status, s);
    return hipGetLastError() == hipSuccess ? HOH_OK : HOH_E_HIP;
  }
  if (hipMemcpyAsync(c->pinned, c->misc.p, 16, hipMemcpyDeviceToHost, s) != hipSuccess) return HOH_E_HIP;
  if (hipStreamSynchronize(s) != hipSuccess) return HOH_E_HIP;
  const uint32_t gerr = (uint32_t)c->pinned[0];
  *total_out = c->pinned[1];
  if (gerr) {
    const uint32_t tf = gerr >> 8;
    if (tf & TF_UNREPRODUCIBLE) return HOH_E_UNREPRODUCIBLE;
    if (tf & TF_UNSUPPORTED) return HOH_E_UNSUPPORTED;
    if (gerr & 2) return HOH_E_RANGE;
    return HOH_E_HIP;
  }
  if (*total_out > cap) return HOH_E_CAP;
  return HOH_OK;
}

int hoh_encode_tiles(hoh_ctx* c, const uint8_t* d_rgb, int W, int H, int t0, int ntiles, uint8_t* d_out,
                     size_t cap, uint32_t* d_tile_sizes, size_t* out_size, void* stream) {
  return hoh_encode_tiles_ix(c, d_rgb, W, H, t0, ntiles, d_out, cap, d_tile_sizes, out_size, nullptr, stream);
}

int hoh_encode_tiles_ix(hoh_ctx* c, const uint8_t* d_rgb, int W, int H, int t0, int ntiles, uint8_t* d_out,
                        size_t cap, uint32_t* d_tile_sizes, size_t* out_size, hoh_index* idx, void* stream) {
  return hoh_encode_tiles_speed(c, d_rgb, W, H, 0, t0, ntiles, d_out, cap, d_tile_sizes, out_size, idx, stream);
}

int hoh_encode_tiles_speed(hoh_ctx* c, const uint8_t* d_rgb, int W, int H, int speed, int t0, int ntiles,
                           uint8_t* d_out, size_t cap, uint32_t* d_tile_sizes, size_t* out_size, hoh_index* idx,
                           void* stream) {
  if (!c || !d_rgb || !d_out || !out_size || W <= 0 || H <= 0 || speed < 0 || speed > 4) return HOH_E_ARG;
  if (speed && idx) idx->nstreams = 0;
  (void)hipSetDevice(c->device);
  int xt, yt, tw, th;
  if (!hoh_tiling(W, H, &xt, &yt, &tw, &th)) return HOH_E_ARG;
  uint64_t total = 0;
  int r = encode_tiles_impl(c, d_rgb, W, H, t0, ntiles, d_out, cap, 0, 0, d_tile_sizes, &total, speed ? nullptr : idx,
                            pick(c, stream), speed);
  *out_size = (size_t)total;
  return r;
}

int hoh_encode_tiles_async(hoh_ctx* c, const uint8_t* d_rgb, int W, int H, int speed, int t0, int ntiles,
                           uint8_t* d_out, size_t cap, uint32_t* d_tile_sizes, hoh_index* idx, uint64_t* d_status,
                           void* stream) {
  if (!c || !d_rgb || !d_out || !d_tile_sizes || !d_status || W <= 0 || H <= 0 || speed < 0 || speed > 4)
    return HOH_E_ARG;
  if (speed && idx) idx->nstreams = 0;
  (void)hipSetDevice(c->device);
  int xt, yt, tw, th;
  if (!hoh_tiling(W, H, &xt, &yt, &tw, &th)) return HOH_E_ARG;
  uint64_t total = 0;
  return encode_tiles_impl(c, d_rgb, W, H, t0, ntiles, d_out, cap, 0, 0, d_tile_sizes, &total, speed ? nullptr : idx,
                           pick(c, stream), speed, d_status);
}

// tiles per -s>=1 stack (measurement knob SPEED_STACK_TILES; ~8 MB of workspace per tile): 1024
// = one 8192^2 image, which fills the device alone (stacks of two measured 3-6 % slower in the
// pipelined speed legs, profiles/r06/speed_batches.txt); small images stack up to it
static int speed_stack() { return HOH_KNOB(SPEED_STACK_TILES, 1024); }

// n images' shards per call (choh.cpp:464-500's tile loop over a band of tile rows, run over a
// batch).  When the band is whole tile rows of 256 (H a multiple of 256), the n bands stacked in
// d_rgb are the tile grid of one W x (n * rows) image, so every kernel covers all n bands' tiles in
// one launch, exactly as hoh_encode_images_async stacks whole images; blob i gets its own layout
// (k_layout: one workgroup per band) at d_out + i * stride.  Otherwise the bands run one after
// another on the stream (same bytes).
int hoh_encode_tiles_images_async(hoh_ctx* c, int n, const uint8_t* d_rgb, int W, int H, int speed, int t0,
                                  int ntiles, uint8_t* d_out, size_t stride, uint32_t* d_tile_sizes, hoh_index* idx,
                                  uint64_t* d_status, void* stream) {
  if (!c || n <= 0 || !d_rgb || !d_out || !d_tile_sizes || !d_status || W <= 0 || H <= 0 || speed < 0 || speed > 4 ||
      stride == 0)
    return HOH_E_ARG;
  int xt, yt, tw, th;
  if (!hoh_tiling(W, H, &xt, &yt, &tw, &th)) return HOH_E_UNSUPPORTED;     // header-only files carry no tiles
  if (t0 < 0 || ntiles <= 0 || t0 + ntiles > xt * yt || t0 % xt || ntiles % xt) return HOH_E_ARG;
  const int y0 = (t0 / xt) * th, rows = std::min(H, (t0 + ntiles) / xt * th) - y0;
  const size_t band = (size_t)W * rows * 3;
  if (n == 1 || !batch_stacks(W, H)) {
    if (idx && n > 1 && !speed) return HOH_E_UNSUPPORTED;      // a side index holds one shard here
    for (int i = 0; i < n; i++) {
      const int r = hoh_encode_tiles_async(c, d_rgb + i * band - (size_t)y0 * W * 3, W, H, speed, t0, ntiles,
                                           d_out + i * stride, stride, d_tile_sizes + (size_t)i * ntiles, idx,
                                           d_status + 2 * i, stream);
      if (r) return r;
    }
    return HOH_OK;
  }
  if ((int64_t)rows * n > (1ll << 30) || (int64_t)ntiles * n > (1 << 24)) return HOH_E_ARG;
  (void)hipSetDevice(c->device);
  if (speed && idx) idx->nstreams = 0;                 // -s>=1 files get no side index
  // -s>=1 workspaces are ~8 MB per tile: stacks of at most speed_stack() tiles, one after another
  const int per = speed ? std::max(1, speed_stack() / ntiles) : n;
  for (int i0 = 0; i0 < n; i0 += per) {
    const int k = std::min(per, n - i0);
    uint64_t total = 0;
    const int r = k == 1 ? hoh_encode_tiles_async(c, d_rgb + i0 * band - (size_t)y0 * W * 3, W, H, speed, t0, ntiles,
                                                  d_out + i0 * stride, stride, d_tile_sizes + (size_t)i0 * ntiles,
                                                  nullptr, d_status + 2 * i0, stream)
                         : encode_tiles_impl(c, d_rgb + i0 * band, W, rows * k, 0, ntiles * k, d_out + i0 * stride,
                                             stride, 0, 0, d_tile_sizes + (size_t)i0 * ntiles, &total,
                                             speed ? nullptr : idx, pick(c, stream), speed, d_status + 2 * i0, k,
                                             stride);
    if (r) return r;
  }
  return HOH_OK;
}

int hoh_encode_image_ix(hoh_ctx* c, const uint8_t* d_rgb, int W, int H, int speed, uint8_t* d_out,
                        size_t cap, size_t* out_size, size_t* printed, hoh_index* idx, void* stream) {
  if (!c || !d_rgb || !d_out || !out_size || W <= 0 || H <= 0) return HOH_E_ARG;
  if (speed < 0 || speed > 4) return HOH_E_ARG;                         // choh.cpp:408-427
  (void)hipSetDevice(c->device);
  hipStream_t s = pick(c, stream);
  uint8_t hb[32];
  int xt, yt, tw, th;
  const int tiled = hoh_tiling(W, H, &xt, &yt, &tw, &th);
  size_t hl = header_fixed(W, H, hb);
  if (tiled) { hb[hl++] = (uint8_t)(xt - 1); hb[hl++] = (uint8_t)(yt - 1); }
  if (cap < hl) return HOH_E_CAP;
  uint64_t total = 0;
  int r;
  if (tiled) {
    launch_put_bytes(d_out, hb, (int)hl, s);      // the header, ahead of the tiles (one host sync per call)
    r = encode_tiles_impl(c, d_rgb, W, H, 0, xt * yt, d_out, cap, hl, 1, nullptr, &total, idx, s, speed);
    if (speed && idx) idx->nstreams = 0;
    *out_size = (size_t)total;
    if (printed) *printed = (size_t)total;
  } else {
    // choh.cpp:508-520: the single tile is coded and discarded; only the header is written (Q13)
    ScratchFrame f(c);
    const size_t b = hoh_encode_bound(W, H);
    uint8_t* scratch = f.get<uint8_t>(b);
    if (!scratch) return HOH_E_HIP;
    r = encode_tiles_impl(c, d_rgb, W, H, 0, 1, scratch, b, 0, 0, nullptr, &total, nullptr, s, speed);
    if (r == HOH_OK && hipMemcpyAsync(d_out, hb, hl, hipMemcpyHostToDevice, s) != hipSuccess) r = HOH_E_HIP;
    if (r == HOH_OK && hipStreamSynchronize(s) != hipSuccess) r = HOH_E_HIP;
    *out_size = hl;
    if (printed) *printed = hl + (size_t)total;
    if (idx) idx->nstreams = 0;
  }
  return r;
}

int hoh_encode_image_async(hoh_ctx* c, const uint8_t* d_rgb, int W, int H, int speed, uint8_t* d_out, size_t cap,
                           hoh_index* idx, uint64_t* d_status, void* stream) {
  if (!c || !d_rgb || !d_out || !d_status || W <= 0 || H <= 0 || speed < 0 || speed > 4) return HOH_E_ARG;
  (void)hipSetDevice(c->device);
  hipStream_t s = pick(c, stream);
  uint8_t hb[32];
  int xt, yt, tw, th;
  if (!hoh_tiling(W, H, &xt, &yt, &tw, &th)) return HOH_E_UNSUPPORTED;  // header-only files: use the sync call
  size_t hl = header_fixed(W, H, hb);
  hb[hl++] = (uint8_t)(xt - 1);
  hb[hl++] = (uint8_t)(yt - 1);
  if (cap < hl) return HOH_E_CAP;
  if (speed && idx) idx->nstreams = 0;
  launch_put_bytes(d_out, hb, (int)hl, s);
  uint64_t total = 0;
  return encode_tiles_impl(c, d_rgb, W, H, 0, xt * yt, d_out, cap, hl, 1, nullptr, &total, speed ? nullptr : idx, s,
                           speed, d_status);
}

int hoh_encode_images_async(hoh_ctx* c, int n, const uint8_t* d_rgb, int W, int H, int speed, uint8_t* d_out,
                            size_t stride, hoh_index* idx, uint64_t* d_status, void* stream) {
  if (!c || n <= 0 || !d_rgb || !d_out || !d_status || W <= 0 || H <= 0 || speed < 0 || speed > 4) return HOH_E_ARG;
  int xt, yt, tw, th;
  if (!hoh_tiling(W, H, &xt, &yt, &tw, &th)) return HOH_E_UNSUPPORTED;
  const size_t img_bytes = (size_t)W * H * 3;
  if (n == 1 || !batch_stacks(W, H)) {
    // one image after another on the stream (same bytes); a side index holds one image only
    if (idx && n > 1 && !speed) return HOH_E_UNSUPPORTED;
    for (int i = 0; i < n; i++) {
      const int r = hoh_encode_image_async(c, d_rgb + i * img_bytes, W, H, speed, d_out + i * stride, stride, idx,
                                           d_status + 2 * i, stream);
      if (r) return r;
    }
    return HOH_OK;
  }
  if ((int64_t)H * n > (1ll << 30) || (int64_t)xt * yt * n > (1 << 24)) return HOH_E_ARG;
  (void)hipSetDevice(c->device);
  hipStream_t s = pick(c, stream);
  uint8_t hb[32];
  size_t hl = header_fixed(W, H, hb);
  hb[hl++] = (uint8_t)(xt - 1);
  hb[hl++] = (uint8_t)(yt - 1);
  if (stride < hl) return HOH_E_CAP;
  launch_put_bytes(d_out, hb, (int)hl, s, n, stride);
  if (speed && idx) idx->nstreams = 0;                 // -s>=1 files get no side index
  // -s>=1 workspaces are ~8 MB per tile: stacks of at most speed_stack() tiles, one after another
  const int per = speed ? std::max(1, speed_stack() / (xt * yt)) : n;
  for (int i0 = 0; i0 < n; i0 += per) {
    const int k = std::min(per, n - i0);
    uint64_t total = 0;
    const int r = k == 1 ? encode_tiles_impl(c, d_rgb + i0 * img_bytes, W, H, 0, xt * yt, d_out + i0 * stride, stride,
                                             hl, 1, nullptr, &total, nullptr, s, speed, d_status + 2 * i0)
                         : encode_tiles_impl(c, d_rgb + i0 * img_bytes, W, H * k, 0, xt * yt * k, d_out + i0 * stride,
                                             stride, hl, 1, nullptr, &total, speed ? nullptr : idx, s, speed,
                                             d_status + 2 * i0, k, stride);
    if (r) return r;
  }
  return HOH_OK;
}

int hoh_encode_image(hoh_ctx* c, const uint8_t* d_rgb, int W, int H, int speed, uint8_t* d_out, size_t cap,
                     size_t* out_size, size_t* printed, void* stream) {
  return hoh_encode_image_ix(c, d_rgb, W, H, speed, d_out, cap, out_size, printed, nullptr, stream);
}

int hoh_synth_rgb(hoh_ctx* c, uint8_t* d_rgb, int W, int H, uint64_t seed, int noise, void* stream) {
  return hoh_synth_rgb_rows(c, d_rgb, W, 0, H, seed, noise, stream);
}

int hoh_synth_rgb_rows(hoh_ctx* c, uint8_t* d_rgb, int W, int y0, int rows, uint64_t seed, int noise, void* stream) {
  if (!c || !d_rgb || W <= 0 || rows <= 0 || y0 < 0 || noise < 0) return HOH_E_ARG;
  (void)hipSetDevice(c->device);
  hipStream_t s = pick(c, stream);
  launch_synth(d_rgb, W, rows, y0, seed, noise, s);
  if (hipGetLastError() != hipSuccess) return HOH_E_HIP;
  return hipStreamSynchronize(s) == hipSuccess ? HOH_OK : HOH_E_HIP;
}

int hoh_natural_rgb_rows(hoh_ctx* c, uint8_t* d_rgb, int W, int y0, int rows, uint64_t seed, void* stream) {
  if (!c || !d_rgb || W <= 0 || rows <= 0 || y0 < 0 || W >= (1 << 24) || y0 + rows >= (1 << 24)) return HOH_E_ARG;
  (void)hipSetDevice(c->device);
  hipStream_t s = pick(c, stream);
  launch_natural(d_rgb, W, rows, y0, seed, s);
  if (hipGetLastError() != hipSuccess) return HOH_E_HIP;
  return hipStreamSynchronize(s) == hipSuccess ? HOH_OK : HOH_E_HIP;
}

}  // extern "C"

// ---------------------------------------------------------------- entropy streams (batched)

// nstreams streams of d_syms (device), all with one range / prob_bits, written at
// d_out + out_off[i] (device).  Host arrays: off (symbol offsets, multiples of 8), cnt, out_off.
int encode_streams_impl(hoh_ctx* c, const uint16_t* d_syms, const uint64_t* off, const uint32_t* cnt, int nstreams,
                        uint32_t range, uint32_t pb, uint8_t* d_out, const uint64_t* out_off, uint32_t* sizes,
                        hipStream_t s) {
  if (range == 0 || range > 4096 || pb == 0 || pb > 31) return HOH_E_RANGE;
  if (nstreams <= 0) return HOH_E_ARG;
  uint32_t nmax = 0;
  for (int i = 0; i < nstreams; i++) { if (off[i] % 8) return HOH_E_ARG; nmax = cnt[i] > nmax ? cnt[i] : nmax; }
  const size_t per_ck = nmax / HOH_SEG + 2;
  const size_t slab = (size_t)nmax + 8;
  const uint32_t hcap = (uint32_t)rup(64 + (2 * 8 * 16 + (size_t)range * (pb > 16 ? pb : 16)) / 8 + 16, 16);
  int e;
  if ((e = ensure(c->streams, (size_t)nstreams * sizeof(StreamInfo)))) return e;
  if ((e = ensure(c->hdr, (size_t)nstreams * hcap))) return e;
  if ((e = ensure(c->tab_gen, (size_t)nstreams * range * sizeof(EncGen)))) return e;
  if ((e = ensure(c->slabs, (size_t)nstreams * slab * 4))) return e;
  if ((e = ensure(c->misc, 64))) return e;
  // prob_bits 7..19 with range <= 512 (every -s0 plane, config 2's single stream, the -s>=1
  // ladder) takes the tuned chain k_rans_fast (k_tables may still hand a stream back), the rest
  // the reference reciprocal step (k_rans_gen)
  const bool fast = pb >= 7 && pb <= 19 && range <= HOH_FAST_RANGE;
  if (fast && (e = ensure(c->tab_fast, (size_t)nstreams * HOH_FAST_STRIDE * sizeof(EncFast)))) return e;
  std::vector<StreamInfo> st((size_t)nstreams);
  for (int i = 0; i < nstreams; i++) {
    memset(&st[i], 0, sizeof(StreamInfo));
    st[i].sym_off = off[i];
    st[i].slab_off = (uint64_t)i * slab;
    st[i].slab_cap = (uint32_t)slab;
    st[i].out_off = out_off[i];
    st[i].n = cnt[i];
    st[i].range = range;
    st[i].pb = pb;
    st[i].ckpt_off = (uint32_t)((size_t)i * per_ck);
    st[i].mode = SM_EMPTY;
    st[i].fast = fast ? 1 : 0;
  }
  EncodeJob j{};
  memset(&j, 0, sizeof(j));
  j.sym = (uint16_t*)d_syms;
  j.streams = (StreamInfo*)c->streams.p;
  j.hdr = (uint8_t*)c->hdr.p;
  j.hdr_cap = hcap;
  j.tab_gen = (EncGen*)c->tab_gen.p;
  j.tab_fast = fast ? (EncFast*)c->tab_fast.p : nullptr;
  j.tab_wide = (size_t)nstreams * HOH_FAST_STRIDE * sizeof(EncFast) > 0xffffffffull;
  j.gen_stride = range;
  j.slabs = (uint32_t*)c->slabs.p;
  j.ckpt = nullptr;                           // stream-level decodes are serial: no checkpoints
  j.gerr = (uint32_t*)c->misc.p;
  j.total = (uint64_t*)((uint8_t*)c->misc.p + 8);
  j.out = d_out;
  j.cap = ~0ull;
  j.spt = 1;
  if (hipMemcpyAsync(c->streams.p, st.data(), st.size() * sizeof(StreamInfo), hipMemcpyHostToDevice, s) != hipSuccess) return HOH_E_HIP;
  if (hipMemsetAsync(c->misc.p, 0, 64, s) != hipSuccess) return HOH_E_HIP;
  launch_tables(j, nstreams, s);
  if (fast) launch_rans_fast(j, nstreams, s, SidMap{0, 0}, nstreams, SidMap{0, 0}, pb == 15 ? 0 : 1);
  launch_rans_gen(j, nstreams, s);            // skips the streams k_rans_fast coded
  launch_finalize(j, nstreams, s);
  launch_streambytes(j, nstreams, s);
  if (hipGetLastError() != hipSuccess) return HOH_E_HIP;
  if (hipMemcpyAsync(st.data(), c->streams.p, st.size() * sizeof(StreamInfo), hipMemcpyDeviceToHost, s) != hipSuccess) return HOH_E_HIP;
  if (hipMemcpyAsync(c->pinned, c->misc.p, 8, hipMemcpyDeviceToHost, s) != hipSuccess) return HOH_E_HIP;
  if (hipStreamSynchronize(s) != hipSuccess) return HOH_E_HIP;
  if (c->pinned[0] & 2) return HOH_E_RANGE;
  if (c->pinned[0]) return HOH_E_RANGE;
  for (int i = 0; i < nstreams; i++) {
    if (st[i].err) return HOH_E_RANGE;
    sizes[i] = st[i].size;
  }
  return HOH_OK;
}

extern "C" {

size_t hoh_entropy_bound(size_t n, size_t range, uint32_t pb) {
  return 64 + (2 * 8 * 17 + range * (pb > 16 ? pb : 16) + 7) / 8 + 4 * (n + 2) + (hoh_bitlen(range) * n + 7) / 8;
}

int hoh_encode_entropy_batch(hoh_ctx* c, const uint16_t* d_syms, const uint64_t* h_off, const uint32_t* h_cnt,
                             int nstreams, uint32_t range, uint32_t pb, uint8_t* d_out, const uint64_t* h_out_off,
                             uint32_t* h_sizes, void* stream) {
  if (!c || !d_syms || !h_off || !h_cnt || !d_out || !h_out_off || !h_sizes) return HOH_E_ARG;
  (void)hipSetDevice(c->device);
  return encode_streams_impl(c, d_syms, h_off, h_cnt, nstreams, range, pb, d_out, h_out_off, h_sizes, pick(c, stream));
}

int hoh_encode_entropy(hoh_ctx* c, const uint16_t* symbols, size_t n, size_t range, uint32_t pb, uint8_t* out,
                       size_t cap, size_t* written) {
  if (!c || (!symbols && n) || !out || !written) return HOH_E_ARG;
  if (n >= (1u << 31)) return HOH_E_ARG;
  (void)hipSetDevice(c->device);
  hipStream_t s = c->own;
  const size_t bound = hoh_entropy_bound(n, range, pb);
  ScratchFrame f(c);
  uint16_t* ds = f.get<uint16_t>(n * 2 + 16);
  uint8_t* dout = f.get<uint8_t>(bound);
  if (!ds || !dout) return HOH_E_HIP;
  int r = HOH_OK;
  if (n && hipMemcpyAsync(ds, symbols, n * 2, hipMemcpyHostToDevice, s) != hipSuccess) r = HOH_E_HIP;
  uint64_t off = 0, oo = 0;
  uint32_t cnt = (uint32_t)n, size = 0;
  if (!r) r = encode_streams_impl(c, ds, &off, &cnt, 1, (uint32_t)range, pb, dout, &oo, &size, s);
  if (!r) {
    *written = size;
    if (size > cap) r = HOH_E_CAP;
    else if (hipMemcpy(out, dout, size, hipMemcpyDeviceToHost) != hipSuccess) r = HOH_E_HIP;
  }
  return r;
}

// ---------------------------------------------------------------- host-entry scratch

ScratchFrame::ScratchFrame(hoh_ctx* ctx) : c(ctx), cur(ctx->scr.cur), used(ctx->scr.used) {}
ScratchFrame::~ScratchFrame() { c->scr.cur = cur; c->scr.used = used; }

void* ScratchFrame::alloc(size_t n) {
  Scratch& s = c->scr;
  n = rup(n ? n : 16, 256);
  for (;;) {
    if (s.cur == s.chunks.size()) s.chunks.push_back(Buf{});
    Buf& b = s.chunks[s.cur];
    if (s.used + n <= b.n) {
      void* p = (uint8_t*)b.p + s.used;
      s.used += n;
      return p;
    }
    if (s.used == 0) {
      // nothing of this chunk (nor of any later one) is live: grow it in place
      const size_t want = std::max(n, std::max(b.n * 2, (size_t)1 << 20));
      if (ensure(b, want) != HOH_OK) return nullptr;
      continue;
    }
    s.cur++;
    s.used = 0;
  }
}

// ---------------------------------------------------------------- decode side index

int hoh_index_create(hoh_index** idx) {
  if (!idx) return HOH_E_ARG;
  *idx = new hoh_index();
  return HOH_OK;
}

void hoh_index_destroy(hoh_index* idx) {
  if (!idx) return;
  freebuf(idx->ck);
  freebuf(idx->streams);
  delete idx;
}

size_t hoh_index_bytes(const hoh_index* idx) {
  return idx ? idx->ck_count * sizeof(Checkpoint) + (size_t)idx->nstreams * sizeof(IndexStream) : 0;
}

}  // extern "C"

// index capture: copy every plane stream's checkpoints + payload location (device to device)
int index_reserve(hoh_index* idx, size_t nstreams, size_t nck) {
  int e;
  if ((e = ensure(idx->streams, nstreams * sizeof(IndexStream)))) return e;
  return ensure(idx->ck, nck * sizeof(Checkpoint));
}
Checkpoint* index_ckpt_buf(hoh_index* idx) { return (Checkpoint*)idx->ck.p; }

// the encoder already wrote the checkpoints into the index (j.ckpt); record where each stream's
// payload sits in the file
int index_capture(hoh_index* idx, const EncodeJob& j, hipStream_t s) {
  const int S = j.ntiles * SK_PER_TILE;
  const size_t per = j.npix_cap / HOH_SEG + 2;
  int e;
  if ((e = index_reserve(idx, (size_t)S, (size_t)S * per))) return e;
  idx->nstreams = S;
  idx->ck_count = (size_t)S * per;
  idx->nimg = j.nimg > 1 ? j.nimg : 1;
  idx->stride = j.nimg > 1 ? j.out_stride : 0;
  launch_index_capture(j, (IndexStream*)idx->streams.p, per, s);
  return hipGetLastError() == hipSuccess ? HOH_OK : HOH_E_HIP;
}

const IndexStream* index_streams(const hoh_index* idx) { return idx ? (const IndexStream*)idx->streams.p : nullptr; }
int index_batch(const hoh_index* idx, uint64_t* stride) { if (stride) *stride = idx ? idx->stride : 0; return idx ? idx->nimg : 1; }
const Checkpoint* index_ckpts(const hoh_index* idx) { return idx ? (const Checkpoint*)idx->ck.p : nullptr; }
int index_nstreams(const hoh_index* idx) { return idx ? idx->nstreams : 0; }
DecWork& ctx_dec(hoh_ctx* c) { return c->dec; }
hipStream_t ctx_stream(hoh_ctx* c, void* s) { return pick(c, s); }
uint64_t* ctx_pinned(hoh_ctx* c) { return c->pinned; }
int ctx_device(hoh_ctx* c) { return c->device; }
int ctx_cus(hoh_ctx* c) { return c->cus; }
int ctx_noix(hoh_ctx* c) { return c->noix; }
void ctx_mark(hoh_ctx* c, hipStream_t s, const char* name, bool reset) { prof_mark(c, s, name, reset); }
