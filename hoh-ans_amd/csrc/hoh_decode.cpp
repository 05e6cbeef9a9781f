// C ABI: decoders and the plane-level entry points (include/hoh_ans.h).  Compute runs in
// k_decode.hip / k_plane.hip; host code here only moves caller buffers and checks framing bytes.
#include "hoh_dec.h"
#include "../../include/hoh_ans.h"

#include <string.h>
#include <vector>

int decode_image_impl(hoh_ctx* c, const uint8_t* d_in, size_t size, uint8_t* d_rgb, size_t cap, int* Wp, int* Hp,
                      const hoh_index* idx, hipStream_t s);
int decode_image_async_impl(hoh_ctx* c, const uint8_t* d_in, size_t size, int W, int H, uint8_t* d_rgb, size_t cap,
                            const hoh_index* idx, uint64_t* d_status, hipStream_t s);
int decode_images_async_impl(hoh_ctx* c, int n, const uint8_t* d_in, size_t stride, int W, int H, uint8_t* d_rgb,
                             const hoh_index* idx, uint64_t* d_status, hipStream_t s);
int decode_tiles_impl(hoh_ctx* c, const uint8_t* d_blob, size_t size, int W, int H, int t0, int ntiles,
                      const uint32_t* h_sizes, uint8_t* d_rgb, const hoh_index* idx, hipStream_t s);
int decode_tiles_async_impl(hoh_ctx* c, const uint8_t* d_blob, size_t size, int W, int H, int t0, int ntiles,
                            const uint32_t* d_sizes, uint8_t* d_rgb, const hoh_index* idx, uint64_t* d_status,
                            hipStream_t s);
int decode_tiles_images_async_impl(hoh_ctx* c, int n, const uint8_t* d_blob, size_t stride, int W, int H, int t0,
                                   int ntiles, const uint32_t* d_sizes, uint8_t* d_rgb, const hoh_index* idx,
                                   uint64_t* d_status, hipStream_t s);
int decode_stream_impl(hoh_ctx* c, const uint8_t* d_in, size_t size, size_t* bp, uint16_t* d_out, size_t cap,
                       size_t* n, hipStream_t s);
int encode_streams_impl(hoh_ctx* c, const uint16_t* d_syms, const uint64_t* off, const uint32_t* cnt, int nstreams,
                        uint32_t range, uint32_t pb, uint8_t* d_out, const uint64_t* out_off, uint32_t* sizes,
                        hipStream_t s);
void launch_predict(const uint16_t* d, int w, int h, int depth, uint16_t* out, hipStream_t s);
void launch_unpredict_serial(const uint16_t* res, size_t nres, const uint16_t* br, int w, int h, int depth,
                             uint16_t* o, uint32_t* err, hipStream_t s);
void launch_green(const uint8_t* rgb, size_t n, uint16_t* G, uint16_t* R, uint16_t* B, hipStream_t s);
void launch_addgreen(const uint16_t* G, const uint16_t* R, const uint16_t* B, size_t n, uint8_t* o, hipStream_t s);
void launch_compact(const uint16_t* in, const uint8_t* nuke, size_t n, uint16_t* out, uint64_t* count, hipStream_t s);
int layer_encode_search(hoh_ctx* c, const uint16_t* data, size_t n, int w, int h, int depth, int cruncher,
                        const uint8_t* nuke, uint8_t* out, size_t cap, size_t* written);

namespace {

// device buffer of a host-buffer entry point, carved from the context's grow-only scratch
// (ScratchFrame, hoh_dec.h): no device allocation once the context has seen the call's shape
struct DevMem {
  void* p = nullptr;
  DevMem(ScratchFrame& f, size_t n) : p(f.alloc(n)) {}
  template <class T> T* as() { return (T*)p; }
};

uint64_t rdv(const uint8_t* b, size_t size, size_t& p, bool& ok) {   // varint.hpp:6-27
  if (p >= size) { ok = false; return 0; }
  uint64_t b0 = b[p++];
  if (!(b0 & 0x80)) return b0;
  if (p >= size) { ok = false; return 0; }
  uint64_t b1 = b[p++];
  if (!(b1 & 0x80)) return ((b0 & 0x7f) << 7) + b1;
  if (p >= size) { ok = false; return 0; }
  uint64_t b2 = b[p++];
  return ((b0 & 0x7f) << 14) + ((b1 & 0x7f) << 7) + b2;
}

}  // namespace

extern "C" {

int hoh_decode_image_ix(hoh_ctx* c, const uint8_t* d_hoh, size_t size, uint8_t* d_rgb, size_t cap, int* W, int* H,
                        const hoh_index* idx, void* stream) {
  if (!c || !d_hoh || !d_rgb || !W || !H) return HOH_E_ARG;
  (void)hipSetDevice(ctx_device(c));
  return decode_image_impl(c, d_hoh, size, d_rgb, cap, W, H, idx, ctx_stream(c, stream));
}

int hoh_decode_image_async(hoh_ctx* c, const uint8_t* d_hoh, size_t size, int W, int H, uint8_t* d_rgb, size_t cap,
                           const hoh_index* idx, uint64_t* d_status, void* stream) {
  if (!c || !d_hoh || !d_rgb || !d_status || W <= 0 || H <= 0) return HOH_E_ARG;
  (void)hipSetDevice(ctx_device(c));
  return decode_image_async_impl(c, d_hoh, size, W, H, d_rgb, cap, idx, d_status, ctx_stream(c, stream));
}

int hoh_decode_images_async(hoh_ctx* c, int n, const uint8_t* d_hoh, size_t stride, int W, int H, uint8_t* d_rgb,
                            const hoh_index* idx, uint64_t* d_status, void* stream) {
  if (!c || n <= 0 || !d_hoh || !d_rgb || !d_status || W <= 0 || H <= 0 || stride == 0) return HOH_E_ARG;
  (void)hipSetDevice(ctx_device(c));
  return decode_images_async_impl(c, n, d_hoh, stride, W, H, d_rgb, idx, d_status, ctx_stream(c, stream));
}

int hoh_decode_tiles(hoh_ctx* c, const uint8_t* d_blob, size_t size, int W, int H, int t0, int ntiles,
                     const uint32_t* h_tile_sizes, uint8_t* d_rgb, const hoh_index* idx, void* stream) {
  if (!c || !d_blob || !d_rgb || !h_tile_sizes || W <= 0 || H <= 0) return HOH_E_ARG;
  (void)hipSetDevice(ctx_device(c));
  return decode_tiles_impl(c, d_blob, size, W, H, t0, ntiles, h_tile_sizes, d_rgb, idx, ctx_stream(c, stream));
}

int hoh_decode_tiles_async(hoh_ctx* c, const uint8_t* d_blob, size_t size, int W, int H, int t0, int ntiles,
                           const uint32_t* d_tile_sizes, uint8_t* d_rgb, const hoh_index* idx, uint64_t* d_status,
                           void* stream) {
  if (!c || !d_blob || !d_rgb || !d_tile_sizes || !d_status || W <= 0 || H <= 0) return HOH_E_ARG;
  (void)hipSetDevice(ctx_device(c));
  return decode_tiles_async_impl(c, d_blob, size, W, H, t0, ntiles, d_tile_sizes, d_rgb, idx, d_status,
                                 ctx_stream(c, stream));
}

int hoh_decode_tiles_images_async(hoh_ctx* c, int n, const uint8_t* d_blob, size_t stride, int W, int H, int t0,
                                  int ntiles, const uint32_t* d_tile_sizes, uint8_t* d_rgb, const hoh_index* idx,
                                  uint64_t* d_status, void* stream) {
  if (!c || n <= 0 || !d_blob || !d_rgb || !d_tile_sizes || !d_status || W <= 0 || H <= 0 || stride == 0)
    return HOH_E_ARG;
  (void)hipSetDevice(ctx_device(c));
  return decode_tiles_images_async_impl(c, n, d_blob, stride, W, H, t0, ntiles, d_tile_sizes, d_rgb, idx, d_status,
                                        ctx_stream(c, stream));
}

int hoh_decode_image(hoh_ctx* c, const uint8_t* d_hoh, size_t size, uint8_t* d_rgb, size_t cap, int* W, int* H,
                     void* stream) {
  return hoh_decode_image_ix(c, d_hoh, size, d_rgb, cap, W, H, nullptr, stream);
}

int hoh_entropy_count(const uint8_t* in, size_t in_size, size_t bp, size_t* n) {
  if (!in || !n) return HOH_E_ARG;
  bool ok = true;
  (void)rdv(in, in_size, bp, ok);
  *n = (size_t)rdv(in, in_size, bp, ok);
  return ok ? HOH_OK : HOH_E_CORRUPT;
}

// Framing walk of one stream (entropy_decoding.hpp:143-154 header, :174-250 table field widths,
// :256 payload size; stored streams :278-290), no symbol decoding: the bit fields are counted,
// not read.  Field reads start on a fresh byte (slag_bits = 0), so a run of b bits takes
// ceil(b / 8) bytes.
int hoh_entropy_parse(const uint8_t* in, size_t in_size, size_t bp, hoh_entropy_header* h) {
  if (!in || !h) return HOH_E_ARG;
  bool ok = true;
  size_t p = bp;
  const uint64_t range = rdv(in, in_size, p, ok) + 1;
  const uint64_t count = rdv(in, in_size, p, ok);
  if (!ok) return HOH_E_CORRUPT;
  uint32_t mb = 0;
  for (uint64_t v = range - 1; v; v >>= 1) mb++;
  *h = hoh_entropy_header{};
  h->range = range;
  h->count = count;
  h->symbol_bits = mb;
  if (count == 0) {                                                    // header only (entropy_encoding.hpp:19-23)
    h->table_end = h->stream_end = p;
    return HOH_OK;
  }
  if (p >= in_size) return HOH_E_CORRUPT;
  const uint8_t meta = in[p++];
  h->entropy_mode = meta >> 7;
  h->prob_bits = (meta & 0x3c) >> 2;
  h->table_mode = meta & 3;
  if (!h->entropy_mode) {                                              // stored (:278-290)
    h->table_end = p;
    h->payload_bytes = (count * mb + 7) / 8;
    h->stream_end = p + h->payload_bytes;
    return h->stream_end <= in_size ? HOH_OK : HOH_E_CORRUPT;
  }
  uint64_t bits = 0;
  if (h->table_mode == 1) {
    bits = range * mb;                                                 // raw widths (:180-195)
  } else if (h->table_mode == 2) {                                     // clamped widths (:196-244)
    const uint32_t pb = h->prob_bits;
    const int nclamp = ((int)pb - 1) / 4 + 2;
    std::vector<uint32_t> lo(nclamp), hi(nclamp);
    uint64_t q = (uint64_t)p * 8;                                      // bit cursor
    auto field = [&](uint32_t w) -> uint32_t {
      uint32_t v = 0;
      for (uint32_t i = 0; i < w; i++, q++) {
        if (q / 8 >= in_size) { ok = false; return 0; }
        v = (v << 1) | ((in[q / 8] >> (7 - q % 8)) & 1);
      }
      return v;
    };
    for (int i = 0; i < nclamp; i++) { lo[i] = field(mb); hi[i] = field(mb); }
    if (ok && lo[0] == hi[0] && lo[0] < range) {
      // single-symbol table: one field of the widest class, whose 2^pb value overflowed it
      //  -- recognised as the GPU decoder does (k_dparse)
      const uint32_t w = nclamp >= 3 ? 4 * (nclamp - 1) : 4;
      bits += w > pb ? pb : w;
    } else
    for (uint64_t i = 0; i < range && ok; i++) {
      uint32_t w = 0;
      if (lo[0] <= i && hi[0] >= i) w = 1;
      if (lo[1] <= i && hi[1] >= i) w = 4;
      for (int j = 2; j < nclamp; j++)
        if (lo[j] <= i && hi[j] >= i) w = 4 * j;
      bits += w > pb ? pb : w;
    }
    if (!ok) return HOH_E_CORRUPT;
    bits += (uint64_t)2 * nclamp * mb;
  } else if (h->table_mode == 3) {
    return HOH_E_CORRUPT;                                              // unimplemented there (:245-247)
  }
  p += (size_t)((bits + 7) / 8);
  h->table_end = p;
  if (p > in_size) return HOH_E_CORRUPT;
  h->payload_bytes = rdv(in, in_size, p, ok);
  h->stream_end = p + h->payload_bytes;
  return ok && h->stream_end <= in_size ? HOH_OK : HOH_E_CORRUPT;
}

int hoh_decode_entropy(hoh_ctx* c, const uint8_t* in, size_t in_size, size_t* bp, uint16_t* out, size_t cap,
                       size_t* n) {
  if (!c || !in || !bp || !n || *bp >= in_size) return HOH_E_ARG;
  (void)hipSetDevice(ctx_device(c));
  hipStream_t s = ctx_stream(c, nullptr);
  size_t cnt = 0;
  int r = hoh_entropy_count(in, in_size, *bp, &cnt);
  if (r) return r;
  if (cnt > cap) return HOH_E_CAP;
  ScratchFrame sf(c);
  DevMem din(sf, in_size + 8), dout(sf, cnt * 2 + 16);
  if (!din.p || !dout.p) return HOH_E_HIP;
  if (hipMemcpy(din.p, in, in_size, hipMemcpyHostToDevice) != hipSuccess) return HOH_E_HIP;
  if (hipMemset((uint8_t*)din.p + in_size, 0, 8) != hipSuccess) return HOH_E_HIP;
  size_t p = *bp, m = 0;
  r = decode_stream_impl(c, din.as<uint8_t>(), in_size, &p, dout.as<uint16_t>(), cnt, &m, s);
  if (r) return r;
  if (m && hipMemcpy(out, dout.p, m * 2, hipMemcpyDeviceToHost) != hipSuccess) return HOH_E_HIP;
  *n = m;
  *bp = p;
  return HOH_OK;
}

int hoh_predict_fastpath(hoh_ctx* c, const uint16_t* data, int w, int h, int depth, uint16_t* out) {
  if (!c || !data || !out || w <= 0 || h <= 0 || depth < 1 || depth > 15) return HOH_E_ARG;
  (void)hipSetDevice(ctx_device(c));
  hipStream_t s = ctx_stream(c, nullptr);
  const size_t n = (size_t)w * h;
  ScratchFrame sf(c);
  DevMem a(sf, n * 2), b(sf, n * 2);
  if (!a.p || !b.p) return HOH_E_HIP;
  if (hipMemcpyAsync(a.p, data, n * 2, hipMemcpyHostToDevice, s) != hipSuccess) return HOH_E_HIP;
  launch_predict(a.as<uint16_t>(), w, h, depth, b.as<uint16_t>(), s);
  if (hipMemcpyAsync(out, b.p, n * 2, hipMemcpyDeviceToHost, s) != hipSuccess) return HOH_E_HIP;
  return hipStreamSynchronize(s) == hipSuccess ? HOH_OK : HOH_E_HIP;
}

int hoh_unpredict_fastpath(hoh_ctx* c, const uint16_t* res, size_t nres, const uint16_t* backref, int w, int h,
                           int depth, uint16_t* out) {
  if (!c || (!res && nres) || !out || w <= 0 || h <= 0 || depth < 1 || depth > 15) return HOH_E_ARG;
  (void)hipSetDevice(ctx_device(c));
  hipStream_t s = ctx_stream(c, nullptr);
  const size_t n = (size_t)w * h;
  ScratchFrame sf(c);
  DevMem dr(sf, nres * 2), db(sf, backref ? n * 2 : 16), dout(sf, n * 2), de(sf, 16);
  if (!dr.p || !db.p || !dout.p || !de.p) return HOH_E_HIP;
  if (nres && hipMemcpyAsync(dr.p, res, nres * 2, hipMemcpyHostToDevice, s) != hipSuccess) return HOH_E_HIP;
  if (backref && hipMemcpyAsync(db.p, backref, n * 2, hipMemcpyHostToDevice, s) != hipSuccess) return HOH_E_HIP;
  launch_unpredict_serial(dr.as<uint16_t>(), nres, backref ? db.as<uint16_t>() : nullptr, w, h, depth,
                          dout.as<uint16_t>(), de.as<uint32_t>(), s);
  uint32_t err = 1;
  if (hipMemcpyAsync(&err, de.p, 4, hipMemcpyDeviceToHost, s) != hipSuccess) return HOH_E_HIP;
  if (hipMemcpyAsync(out, dout.p, n * 2, hipMemcpyDeviceToHost, s) != hipSuccess) return HOH_E_HIP;
  if (hipStreamSynchronize(s) != hipSuccess) return HOH_E_HIP;
  return err ? HOH_E_CORRUPT : HOH_OK;
}

int hoh_subtract_green(hoh_ctx* c, const uint8_t* rgb, size_t npix, uint16_t* G, uint16_t* R, uint16_t* B) {
  if (!c || !rgb || !G || !R || !B) return HOH_E_ARG;
  (void)hipSetDevice(ctx_device(c));
  hipStream_t s = ctx_stream(c, nullptr);
  ScratchFrame sf(c);
  DevMem a(sf, npix * 3), g(sf, npix * 2), r(sf, npix * 2), b(sf, npix * 2);
  if (!a.p || !g.p || !r.p || !b.p) return HOH_E_HIP;
  if (hipMemcpyAsync(a.p, rgb, npix * 3, hipMemcpyHostToDevice, s) != hipSuccess) return HOH_E_HIP;
  launch_green(a.as<uint8_t>(), npix, g.as<uint16_t>(), r.as<uint16_t>(), b.as<uint16_t>(), s);
  if (hipMemcpyAsync(G, g.p, npix * 2, hipMemcpyDeviceToHost, s) != hipSuccess) return HOH_E_HIP;
  if (hipMemcpyAsync(R, r.p, npix * 2, hipMemcpyDeviceToHost, s) != hipSuccess) return HOH_E_HIP;
  if (hipMemcpyAsync(B, b.p, npix * 2, hipMemcpyDeviceToHost, s) != hipSuccess) return HOH_E_HIP;
  return hipStreamSynchronize(s) == hipSuccess ? HOH_OK : HOH_E_HIP;
}

int hoh_add_green(hoh_ctx* c, const uint16_t* G, const uint16_t* R, const uint16_t* B, size_t npix, uint8_t* rgb) {
  if (!c || !rgb || !G || !R || !B) return HOH_E_ARG;
  (void)hipSetDevice(ctx_device(c));
  hipStream_t s = ctx_stream(c, nullptr);
  ScratchFrame sf(c);
  DevMem a(sf, npix * 3), g(sf, npix * 2), r(sf, npix * 2), b(sf, npix * 2);
  if (!a.p || !g.p || !r.p || !b.p) return HOH_E_HIP;
  if (hipMemcpyAsync(g.p, G, npix * 2, hipMemcpyHostToDevice, s) != hipSuccess) return HOH_E_HIP;
  if (hipMemcpyAsync(r.p, R, npix * 2, hipMemcpyHostToDevice, s) != hipSuccess) return HOH_E_HIP;
  if (hipMemcpyAsync(b.p, B, npix * 2, hipMemcpyHostToDevice, s) != hipSuccess) return HOH_E_HIP;
  launch_addgreen(g.as<uint16_t>(), r.as<uint16_t>(), b.as<uint16_t>(), npix, a.as<uint8_t>(), s);
  if (hipMemcpyAsync(rgb, a.p, npix * 3, hipMemcpyDeviceToHost, s) != hipSuccess) return HOH_E_HIP;
  return hipStreamSynchronize(s) == hipSuccess ? HOH_OK : HOH_E_HIP;
}

// layer_encode.hpp:11-412 at cruncher_mode 0: 0x10, 00 00 00 10, entropy(cleaned MED residuals)
int hoh_layer_encode(hoh_ctx* c, const uint16_t* data, size_t size, int w, int h, int depth, size_t cruncher,
                     const uint8_t* nuke, uint8_t* out, size_t cap, size_t* written) {
  if (!c || !data || !out || !written || w <= 0 || h <= 0 || (size_t)w * h != size || depth < 1 || depth > 12)
    return HOH_E_ARG;
  (void)hipSetDevice(ctx_device(c));
  if (cruncher > 4) return HOH_E_ARG;
  if (cruncher != 0) return layer_encode_search(c, data, size, w, h, depth, (int)cruncher, nuke, out, cap, written);
  hipStream_t s = ctx_stream(c, nullptr);
  const size_t bound = hoh_entropy_bound(size, (size_t)1 << depth, 15);
  ScratchFrame sf(c);
  DevMem a(sf, size * 2), res(sf, size * 2 + 16), cl(sf, size * 2 + 16), nk(sf, nuke ? size : 16), cnt(sf, 16), eout(sf, bound);
  if (!a.p || !res.p || !cl.p || !nk.p || !cnt.p || !eout.p) return HOH_E_HIP;
  if (hipMemcpyAsync(a.p, data, size * 2, hipMemcpyHostToDevice, s) != hipSuccess) return HOH_E_HIP;
  if (nuke && hipMemcpyAsync(nk.p, nuke, size, hipMemcpyHostToDevice, s) != hipSuccess) return HOH_E_HIP;
  launch_predict(a.as<uint16_t>(), w, h, depth, res.as<uint16_t>(), s);
  launch_compact(res.as<uint16_t>(), nuke ? nk.as<uint8_t>() : nullptr, size, cl.as<uint16_t>(), cnt.as<uint64_t>(), s);
  uint64_t nc = 0;
  if (hipMemcpyAsync(&nc, cnt.p, 8, hipMemcpyDeviceToHost, s) != hipSuccess) return HOH_E_HIP;
  if (hipStreamSynchronize(s) != hipSuccess) return HOH_E_HIP;
  uint64_t off = 0, oo = 0;
  uint32_t n32 = (uint32_t)nc, sz = 0;
  int r = encode_streams_impl(c, cl.as<uint16_t>(), &off, &n32, 1, 1u << depth, 15, eout.as<uint8_t>(), &oo, &sz, s);
  if (r) return r;
  const size_t possible = ((size_t)depth * size + ((size_t)depth * size) % 8 + 1024) / 8;   // :22
  if (sz >= possible) return HOH_E_UNREPRODUCIBLE;                     // :115-120 keeps garbage
  *written = 5 + (size_t)sz;
  if (*written > cap) return HOH_E_CAP;
  const uint8_t hdr[5] = {0x10, 0, 0, 0x00, 0x10};                    // :57, :320-325
  memcpy(out, hdr, 5);
  if (hipMemcpy(out + 5, eout.p, sz, hipMemcpyDeviceToHost) != hipSuccess) return HOH_E_HIP;
  return HOH_OK;
}

// layer_decode.hpp:128-278; returns the full-depth plane (no u8 truncation, Q10).  Layers with a
// predictor map (-s>=1) go through the general unpredict_all; the 1x1 MED map of -s0 layers through
// the fast path with MED on every row (Q9 fixed).
int hoh_layer_decode(hoh_ctx* c, const uint8_t* in, size_t in_size, size_t bp, int w, int h, int depth,
                     const uint16_t* backref, uint16_t* out) {
  if (!c || !in || !out || w <= 0 || h <= 0 || bp + 1 > in_size) return HOH_E_ARG;
  const uint8_t tr = in[bp];
  if (tr & 0xe0) return HOH_E_UNSUPPORTED;                             // compaction modes 1-7 (:141-195)
  size_t p = bp + 1, cnt = 0, n = 0;
  int r;
  auto stream = [&](std::vector<uint16_t>& v) -> int {
    int e = hoh_entropy_count(in, in_size, p, &cnt);
    if (e) return e;
    v.resize(cnt + 1);
    return hoh_decode_entropy(c, in, in_size, &p, v.data(), cnt, &n);
  };
  std::vector<uint16_t> res;
  if (!(tr & 0x10)) {                                                  // no prediction (:265-276)
    if ((r = stream(res))) return r;
    if (n != (size_t)w * h) return HOH_E_CORRUPT;
    memcpy(out, res.data(), n * 2);
    return HOH_OK;
  }
  if (p + 2 > in_size) return HOH_E_CORRUPT;
  const int xt = in[p] + 1, yt = in[p + 1] + 1;                        // :198-199
  p += 2;
  std::vector<uint16_t> map((size_t)xt * yt);
  if (xt == 1 && yt == 1) {                                            // :203-209
    if (p + 2 > in_size) return HOH_E_CORRUPT;
    map[0] = (uint16_t)((in[p] << 8) | in[p + 1]);
    p += 2;
  } else {                                                             // :210-229
    if (p + 1 > in_size) return HOH_E_CORRUPT;
    const int used = in[p++];
    if (p + 2 * (size_t)used > in_size) return HOH_E_CORRUPT;
    std::vector<uint16_t> comb(used);
    for (int i = 0; i < used; i++, p += 2) comb[i] = (uint16_t)((in[p] << 8) | in[p + 1]);
    std::vector<uint16_t> sym;
    if ((r = stream(sym))) return r;
    if (n != map.size()) return HOH_E_CORRUPT;
    for (size_t i = 0; i < n; i++) {
      if (sym[i] >= used) return HOH_E_CORRUPT;
      map[i] = comb[sym[i]];
    }
  }
  if ((r = stream(res))) return r;
  return hoh_unpredict_all(c, res.data(), n, backref, w, h, depth, xt, yt, map.data(), out);
}

}  // extern "C"
