// C ABI of the plane-level -s>=1 functions (include/hoh_ans.h): channelpredict_section /
// channelpredict_all (prediction.hpp:46-229), unpredict_all with any predictor map
// (unprediction.hpp:6-91), layer_encode at cruncher_mode 1..4 (layer_encode.hpp:11-412) and
// decode_layer for predictor-map layers (layer_decode.hpp:128-278).  All compute runs in
// k_search.hip / k_plane.hip and the stream kernels; this file moves caller buffers, computes the
// entropy table with the host's log2 (the reference's exact doubles) and sequences the prob_bits
// ladder.
#include "hoh_dec.h"
#include "../../include/hoh_ans.h"

#include <math.h>
#include <string.h>
#include <vector>

int encode_streams_impl(hoh_ctx* c, const uint16_t* d_syms, const uint64_t* off, const uint32_t* cnt, int nstreams,
                        uint32_t range, uint32_t pb, uint8_t* d_out, const uint64_t* out_off, uint32_t* sizes,
                        hipStream_t s);
void launch_predict(const uint16_t* d, int w, int h, int depth, uint16_t* out, hipStream_t s);
void launch_compact(const uint16_t* in, const uint8_t* nuke, size_t n, uint16_t* out, uint64_t* count, hipStream_t s);
void launch_section_one(const uint16_t* D, int w, int h, int depth, int xt, int yt, int cx, int cy, uint32_t mask,
                        uint16_t* out, uint64_t* count, uint16_t* top, uint8_t* bp, hipStream_t s);
void launch_all_plane(const uint16_t* D, int w, int h, int depth, int xt, int yt, const uint16_t* map, uint16_t* out,
                      hipStream_t s);
void launch_unpredict_all(const uint16_t* res, uint64_t nres, const uint16_t* backref, int w, int h, int depth,
                          int xt, int yt, const uint16_t* map, uint16_t* out, uint16_t* top, uint8_t* bp,
                          uint32_t* err, hipStream_t s);
void launch_search_plane(const uint16_t* D, int w, int h, int depth, int xt, int yt, int npred, const double* ent,
                         double* cost, uint16_t* plist, uint8_t* pidx, hipStream_t s);
void launch_hist16(const uint16_t* in, uint64_t n, uint32_t* hist, hipStream_t s);

namespace {

// device buffer carved from the context's grow-only scratch (ScratchFrame, hoh_dec.h)
struct Dev {
  void* p = nullptr;
  Dev(ScratchFrame& f, size_t n) : p(f.alloc(n)) {}
  template <class T> T* as() { return (T*)p; }
};

const uint16_t kMasksH[14] = {0x0001, 0x0002, 0x0020, 0x0010, 0xffbf, 0x0003, 0xfffd,
                              0xfffb, 0xfff7, 0xffef, 0xffdf, 0xff7f, 0xfdff, 0xffff};   // layer_encode.hpp:159-175

// -log2((1 + count) / n) from a device histogram (layer_encode.hpp:133-147), uploaded
int entropy_table(const uint16_t* d_res, size_t n, int range, double* d_ent, uint32_t* d_hist, hipStream_t s) {
  if (hipMemsetAsync(d_hist, 0, (size_t)range * 4, s) != hipSuccess) return HOH_E_HIP;
  launch_hist16(d_res, n, d_hist, s);
  std::vector<uint32_t> h(range);
  if (hipMemcpyAsync(h.data(), d_hist, (size_t)range * 4, hipMemcpyDeviceToHost, s) != hipSuccess) return HOH_E_HIP;
  if (hipStreamSynchronize(s) != hipSuccess) return HOH_E_HIP;
  std::vector<double> e(range);
  for (int i = 0; i < range; i++) e[i] = -log2((double)(1 + h[i]) / (double)n);
  if (hipMemcpyAsync(d_ent, e.data(), (size_t)range * 8, hipMemcpyHostToDevice, s) != hipSuccess) return HOH_E_HIP;
  return HOH_OK;
}

// one entropy stream of n device symbols -> host bytes
int encode_one(hoh_ctx* c, const uint16_t* d_sym, uint32_t n, uint32_t range, uint32_t pb, std::vector<uint8_t>& out,
               hipStream_t s) {
  const size_t bound = hoh_entropy_bound(n, range, pb);
  ScratchFrame sf(c);
  Dev d(sf, bound);
  if (!d.p) return HOH_E_HIP;
  uint64_t off = 0, oo = 0;
  uint32_t sz = 0;
  int r = encode_streams_impl(c, d_sym, &off, &n, 1, range, pb, d.as<uint8_t>(), &oo, &sz, s);
  if (r) return r;
  out.resize(sz);
  if (sz && hipMemcpy(out.data(), d.p, sz, hipMemcpyDeviceToHost) != hipSuccess) return HOH_E_HIP;
  return HOH_OK;
}

}  // namespace

// layer_encode.hpp:11-412 at cruncher_mode >= 1 (called by hoh_layer_encode)
int layer_encode_search(hoh_ctx* c, const uint16_t* data, size_t n, int w, int h, int depth, int cruncher,
                        const uint8_t* nuke, uint8_t* out, size_t cap, size_t* written) {
  hipStream_t s = ctx_stream(c, nullptr);
  const int range = 1 << depth;
  ScratchFrame sf(c);
  Dev dd(sf, n * 2 + 16), dres(sf, n * 2 + 16), dcl(sf, n * 2 + 16), dnk(sf, nuke ? n : 16), dcnt(sf, 16), dhist(sf, (size_t)range * 4),
      dent(sf, (size_t)range * 8);
  if (!dd.p || !dres.p || !dcl.p || !dnk.p || !dcnt.p || !dhist.p || !dent.p) return HOH_E_HIP;
  if (hipMemcpyAsync(dd.p, data, n * 2, hipMemcpyHostToDevice, s) != hipSuccess) return HOH_E_HIP;
  if (nuke && hipMemcpyAsync(dnk.p, nuke, n, hipMemcpyHostToDevice, s) != hipSuccess) return HOH_E_HIP;
  auto clean = [&](uint32_t& nc) -> int {                              // :93-99, :327-333
    launch_compact(dres.as<uint16_t>(), nuke ? dnk.as<uint8_t>() : nullptr, n, dcl.as<uint16_t>(), dcnt.as<uint64_t>(), s);
    uint64_t v = 0;
    if (hipMemcpyAsync(&v, dcnt.p, 8, hipMemcpyDeviceToHost, s) != hipSuccess) return HOH_E_HIP;
    if (hipStreamSynchronize(s) != hipSuccess) return HOH_E_HIP;
    nc = (uint32_t)v;
    return HOH_OK;
  };
  std::vector<uint8_t> hdr{0x10};                                     // :57
  size_t possible = ((size_t)depth * n + ((size_t)depth * n) % 8 + 1024) / 8;   // :22
  std::vector<uint8_t> perm, tmp;
  bool valid = false;
  launch_predict(dd.as<uint16_t>(), w, h, depth, dres.as<uint16_t>(), s);      // :63-75 (fast path)
  uint32_t nc = 0;
  int r = clean(nc);
  if (r) return r;
  if ((r = encode_one(c, dcl.as<uint16_t>(), nc, range, 15, tmp, s))) return r;   // :106-113
  if (tmp.size() < possible) { possible = tmp.size(); perm.swap(tmp); valid = true; }
  const int xt = (w + 39) / 40, yt = (h + 39) / 40;
  if (xt > 1 || yt > 1) {                                             // :124-319
    const int T = xt * yt, npred = cruncher * 5 < 14 ? cruncher * 5 : 14;
    ScratchFrame sf_cells(c);
    Dev dcost(sf_cells, (size_t)T * 14 * 8), dpl(sf_cells, (size_t)T * 2), dpi(sf_cells, (size_t)T), dmap(sf_cells, (size_t)T * 2 + 16);
    if (!dcost.p || !dpl.p || !dpi.p || !dmap.p) return HOH_E_HIP;
    for (int pass = 0; pass < (cruncher > 2 ? 2 : 1); pass++) {
      if ((r = entropy_table(dres.as<uint16_t>(), n, range, dent.as<double>(), dhist.as<uint32_t>(), s))) return r;
      launch_search_plane(dd.as<uint16_t>(), w, h, depth, xt, yt, npred, dent.as<double>(), dcost.as<double>(),
                          dpl.as<uint16_t>(), dpi.as<uint8_t>(), s);
      launch_all_plane(dd.as<uint16_t>(), w, h, depth, xt, yt, dpl.as<uint16_t>(), dres.as<uint16_t>(), s);
    }
    std::vector<uint8_t> pidx((size_t)T);
    if (hipMemcpyAsync(pidx.data(), dpi.p, (size_t)T, hipMemcpyDeviceToHost, s) != hipSuccess) return HOH_E_HIP;
    if (hipStreamSynchronize(s) != hipSuccess) return HOH_E_HIP;
    hdr.push_back((uint8_t)(xt - 1));                                 // :276-277
    hdr.push_back((uint8_t)(yt - 1));
    int used[14] = {0}, nused = 0, rank[14] = {0};
    for (int i = 0; i < T; i++) used[pidx[i]] = 1;
    for (int m = 0; m < 14; m++) if (used[m]) { rank[m] = nused++; }
    hdr.push_back((uint8_t)nused);                                    // :291-297
    for (int m = 0; m < 14; m++) if (used[m]) { hdr.push_back((uint8_t)(kMasksH[m] >> 8)); hdr.push_back((uint8_t)(kMasksH[m] & 255)); }
    std::vector<uint16_t> mp((size_t)T);
    for (int i = 0; i < T; i++) mp[i] = (uint16_t)rank[pidx[i]];
    if (hipMemcpyAsync(dmap.p, mp.data(), (size_t)T * 2, hipMemcpyHostToDevice, s) != hipSuccess) return HOH_E_HIP;
    std::vector<uint8_t> ms;
    if ((r = encode_one(c, dmap.as<uint16_t>(), (uint32_t)T, (uint32_t)nused, 8, ms, s))) return r;   // :308-317
    hdr.insert(hdr.end(), ms.begin(), ms.end());
  } else {
    const uint8_t f[4] = {0, 0, 0x00, 0x10};                          // :320-325
    hdr.insert(hdr.end(), f, f + 4);
  }
  if ((r = clean(nc))) return r;                                      // :326-392
  std::vector<uint8_t> t1, t2;
  if ((r = encode_one(c, dcl.as<uint16_t>(), nc, range, 16, t1, s))) return r;
  if ((r = encode_one(c, dcl.as<uint16_t>(), nc, range, 15, t2, s))) return r;
  const bool up = t1.size() < t2.size();
  const size_t t12 = up ? t1.size() : t2.size();
  if (t12 < possible) possible = t12;                                 // not swapped (Q14)
  for (int k = 0; k < 3; k++) {
    const uint32_t pb = up ? 17 + k : 14 - k;
    if ((r = encode_one(c, dcl.as<uint16_t>(), nc, range, pb, tmp, s))) return r;
    if (tmp.size() < possible) { possible = tmp.size(); perm.swap(tmp); valid = true; }
  }
  if (!valid) return HOH_E_UNREPRODUCIBLE;                            // permanent never written
  *written = hdr.size() + possible;
  if (*written > cap) return HOH_E_CAP;
  memcpy(out, hdr.data(), hdr.size());
  memcpy(out + hdr.size(), perm.data(), possible);                   // :396-398 (prefix, Q14)
  return HOH_OK;
}

extern "C" {

int hoh_predict_section(hoh_ctx* c, const uint16_t* data, int w, int h, int depth, int xt, int yt, int cx, int cy,
                        uint16_t mask, uint16_t* out, size_t* count) {
  if (!c || !data || !out || !count || w <= 0 || h <= 0 || xt <= 0 || yt <= 0 || depth < 1 || depth > 15) return HOH_E_ARG;
  const int tw = (w + xt - 1) / xt, th = (h + yt - 1) / yt;
  if (cx < 0 || cy < 0 || cx * tw >= w || cy * th >= h) return HOH_E_ARG;
  (void)hipSetDevice(ctx_device(c));
  hipStream_t s = ctx_stream(c, nullptr);
  if (mask == 0x0010 && xt == 1 && yt == 1) {                          // prediction.hpp:59-68
    *count = (size_t)w * h;
    return hoh_predict_fastpath(c, data, w, h, depth, out);
  }
  const size_t n = (size_t)w * h;
  ScratchFrame sf(c);
  Dev dd(sf, n * 2), dout(sf, (size_t)tw * th * 2), dc(sf, 16), dtop(sf, (size_t)tw * 2), dbp(sf, (size_t)tw);
  if (!dd.p || !dout.p || !dc.p || !dtop.p || !dbp.p) return HOH_E_HIP;
  if (hipMemcpyAsync(dd.p, data, n * 2, hipMemcpyHostToDevice, s) != hipSuccess) return HOH_E_HIP;
  launch_section_one(dd.as<uint16_t>(), w, h, depth, xt, yt, cx, cy, mask, dout.as<uint16_t>(), dc.as<uint64_t>(),
                     dtop.as<uint16_t>(), dbp.as<uint8_t>(), s);
  uint64_t k = 0;
  if (hipMemcpyAsync(&k, dc.p, 8, hipMemcpyDeviceToHost, s) != hipSuccess) return HOH_E_HIP;
  if (hipStreamSynchronize(s) != hipSuccess) return HOH_E_HIP;
  *count = (size_t)k;
  return hipMemcpy(out, dout.p, k * 2, hipMemcpyDeviceToHost) == hipSuccess ? HOH_OK : HOH_E_HIP;
}

int hoh_predict_all(hoh_ctx* c, const uint16_t* data, int w, int h, int depth, int xt, int yt,
                    const uint16_t* tile_map, uint16_t* out) {
  if (!c || !data || !tile_map || !out || w <= 0 || h <= 0 || xt <= 0 || yt <= 0 || depth < 1 || depth > 15) return HOH_E_ARG;
  (void)hipSetDevice(ctx_device(c));
  hipStream_t s = ctx_stream(c, nullptr);
  const size_t n = (size_t)w * h, nm = (size_t)xt * yt;
  ScratchFrame sf(c);
  Dev dd(sf, n * 2), dout(sf, n * 2), dm(sf, nm * 2);
  if (!dd.p || !dout.p || !dm.p) return HOH_E_HIP;
  if (hipMemcpyAsync(dd.p, data, n * 2, hipMemcpyHostToDevice, s) != hipSuccess) return HOH_E_HIP;
  if (hipMemcpyAsync(dm.p, tile_map, nm * 2, hipMemcpyHostToDevice, s) != hipSuccess) return HOH_E_HIP;
  launch_all_plane(dd.as<uint16_t>(), w, h, depth, xt, yt, dm.as<uint16_t>(), dout.as<uint16_t>(), s);
  if (hipStreamSynchronize(s) != hipSuccess) return HOH_E_HIP;
  return hipMemcpy(out, dout.p, n * 2, hipMemcpyDeviceToHost) == hipSuccess ? HOH_OK : HOH_E_HIP;
}

int hoh_unpredict_all(hoh_ctx* c, const uint16_t* res, size_t nres, const uint16_t* backref, int w, int h, int depth,
                      int xt, int yt, const uint16_t* tile_map, uint16_t* out) {
  if (!c || !res || !tile_map || !out || w <= 0 || h <= 0 || xt <= 0 || yt <= 0 || depth < 1 || depth > 15) return HOH_E_ARG;
  if (xt == 1 && yt == 1 && tile_map[0] == 0x0010)                     // -s0 layers: MED on every row (Q9 fixed)
    return hoh_unpredict_fastpath(c, res, nres, backref, w, h, depth, out);
  (void)hipSetDevice(ctx_device(c));
  hipStream_t s = ctx_stream(c, nullptr);
  const size_t n = (size_t)w * h, nm = (size_t)xt * yt;
  ScratchFrame sf(c);
  Dev dr(sf, nres * 2 + 16), db(sf, backref ? n * 2 : 16), dout(sf, n * 2), dm(sf, nm * 2), dtop(sf, (size_t)w * 2), dbp(sf, (size_t)w), de(sf, 16);
  if (!dr.p || !db.p || !dout.p || !dm.p || !dtop.p || !dbp.p || !de.p) return HOH_E_HIP;
  if (nres && hipMemcpyAsync(dr.p, res, nres * 2, hipMemcpyHostToDevice, s) != hipSuccess) return HOH_E_HIP;
  if (backref && hipMemcpyAsync(db.p, backref, n * 2, hipMemcpyHostToDevice, s) != hipSuccess) return HOH_E_HIP;
  if (hipMemcpyAsync(dm.p, tile_map, nm * 2, hipMemcpyHostToDevice, s) != hipSuccess) return HOH_E_HIP;
  launch_unpredict_all(dr.as<uint16_t>(), nres, backref ? db.as<uint16_t>() : nullptr, w, h, depth, xt, yt,
                       dm.as<uint16_t>(), dout.as<uint16_t>(), dtop.as<uint16_t>(), dbp.as<uint8_t>(), de.as<uint32_t>(), s);
  uint32_t err = 1;
  if (hipMemcpyAsync(&err, de.p, 4, hipMemcpyDeviceToHost, s) != hipSuccess) return HOH_E_HIP;
  if (hipStreamSynchronize(s) != hipSuccess) return HOH_E_HIP;
  if (err) return HOH_E_CORRUPT;
  return hipMemcpy(out, dout.p, n * 2, hipMemcpyDeviceToHost) == hipSuccess ? HOH_OK : HOH_E_HIP;
}

}  // extern "C"
