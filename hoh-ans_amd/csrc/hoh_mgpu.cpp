// Multi-GPU choh / dhoh in ONE process (include/hoh_ans.h, hoh_mgpu_*): tiles are independent
// (choh.cpp:464-500), so device r owns a contiguous band of tile rows, encodes it into a blob
// (hoh_encode_tiles_speed on its own context), and one RCCL group of point-to-point transfers over
// xGMI puts every blob behind the header + tile table (hoh_file_prefix, choh.cpp:437-498) in the
// file on the first device: byte-identical to a one-GPU encode.  Decode is the mirror: the tile
// table is parsed on the host (dhoh.cpp:42-65), one RCCL group sends each device its tiles'
// bytes, each device decodes its band (hoh_decode_tiles) and copies its rows to the host image.
//
// RCCL (librccl.so, the communicators of ncclCommInitAll) is loaded at hoh_mgpu_create, so
// single-GPU users of libhohgpu need no RCCL.  When a device appears twice in the list (several
// shards on one GPU -- the way to exercise the gather on a one-GPU machine) RCCL cannot build a
// communicator and the blobs move by device copies instead; the bytes are the same.  The same
// peer-copy transport serves distinct devices when librccl is absent or ncclCommInitAll fails.
#include "hoh_internal.h"
#include "../../include/hoh_ans.h"
#include <rccl/rccl.h>

#include <dlfcn.h>
#include <string.h>
#include <thread>
#include <vector>

namespace {

struct Rccl {
  void* h = nullptr;
  ncclResult_t (*init_all)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;

  bool load() {
    if (h) return true;
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
      h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (h) break;
    }
    if (!h) return false;
    init_all = (decltype(init_all))dlsym(h, "ncclCommInitAll");
    destroy = (decltype(destroy))dlsym(h, "ncclCommDestroy");
    group_start = (decltype(group_start))dlsym(h, "ncclGroupStart");
    group_end = (decltype(group_end))dlsym(h, "ncclGroupEnd");
    send = (decltype(send))dlsym(h, "ncclSend");
    recv = (decltype(recv))dlsym(h, "ncclRecv");
    return init_all && destroy && group_start && group_end && send && recv;
  }
};

Rccl g_rccl;

struct DBuf {
  void* p = nullptr;
  size_t n = 0;
  int grow(size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (n >= bytes) return HOH_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    if (hipMalloc(&p, bytes) != hipSuccess) return HOH_E_HIP;
    n = bytes;
    return HOH_OK;
  }
};

}  // namespace

struct hoh_mgpu {
  int n = 0;
  std::vector<int> dev;
  std::vector<hoh_ctx*> ctx;
  std::vector<hipStream_t> st;
  std::vector<ncclComm_t> comm;   // empty: device copies (a device listed twice)
  std::vector<DBuf> rgb, blob, sizes, drgb;
};

// band of tile rows of device r (the same split as hoh_ans/dist.py: shard)
static void band(int yt, int xt, int r, int n, int* t0, int* nt) {
  const int r0 = r * yt / n, r1 = (r + 1) * yt / n;
  *t0 = r0 * xt;
  *nt = (r1 - r0) * xt;
}

extern "C" {

int hoh_mgpu_create(hoh_mgpu** out, int ndev, const int* devices) {
  if (!out || ndev <= 0 || !devices) return HOH_E_ARG;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return HOH_E_NODEV;
  for (int r = 0; r < ndev; r++)
    if (devices[r] < 0 || devices[r] >= count) return HOH_E_NODEV;
  hoh_mgpu* m = new hoh_mgpu();
  m->n = ndev;
  m->dev.assign(devices, devices + ndev);
  m->ctx.assign(ndev, nullptr);
  m->st.assign(ndev, nullptr);
  m->rgb.resize(ndev); m->blob.resize(ndev); m->sizes.resize(ndev); m->drgb.resize(ndev);
  int e = HOH_OK;
  for (int r = 0; r < ndev && !e; r++) {
    e = hoh_ctx_create(&m->ctx[r], devices[r]);
    if (!e && hipStreamCreateWithFlags(&m->st[r], hipStreamNonBlocking) != hipSuccess) e = HOH_E_HIP;
  }
  bool distinct = true;
  for (int a = 0; a < ndev; a++)
    for (int b = a + 1; b < ndev; b++) distinct &= devices[a] != devices[b];
  // distinct devices: one RCCL communicator each; without librccl, or when ncclCommInitAll
  // fails, the blobs move by peer copies instead (transport 0) -- the bytes are the same
  if (!e && distinct && g_rccl.load()) {
    m->comm.assign(ndev, nullptr);
    if (g_rccl.init_all(m->comm.data(), ndev, devices) != ncclSuccess) m->comm.clear();
  }
  if (e) { hoh_mgpu_destroy(m); return e; }
  *out = m;
  return HOH_OK;
}

void hoh_mgpu_destroy(hoh_mgpu* m) {
  if (!m) return;
  for (auto c : m->comm) if (c) (void)g_rccl.destroy(c);
  for (int r = 0; r < m->n; r++) {
    (void)hipSetDevice(m->dev[r]);
    for (DBuf* b : {&m->rgb[r], &m->blob[r], &m->sizes[r], &m->drgb[r]}) if (b->p) (void)hipFree(b->p);
    if (m->st[r]) (void)hipStreamDestroy(m->st[r]);
    if (m->ctx[r]) hoh_ctx_destroy(m->ctx[r]);
  }
  delete m;
}

int hoh_mgpu_transport(const hoh_mgpu* m) { return m && !m->comm.empty() ? 1 : 0; }

// every device's stream drained: an error return after transfers were enqueued must not leave
// them running into buffers the next call (or hoh_mgpu_destroy) reuses
static int drain(hoh_mgpu* m, int e) {
  for (int r = 0; r < m->n; r++) {
    (void)hipSetDevice(m->dev[r]);
    if (hipStreamSynchronize(m->st[r]) != hipSuccess && !e) e = HOH_E_HIP;
  }
  return e;
}

int hoh_mgpu_encode_image(hoh_mgpu* m, const uint8_t* h_rgb, int W, int H, int speed, uint8_t* d_out, size_t cap,
                          size_t* out_size, size_t* printed) {
  if (!m || !h_rgb || !d_out || !out_size || W <= 0 || H <= 0 || speed < 0 || speed > 4) return HOH_E_ARG;
  int xt, yt, tw, th;
  if (!hoh_tiling(W, H, &xt, &yt, &tw, &th) || yt < m->n) {
    // untiled (header-only) or fewer tile rows than devices: the first device alone
    (void)hipSetDevice(m->dev[0]);
    int e;
    if ((e = m->rgb[0].grow((size_t)W * H * 3))) return e;
    if (hipMemcpy(m->rgb[0].p, h_rgb, (size_t)W * H * 3, hipMemcpyHostToDevice) != hipSuccess) return HOH_E_HIP;
    return hoh_encode_image(m->ctx[0], (const uint8_t*)m->rgb[0].p, W, H, speed, d_out, cap, out_size, printed,
                            m->st[0]);
  }
  const int n = m->n;
  std::vector<int> t0(n), nt(n), y0(n), rows(n), err(n, HOH_OK);
  std::vector<size_t> bsz(n, 0);
  std::vector<std::vector<uint32_t>> ts(n);
  for (int r = 0; r < n; r++) {
    band(yt, xt, r, n, &t0[r], &nt[r]);
    y0[r] = (t0[r] / xt) * th;
    rows[r] = std::min(H, (t0[r] + nt[r]) / xt * th) - y0[r];
  }
  // each device: its rows in, its tiles out (a host thread per device: the calls synchronise)
  auto work = [&](int r) {
    (void)hipSetDevice(m->dev[r]);
    const size_t raw = (size_t)W * rows[r] * 3;
    const size_t bcap = hoh_encode_bound(W, rows[r]);
    int e;
    if ((e = m->rgb[r].grow(raw)) || (e = m->blob[r].grow(bcap)) || (e = m->sizes[r].grow((size_t)nt[r] * 4))) {
      err[r] = e;
      return;
    }
    if (hipMemcpyAsync(m->rgb[r].p, h_rgb + (size_t)y0[r] * W * 3, raw, hipMemcpyHostToDevice, m->st[r]) != hipSuccess) {
      err[r] = HOH_E_HIP;
      return;
    }
    const uint8_t* base = (const uint8_t*)m->rgb[r].p - (size_t)y0[r] * W * 3;
    e = hoh_encode_tiles_speed(m->ctx[r], base, W, H, speed, t0[r], nt[r], (uint8_t*)m->blob[r].p, bcap,
                               (uint32_t*)m->sizes[r].p, &bsz[r], nullptr, m->st[r]);
    if (!e) {
      ts[r].resize(nt[r]);
      if (hipMemcpy(ts[r].data(), m->sizes[r].p, (size_t)nt[r] * 4, hipMemcpyDeviceToHost) != hipSuccess) e = HOH_E_HIP;
    }
    err[r] = e;
  };
  {
    std::vector<std::thread> th;
    for (int r = 1; r < n; r++) th.emplace_back(work, r);
    work(0);
    for (auto& t : th) t.join();
  }
  for (int r = 0; r < n; r++) if (err[r]) return drain(m, err[r]);
  // the file: prefix, then the blobs in device order (tile order)
  std::vector<uint32_t> all;
  for (int r = 0; r < n; r++) all.insert(all.end(), ts[r].begin(), ts[r].end());
  std::vector<uint8_t> prefix(64 + 3 * all.size());
  const size_t pl = hoh_file_prefix(W, H, all.data(), (int)all.size(), prefix.data(), prefix.size());
  if (!pl) return HOH_E_ARG;
  std::vector<size_t> off(n + 1, pl);
  for (int r = 0; r < n; r++) off[r + 1] = off[r] + bsz[r];
  *out_size = off[n];
  if (printed) *printed = off[n];
  if (off[n] > cap) return HOH_E_CAP;
  (void)hipSetDevice(m->dev[0]);
  // the prefix (a few KB, host vector) synchronously: nothing else touches those bytes
  if (hipMemcpy(d_out, prefix.data(), pl, hipMemcpyHostToDevice) != hipSuccess) return HOH_E_HIP;
  if (bsz[0] && hipMemcpyAsync(d_out + off[0], m->blob[0].p, bsz[0], hipMemcpyDeviceToDevice, m->st[0]) != hipSuccess)
    return drain(m, HOH_E_HIP);
  if (!m->comm.empty()) {
    if (g_rccl.group_start() != ncclSuccess) return drain(m, HOH_E_HIP);
    ncclResult_t rr = ncclSuccess;
    for (int r = 1; r < n && rr == ncclSuccess; r++) {
      if (!bsz[r]) continue;
      rr = g_rccl.send(m->blob[r].p, bsz[r], ncclUint8, 0, m->comm[r], m->st[r]);
      if (rr == ncclSuccess) rr = g_rccl.recv(d_out + off[r], bsz[r], ncclUint8, r, m->comm[0], m->st[0]);
    }
    if (g_rccl.group_end() != ncclSuccess || rr != ncclSuccess) return drain(m, HOH_E_HIP);
  } else {
    for (int r = 1; r < n; r++)
      if (bsz[r] && hipMemcpyPeerAsync(d_out + off[r], m->dev[0], m->blob[r].p, m->dev[r], bsz[r], m->st[0]) != hipSuccess)
        return drain(m, HOH_E_HIP);
  }
  return drain(m, HOH_OK);
}

int hoh_mgpu_decode_image(hoh_mgpu* m, const uint8_t* d_hoh, size_t size, uint8_t* h_rgb, size_t cap, int* Wp,
                          int* Hp) {
  if (!m || !d_hoh || !h_rgb || !Wp || !Hp) return HOH_E_ARG;
  // header + tile table on the host (dhoh.cpp:297-366): at most 16 + 3 bytes per tile
  (void)hipSetDevice(m->dev[0]);
  std::vector<uint8_t> hb(std::min<size_t>(size, 64));
  if (hipMemcpy(hb.data(), d_hoh, hb.size(), hipMemcpyDeviceToHost) != hipSuccess) return HOH_E_HIP;
  int W, H, xt, yt;
  int e = hoh_peek_header(hb.data(), hb.size(), &W, &H, &xt, &yt);
  if (e) return e;
  *Wp = W;
  *Hp = H;
  if ((size_t)W * H * 3 > cap) return HOH_E_CAP;
  int txt, tyt, tw, th;
  if (!hoh_tiling(W, H, &txt, &tyt, &tw, &th) || tyt < m->n) {
    int e2;
    if ((e2 = m->drgb[0].grow((size_t)W * H * 3))) return e2;
    int w2, h2;
    e2 = hoh_decode_image(m->ctx[0], d_hoh, size, (uint8_t*)m->drgb[0].p, (size_t)W * H * 3, &w2, &h2, m->st[0]);
    if (e2) return e2;
    return hipMemcpy(h_rgb, m->drgb[0].p, (size_t)W * H * 3, hipMemcpyDeviceToHost) == hipSuccess ? HOH_OK : HOH_E_HIP;
  }
  const int ntiles = xt * yt;
  const size_t tcap = std::min<size_t>(size, 64 + 3 * (size_t)ntiles);
  std::vector<uint8_t> tb(tcap);
  if (hipMemcpy(tb.data(), d_hoh, tcap, hipMemcpyDeviceToHost) != hipSuccess) return HOH_E_HIP;
  size_t p = 6;
  auto rv = [&](uint64_t& v) -> bool {                                  // varint.hpp:6-27
    if (p >= tcap) return false;
    uint64_t b0 = tb[p++];
    if (!(b0 & 0x80)) { v = b0; return true; }
    if (p >= tcap) return false;
    uint64_t b1 = tb[p++];
    if (!(b1 & 0x80)) { v = ((b0 & 0x7f) << 7) + b1; return true; }
    if (p >= tcap) return false;
    v = ((b0 & 0x7f) << 14) + ((b1 & 0x7f) << 7) + tb[p++];
    return true;
  };
  uint64_t v;
  if (!rv(v) || !rv(v) || p + 2 > tcap) return HOH_E_CORRUPT;              // W-1, H-1
  // x_tiles-1, y_tiles-1 must be the tiling of W x H (as decode_image_impl checks: one byte each,
  // so 256 tiles on an axis wrap to 0, choh.cpp:457-458)
  if (xt != txt || yt != tyt || tb[p] != (uint8_t)(txt - 1) || tb[p + 1] != (uint8_t)(tyt - 1)) return HOH_E_CORRUPT;
  p += 2;
  std::vector<uint64_t> tsz(ntiles);
  uint64_t sum = 0;
  for (int i = 0; i + 1 < ntiles; i++) {
    if (!rv(v)) return HOH_E_CORRUPT;
    tsz[i] = v;
    sum += v;
  }
  if (p + sum > size) return HOH_E_CORRUPT;
  tsz[ntiles - 1] = size - p - sum;                                      // the last tile runs to the end
  const int n = m->n;
  std::vector<int> t0(n), nt(n), y0(n), rows(n), err(n, HOH_OK);
  std::vector<size_t> boff(n), bsz(n);
  size_t acc = p;
  for (int r = 0; r < n; r++) {
    band(yt, xt, r, n, &t0[r], &nt[r]);
    y0[r] = (t0[r] / xt) * th;
    rows[r] = std::min(H, (t0[r] + nt[r]) / xt * th) - y0[r];
    boff[r] = acc;
    bsz[r] = 0;
    for (int i = t0[r]; i < t0[r] + nt[r]; i++) bsz[r] += tsz[i];
    acc += bsz[r];
  }
  // every device's tile bytes: one RCCL group from the first device (or device copies)
  for (int r = 1; r < n; r++) {
    (void)hipSetDevice(m->dev[r]);
    if ((e = m->blob[r].grow(bsz[r] + 16))) return e;
  }
  if (!m->comm.empty()) {
    if (g_rccl.group_start() != ncclSuccess) return HOH_E_HIP;
    ncclResult_t rr = ncclSuccess;
    for (int r = 1; r < n && rr == ncclSuccess; r++) {
      if (!bsz[r]) continue;
      rr = g_rccl.send(d_hoh + boff[r], bsz[r], ncclUint8, r, m->comm[0], m->st[0]);
      if (rr == ncclSuccess) rr = g_rccl.recv(m->blob[r].p, bsz[r], ncclUint8, 0, m->comm[r], m->st[r]);
    }
    if (g_rccl.group_end() != ncclSuccess || rr != ncclSuccess) return drain(m, HOH_E_HIP);
  } else {
    (void)hipSetDevice(m->dev[0]);
    for (int r = 1; r < n; r++)
      if (bsz[r] && hipMemcpyPeerAsync(m->blob[r].p, m->dev[r], d_hoh + boff[r], m->dev[0], bsz[r], m->st[0]) != hipSuccess)
        return drain(m, HOH_E_HIP);
    if (hipStreamSynchronize(m->st[0]) != hipSuccess) return drain(m, HOH_E_HIP);
  }
  auto work = [&](int r) {
    (void)hipSetDevice(m->dev[r]);
    if (hipStreamSynchronize(m->st[r]) != hipSuccess) { err[r] = HOH_E_HIP; return; }
    const size_t raw = (size_t)W * rows[r] * 3;
    int e2;
    if ((e2 = m->drgb[r].grow(raw))) { err[r] = e2; return; }
    std::vector<uint32_t> s32(nt[r]);
    for (int i = 0; i < nt[r]; i++) s32[i] = (uint32_t)tsz[t0[r] + i];
    const uint8_t* src = r == 0 ? d_hoh + boff[0] : (const uint8_t*)m->blob[r].p;
    uint8_t* base = (uint8_t*)m->drgb[r].p - (size_t)y0[r] * W * 3;
    e2 = hoh_decode_tiles(m->ctx[r], src, bsz[r], W, H, t0[r], nt[r], s32.data(), base, nullptr, m->st[r]);
    if (!e2 && hipMemcpy(h_rgb + (size_t)y0[r] * W * 3, m->drgb[r].p, raw, hipMemcpyDeviceToHost) != hipSuccess)
      e2 = HOH_E_HIP;
    err[r] = e2;
  };
  {
    std::vector<std::thread> thr;
    for (int r = 1; r < n; r++) thr.emplace_back(work, r);
    work(0);
    for (auto& t : thr) t.join();
  }
  for (int r = 0; r < n; r++) if (err[r]) return drain(m, err[r]);
  return HOH_OK;
}

}  // extern "C"
