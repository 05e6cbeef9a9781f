// Encoder front end, one workgroup (4 waves) per tile (choh.cpp:464-500 tiles are independent),
// streaming the tile in raster blocks of 256 positions:
//  * subtract-green (channel.hpp:73-79) + MED fast-path residuals for the three planes
//    (prediction.hpp:6-44), written to the residual arena, histograms in LDS.  A pixel is kept
//    as {R' | B' << 16, rgb}: the two 9-bit planes go through packed 16-bit arithmetic (the
//    uint16 gradient wrap of Q8 is exactly the packed u16 wrap), G through SDWA byte selects;
//  * grey test (channel.hpp:21-31); the distinct-colour count capped at 257 (choh.cpp:17-46)
//    and the palette order come from k_colours, launched just before (early exit per tile);
//  * LZ candidate detection for find_lz_rgb at -s0 (lz.hpp:32-53): a position q is a candidate
//    iff some back distance b in [1, min(64, q)] gives 4 equal RGB pixels q..q+3 vs q-b..q-b+3.
//    Each wave fingerprints the 4-pixel windows of its 64 positions and of the 64 before them,
//    counts the 128 fingerprints in a wave-private LDS hash table and checks exactly
//    (b = 1..64, first hit wins) only positions whose fingerprint occurs twice; equal windows
//    have equal fingerprints, so the candidate set is exact.  The greedy selection runs in
//    k_lz.hip over the (sparse) candidate bitmap.
// Pixels live in an LDS ring (stored twice, plus a third copy of slots 0..3 for the LZ check's
// window, so reads at q+k and q-d never wrap); every pixel is
// read from HBM once (one unaligned dword), one block ahead of its use.  Tiles wider than the
// ring allows (only untiled images) read their neighbours from memory instead.
#include "hoh_internal.h"

// Ring of RING positions (stored twice): a block's writes land while the slowest wave may still
// read the previous block's neighbourhood, so the span in use is [q - 256 - max(w + 1, 67), q + 512)
// and RING >= 768 + max(w + 1, 67).  Tiles up to 271 wide (every tiled image) use 1040 positions
// (8 KB; with the 256-bin G histogram a workgroup needs 26.4 KB: six per CU), up to 1279 wide 2048.
#define RING_SMALL 1040
#define RING_SMALL_MAX_W 271
#define RING 2048
#define RING_MAX_W 1200
#define WTAB 512                // slots of a wave's fingerprint table (128 keys)
#define CSET 512                // colour set slots (<= 257 colours are counted)
#define NT 256
#define PF 4                    // blocks of HBM loads in flight per thread

typedef unsigned short us2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ us2 as_us2(uint32_t v) { return __builtin_bit_cast(us2, v); }
__device__ __forceinline__ uint32_t as_u32(us2 v) { return __builtin_bit_cast(uint32_t, v); }

__device__ __forceinline__ uint16_t med16(uint16_t a, uint16_t b, uint16_t c) {
  // predictor_operations.hpp:37-60, uint16_t overload (selected by overload resolution: Q8)
  if (a > b) return b > c ? b : (c > a ? a : c);
  return b < c ? b : (c > a ? c : a);
}

// R' | B' << 16 of a packed pixel r | g << 8 | b << 16 (R' = r - g + 256, B' = b - g + 256)
__device__ __forceinline__ uint32_t rb_form(uint32_t rgb) {
  const uint32_t g = (rgb >> 8) & 255u;
  return ((rgb & 0x00ff00ffu) | 0x01000100u) - g * 0x10001u;
}

__device__ __forceinline__ uint32_t fp32(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  uint32_t h = a * 0x9E3779B1u;
  h = (h ^ b) * 0x85EBCA77u;
  h = (h ^ c) * 0xC2B2AE3Du;
  h = (h ^ d) * 0x27D4EB2Fu;
  return (h ^ (h >> 15)) | 1u;                     // never 0 (the empty-slot key)
}

// insert key k into a wave table (open addressing, keys are odd), return its slot; a key
// inserted a second time sets the slot's duplicate bit
__device__ __forceinline__ uint32_t wt_insert(uint32_t* key, uint32_t* dup, uint32_t k) {
  uint32_t sl = (k >> 1) & (WTAB - 1);
  {
    const uint32_t old = atomicCAS(&key[sl], 0u, k);     // the common case: first probe
    if (old == 0u) return sl;
    if (old == k) { atomicOr(&dup[sl >> 5], 1u << (sl & 31)); return sl; }
    sl = (sl + 1) & (WTAB - 1);
  }
  for (int probe = 1; probe < WTAB; probe++) {
    const uint32_t old = atomicCAS(&key[sl], 0u, k);
    if (old == 0u) return sl;
    if (old == k) { atomicOr(&dup[sl >> 5], 1u << (sl & 31)); return sl; }
    sl = (sl + 1) & (WTAB - 1);
  }
  return WTAB;
}

// pixel at raster position q of a tile read from memory (tiles too wide for the ring)
__device__ __forceinline__ uint32_t px_mem(const uint8_t* img, size_t pitch, int w, uint32_t npix, uint32_t q) {
  if (q >= npix) return 0;                           // incl. positions before the tile (wrapped)
  const uint32_t y = q / (uint32_t)w, x = q - y * (uint32_t)w;
  const uint8_t* p = img + (size_t)y * pitch + (size_t)x * 3;
  return p[0] | (p[1] << 8) | (p[2] << 16);
}

template <bool RINGED, uint32_t RG>
__device__ __forceinline__ void front_tile(const EncodeJob& j, uint32_t* ring) {
  __shared__ uint32_t wkey[4][WTAB + 1];
  __shared__ uint32_t wdup[4][WTAB / 32];
  __shared__ uint32_t hist[3 * 512 - 256];         // G: 256 bins at 0, R': 512 at 256, B': 512 at 768
  __shared__ int s_notgrey, s_ncand;

  const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int gt = j.t0 + t;
  const int x0 = (gt % j.xt) * j.tw, y0 = (gt / j.xt) * j.th;
  const int w = min(j.tw, j.W - x0), h = min(j.th, j.H - y0);
  const uint32_t npix = (uint32_t)w * h;
  for (int i = tid; i < 3 * 512 - 256; i += NT) hist[i] = 0;
  for (int i = lane; i <= WTAB; i += 64) wkey[wv][i] = 0;
  if (lane < WTAB / 32) wdup[wv][lane] = 0;
  if (tid == 0) { s_notgrey = 0; s_ncand = 0; }

  uint16_t* res0 = j.sym + med_plane_off(j, t, 0);
  uint16_t* res1 = j.sym + med_plane_off(j, t, 1);
  uint16_t* res2 = j.sym + med_plane_off(j, t, 2);
  uint64_t* cand = j.candbits + (size_t)t * (j.npix_cap / 64);
  const uint8_t* img = j.rgb + ((size_t)y0 * j.W + x0) * 3;
  const size_t pitch = (size_t)j.W * 3;
  const bool lz = j.speed == 0;     // -s>=1: k_lzcand screens a longer window

  // loader cursor: this thread's pixel of the block being loaded (raster blk*256 + tid) as a
  // byte offset from the tile origin
  int lx = tid;
  uint32_t loff = 0;
  while (lx >= w) { lx -= w; loff += (uint32_t)pitch; }
  loff += (uint32_t)lx * 3;
  const uint32_t wrap = (uint32_t)pitch - (uint32_t)w * 3;
  // branch-free pixel fetch: an unaligned dword whose top 3 bytes are the pixel (the image's
  // very first pixel takes the dword at its own address instead); positions past the tile
  // fetch the tile's first pixel and return 0
  // Only the tile's own pixels may be read (a shard's buffer starts at its first row), so a
  // pixel that starts a tile row reads the dword at itself (its 3 bytes + the next pixel's
  // first), every other pixel the dword ending with it (the previous pixel's last byte + its 3);
  // positions past the tile read the tile's first pixel and return 0.  1-pixel-wide tiles
  // (untiled W = 1 images) read bytes.
  auto load_px = [&](uint32_t q) -> uint32_t {
    const bool in = q < npix;
    if (w < 2) return in ? (img[loff] | (img[loff + 1] << 8) | (img[loff + 2] << 16)) : 0u;
    const bool at_self = !in || lx == 0;
    const uint32_t a = !in ? 0u : (lx == 0 ? loff : loff - 1);
    uint32_t v;
    __builtin_memcpy(&v, img + a, 4);
    v = at_self ? (v & 0xffffffu) : (v >> 8);
    return in ? v : 0u;
  };
  const bool wide_rows = w >= NT;                    // a block advance wraps at most one row
  auto advance = [&]() {
    lx += NT;
    loff += NT * 3;
    if (wide_rows) {
      const bool wr = lx >= w;
      lx -= wr ? w : 0;
      loff += wr ? wrap : 0u;
    } else {
      while (lx >= w) { lx -= w; loff += wrap; }
    }
  };
  uint32_t own = 0, nv[PF];
  if (RINGED) {
    own = load_px(tid);
    ring[tid] = own;                                 // tid < 256 < RG
    ring[tid + RG] = own;
    if (tid < 4) ring[tid + 2 * RG] = own;
    advance();
#pragma unroll
    for (int k = 1; k <= PF; k++) {
      nv[k % PF] = load_px((uint32_t)k * NT + tid);
      advance();
    }
  }
  // compute cursor: (x, y) of position base + tid
  uint32_t cx = tid, cy = 0;
  while (cx >= (uint32_t)w) { cx -= w; cy++; }
  __syncthreads();

  uint32_t ri = tid;                                 // (blk * NT + tid) % RG, kept incrementally
  uint32_t notgrey = 0;
  int ncand = 0;
  const uint32_t nblk = (npix + NT - 1) / NT;
  auto body = [&](const uint32_t blk, uint32_t& slot) {
    const uint32_t base = blk * NT;
    const uint32_t q = base + tid;
    uint32_t v;
    if (RINGED) {   // land block blk+1, issue block blk+1+PF into its slot
      const uint32_t rn = ri + NT >= RG ? ri + NT - RG : ri + NT;   // position base + NT + tid
      ring[rn] = slot;
      ring[rn + RG] = slot;
      if (rn < 4) ring[rn + 2 * RG] = slot;
      v = own;
      own = slot;
      slot = load_px(base + (1 + PF) * NT + tid);
      advance();
    } else {
      v = px_mem(img, pitch, w, npix, q);
    }
    // forward / backward neighbours by raster distance: ring copies [ri] and [ri + RG] hold
    // the same pixels, so q + k and q - d never wrap; the LZ check's window q - b + 3 (b >= 1)
    // reaches index ri + RG + 2, so slots 0..3 have a third copy at 2 RG
    const uint32_t rq = ri;
    ri = ri + NT >= RG ? ri + NT - RG : ri + NT;
    auto F = [&](uint32_t k) -> uint32_t { return RINGED ? ring[rq + k] : px_mem(img, pitch, w, npix, q + k); };
    auto B = [&](uint32_t d) -> uint32_t { return RINGED ? ring[rq + RG - d] : px_mem(img, pitch, w, npix, q - d); };
    __syncthreads();
    const bool act = q < npix;
    if (act) {
      const uint32_t g = (v >> 8) & 255u;
      notgrey |= (v ^ (g * 0x010101u)) & 0xffffffu;
      // neighbours; outside the tile the reference uses c/2 in every plane (prediction.hpp:21-28),
      // i.e. the grey pixel 128,128,128 (G = 128, R' = B' = 256)
      const bool hasL = cx > 0, hasT = cy > 0;
      const uint32_t bL = B(1), bT = B(w), bTL = B(w + 1);     // unconditional reads, then select
      const uint32_t vL = hasL ? bL : 0x808080u;
      const uint32_t vT = hasT ? bT : 0x808080u;
      const uint32_t vTL = (hasL && hasT) ? bTL : 0x808080u;
      // G: median of (T, L, (uint16)(T + L - TL))
      const uint32_t gL = (vL >> 8) & 255u, gT = (vT >> 8) & 255u, gTL = (vTL >> 8) & 255u;
      const uint32_t gg = (gT + gL - gTL) & 0xffffu;
      const uint32_t pg = max(min(gT, gL), min(max(gT, gL), gg));
      const uint32_t rg = (g - pg + 128u) & 255u;
      // R', B' packed: the same median per 16-bit lane
      const us2 tt = as_us2(rb_form(vT)), ll = as_us2(rb_form(vL)), tl = as_us2(rb_form(vTL));
      const us2 gr = tt + ll - tl;
      const us2 mn = __builtin_elementwise_min(tt, ll), mx = __builtin_elementwise_max(tt, ll);
      const us2 pr = __builtin_elementwise_max(mn, __builtin_elementwise_min(mx, gr));
      const uint32_t rrb = as_u32(as_us2(rb_form(v)) - pr + (us2)(256)) & 0x01ff01ffu;
      const uint32_t rr = rrb & 0xffffu, rb = rrb >> 16;
      res0[q] = (uint16_t)rg;
      res1[q] = (uint16_t)rr;
      res2[q] = (uint16_t)rb;
      atomicAdd(&hist[rg], 1u);
      atomicAdd(&hist[256 + rr], 1u);
      atomicAdd(&hist[768 + rb], 1u);
    }
    cx += NT;
    if (wide_rows) {
      const bool wr = cx >= (uint32_t)w;
      cx -= wr ? w : 0;
      cy += wr ? 1 : 0;
    } else {
      while (cx >= (uint32_t)w) { cx -= w; cy++; }
    }
    if (!lz) return;
    // LZ screen: this position's window, then (after the barrier) the window 64 back
    const bool win = q + 3 < npix;                 // a 4-pixel window starts here
    const uint32_t v1 = win ? F(1) : 0, v2 = win ? F(2) : 0, v3 = win ? F(3) : 0;
    const uint32_t hq = win ? fp32(v, v1, v2, v3) : 0u;
    // the window 64 back is another wave's: recomputing its fingerprint beats a second barrier
    const bool winp = q >= 64 && q - 61 < npix;
    const uint32_t hp = winp ? fp32(B(64), B(63), B(62), B(61)) : 0u;
    uint32_t* key = wkey[wv];
    uint32_t* dup = wdup[wv];
    uint32_t sq = WTAB, sp = WTAB;
    if (hq) sq = wt_insert(key, dup, hq);
    if (hp) sp = wt_insert(key, dup, hp);
    const bool hit = hq && sq < WTAB && ((dup[sq >> 5] >> (sq & 31)) & 1);
    const uint64_t flag = __ballot(hit);
    uint64_t word = 0;
    if (flag) {
      // exact check for the flagged lanes (lz.hpp:37-42 with offset < 4)
      bool c = false;
      if (hit) {
        const uint32_t bmax = q < 64 ? q : 64;
        for (uint32_t b = 1; b <= bmax && !c; b++)
          c = B(b) == v && B(b - 1) == v1 && B(b - 2) == v2 && B(b - 3) == v3;
      }
      word = __ballot(c);
    }
    // clear the slots this wave used (wave-ordered LDS: the reads above are done)
    key[sq] = 0;                                    // slot WTAB is a spare: no branch
    key[sp] = 0;
    if (lane < WTAB / 32) dup[lane] = 0;
    if (lane == 0 && (q >> 6) < (npix + 63) / 64) cand[q >> 6] = word;
    ncand += lane == 0 ? __popcll(word) : 0;
  };
  for (uint32_t blk = 0; blk < nblk; blk += PF) {
#pragma unroll
    for (int u = 0; u < PF; u++)
      if (blk + u < nblk) body(blk + u, nv[(u + 1) % PF]);
  }
  if (notgrey) atomicOr(&s_notgrey, 1);
  if (ncand) atomicAdd(&s_ncand, ncand);
  __syncthreads();
  for (int i = tid; i < 3 * 512; i += NT) {
    const int k = i / 512, s = i % 512;
    j.hist[(size_t)(t * j.spt + med_kind(j, k)) * 512 + s] = k == 0 ? (s < 256 ? hist[s] : 0u) : hist[k * 512 - 256 + s];
  }
  if (tid == 0) {
    TileInfo ti;
    ti.x0 = x0; ti.y0 = y0; ti.w = w; ti.h = h;
    ti.colours = j.ncol[t];                          // k_colours ran before this kernel
    uint32_t fl = 0;
    if (!s_notgrey) fl |= TF_GREY;
    if (!s_notgrey && ti.colours != -1 && ti.colours <= 2) fl |= TF_BINARY;
    if (!s_notgrey && !(fl & TF_BINARY)) fl |= TF_UNREPRODUCIBLE;   // choh.cpp:196-205 copies garbage
    if (s_notgrey && ti.colours != -1) fl |= TF_PALETTE_CAND;
    ti.flags = fl;
    ti.nmatch = 0;
    ti.ncand = (uint32_t)s_ncand;
    ti.size = 0; ti.lz_bytes = 0; ti.off = 0;
    ti.mode = (fl & TF_GREY) ? 0 : 128;
    ti.pad = 0;
    j.tiles[t] = ti;
  }
}

// Distinct colours of each tile, capped at 257 (choh.cpp:17-46), and for tiles with <= 256 the
// palette in first-occurrence order (choh.cpp:64-88).  One workgroup per tile walks raster blocks
// and stops as soon as a tile has shown 257 colours, which natural tiles do within a block or
// two, so k_front carries no colour set (and fits seven workgroups per CU).
__global__ __launch_bounds__(NT) void k_colours(EncodeJob j) {
  __shared__ uint32_t hset[CSET];
  __shared__ uint32_t hpos[CSET];                   // first raster position of each colour
  __shared__ uint32_t pc[256], pp[256];
  __shared__ int s_ncol, s_np;
  const int t = blockIdx.x, tid = threadIdx.x;
  const int gt = j.t0 + t;
  const int x0 = (gt % j.xt) * j.tw, y0 = (gt / j.xt) * j.th;
  const int w = min(j.tw, j.W - x0), h = min(j.th, j.H - y0);
  const uint32_t npix = (uint32_t)w * h;
  const uint8_t* img = j.rgb + ((size_t)y0 * j.W + x0) * 3;
  const size_t pitch = (size_t)j.W * 3;
  for (int i = tid; i < CSET; i += NT) { hset[i] = 0xffffffffu; hpos[i] = 0xffffffffu; }
  if (tid == 0) { s_ncol = 0; s_np = 0; }
  uint32_t x = tid, y = 0;
  while (x >= (uint32_t)w) { x -= w; y++; }
  __syncthreads();
  const int lane = tid & 63;
  // four 256-pixel blocks per barrier (their loads together); a pixel whose colour equals the
  // previous lane's (the previous raster position, or its block's) skips the insert: that lane
  // holds the smaller first position (flat tiles no longer send 256 CAS to one LDS word)
  for (uint32_t q0 = 0; q0 < npix; q0 += 4 * NT) {
    uint32_t v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint32_t q = q0 + (uint32_t)u * NT + tid;
      v[u] = 0xffffffffu;
      if (q < npix) {
        const uint8_t* p = img + (size_t)y * pitch + (size_t)x * 3;
        v[u] = p[0] | (p[1] << 8) | (p[2] << 16);
      }
      x += NT;
      while (x >= (uint32_t)w) { x -= w; y++; }
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint32_t q = q0 + (uint32_t)u * NT + tid;
      const uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp((int)v[u], (int)v[u], 0x138, 0xf, 0xf, false);
      // (past 256 colours the tile is decided: stop filling the 512-slot set)
      if (q < npix && (lane == 0 || v[u] != prev) && *(volatile int*)&s_ncol <= 256) {
        uint32_t hsh = (v[u] * 2654435761u) >> 23;
        for (int probe = 0; probe < CSET; probe++) {
          const uint32_t old = atomicCAS(&hset[hsh], 0xffffffffu, v[u]);
          if (old == 0xffffffffu) { atomicAdd(&s_ncol, 1); atomicMin(&hpos[hsh], q); break; }
          if (old == v[u]) { atomicMin(&hpos[hsh], q); break; }
          hsh = (hsh + 1) & (CSET - 1);
        }
      }
    }
    __syncthreads();
    if (s_ncol > 256) break;                         // block-uniform after the barrier
  }
  if (s_ncol > 256) {
    if (tid == 0) j.ncol[t] = -1;
    return;
  }
  // rank of a colour = number of colours whose first position is smaller
  for (int i = tid; i < CSET; i += NT) {
    if (hset[i] != 0xffffffffu) {
      const int k = atomicAdd(&s_np, 1);
      pc[k] = hset[i];
      pp[k] = hpos[i];
    }
  }
  __syncthreads();
  if (tid < s_np) {
    const uint32_t me = pp[tid];
    uint32_t rank = 0;
    for (int m = 0; m < s_np; m++) rank += pp[m] < me;
    j.palette[(size_t)t * 256 + rank] = pc[tid];
  }
  if (tid == 0) j.ncol[t] = s_ncol;
}

template <uint32_t RG>
__global__ __launch_bounds__(NT) void k_front(EncodeJob j) {
  __shared__ uint32_t ring[2 * RG + 4];
  front_tile<true, RG>(j, ring);
}

__global__ __launch_bounds__(NT) void k_front_wide(EncodeJob j) { front_tile<false, 1>(j, nullptr); }

// Indexed plane of a palette-candidate tile (choh.cpp:48-102 palette_encode + layer_encode -s0):
// index = first-occurrence rank of the pixel's colour, then the MED fast-path residual at depth 8
// (prediction.hpp:6-44) and its histogram.  One workgroup per tile; pass 1 writes the indices
// into the tile's indexed-plane slot, pass 2 turns them into residuals in place, walking blocks
// from the last to the first so every neighbour (q-1, q-w, q-w-1) is still an index when read.
__device__ __forceinline__ void palette_tile(const EncodeJob& j, int t, uint32_t* hk, uint32_t* hv, uint32_t* phist);

// a small grid strides over the tiles (palette candidates are rare): no idle workgroup per tile
__global__ __launch_bounds__(NT) void k_palette(EncodeJob j) {
  __shared__ uint32_t hk[1024];
  __shared__ uint32_t hv[1024];
  __shared__ uint32_t phist[256];
  for (int t = blockIdx.x; t < j.ntiles; t += gridDim.x) {
    palette_tile(j, t, hk, hv, phist);
    __syncthreads();
  }
}

__device__ __forceinline__ void palette_tile(const EncodeJob& j, int t, uint32_t* hk, uint32_t* hv, uint32_t* phist) {
  const int tid = threadIdx.x;
  const TileInfo ti = j.tiles[t];
  if (!(ti.flags & TF_PALETTE_CAND) || (ti.flags & TF_GREY)) return;
  const int w = ti.w, h = ti.h, ncol = ti.colours;
  const uint32_t npix = (uint32_t)w * h;
  for (int i = tid; i < 1024; i += NT) hk[i] = 0xffffffffu;
  phist[tid] = 0;
  __syncthreads();
  if (tid < ncol) {
    const uint32_t c = j.palette[(size_t)t * 256 + tid];
    uint32_t hsh = (c * 2654435761u) >> 22;
    while (atomicCAS(&hk[hsh], 0xffffffffu, c) != 0xffffffffu) hsh = (hsh + 1) & 1023;
    hv[hsh] = (uint32_t)tid;
  }
  __syncthreads();
  uint16_t* pl = j.sym + med_plane_off(j, t, 3);
  const uint8_t* img = j.rgb + ((size_t)ti.y0 * j.W + ti.x0) * 3;
  const size_t pitch = (size_t)j.W * 3;
  int x = tid, y = 0;
  while (x >= w) { x -= w; y++; }
  for (uint32_t q = tid; q < npix; q += NT) {
    const uint8_t* p = img + (size_t)y * pitch + (size_t)x * 3;
    const uint32_t c = p[0] | (p[1] << 8) | (p[2] << 16);
    uint32_t hsh = (c * 2654435761u) >> 22;
    for (int probe = 0; probe < 1024 && hk[hsh] != c; probe++) hsh = (hsh + 1) & 1023;
    pl[q] = (uint16_t)hv[hsh];
    if (j.idx8) j.idx8[(size_t)t * j.npix_cap + q] = (uint8_t)hv[hsh];
    x += NT;
    while (x >= w) { x -= w; y++; }
  }
  __syncthreads();
  const uint32_t nblk = (npix + NT - 1) / NT;
  for (int b = (int)nblk - 1; b >= 0; b--) {
    const uint32_t q = (uint32_t)b * NT + tid;
    uint32_t r = 0;
    if (q < npix) {
      const uint32_t qx = q % (uint32_t)w, qy = q / (uint32_t)w;
      const uint16_t v = pl[q];
      const uint16_t L = qx ? pl[q - 1] : (uint16_t)128;
      const uint16_t T = qy ? pl[q - w] : (uint16_t)128;
      const uint16_t TL = (qx && qy) ? pl[q - w - 1] : (uint16_t)128;
      r = ((int)v - (int)med16(T, L, (uint16_t)(T + L - TL)) + 128 + 256) & 255;
    }
    __syncthreads();
    if (q < npix) { pl[q] = (uint16_t)r; atomicAdd(&phist[r], 1u); }
    __syncthreads();
  }
  uint32_t* hs = j.hist + (size_t)(t * j.spt + med_kind(j, 3)) * 512;
  for (int i = tid; i < 512; i += NT) hs[i] = i < 256 ? phist[i] : 0u;
}

void launch_palette(const EncodeJob& j, hipStream_t s) {
  hipLaunchKernelGGL(k_palette, dim3(j.ntiles < 128 ? j.ntiles : 128), dim3(NT), 0, s, j);
}

// ---------------------------------------------------------------- full 256 x 256 tiles
//
// Every tile of an image whose sides are multiples of 256 (the bench's 8192^2 and 16384^2) is a
// full 256 x 256 tile, and k_front256 walks it with every neighbour in registers instead of an
// LDS pixel ring behind block barriers.  Wave v of the tile's workgroup owns rows 64v .. 64v+63 and
// walks them in raster order one 64-pixel chunk (a quarter row) at a time: L is a DPP wave shift
// of the chunk (lane 0 takes lane 63 of the chunk to the left), T the same lane of the row above
// (kept from the previous row; the stripe's first row reads it from memory), TL a shift of T.  The
// LZ screen keeps the exact test of k_front (a window q..q+3 is a candidate iff it equals one of
// the 64 windows before it): the chunk's 64 window fingerprints go into a wave-private table and
// are looked up in the previous chunk's table, so each window is fingerprinted and inserted once
// (k_front needs two of each); the two tables alternate, each cleared slot by slot by the lanes
// that filled it.  Positions whose fingerprint occurs twice get the exact pixel comparison from a
// per-wave LDS pixel ring.  Candidate words, residuals, histograms and tile flags are the same
// as k_front's.
#define F2_TAB 256            // slots of a chunk's fingerprint table (64 keys)
#define F2_RING 256           // positions of a wave's pixel ring (the exact LZ check)

__device__ __forceinline__ uint32_t wshl1(uint32_t v, uint32_t old) {   // lane l <- lane l+1, lane 63 <- old
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x130, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t wshr1(uint32_t v, uint32_t old) {   // lane l <- lane l-1, lane 0 <- old
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t lane_of(uint32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }

// slot of key k in a (read-only) table, F2_TAB if absent
__device__ __forceinline__ uint32_t wt_find(const uint32_t* key, uint32_t k) {
  uint32_t sl = (k >> 1) & (F2_TAB - 1);
  for (int probe = 0; probe < F2_TAB; probe++) {
    const uint32_t o = key[sl];
    if (o == k) return sl;
    if (o == 0u) return F2_TAB;
    sl = (sl + 1) & (F2_TAB - 1);
  }
  return F2_TAB;
}

// insert into a chunk table (open addressing, one slot per distinct key); returns the slot
// (F2_TAB if none)
__device__ __forceinline__ uint32_t wt_put(uint32_t* key, uint32_t k) {
  uint32_t sl = (k >> 1) & (F2_TAB - 1);
  for (int probe = 0; probe < F2_TAB; probe++) {
    const uint32_t old = atomicCAS(&key[sl], 0u, k);
    if (old == 0u || old == k) return sl;
    sl = (sl + 1) & (F2_TAB - 1);
  }
  return F2_TAB;
}

// LDS max over the lanes that hold a slot's key (of `lane` or of 63 - lane; the word is cleared to 0)
__device__ __forceinline__ void wt_max(uint32_t* pos, uint32_t sl, uint32_t v) {
  __hip_atomic_fetch_max(&pos[sl], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__global__ __launch_bounds__(NT) void k_front256(EncodeJob j) {
  __shared__ uint32_t tab[4][2][F2_TAB + 1];        // per wave: two alternating chunk tables
  // per slot, one word: while its table is the current chunk's, 63 - the key's smallest lane; then
  // (rewritten after the chunk's checks) the largest lane, for the next chunk's lookups
  __shared__ uint32_t tpos[4][2][F2_TAB + 1];
  __shared__ uint32_t pring[4][F2_RING];
#ifndef F2_HC
#define F2_HC 1               // histogram copies (lane & (F2_HC - 1) picks one): fewer same-address atomics
#endif
#ifndef F2_AGG
#define F2_AGG 0              // 1: wave-aggregated histogram adds for lane 0's bin (+ 64 spare words)
#endif
  __shared__ uint32_t hist[F2_HC][3 * 512 - 256 + 64 * F2_AGG];
  __shared__ int s_notgrey, s_ncand;
  const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int gt = j.t0 + t;
  const int x0 = (gt % j.xt) * 256, y0 = (gt / j.xt) * 256;
  const uint32_t npix = 256u * 256u;
  for (int i = tid; i < F2_HC * (3 * 512 - 256 + 64 * F2_AGG); i += NT) (&hist[0][0])[i] = 0;
  uint32_t* hl = hist[lane & (F2_HC - 1)];
  for (int i = lane; i < 2 * (F2_TAB + 1); i += 64) tab[wv][i / (F2_TAB + 1)][i % (F2_TAB + 1)] = 0;
  for (int i = lane; i < 2 * (F2_TAB + 1); i += 64) tpos[wv][i / (F2_TAB + 1)][i % (F2_TAB + 1)] = 0;
  if (tid == 0) { s_notgrey = 0; s_ncand = 0; }
  uint16_t* res0 = j.sym + med_plane_off(j, t, 0);
  uint16_t* res1 = j.sym + med_plane_off(j, t, 1);
  uint16_t* res2 = j.sym + med_plane_off(j, t, 2);
  uint64_t* cand = j.candbits + (size_t)t * (j.npix_cap / 64);
  const uint8_t* img = j.rgb + ((size_t)y0 * j.W + x0) * 3;
  const size_t pitch = (size_t)j.W * 3;
  const bool lz = j.speed == 0 && !(j.exp & 2);     // what-if EXP & 2 (measurement): no LZ screen
  uint32_t* ring = pring[wv];
  // pixel (x = 64k + lane, y) of the tile: one unaligned dword that never leaves the tile (x = 0
  // reads its own 3 bytes + the next pixel's first, others the previous pixel's last byte + theirs)
  auto load_row = [&](int y, uint32_t* o) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int x = 64 * k + lane;
      const uint8_t* p = img + (size_t)y * pitch + (size_t)x * 3;
      uint32_t v;
      __builtin_memcpy(&v, x ? p - 1 : p, 4);
      o[k] = x ? (v >> 8) : (v & 0xffffffu);
    }
  };
  const uint32_t GREY = 0x808080u;
  const int ya = 64 * wv, yb = ya + 64;
  uint32_t prow[4], cur[4], nxt[4];
  if (ya > 0) load_row(ya - 1, prow);
  else { prow[0] = prow[1] = prow[2] = prow[3] = GREY; }
  load_row(ya, cur);
  load_row(ya + 1, nxt);                              // ya + 1 < 256 always
  __syncthreads();
  uint32_t notgrey = 0;
  int ncand = 0;
  int cb = 0;                                         // table of the current chunk
  uint32_t slot_prev = F2_TAB;                        // this lane's slot in the previous chunk's table
  // the chunk before the stripe (row ya-1, quarter 3): its windows go into the "previous" table
  // and its pixels into the ring, so the stripe's first chunk sees all 64 windows behind it
  if (lz) {
    if (ya > 0) {
      const uint32_t pv = prow[3];
      const uint32_t a1 = wshl1(pv, lane_of(cur[0], 0));
      const uint32_t a2 = wshl1(a1, lane_of(cur[0], 1));
      const uint32_t a3 = wshl1(a2, lane_of(cur[0], 2));
      const uint32_t k = fp32(pv, a1, a2, a3);
      slot_prev = wt_put(tab[wv][1], k);
      if (slot_prev < F2_TAB) wt_max(tpos[wv][1], slot_prev, lane);
      ring[(uint32_t)(ya * 256 - 64 + lane) & (F2_RING - 1)] = pv;
    }
    ring[(uint32_t)(ya * 256 + lane) & (F2_RING - 1)] = cur[0];
  }
  for (int y = ya; y < yb; y++) {
    const bool hasT = y > 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t q = (uint32_t)y * 256u + 64u * k + lane;
      const uint32_t v = cur[k];
      const uint32_t g = (v >> 8) & 255u;
      notgrey |= (v ^ (g * 0x010101u)) & 0xffffffu;
      // neighbours (prediction.hpp:21-28: outside the tile the grey pixel 128,128,128)
      const uint32_t lft = k ? lane_of(cur[k - 1], 63) : GREY;
      const uint32_t tlf = k ? lane_of(prow[k - 1], 63) : GREY;
      const uint32_t vL = wshr1(v, lft);              // x = 0 (k = 0, lane 0) gets grey
      const uint32_t vT = hasT ? prow[k] : GREY;
      const uint32_t vTL = hasT ? wshr1(prow[k], tlf) : GREY;
      const uint32_t gL = (vL >> 8) & 255u, gT = (vT >> 8) & 255u, gTL = (vTL >> 8) & 255u;
      const uint32_t gg = (gT + gL - gTL) & 0xffffu;
      const uint32_t pg = max(min(gT, gL), min(max(gT, gL), gg));
      const uint32_t rg = (g - pg + 128u) & 255u;
      const us2 tt = as_us2(rb_form(vT)), ll = as_us2(rb_form(vL)), tl = as_us2(rb_form(vTL));
      const us2 gr = tt + ll - tl;
      const us2 mn = __builtin_elementwise_min(tt, ll), mx = __builtin_elementwise_max(tt, ll);
      const us2 pr = __builtin_elementwise_max(mn, __builtin_elementwise_min(mx, gr));
      const uint32_t rrb = as_u32(as_us2(rb_form(v)) - pr + (us2)(256)) & 0x01ff01ffu;
      const uint32_t rr = rrb & 0xffffu, rb = rrb >> 16;
      res0[q] = (uint16_t)rg;
      res1[q] = (uint16_t)rr;
      res2[q] = (uint16_t)rb;
#if F2_AGG
      // lanes holding lane 0's bin add once, through lane 0 (smooth tiles put most of a chunk on
      // one bin, and same-address LDS atomics serialise); the others' adds of 0 go to spare words
      auto hadd = [&](uint32_t i) {
        const uint32_t i0 = __builtin_amdgcn_readfirstlane(i);
        const uint32_t n0 = (uint32_t)__popcll(__ballot(i == i0));
        const bool dup = i == i0 && lane != 0;
        atomicAdd(&hl[dup ? 3 * 512 - 256 + lane : i], lane == 0 ? n0 : dup ? 0u : 1u);
      };
      hadd(rg);
      hadd(256 + rr);
      hadd(768 + rb);
#else
      atomicAdd(&hl[rg], 1u);
      atomicAdd(&hl[256 + rr], 1u);
      atomicAdd(&hl[768 + rb], 1u);
#endif
      if (!lz) continue;
      // the window q .. q+3 (the next chunk's first pixels for the last lanes)
      const uint32_t nx = k < 3 ? cur[k + 1] : nxt[0];
      const uint32_t v1 = wshl1(v, lane_of(nx, 0));
      const uint32_t v2 = wshl1(v1, lane_of(nx, 1));
      const uint32_t v3 = wshl1(v2, lane_of(nx, 2));
      ring[(q + 64u) & (F2_RING - 1)] = (q + 64u < npix) ? nx : 0u;   // the ring runs a chunk ahead
      const bool win = q + 3 < npix;
      const uint32_t hq = win ? fp32(v, v1, v2, v3) : 0u;
      uint32_t* tc = tab[wv][cb];
      uint32_t* pc = tpos[wv][cb];
      const uint32_t* tp = tab[wv][cb ^ 1];
      const uint32_t* pp = tpos[wv][cb ^ 1];
#if F2_AGG
      // lanes holding lane 0's key leave the table work to lane 0 (flat runs give most of a chunk
      // one key, and same-address LDS atomics serialise): lane 0's min lane is itself, and it writes
      // the group's max lane for the next chunk
      const uint32_t h0 = __builtin_amdgcn_readfirstlane(hq);
      const uint64_t m0 = __ballot(hq == h0);
      const bool kdup = hq == h0 && lane != 0;
      uint32_t sq = hq && !kdup ? wt_put(tc, hq) : F2_TAB;
      {
        const uint32_t s0 = __builtin_amdgcn_readfirstlane(sq);
        if (kdup) sq = s0;
      }
      if (sq < F2_TAB && !kdup) wt_max(pc, sq, 63u - lane);
#else
      const uint32_t sq = hq ? wt_put(tc, hq) : F2_TAB;
      const bool kdup = false;
      const uint64_t m0 = 1;
      if (sq < F2_TAB) wt_max(pc, sq, 63u - lane);
#endif
      const uint32_t sp = hq ? wt_find(tp, hq) : F2_TAB;
      // Equal windows have equal fingerprints, so the windows before q equal to q's can only be
      // at the positions holding hq: in this chunk at lanes min..lane-1 (the earliest is checked),
      // in the previous chunk at lanes >= lane (distance <= 64; the latest, i.e. nearest, is
      // checked).  When a checked window differs (a fingerprint collision) the lane falls back
      // to the full test over b = 1..64 (lz.hpp:37-42 with offset < 4).
      const uint32_t fcur = sq < F2_TAB ? 63u - pc[sq] : 64u;
      const uint32_t lprev = sp < F2_TAB ? pp[sp] : 0u;
      const bool ccur = fcur < (uint32_t)lane, cprev = sp < F2_TAB && lprev >= (uint32_t)lane;
      const uint64_t flag = __ballot(ccur || cprev);
      uint64_t word = 0;
      if (flag) {
        auto same = [&](uint32_t p) {
          return ring[p & (F2_RING - 1)] == v && ring[(p + 1) & (F2_RING - 1)] == v1 &&
                 ring[(p + 2) & (F2_RING - 1)] == v2 && ring[(p + 3) & (F2_RING - 1)] == v3;
        };
        const uint32_t q0 = q - lane;
        bool c = false, full = false;
        if (ccur || cprev) {
          c = same(ccur ? q0 + fcur : q0 - 64u + lprev);
          if (!c && ccur && cprev) c = same(q0 - 64u + lprev);
          full = !c;
        }
        if (__ballot(full)) {
          if (full) {
            const uint32_t bmax = q < 64 ? q : 64;
            for (uint32_t b = 1; b <= bmax && !c; b++) c = same(q - b);
          }
        }
        word = __ballot(c);
      }
      // this chunk's words turn into the largest lane for the next chunk's lookups (program order
      // on one address: the fcur reads above come first)
      if (sq < F2_TAB && !kdup) { pc[sq] = 0; wt_max(pc, sq, lane ? (uint32_t)lane : 63u - (uint32_t)__builtin_clzll(m0)); }
      if (lane == 0) cand[q >> 6] = word;
      ncand += lane == 0 ? __popcll(word) : 0;
      // empty the previous chunk's table for the next chunk (wave-ordered: every lookup is done)
      uint32_t* tpw = tab[wv][cb ^ 1];
      tpw[slot_prev] = 0;                             // slot F2_TAB is a spare: no branch
      tpos[wv][cb ^ 1][slot_prev] = 0;
      slot_prev = kdup ? F2_TAB : sq;
      cb ^= 1;
    }
#pragma unroll
    for (int k = 0; k < 4; k++) { prow[k] = cur[k]; cur[k] = nxt[k]; }
    if (y + 2 < 256) load_row(y + 2, nxt);
  }
  if (notgrey) atomicOr(&s_notgrey, 1);
  if (ncand) atomicAdd(&s_ncand, ncand);
  __syncthreads();
  for (int i = tid; i < 3 * 512; i += NT) {
    const int k = i / 512, sv = i % 512;
    uint32_t v = 0;
#pragma unroll
    for (int hc = 0; hc < F2_HC; hc++) v += k == 0 ? (sv < 256 ? hist[hc][sv] : 0u) : hist[hc][k * 512 - 256 + sv];
    j.hist[(size_t)(t * j.spt + med_kind(j, k)) * 512 + sv] = v;
  }
  if (tid == 0) {
    TileInfo ti;
    ti.x0 = x0; ti.y0 = y0; ti.w = 256; ti.h = 256;
    ti.colours = j.ncol[t];
    uint32_t fl = 0;
    if (!s_notgrey) fl |= TF_GREY;
    if (!s_notgrey && ti.colours != -1 && ti.colours <= 2) fl |= TF_BINARY;
    if (!s_notgrey && !(fl & TF_BINARY)) fl |= TF_UNREPRODUCIBLE;   // choh.cpp:196-205 copies garbage
    if (s_notgrey && ti.colours != -1) fl |= TF_PALETTE_CAND;
    ti.flags = fl;
    ti.nmatch = 0;
    ti.ncand = (uint32_t)s_ncand;
    ti.size = 0; ti.lz_bytes = 0; ti.off = 0;
    ti.mode = (fl & TF_GREY) ? 0 : 128;
    ti.pad = 0;
    j.tiles[t] = ti;
  }
}

void launch_front(const EncodeJob& j, hipStream_t s) {
  hipLaunchKernelGGL(k_colours, dim3(j.ntiles), dim3(NT), 0, s, j);
  if (j.tw == 256 && j.th == 256) hipLaunchKernelGGL(k_front256, dim3(j.ntiles), dim3(NT), 0, s, j);
  else if (j.tw <= RING_SMALL_MAX_W) hipLaunchKernelGGL(k_front<RING_SMALL>, dim3(j.ntiles), dim3(NT), 0, s, j);
  else if (j.tw <= RING_MAX_W) hipLaunchKernelGGL(k_front<RING>, dim3(j.ntiles), dim3(NT), 0, s, j);
  else hipLaunchKernelGGL(k_front_wide, dim3(j.ntiles), dim3(NT), 0, s, j);
}
