// Encoder front end, one workgroup (4 waves) per 256x256 tile (choh.cpp:464-500 tiles are
// independent), streaming the tile in raster blocks of 256 pixels (one barrier per block):
//  * subtract-green (channel.hpp:73-79) + MED fast-path residuals for the three planes
//    (prediction.hpp:6-44), written to the residual arena, histograms in LDS;
//  * grey test (channel.hpp:21-31) and distinct-colour count capped at 257 (choh.cpp:17-46);
//  * LZ candidate detection for find_lz_rgb at -s0 (lz.hpp:32-53): a position q is a candidate
//    iff some back distance b in [1, min(64, q)] gives 4 equal RGB pixels q..q+3 vs q-b..q-b+3.
//    Each wave fingerprints the 4-pixel windows of its 64 positions and of the 64 before them,
//    counts the 128 fingerprints in a wave-private LDS hash table, and checks exactly (b = 1..64,
//    first hit wins) only the positions whose fingerprint occurs twice; equal windows have equal
//    fingerprints, so the candidate set is exact.  The greedy selection runs in k_lz.hip over
//    the (sparse) candidate bitmap.
// Pixels live in an LDS ring (stored twice, so reads at q+k and q-d never wrap); every pixel is
// read from HBM once, one block ahead of its use.
#include "hoh_internal.h"

#define RING 2048               // pixels: >= the 1024-pixel span [q - 512, q + 512) in use
#define WTAB 512                // slots of a wave's fingerprint table (128 keys)
#define NT 256

__device__ __forceinline__ uint16_t med16(uint16_t a, uint16_t b, uint16_t c) {
  // predictor_operations.hpp:37-60, uint16_t overload (selected by overload resolution: Q8)
  if (a > b) return b > c ? b : (c > a ? a : c);
  return b < c ? b : (c > a ? c : a);
}

__device__ __forceinline__ uint32_t plane_val(uint32_t px, int k) {
  uint32_t r = px & 255, g = (px >> 8) & 255, b = px >> 16;
  return k == 0 ? g : k == 1 ? r - g + 256 : b - g + 256;
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
  for (int probe = 0; probe < WTAB; probe++) {
    const uint32_t old = atomicCAS(&key[sl], 0u, k);
    if (old == 0u) return sl;
    if (old == k) { atomicOr(&dup[sl >> 5], 1u << (sl & 31)); return sl; }
    sl = (sl + 1) & (WTAB - 1);
  }
  return WTAB;
}

__global__ __launch_bounds__(NT) void k_front(EncodeJob j) {
  __shared__ uint32_t ring[2 * RING];
  __shared__ uint32_t wkey[4][WTAB];
  __shared__ uint32_t wdup[4][WTAB / 32];
  __shared__ uint32_t hist[3][512];
  __shared__ uint32_t hset[1024];
  __shared__ uint32_t hpos[1024];                   // first raster position of each colour
  __shared__ int s_ncol, s_notgrey, s_ncand, s_np;

  const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int gt = j.t0 + t;
  const int x0 = (gt % j.xt) * j.tw, y0 = (gt / j.xt) * j.th;
  const int w = min(j.tw, j.W - x0), h = min(j.th, j.H - y0);
  const uint32_t npix = (uint32_t)w * h;
  for (int i = tid; i < 3 * 512; i += NT) (&hist[0][0])[i] = 0;
  for (int i = tid; i < 1024; i += NT) { hset[i] = 0xffffffffu; hpos[i] = 0xffffffffu; }
  for (int i = lane; i < WTAB; i += 64) wkey[wv][i] = 0;
  if (lane < WTAB / 32) wdup[wv][lane] = 0;
  if (tid == 0) { s_ncol = 0; s_notgrey = 0; s_ncand = 0; s_np = 0; }

  uint16_t* res[3];
  for (int k = 0; k < 3; k++) res[k] = j.sym + med_plane_off(j, t, k);
  uint64_t* cand = j.candbits + (size_t)t * (j.npix_cap / 64);
  const uint8_t* img = j.rgb + ((size_t)y0 * j.W + x0) * 3;
  const size_t pitch = (size_t)j.W * 3;

  // loader cursor: this thread's pixel of the block being loaded (raster blk*256 + tid)
  int lx = tid, ly = 0;
  while (lx >= w) { lx -= w; ly++; }
  auto load_px = [&](uint32_t q) -> uint32_t {
    if (q >= npix) return 0;
    const uint8_t* p = img + (size_t)ly * pitch + (size_t)lx * 3;
    return p[0] | (p[1] << 8) | (p[2] << 16);
  };
  auto advance = [&]() { lx += NT; while (lx >= w) { lx -= w; ly++; } };
  {
    const uint32_t v0 = load_px(tid);
    ring[tid & (RING - 1)] = v0;
    ring[(tid & (RING - 1)) + RING] = v0;
    advance();
  }
  uint32_t nextv = load_px(NT + tid);
  advance();
  // compute cursor: (x, y) of position base + tid
  uint32_t cx = tid, cy = 0;
  while (cx >= (uint32_t)w) { cx -= w; cy++; }
  __syncthreads();

  int notgrey = 0, ncand = 0;
  const uint32_t nblk = (npix + NT - 1) / NT;
  for (uint32_t blk = 0; blk < nblk; blk++) {
    const uint32_t base = blk * NT;
    {   // land block blk+1, issue block blk+2
      const uint32_t qn = base + NT + tid;
      ring[qn & (RING - 1)] = nextv;
      ring[(qn & (RING - 1)) + RING] = nextv;
      nextv = load_px(base + 2 * NT + tid);
      advance();
    }
    __syncthreads();
    const uint32_t q = base + tid;
    const bool act = q < npix;
    const uint32_t ri = q & (RING - 1);
    const uint32_t* fwd = ring + ri;              // fwd[k] = pixel q + k
    const uint32_t* bwd = ring + ri + RING;       // bwd[-d] = pixel q - d
    const uint32_t v = fwd[0];
    if (act) {
      const uint32_t pr = v & 255, pg = (v >> 8) & 255, pbb = v >> 16;
      notgrey |= (pr != pg) | (pr != pbb);
      if (s_ncol <= 256 && !(j.dbg & 1)) {         // distinct colours, stop past 256
        uint32_t hsh = (v * 2654435761u) >> 22;
        for (int probe = 0; probe < 1024; probe++) {
          uint32_t old = atomicCAS(&hset[hsh], 0xffffffffu, v);
          if (old == 0xffffffffu) { atomicAdd(&s_ncol, 1); atomicMin(&hpos[hsh], q); break; }
          if (old == v) { atomicMin(&hpos[hsh], q); break; }
          hsh = (hsh + 1) & 1023;
        }
      }
      const bool hasL = cx > 0, hasT = cy > 0;
      const uint32_t vL = hasL ? bwd[-1] : 0;
      const uint32_t vT = hasT ? bwd[-w] : 0;
      const uint32_t vTL = (hasL && hasT) ? bwd[-w - 1] : 0;
#pragma unroll
      for (int k = 0; k < 3; k++) {
        const int c = k ? 512 : 256, half = c / 2;
        uint16_t L = hasL ? (uint16_t)plane_val(vL, k) : (uint16_t)half;
        uint16_t T = hasT ? (uint16_t)plane_val(vT, k) : (uint16_t)half;
        uint16_t TL = (hasL && hasT) ? (uint16_t)plane_val(vTL, k) : (uint16_t)half;
        uint16_t p = med16(T, L, (uint16_t)(T + L - TL));
        uint32_t r = ((int)plane_val(v, k) - (int)p + half + c) & (c - 1);
        res[k][q] = (uint16_t)r;
        if (!(j.dbg & 2)) atomicAdd(&hist[k][r], 1u);
      }
    }
    cx += NT;
    while (cx >= (uint32_t)w) { cx -= w; cy++; }
    // LZ screen (wave-private): windows at q and at q - 64
    const bool win = q + 3 < npix;                 // a 4-pixel window starts here
    const uint32_t hq = win ? fp32(v, fwd[1], fwd[2], fwd[3]) : 0u;
    const bool winp = q >= 64 && q - 61 < npix;    // window at q - 64 lies in the tile
    const uint32_t hp = winp ? fp32(bwd[-64], bwd[-63], bwd[-62], bwd[-61]) : 0u;
    uint32_t* key = wkey[wv];
    uint32_t* dup = wdup[wv];
    uint32_t sq = WTAB, sp = WTAB;
    if (!(j.dbg & 4) && j.speed == 0) {         // -s>=1: k_lzcand screens a longer window
      if (hq) sq = wt_insert(key, dup, hq);
      if (hp) sp = wt_insert(key, dup, hp);
    }
    const bool hit = hq && sq < WTAB && ((dup[sq >> 5] >> (sq & 31)) & 1);
    const uint64_t flag = __ballot(hit);
    uint64_t word = 0;
    if (flag) {
      // exact check for the flagged lanes (lz.hpp:37-42 with offset < 4)
      bool c = false;
      if (hit) {
        const uint32_t bmax = q < 64 ? q : 64;
        const uint32_t v1 = fwd[1], v2 = fwd[2], v3 = fwd[3];
        for (uint32_t b = 1; b <= bmax && !c; b++)
          c = bwd[-(int)b] == v && bwd[1 - (int)b] == v1 && bwd[2 - (int)b] == v2 && bwd[3 - (int)b] == v3;
      }
      word = __ballot(c);
    }
    // clear the slots this wave used (wave-ordered LDS: the reads above are done)
    if (sq < WTAB) key[sq] = 0;
    if (sp < WTAB) key[sp] = 0;
    if (lane < WTAB / 32) dup[lane] = 0;
    if (lane == 0 && (q >> 6) < (npix + 63) / 64) cand[q >> 6] = word;
    ncand += lane == 0 ? __popcll(word) : 0;
  }
  if (notgrey) atomicOr(&s_notgrey, 1);
  if (ncand) atomicAdd(&s_ncand, ncand);
  __syncthreads();
  for (int i = tid; i < 3 * 512; i += NT) {
    const int k = i / 512, s = i % 512;
    j.hist[(size_t)(t * j.spt + med_kind(j, k)) * 512 + s] = hist[k][s];
  }
  if (s_ncol <= 256 && s_notgrey) {
    // palette in first-occurrence order (choh.cpp:64-88): rank of a colour = number of colours
    // whose first position is smaller (the ring is free now)
    uint32_t* pc = ring;
    uint32_t* pp = ring + 256;
    for (int i = tid; i < 1024; i += NT) {
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
  }
  if (tid == 0) {
    TileInfo ti;
    ti.x0 = x0; ti.y0 = y0; ti.w = w; ti.h = h;
    ti.colours = s_ncol > 256 ? -1 : s_ncol;
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

// Indexed plane of a palette-candidate tile (choh.cpp:48-102 palette_encode + layer_encode -s0):
// index = first-occurrence rank of the pixel's colour, then the MED fast-path residual at depth 8
// (prediction.hpp:6-44) and its histogram.  One workgroup per tile; pass 1 writes the indices
// into the tile's indexed-plane slot, pass 2 turns them into residuals in place, walking blocks
// from the last to the first so every neighbour (q-1, q-w, q-w-1) is still an index when read.
__global__ __launch_bounds__(NT) void k_palette(EncodeJob j) {
  __shared__ uint32_t hk[1024];
  __shared__ uint32_t hv[1024];
  __shared__ uint32_t phist[256];
  const int t = blockIdx.x, tid = threadIdx.x;
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
  hipLaunchKernelGGL(k_palette, dim3(j.ntiles), dim3(NT), 0, s, j);
}

void launch_front(const EncodeJob& j, hipStream_t s) {
  hipLaunchKernelGGL(k_front, dim3(j.ntiles), dim3(NT), 0, s, j);
}
