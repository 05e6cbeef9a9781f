// Greedy RGB LZ of find_lz_rgb at -s0 (lz.hpp:6-170), one wave per tile.
// k_front marked every position whose longest match is >= 4; here the greedy scan walks those
// candidates in order: at a candidate the 64 lanes measure the run length at the 64 back
// distances (lane = back-1) and reduce to (longest, smallest back) exactly like lz.hpp:35-53.
// Then the three LZ symbol streams are generated, and if any pixel was matched ("nuked") the
// residual streams of the three planes are compacted and their histograms corrected
// (layer_encode.hpp:93-99).  Also fills the StreamInfo of the tile's streams.
#include "hoh_internal.h"

#include <algorithm>

__device__ __forceinline__ uint32_t img_px(const EncodeJob& j, int x0, int y0, int w, uint32_t q) {
  const uint8_t* p = j.rgb + ((size_t)(y0 + (int)(q / w)) * j.W + x0 + (int)(q % w)) * 3;
  return p[0] | (p[1] << 8) | (p[2] << 16);
}

#ifndef LZ_SEG
#define LZ_SEG 4          // waves per tile (segments scanned speculatively, section below)
#endif
#ifndef LZ_FILL
#define LZ_FILL 2         // 64-position chunks per batch of ring loads (2: a 512-position ring, 24 KB per tile: natural -s0 pipeline +5% against 4)
#endif
#define LZR (LZ_FILL >= 4 ? 1024 : 512)   // pixel ring of a k_lz wave: [q - 64, q + 260 + 64 LZ_FILL)

#define LZ_BITS_MAX 1024   // candidate words kept in LDS (tiles up to 65,536 pixels)
// The greedy walk is serial (the next decision is at the first candidate after the last match),
// but the walk from any position is a function of that position alone, so a tile is cut into
// LZ_SEG segments of whole 64-position words walked at once, each from its own first position
// (one wave each, matches packed into lzspec), every visited candidate marked in an LDS bitmap.
// Wave 0 then stitches: segment s's true walk enters at the exit of s - 1's; from there it is
// re-walked until it reaches a candidate segment s's own walk visited (from then on the two
// coincide: that walk's matches from this candidate on, and its exit, are the true ones) or
// leaves the segment.  Matches are decided exactly as before, so the list is the serial one.
__global__ __launch_bounds__(64 * LZ_SEG) void k_lz(EncodeJob j) {
  __shared__ uint32_t ring[LZ_SEG][LZR + 16];        // + a mirror of entries 0..15
  __shared__ uint64_t cbits[LZ_BITS_MAX];
  __shared__ uint32_t vis[2 * LZ_BITS_MAX];          // visited candidates (segmented walks only)
  __shared__ uint32_t s_cnt[LZ_SEG], s_exit[LZ_SEG];
#ifdef LZ_DBG
  __shared__ uint32_t s_dbg[LZ_SEG][3];
  const uint64_t dbg_t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t dbg_vis = 0, dbg_fix = 0, dbg_rounds = 0;
#endif
  const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  TileInfo ti = j.tiles[t];
  const uint32_t npix = (uint32_t)ti.w * ti.h;
  const uint32_t nwords = (npix + 63) / 64;
  uint64_t* bits = j.candbits + (size_t)t * (j.npix_cap / 64);
  uint32_t* mt = j.matches + (size_t)t * 3 * (j.lz_cap + 1);
  int bonus = 0;                                                      // choh.cpp:139-154
  if (ti.colours != -1) {
    if (ti.colours <= 4) bonus = 32;
    else if (ti.colours <= 8) bonus = 20;
    else if (ti.colours <= 16) bonus = 10;
    else if (ti.colours <= 32) bonus = 2;
  }
  const uint32_t thr = 4 + bonus;
  // the candidate bitmap in LDS: the scan searches it once per step (natural tiles: thousands)
  const bool lds_bits = nwords <= LZ_BITS_MAX;
  // segmented walks need the LDS bitmaps and 16-bit positions (lzspec entries)
  const uint32_t nseg = (lds_bits && nwords >= 4 * LZ_SEG) ? LZ_SEG : 1;
  const uint32_t segcap = j.lz_cap / LZ_SEG;
  uint32_t* spec = j.lzspec + (size_t)t * j.lz_cap;
  auto seg_lo = [&](uint32_t s) { return s >= nseg ? npix : (nwords * s / nseg) * 64; };
  if (ti.ncand) {
    for (uint32_t i = tid; i < nwords; i += 64 * LZ_SEG) cbits[i] = lds_bits ? bits[i] : 0;
    if (nseg > 1)
      for (uint32_t i = tid; i < 2 * nwords; i += 64 * LZ_SEG) vis[i] = 0;
  }
  __syncthreads();
  // The run lengths compare pixels q + k with q + k - b (b <= 64, k < 259): they come from the
  // wave's LDS ring holding the tile positions [wlo, wend) (wend - wlo <= LZR), loaded 256 at a
  // time as the scan moves and only around candidates (natural tiles hold thousands of copies and
  // per-step global reads made this kernel ~16 ms per image)
  uint32_t* rg = ring[wv];
  const int x0 = ti.x0, y0 = ti.y0, tw = ti.w;
  uint32_t wend = 0;
  auto fill_to = [&](uint32_t lo, uint32_t need) {
    if (lo > wend) wend = lo & ~63u;                  // nothing needed in between
    while (wend < need) {                             // 64 LZ_FILL positions per batch of loads
      // unconditional loads (positions past the tile read its last pixel and are replaced after):
      // a load under a lane condition is awaited inside its branch, one round trip per chunk
      uint32_t v[LZ_FILL];
#pragma unroll
      for (int u = 0; u < LZ_FILL; u++) v[u] = img_px(j, x0, y0, tw, min(wend + 64u * u + (uint32_t)lane, npix - 1));
#pragma unroll
      for (int u = 0; u < LZ_FILL; u++) {
        const uint32_t p = wend + 64u * u + (uint32_t)lane, e = p & (LZR - 1);
        const uint32_t x = p < npix ? v[u] : 0xff000000u;
        rg[e] = x;
        if (e < 16) rg[e + LZR] = x;                  // the mirror: 16 entries read from any base
      }
      wend += 64 * LZ_FILL;
    }
    // the wave's own ring: its LDS accesses are ordered without a barrier
  };
  uint32_t cwi = 0xffffffffu;                         // the bitmap word last read, kept in registers
  uint64_t cw = 0;
  // first candidate q >= pos (0xffffffff: none)
  auto next_cand = [&](uint32_t pos) -> uint32_t {
    if (pos >= npix) return 0xffffffffu;
    if (lds_bits) {                                   // usually in pos's own word
      // (kept in VGPRs: readfirstlane on the word or on q measured 1.7x / 1.05x slower)
      if ((pos >> 6) != cwi) { cwi = pos >> 6; cw = cbits[cwi]; }
      const uint64_t wv2 = cw & (~0ull << (pos & 63));
      if (wv2) return (pos & ~63u) + (uint32_t)(__ffsll((unsigned long long)wv2) - 1);
    }
    for (uint32_t wi = pos >> 6; wi < nwords; wi += 64) {
      uint64_t w2 = (wi + lane < nwords) ? (lds_bits ? cbits[wi + lane] : bits[wi + lane]) : 0;
      if (wi + lane == (pos >> 6)) w2 &= ~0ull << (pos & 63);
      const uint64_t bal = __ballot(w2 != 0);
      if (bal) {
        const int l = __ffsll((unsigned long long)bal) - 1;
        const uint64_t word = __shfl(w2, l);
        return (wi + l) * 64 + (__ffsll((unsigned long long)word) - 1);
      }
    }
    return 0xffffffffu;
  };
  // (longest, smallest back) at candidate q, lz.hpp:35-53: lane = back - 1
  auto measure = [&](uint32_t q) -> uint32_t {
    fill_to(q >= 64 ? q - 64 : 0, q + 260);
    const uint32_t b = lane + 1;
    const uint32_t lim = min(259u, npix - q);
    uint32_t L = 0;
    // Inside a run of equal pixels (q - 1 equals q): for every back b whose q - b .. q - 1 are
    // all that pixel the copy runs exactly to the end of q's own run (the older side still holds
    // the pixel where q's run has ended), so those lanes take q's run length (64 positions per
    // LDS read) instead of comparing 16 at a time up to 259.
    bool inrun = false;
    const uint32_t c0 = rg[q & (LZR - 1)];
    if (q >= 1 && rg[(q - 1) & (LZR - 1)] == c0) {                     // wave-uniform
      const uint64_t m = __ballot(b <= q && rg[(q - b) & (LZR - 1)] == c0);
      const uint32_t B = ~m ? (uint32_t)(__ffsll((unsigned long long)~m) - 1) : 64u;   // backs 1..B in the run
      uint32_t rq = 0;
      for (;;) {
        const uint64_t e = __ballot(rq + lane < lim && rg[(q + rq + lane) & (LZR - 1)] == c0);
        if (~e) { rq += (uint32_t)(__ffsll((unsigned long long)~e) - 1); break; }
        rq += 64;
      }
      inrun = b <= B;
      if (inrun) L = rq;
    }
    if (b <= q && !inrun) {
      // sixteen positions per LDS round trip from two bases (the mirror spares every read its
      // wrap), the first unequal one by a select chain
      for (;;) {
        const uint32_t* pa = rg + ((q + L) & (LZR - 1));
        const uint32_t* pc = rg + ((q + L - b) & (LZR - 1));
        uint32_t a[16], c[16];
#pragma unroll
        for (int u = 0; u < 16; u++) { a[u] = pa[u]; c[u] = pc[u]; }
        uint32_t r0 = 8, r1 = 16;                     // two chains: no compare-to-select stalls
#pragma unroll
        for (int u = 7; u >= 0; u--) {
          r1 = a[u + 8] != c[u + 8] ? (uint32_t)u + 8 : r1;
          r0 = a[u] != c[u] ? (uint32_t)u : r0;
        }
        const uint32_t run = r0 < 8 ? r0 : r1;
        L = min(L + run, lim);
#ifdef LZ_DBG
        if (lane == 0) dbg_rounds++;
#endif
        if (run < 16 || L >= lim) break;
      }
    }
    return wave_max_u32((L << 8) | (255u - b));
  };
  uint32_t nm = 0;
  bool overflow = false;
  auto emit = [&](uint32_t q, uint32_t longest, uint32_t best) {
    if (nm < j.lz_cap) {
      if (lane == 0) { mt[3 * nm] = q; mt[3 * nm + 1] = longest; mt[3 * nm + 2] = best; }
    } else {
      overflow = true;
    }
    nm++;
  };
  // ---- phase 1: every segment's own walk (nseg == 1: the serial walk, straight into mt)
  if (ti.ncand && (uint32_t)wv < nseg) {
    const uint32_t lo = seg_lo(wv), hi = seg_lo(wv + 1);
    uint32_t pos = lo, cnt = 0;
    while (pos < hi) {
      const uint32_t q = next_cand(pos);
      if (q >= hi) break;
      if (nseg > 1 && lane == 0) atomicOr(&vis[q >> 5], 1u << (q & 31));   // no round trip
#ifdef LZ_DBG
      dbg_vis++;
#endif
      const uint32_t key = measure(q);
      const uint32_t longest = key >> 8, best = 255u - (key & 255);
      if (longest >= thr) {
        if (nseg == 1) emit(q, longest, best);
        else if (cnt < segcap && lane == 0) spec[wv * segcap + cnt] = q | ((longest - 4) << 16) | ((best - 1) << 24);
        cnt++;
        pos = q + longest;
      } else {
        pos = q + 1;
      }
    }
    if (lane == 0) { s_cnt[wv] = cnt; s_exit[wv] = max(pos, hi); }
  }
#ifdef LZ_DBG
  if (lane == 0) {
    s_dbg[wv][0] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - dbg_t0);
    s_dbg[wv][1] = dbg_vis;
    s_dbg[wv][2] = dbg_rounds;
  }
#endif
  if (nseg > 1) {
    __syncthreads();
    if (wv) return;
    // ---- phase 2 (wave 0): stitch the segments
    uint32_t pos = 0;
    for (uint32_t s = 0; s < (ti.ncand ? nseg : 0u); s++) {
      const uint32_t hi = seg_lo(s + 1), cnt = s_cnt[s];
      if (cnt > segcap) { overflow = true; nm += cnt; continue; }     // cannot happen: lz_cap >= npix / 4 + 16
      uint32_t from = 0;                                              // first valid entry of s's walk
      bool conv = s == 0;
      if (s > 0) {
        while (pos < hi) {
          const uint32_t q = next_cand(pos);
          if (q >= hi) { pos = hi; break; }
          if ((vis[q >> 5] >> (q & 31)) & 1) { conv = true; pos = q; break; }
#ifdef LZ_DBG
          dbg_fix++;
#endif
          const uint32_t key = measure(q);
          const uint32_t longest = key >> 8, best = 255u - (key & 255);
          if (longest >= thr) { emit(q, longest, best); pos = q + longest; }
          else pos = q + 1;
        }
        if (conv) {                                                   // first entry at or after pos
          from = cnt;
          for (uint32_t i0 = 0; i0 < cnt; i0 += 64) {
            const uint32_t i = i0 + lane;
            const uint64_t m = __ballot(i < cnt && (spec[s * segcap + i] & 0xffffu) >= pos);
            if (m) { from = i0 + (uint32_t)(__ffsll((unsigned long long)m) - 1); break; }
          }
        }
      }
      if (conv) {
        for (uint32_t i0 = from; i0 < cnt; i0 += 256) {               // four loads in flight
          uint32_t e[4];
#pragma unroll
          for (int u = 0; u < 4; u++) e[u] = spec[s * segcap + min(i0 + 64u * u + lane, cnt - 1)];
#pragma unroll
          for (int u = 0; u < 4; u++) {
            const uint32_t i = i0 + 64u * u + lane, k = nm + (i - from);
            if (i < cnt && k < j.lz_cap) { mt[3 * k] = e[u] & 0xffffu; mt[3 * k + 1] = ((e[u] >> 16) & 255u) + 4; mt[3 * k + 2] = (e[u] >> 24) + 1; }
          }
        }
        nm += cnt - from;
        if (nm > j.lz_cap) overflow = true;
        pos = s_exit[s];
      }
    }
#ifdef LZ_DBG
    if (lane == 0) {
      uint32_t w = 0;
      for (uint32_t k = 1; k < nseg; k++) if (s_dbg[k][0] > s_dbg[w][0]) w = k;
      mt[3 * j.lz_cap] = s_dbg[w][0];
      mt[3 * j.lz_cap + 1] = s_dbg[w][1] | (dbg_fix << 16);
      mt[3 * j.lz_cap + 2] = s_dbg[w][2];
    }
#endif
  } else if (wv) {
    return;
  }
  // --- LZ symbol streams (lz.hpp:75-95): future (gaps, 255-chunked), length-4, back%256
  uint16_t* lz0 = j.sym + (size_t)j.ntiles * 3 * j.npix_cap + (size_t)(t * 3) * j.lz_cap;
  uint16_t* lz1 = lz0 + j.lz_cap;
  uint16_t* lz2 = lz1 + j.lz_cap;
  uint32_t nf = 0, prev_end = 0;
  const uint32_t nmk = nm < j.lz_cap ? nm : j.lz_cap;
  for (uint32_t m = 0; m <= nmk; m++) {
    const bool tail = m == nmk;
    const uint32_t mpos = tail ? npix : mt[3 * m];
    const uint32_t g = mpos - prev_end;
    const uint32_t n255 = g / 255;
    if (nf + n255 + 1 > j.lz_cap) { overflow = true; break; }
    for (uint32_t k = lane; k < n255; k += 64) lz0[nf + k] = 255;
    nf += n255;
    if (!tail) {
      if (lane == 0) {
        lz0[nf] = (uint16_t)(g % 255);
        lz1[m] = (uint16_t)(mt[3 * m + 1] - 4);
        lz2[m] = (uint16_t)(mt[3 * m + 2] % 256);
      }
      nf++;
      prev_end = mpos + mt[3 * m + 1];
    }
  }
  // --- nuked pixels (compaction of the residual planes runs in k_nuke)
  uint32_t nclean = npix;
  if (nmk && !overflow) {
    uint32_t nk = 0;
    for (uint32_t m = lane; m < nmk; m += 64) nk += mt[3 * m + 1];
    for (int o = 32; o > 0; o >>= 1) nk += __shfl_xor(nk, o);
    nclean = npix - nk;
  }
  if (lane == 0) {
    if (overflow) ti.flags |= TF_OVERFLOW;
    ti.nmatch = nm;
    j.tiles[t] = ti;
    const bool planes = !(ti.flags & TF_GREY);
    const size_t pl_slab = (size_t)j.npix_cap + 8;
    const size_t lz_slab = (size_t)j.lz_cap + 8;
    for (int k = 0; k < j.spt; k++) {
      StreamInfo st;
      memset(&st, 0, sizeof(st));
      if (k < 3) {
        st.sym_off = (size_t)j.ntiles * 3 * j.npix_cap + (size_t)(t * 3 + k) * j.lz_cap;
        st.slab_off = (size_t)j.ntiles * 3 * pl_slab + (size_t)(t * 3 + k) * lz_slab;
        st.slab_cap = (uint32_t)lz_slab;
        st.n = k == 0 ? nf : nmk;
        st.range = 256;
        st.pb = 10;                                                   // lz.hpp:100-142
        st.fast = 1;                                                  // k_tables decides
      } else if (k < SK_I) {
        st.sym_off = (size_t)(t * 3 + k - 3) * j.npix_cap;
        st.slab_off = (size_t)(t * 3 + k - 3) * pl_slab;
        st.slab_cap = (uint32_t)pl_slab;
        st.n = planes ? nclean : 0;
        st.range = planes ? (k == SK_G ? 256 : 512) : 0;              // choh.cpp:221-255; 0 = absent
        st.pb = 15;                                                   // layer_encode.hpp:59
        st.fast = planes ? 1 : 0;
      } else {                                                        // indexed plane (choh.cpp:90-99)
        const bool pal = planes && (ti.flags & TF_PALETTE_CAND);
        st.sym_off = idx_plane_off(j, t);
        st.slab_off = idx_slab_off(j, t);
        st.slab_cap = (uint32_t)pl_slab;
        st.n = pal ? nclean : 0;
        st.range = pal ? 256 : 0;
        st.pb = 15;
        st.fast = pal ? 1 : 0;
      }
      st.mode = SM_EMPTY;
      st.hist_src = k >= SK_G ? (uint32_t)(t * j.spt + k) + 1 : 0;   // planes: k_front's histograms
      st.ckpt_off = (uint32_t)((size_t)(t * j.spt + k) * (j.npix_cap / HOH_SEG + 2));
      j.streams[t * j.spt + k] = st;
    }
  }
}

// Residual compaction of tiles with LZ copies (layer_encode.hpp:93-99): nuked pixels leave
// the three residual planes (four with the indexed plane; order kept) and their histograms.
// One 256-thread workgroup per tile; the nuke bitmap is built in LDS from the match list, then the plane is walked in
// 256-pixel blocks with a block-wide rank of the kept pixels.
__device__ __forceinline__ void nuke_tile(const EncodeJob& j, int t, uint32_t* nk_bits, uint32_t* wsum, bool in_lds);
// 2048-pixel blocks, eight pixels per thread: 16-B plane loads and stores (below)
#define NK_B 2048
template <int NPM>
__device__ __forceinline__ void nuke_tile_v(const EncodeJob& j, int t, uint32_t* nk_bits, uint32_t* wsum,
                                            uint16_t (*nkbuf)[NK_B + 16]);

// nuke bitmap + removed-count histograms in LDS need (npix_cap/32 + 1 + slots*512) words; a
// single tile too large for that (untiled images over ~1.1 M px: the LDS holds 160 KB) takes the
// same walk with the match list searched per pixel and the counts subtracted in global memory.
__host__ __device__ static inline int nuke_slots(const EncodeJob& j) { return j.speed ? 2 * HOH_NPLANE_S : 4; }
#define NK_LDS_MAX (160 * 1024 - 256 - 2 * (NK_B + 16) * 2)   // beside the staging buffers

// A small grid strides over the tiles (most have no match): a launch over every tile dispatches
// ~1000 idle workgroups, which waits for free CUs when other images are in flight.
// registers held to 6 waves per SIMD (80 VGPRs, was 116: four workgroups per CU where the 16 KB
// of LDS allows nine; a 112-byte spill): natural -s0 pipeline 47.8 -> 48.7 GB/s (8 waves, 64
// VGPRs: 47.5)
#ifndef NUKE_WPE
#define NUKE_WPE 6
#endif
#if NUKE_WPE
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NUKE_WPE, NUKE_WPE)))
#else
__global__ __launch_bounds__(256)
#endif
void k_nuke(EncodeJob j, int in_lds) {
  extern __shared__ uint32_t nk_bits[];                  // npix_cap / 32 words, then the counts
  __shared__ uint32_t wsum[4];
  for (int t = blockIdx.x; t < j.ntiles; t += gridDim.x) nuke_tile(j, t, nk_bits, wsum, in_lds != 0);
}
// the 16-B walk (nuke_tile_v): NPM planes at most (-s0: 4, -s>=1: 12)
template <int NPM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NPM > 4 ? 4 : NUKE_WPE, NPM > 4 ? 4 : NUKE_WPE)))
void k_nuke_v(EncodeJob j) {
  extern __shared__ uint32_t nk_bits[];
  __shared__ uint32_t wsum[4];
  __shared__ __attribute__((aligned(16))) uint16_t nkbuf[2][NK_B + 16];
  for (int t = blockIdx.x; t < j.ntiles; t += gridDim.x) nuke_tile_v<NPM>(j, t, nk_bits, wsum, nkbuf);
}

// matches are disjoint and in increasing position order (the greedy scan of k_lz / k_lzscan):
// p is covered iff the last match starting at or before p reaches past it
__device__ __forceinline__ bool nuked_search(const uint32_t* mt, uint32_t nm, uint32_t p) {
  uint32_t lo = 0, hi = nm;                              // first match with start > p
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (mt[3 * mid] <= p) lo = mid + 1; else hi = mid;
  }
  return lo > 0 && p < mt[3 * (lo - 1)] + mt[3 * (lo - 1) + 1];
}

__device__ __forceinline__ void nuke_tile(const EncodeJob& j, int t, uint32_t* nk_bits, uint32_t* wsum,
                                          bool in_lds) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const TileInfo ti = j.tiles[t];
  const uint32_t nm = ti.nmatch;
  if (nm == 0 || (ti.flags & TF_OVERFLOW) || nm > j.lz_cap) return;
  const uint32_t npix = (uint32_t)ti.w * ti.h, nwords = (npix + 31) / 32;
  const uint32_t* mt = j.matches + (size_t)t * 3 * (j.lz_cap + 1);
  const int nslots = nuke_slots(j);
  uint32_t* nh = nk_bits + j.npix_cap / 32 + 1;          // removed counts, [slot][512]
  if (in_lds) {
    for (uint32_t i = tid; i < nwords; i += 256) nk_bits[i] = 0;
    for (uint32_t i = tid; i < (uint32_t)nslots * 512; i += 256) nh[i] = 0;
    __syncthreads();
    // one thread per match (matches are disjoint): natural tiles hold thousands of short copies
    for (uint32_t m = tid; m < nm; m += 256) {
      const uint32_t a = mt[3 * m], e = a + mt[3 * m + 1];
      for (uint32_t p = a; p < e; p++) atomicOr(&nk_bits[p >> 5], 1u << (p & 31));
    }
    __syncthreads();
  }
  const bool grey = ti.flags & TF_GREY, pal = !grey && (ti.flags & TF_PALETTE_CAND);
  // plane slots: -s0 the MED planes G R' B' (+ indexed); -s>=1 the six MED planes, then the six
  // searched planes, each with its stream's histogram.  The kept pixels' ranks are the same in
  // every plane, so each 256-pixel block ranks once and moves all present planes.
  uint16_t* r[2 * HOH_NPLANE_S];
  uint32_t* hk[2 * HOH_NPLANE_S];
  int np = 0;
  for (int k = 0; k < nslots; k++) {
    const int p = k % HOH_NPLANE_S;
    const bool present = !grey && (p < 3 || (p == 3 && pal) || (p >= 4 && j.speed >= 3));
    if (!present) continue;
    if (k < HOH_NPLANE_S || !j.speed) {
      r[np] = j.sym + med_plane_off(j, t, p);
      hk[np] = j.hist + (size_t)(t * j.spt + med_kind(j, p)) * 512;
    } else {
      r[np] = j.sym + fin_plane_off(j, t, p);
      hk[np] = j.hist + (size_t)(t * j.spt + KS_FIN + p) * 512;
    }
    np++;
  }
  if (np == 0) return;
  uint32_t outc = 0;
  // the next block's values are loaded before this block's ranks (they lie above every write of
  // this block: a block's writes land below its own end)
  uint16_t vn[2 * HOH_NPLANE_S];
#pragma unroll
  for (int k = 0; k < 2 * HOH_NPLANE_S; k++) vn[k] = (k < np && (uint32_t)tid < npix) ? r[k][tid] : 0;
  for (uint32_t base = 0; base < npix; base += 256) {
    const uint32_t p = base + tid;
    const bool valid = p < npix;
    uint16_t v[2 * HOH_NPLANE_S];
#pragma unroll
    for (int k = 0; k < 2 * HOH_NPLANE_S; k++) v[k] = vn[k];
#pragma unroll
    for (int k = 0; k < 2 * HOH_NPLANE_S; k++) vn[k] = (k < np && p + 256 < npix) ? r[k][p + 256] : 0;
    const bool nuked = valid && (in_lds ? ((nk_bits[p >> 5] >> (p & 31)) & 1) : nuked_search(mt, nm, p));
    if (nuked) {                                        // counted in LDS, applied once below
#pragma unroll
      for (int k = 0; k < 2 * HOH_NPLANE_S; k++)
        if (k < np) {
          if (in_lds) atomicAdd(&nh[k * 512 + v[k]], 1u);
          else atomicSub(&hk[k][v[k]], 1u);
        }
    }
    const bool keep = valid && !nuked;
    const uint64_t bal = __ballot(keep);
    if (lane == 0) wsum[wv] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t before = 0, tot = 0;
    for (int q = 0; q < 4; q++) { const uint32_t c = wsum[q]; if (q < wv) before += c; tot += c; }
    const uint32_t dest = outc + before + (uint32_t)__popcll(bal & ((1ull << lane) - 1));
    __syncthreads();
    // in place: dest <= p, and every block reads its values before any write of this pass
    // reaches them (writes of block i land below block i's end)
    if (keep) {
#pragma unroll
      for (int k = 0; k < 2 * HOH_NPLANE_S; k++) if (k < np) r[k][dest] = v[k];
    }
    outc += tot;
  }
  __syncthreads();
  if (in_lds) {
#pragma unroll
    for (int k = 0; k < 2 * HOH_NPLANE_S; k++)
      if (k < np)
        for (uint32_t i = tid; i < 512; i += 256)
          if (nh[k * 512 + i]) hk[k][i] -= nh[k * 512 + i];  // this tile's histograms: one writer
  }
  __syncthreads();
}

// The LDS-bitmap walk in 2048-pixel blocks: thread i takes pixels 8i .. 8i+7 of the block, every
// plane's eight values in one 16-B load; the kept ones are ranked once per block (eight bits of
// the nuke bitmap per thread, one block scan), and each plane's kept values are staged in LDS at
// their destination's offset from the 16-B line below it, so they leave as 16-B stores too (the
// first and last partial lines element by element).  Two staging buffers alternate: one barrier
// per plane.  (The 256-pixel walk of nuke_tile moved one u16 per thread per plane behind two
// barriers a block: 2.3 GB in 1.4 ms per natural 8192^2 -s4 launch, twelve planes a tile.)
// In place: a block's writes land below its own end, and every block reads its values first.
template <int NPM>
__device__ __forceinline__ void nuke_tile_v(const EncodeJob& j, int t, uint32_t* nk_bits, uint32_t* wsum,
                                            uint16_t (*nkbuf)[NK_B + 16]) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const TileInfo ti = j.tiles[t];
  const uint32_t nm = ti.nmatch;
  if (nm == 0 || (ti.flags & TF_OVERFLOW) || nm > j.lz_cap) return;
  const uint32_t npix = (uint32_t)ti.w * ti.h, nwords = (npix + 31) / 32;
  const uint32_t* mt = j.matches + (size_t)t * 3 * (j.lz_cap + 1);
  const int nslots = nuke_slots(j);
  uint32_t* nh = nk_bits + j.npix_cap / 32 + 1;          // removed counts, [slot][512]
  for (uint32_t i = tid; i < nwords + 1; i += 256) nk_bits[i] = 0;
  for (uint32_t i = tid; i < (uint32_t)nslots * 512; i += 256) nh[i] = 0;
  __syncthreads();
  for (uint32_t m = tid; m < nm; m += 256) {             // one thread per match (disjoint)
    const uint32_t a = mt[3 * m], e = a + mt[3 * m + 1];
    for (uint32_t p = a; p < e; p++) atomicOr(&nk_bits[p >> 5], 1u << (p & 31));
  }
  __syncthreads();
  const bool grey = ti.flags & TF_GREY, pal = !grey && (ti.flags & TF_PALETTE_CAND);
  // slot k (< nslots <= NPM): -s0 the MED planes G R' B' (+ indexed); -s>=1 the six MED planes,
  // then the six searched planes.  The pointers are recomputed where used (scalar arithmetic), not
  // held: twelve plane and twelve histogram pointers overflowed the scalar registers.
  uint32_t pres = 0;
  for (int k = 0; k < nslots; k++) {
    const int p = k % HOH_NPLANE_S;
    if (!grey && (p < 3 || (p == 3 && pal) || (p >= 4 && j.speed >= 3))) pres |= 1u << k;
  }
  if (pres == 0) return;
  auto plane = [&](int k) -> uint16_t* {
    const int p = k % HOH_NPLANE_S;
    return j.sym + ((k < HOH_NPLANE_S || !j.speed) ? med_plane_off(j, t, p) : fin_plane_off(j, t, p));
  };
  auto histo = [&](int k) -> uint32_t* {
    const int p = k % HOH_NPLANE_S;
    return j.hist + (size_t)(t * j.spt + ((k < HOH_NPLANE_S || !j.speed) ? med_kind(j, p) : KS_FIN + p)) * 512;
  };
  uint32_t outc = 0;
  for (uint32_t base = 0; base < npix; base += NK_B) {
    const uint32_t p0 = base + 8 * (uint32_t)tid;
    const bool full = p0 + 8 <= npix;
    uint4 v[NPM];
#pragma unroll
    for (int k = 0; k < NPM; k++) {
      v[k] = make_uint4(0, 0, 0, 0);
      if ((pres >> k) & 1) {
        const uint16_t* rk = plane(k);
        if (full) v[k] = *(const uint4*)(rk + p0);
        else if (p0 < npix) {
          uint16_t e[8];
#pragma unroll
          for (int i = 0; i < 8; i++) e[i] = p0 + i < npix ? rk[p0 + i] : 0;
          v[k] = make_uint4(e[0] | e[1] << 16, e[2] | e[3] << 16, e[4] | e[5] << 16, e[6] | e[7] << 16);
        }
      }
    }
    const uint32_t valid = p0 >= npix ? 0u : full ? 0xffu : (1u << (npix - p0)) - 1u;
    const uint32_t nk8 = (nk_bits[p0 >> 5] >> (p0 & 31)) & valid;   // p0 % 8 == 0: one word
    const uint32_t keep = valid & ~nk8, cnt = (uint32_t)__popc(keep);
    if (nk8) {                                           // removed values: counted in LDS, applied once below
#pragma unroll
      for (int k = 0; k < NPM; k++)
        if ((pres >> k) & 1) {
          const uint32_t w4[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
          for (int i = 0; i < 8; i++)
            if ((nk8 >> i) & 1) atomicAdd(&nh[k * 512 + ((w4[i >> 1] >> (16 * (i & 1))) & 0xffffu)], 1u);
        }
    }
    // block exclusive scan of the kept counts
    uint32_t incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(incl, o);
      if (lane >= o) incl += u;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    uint32_t before = incl - cnt, tot = 0;
    for (int q = 0; q < 4; q++) { const uint32_t c = wsum[q]; if (q < wv) before += c; tot += c; }
    // global dest outc + i <-> staging slot (outc & 7) + i; 16-B line c of the staging buffer is
    // global elements a0 + 8c .. a0 + 8c + 7 (a0 = outc & ~7)
    const uint32_t sk = (outc & 7u) + before, a0 = outc & ~7u, lo = outc & 7u, hi = lo + tot;
    const uint32_t nln = (hi + 7) / 8;
    uint32_t bsel = 0;                                   // alternates per present plane (slots skip)
#pragma unroll
    for (int k = 0; k < NPM; k++) {
      if ((pres >> k) & 1) {
        uint16_t* b = nkbuf[bsel];
        bsel ^= 1;
        uint16_t* rk = plane(k);
        const uint32_t w4[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
        uint32_t s = sk;
#pragma unroll
        for (int i = 0; i < 8; i++)
          if ((keep >> i) & 1) b[s++] = (uint16_t)(w4[i >> 1] >> (16 * (i & 1)));
        __syncthreads();                                 // also: the other buffer's reads are done
        for (uint32_t c = tid; c < nln; c += 256) {
          const uint32_t e0 = 8 * c;
          if (e0 >= lo && e0 + 8 <= hi) {
            *(uint4*)(rk + a0 + e0) = *(const uint4*)(b + e0);
          } else {
#pragma unroll
            for (int i = 0; i < 8; i++)
              if (e0 + i >= lo && e0 + i < hi) rk[a0 + e0 + i] = b[e0 + i];
          }
        }
      }
    }
    outc += tot;
    __syncthreads();                                     // wsum and the staging buffers are reused
  }
  for (int k = 0; k < NPM; k++)
    if ((pres >> k) & 1) {
      uint32_t* hk = histo(k);
      for (uint32_t i = tid; i < 512; i += 256)
        if (nh[k * 512 + i]) hk[i] -= nh[k * 512 + i];   // this tile's histograms: one writer
    }
  __syncthreads();
}

void launch_lz(const EncodeJob& j, hipStream_t s) {
  hipLaunchKernelGGL(k_lz, dim3(j.ntiles), dim3(64 * LZ_SEG), 0, s, j);
}

void launch_nuke(const EncodeJob& j, hipStream_t s) {
  // Workgroups stride over the tiles (KNOB NUKE_WG_PER_CU x CUs of them): a tile without copies
  // leaves at once, and a grid of one workgroup per tile dispatched ~8,000 such workgroups per
  // batch of eight 8192^2 images behind the other contexts' kernels.
  const size_t lds = ((size_t)j.npix_cap / 32 + 1 + (size_t)nuke_slots(j) * 512) * 4;
  const bool in_lds = lds <= NK_LDS_MAX;
  // -s0 (three or four planes): the 16-B walk (natural 8192^2 encode 7.78 -> 7.67 ms); -s>=1
  // (twelve planes): the 256-pixel walk, whose six waves per SIMD beat the 16-B walk's twelve
  // staged planes per block (1.42 against 1.64 ms alone per natural -s4 launch,
  // profiles/r06b/bench_closing.json speed_roofline_s4)
  const int cap = HOH_KNOB(NUKE_WG_PER_CU, 8) * (j.cus > 0 ? j.cus : 256);
  const dim3 grid(cap > 0 && cap < j.ntiles ? cap : j.ntiles);
  if (!in_lds || j.speed) hipLaunchKernelGGL(k_nuke, grid, dim3(256), in_lds ? lds : 0, s, j, (int)in_lds);
  else hipLaunchKernelGGL(k_nuke_v<4>, grid, dim3(256), lds, s, j);
}
