// -s1..-s4 encoder: cruncher_mode >= 1 of choh (choh.cpp:104-383) and layer_encode
// (layer_encode.hpp:11-412).  Per tile, on top of the -s0 front end (k_front, k_palette):
//  * k_rawmed     MED residuals of the plain R and B planes (-s>=3 RGB mode, choh.cpp:265-293);
//  * k_search     per (tile, plane): entropy estimate from the MED residual histogram, 40-px grid
//                 predictor search (one thread per (cell, mask): the cell walked in raster order,
//                 costs summed in f64 in the reference's order so the selection is bit-identical),
//                 refinement at -s>=3, then channelpredict_all residuals + histogram and the
//                 predictor map;
//  * k_lzfp / k_lzcand / k_lzscan
//                 find_lz_rgb with seek distance 10..14 plus the vertical search (lz.hpp:32-95):
//                 window fingerprints, an exact candidate screen (some earlier equal 4-pixel
//                 window within the seek distance or a whole number of rows above), then the
//                 greedy scan evaluating only candidates, 64 back distances per step;
//  * k_setup_s    stream descriptors: LZ x4, MED at prob_bits 15, size-only encodes of the
//                 searched residuals at prob_bits 16,15,17,18,19,14,13,12, predictor maps;
//  * k_choose_s   the prob_bits ladder and the permanent/dummy buffer logic, including the
//                 stale prefix of Q14; activates the one full encode a layer still needs;
//  * k_layout_s / k_tilebytes_s
//                 colour mode (sub-green / indexed / RGB), layer sizes, offsets, fixed bytes.
// The entropy streams themselves go through k_tables / k_rans_* / k_finalize / k_streambytes.
#include "hoh_internal.h"

#define NT 256

__constant__ uint16_t kMasks[14] = {0x0001, 0x0002, 0x0020, 0x0010, 0xffbf, 0x0003, 0xfffd,
                                    0xfffb, 0xfff7, 0xffef, 0xffdf, 0xff7f, 0xfdff, 0xffff};   // layer_encode.hpp:159-175
__constant__ uint8_t kVarPb[8] = {16, 15, 17, 18, 19, 14, 13, 12};                        // :334-391

__device__ __forceinline__ bool plane_present(const EncodeJob& j, const TileInfo& ti, int p) {
  if (ti.flags & TF_GREY) return false;
  if (p < 3) return true;
  if (p == 3) return (ti.flags & TF_PALETTE_CAND) != 0;
  return j.speed >= 3;
}
__device__ __forceinline__ int plane_depth(int p) { return (p == 1 || p == 2) ? 9 : 8; }

// ---------------------------------------------------------------- predictor primitives (u16)

__device__ __forceinline__ uint32_t med16s(uint32_t a, uint32_t b, uint32_t c) {   // predictor_operations.hpp:37-60
  if (a > b) return b > c ? b : (c > a ? a : c);
  return b < c ? b : (c > a ? c : a);
}
__device__ __forceinline__ uint32_t midp(uint32_t a, uint32_t b) {                 // :8-10
  // a + (b - a) / 2 (truncated) == (a + b + (b < a)) / 2 for a, b < 2^31 (every value here is u16)
  return (a + b + (b < a ? 1u : 0u)) >> 1;
}
__device__ __forceinline__ uint32_t avg3(uint32_t a, uint32_t b, uint32_t c) { return (a + b + c) / 3; }   // :66-68
__device__ __forceinline__ uint32_t paeth(int A, int B, int C) {                   // :89-106
  const int p = A + B - C;
  const int Ap = abs(A - p), Bp = abs(B - p), Cp = abs(C - p);
  if (Ap < Bp) return Ap < Cp ? A : C;
  return Bp < Cp ? B : C;
}

struct Preds { uint32_t v[16]; };

// prediction.hpp:116-133 (section: paeth(L, T, TL)) / :190-207 (all: paeth(L, TL, T))
__device__ __forceinline__ void preds16(uint32_t L, uint32_t T, uint32_t TL, uint32_t TR, bool all, Preds& p) {
  p.v[0] = L; p.v[1] = T; p.v[2] = TL; p.v[3] = TR;
  p.v[4] = med16s(T, L, (T + L - TL) & 0xffffu);
  p.v[5] = midp(L, T); p.v[6] = midp(L, TL); p.v[7] = midp(TL, T); p.v[8] = midp(T, TR);
  p.v[9] = all ? paeth(L, TL, T) : paeth(L, T, TL);
  p.v[10] = avg3(L, L, TL); p.v[11] = avg3(L, TL, TL); p.v[12] = avg3(TL, TL, T);
  p.v[13] = avg3(TL, T, T); p.v[14] = avg3(T, T, TR); p.v[15] = avg3(T, TR, TR);
}

// p.v[k] for a lane-varying k without dynamic register indexing: a 4-level tree of bit blends
// (v_bfi_b32). The masks pass through an empty asm so the compiler cannot see they are 0 / ~0:
// written as selects, it folded the tree into a dynamically indexed private array (Preds and the
// tree levels in scratch, ~12 dependent scratch round trips per pixel step of the cell walk).
__device__ __forceinline__ uint32_t blend(uint32_t a, uint32_t b, uint32_t m) { return (a & ~m) | (b & m); }
__device__ __forceinline__ uint32_t pick(const Preds& p, uint32_t k) {
  uint32_t m0 = 0u - (k & 1u), m1 = 0u - ((k >> 1) & 1u), m2 = 0u - ((k >> 2) & 1u), m3 = 0u - ((k >> 3) & 1u);
  asm volatile("" : "+v"(m0), "+v"(m1), "+v"(m2), "+v"(m3));
  const uint32_t a0 = blend(p.v[0], p.v[1], m0), a1 = blend(p.v[2], p.v[3], m0), a2 = blend(p.v[4], p.v[5], m0),
                 a3 = blend(p.v[6], p.v[7], m0), a4 = blend(p.v[8], p.v[9], m0), a5 = blend(p.v[10], p.v[11], m0),
                 a6 = blend(p.v[12], p.v[13], m0), a7 = blend(p.v[14], p.v[15], m0);
  const uint32_t b0 = blend(a0, a1, m1), b1 = blend(a2, a3, m1), b2 = blend(a4, a5, m1), b3 = blend(a6, a7, m1);
  return blend(blend(b0, b1, m2), blend(b2, b3, m2), m3);
}

// first masked predictor of least |v - p| (prediction.hpp:138-146, :213-224)
// (the smallest key (|v - p_k| << 4) | k over the masked k: |v - p_k| < 2^16 < 2c never fails the
// reference's d < 2c test)
__device__ __forceinline__ uint32_t best_pred(uint32_t v, const Preds& p, uint32_t mask, int c) {
  (void)c;
  uint32_t best = 0xffffffffu;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const uint32_t key = (__builtin_amdgcn_sad_u16(v, p.v[k], 0u) << 4) | (uint32_t)k;
    best = min(best, ((mask >> k) & 1) ? key : 0xffffffffu);
  }
  return best & 15u;
}

// ---------------------------------------------------------------- plane data

// value of plane p at raster position q of tile t (channel.hpp:63-79, choh.cpp:62-88)
__device__ __forceinline__ uint32_t plane_value(const EncodeJob& j, const TileInfo& ti, int t, int p, uint32_t q) {
  if (p == 3) return j.idx8[(size_t)t * j.npix_cap + q];
  const uint32_t y = q / (uint32_t)ti.w, x = q - y * (uint32_t)ti.w;
  const uint8_t* px = j.rgb + ((size_t)(ti.y0 + y) * j.W + ti.x0 + x) * 3;
  const uint32_t r = px[0], g = px[1], b = px[2];
  switch (p) {
    case 0: return g;
    case 1: return r - g + 256;
    case 2: return b - g + 256;
    case 4: return r;
    default: return b;
  }
}

// MED residuals of the plain R and B planes (-s>=3), depth 8, + histograms
__global__ __launch_bounds__(NT) void k_rawmed(EncodeJob j) {
  __shared__ uint32_t hs[2][256];
  const int t = blockIdx.x, tid = threadIdx.x;
  const TileInfo ti = j.tiles[t];
  if (!plane_present(j, ti, 4)) return;
  for (int i = tid; i < 512; i += NT) (&hs[0][0])[i] = 0;
  __syncthreads();
  const uint32_t w = ti.w, npix = w * ti.h;
  for (uint32_t q = tid; q < npix; q += NT) {
    const uint32_t y = q / w, x = q - y * w;
    for (int k = 0; k < 2; k++) {
      const int p = 4 + k;
      const uint32_t v = plane_value(j, ti, t, p, q);
      const uint32_t L = x ? plane_value(j, ti, t, p, q - 1) : 128;
      const uint32_t T = y ? plane_value(j, ti, t, p, q - w) : 128;
      const uint32_t TL = (x && y) ? plane_value(j, ti, t, p, q - w - 1) : 128;
      const uint32_t r = (v - med16s(T, L, (T + L - TL) & 0xffffu) + 128 + 256) & 255;   // prediction.hpp:35
      j.sym[med_plane_off(j, t, p) + q] = (uint16_t)r;
      atomicAdd(&hs[k][r], 1u);
    }
  }
  __syncthreads();
  for (int i = tid; i < 1024; i += NT) {
    const int k = i / 512, s = i % 512;
    j.hist[(size_t)(t * j.spt + KS_MED + 4 + k) * 512 + s] = s < 256 ? hs[k][s] : 0u;
  }
}

// ---------------------------------------------------------------- predictor search

struct SearchLds {         // the pick / refine / final phases of k_search
  uint32_t hist[512];
  uint8_t brow[2][1024];  // the final pass's best predictors of two rows
  uint16_t rows[4][1024]; // the final pass's original rows y - 2..y and row y - 3 arriving
  uint16_t plist[HOH_MAPCAP];
  uint8_t pidx[HOH_MAPCAP];
};

// Search scratch per plane slot pl = t * HOH_NPLANE_S + p, in the tab_gen buffer (written only by
// k_tables, after the search): the 512 entropy weights ent[] and the cells' mask costs [cell][14].
// Per tile the region of its SPT_S streams' tables (860 KB); the scratch of its planes first,
// then (from LZC_MAP_OFF) k_lzcand's map, so the LZ screen can run beside the search.
#define SCR_STRIDE (512 + HOH_MAPCAP * 14)
#define TAB_TILE_BYTES ((size_t)SPT_S * 512 * sizeof(EncGen))
#define LZC_MAP_OFF ((size_t)143360)   // >= HOH_NPLANE_S * SCR_STRIDE * 8, 512-aligned
static_assert(HOH_NPLANE_S * SCR_STRIDE * 8 <= LZC_MAP_OFF, "search scratch below the LZ map");
__device__ __forceinline__ double* search_scr(const EncodeJob& j, int pl) {
  return (double*)((char*)j.tab_gen + (size_t)(pl / HOH_NPLANE_S) * TAB_TILE_BYTES) + (size_t)(pl % HOH_NPLANE_S) * SCR_STRIDE;
}

// cost of mask m on cell (cx, cy): prediction.hpp:46-151 walked in the cell's raster order with
// the reference's cell-local top row / best_pred state, sum of ent[] in f64 (layer_encode.hpp:192-195)
__device__ double cell_cost(const uint16_t* D, int w, int h, int depth, int xt, int yt, int cx, int cy,
                            uint32_t mask, const double* ent, uint16_t* top, uint8_t* bp) {
  const int c = 1 << depth, half = c >> 1;
  const int tw = (w + xt - 1) / xt, th = (h + yt - 1) / yt;
  const int x0 = cx * tw, y0 = cy * th;
  for (int i = 0; i < tw; i++) {
    bp[i] = 4;
    top[i] = cy ? D[(long)y0 * w + x0 + i - w] : (uint16_t)half;   // may run into the cell's own row
  }
  double cost = 0.0;
  for (int ym = 0; ym < th && y0 + ym < h; ym++) {
    uint32_t L, TL;
    if (cx) {
      L = D[(long)(y0 + ym) * w + x0 - 1];
      TL = (ym || cy) ? D[(long)(y0 + ym - 1) * w + x0 - 1] : (uint32_t)half;
    } else {
      L = TL = half;
    }
    const uint16_t* row = D + (long)(y0 + ym) * w + x0;
    const int vw = min(tw, w - x0);
    // the cell's pixels one step ahead of their use (the walk is latency-bound on these loads)
    uint32_t vn = vw > 0 ? row[0] : 0u;
    for (int xm = 0; xm < vw; xm++) {
      const uint32_t v = vn;
      if (xm + 1 < vw) vn = row[xm + 1];
      const uint32_t T = top[xm];
      const int xr = xm + 1 == tw ? 0 : xm + 1;
      const uint32_t TR = top[xr];
      Preds p;
      preds16(L, T, TL, TR, false, p);
      const int xl = xm == 0 ? tw - 1 : xm - 1;
      const uint32_t pr = midp(pick(p, bp[xm]), pick(p, bp[xl]));
      const uint32_t r = ((uint32_t)((int)v - (int)pr + half + c)) & (uint32_t)(c - 1);   // > 0: % c
      cost += ent[r];
      TL = T;
      top[xm] = (uint16_t)v;
      L = v;
      bp[xm] = (uint8_t)best_pred(v, p, mask, c);
    }
  }
  return cost;
}

// cell_cost for a one-predictor mask {k}, k in {0, 1, 4, 5} (kMasks[0..3]): best_pred then always
// returns k (|v - p| < c < 2c), so bp[] is 4 where it still holds its initial value (row 0 of the
// cell; bp[tw - 1] also when the cell is cut by the plane edge, vw < tw) and k elsewhere, and a step
// needs only L, T, TL: predictors 0 (L), 1 (T), 4 (MED) and 5 (midp(L, T)).  Same pixels, same
// f64 additions in the same order as cell_cost.
#define CELL_MAX 40     // tw = ceil(w / ceil(w / 40)) <= 40, likewise th
__device__ double cell_cost_one(const uint16_t* D, int w, int h, int depth, int xt, int yt, int cx, int cy,
                                uint32_t k, const double* ent) {
  const int c = 1 << depth, half = c >> 1;
  const int tw = (w + xt - 1) / xt, th = (h + yt - 1) / yt;
  const int x0 = cx * tw, y0 = cy * th;
  const int vw = min(tw, w - x0);
  // the row above and the current row in registers (the walk has no other state: every value
  // is an original), each row's loads issued together instead of one pixel ahead
  uint32_t up[CELL_MAX], cur[CELL_MAX];
#pragma unroll
  for (int i = 0; i < CELL_MAX; i++) up[i] = (i < tw && cy) ? D[(long)y0 * w + x0 + i - w] : (uint32_t)half;
  double cost = 0.0;
  for (int ym = 0; ym < th && y0 + ym < h; ym++) {
    uint32_t L, TL;
    if (cx) {
      L = D[(long)(y0 + ym) * w + x0 - 1];
      TL = (ym || cy) ? D[(long)(y0 + ym - 1) * w + x0 - 1] : (uint32_t)half;
    } else {
      L = TL = half;
    }
    const uint16_t* row = D + (long)(y0 + ym) * w + x0;
#pragma unroll
    for (int i = 0; i < CELL_MAX; i++) cur[i] = i < vw ? row[i] : 0u;
    const bool a4 = ym == 0, b4first = !(ym > 0 && vw == tw);
#pragma unroll
    for (int xm = 0; xm < CELL_MAX; xm++) {
      if (xm < vw) {
        const uint32_t v = cur[xm], T = up[xm];
        const uint32_t med = med16s(T, L, (T + L - TL) & 0xffffu);
        const uint32_t pk = k == 0 ? L : k == 1 ? T : k == 4 ? med : midp(L, T);
        const uint32_t pa = a4 ? med : pk, pb = (xm == 0 && b4first) ? med : pk;
        const uint32_t pr = midp(pa, pb);
        const uint32_t r = ((uint32_t)((int)v - (int)pr + half + c)) & (uint32_t)(c - 1);
        cost += ent[r];
        TL = T;
        up[xm] = v;
        L = v;
      }
    }
  }
  return cost;
}

// cell_cost for every mask at once (-s2..-s4): the one-predictor masks kMasks[0..3] (cell_cost_one's
// rule) and the full masks kMasks[4 .. 4 + nf) (nf <= 10); out[m] = the cost of kMasks[m].
// best_pred depends only on the pixel and its 16 predictions, never on the walk's state, so one
// pass computes them once for all masks: with keys (|v - p_k| << 4) | k, the first least
// predictor over all sixteen is the smallest key and over all but one index e the smallest key
// other than e's, i.e. the smallest or the second smallest.  kMasks[4..13] are "all but e" for
// e = 6, 1, 2, 3, 4, 5, 7, 9, the pair {0, 1} and all sixteen.  So every mask's best predictor at a
// pixel is one of three candidates: b1 (smallest key), b2 (second smallest) or kp (the pair's), and
// which one follows from b1 alone.  The walk keeps the candidates, not per-mask predictors: one
// LDS word per column holds the row-above value and its pixel's (b1, b2, kp) (4 bits each, all 4
// before a cell's first row, the reference's initial best_pred), and a pixel picks six values
// (the three candidates of the pixel above and of the left neighbour) instead of two per mask.
// Per mask only the residual and its weight remain, summed in f64 in raster order exactly as
// cell_cost sums each mask (the weights gathered one pixel ahead of their additions).  Every LDS
// access is a lane's whole dword (byte / u16 stores of each lane's own bytes changed files from
// run to run in round 4).
#define WM_N 10
__device__ __forceinline__ uint32_t wm_excl(int m) {        // the index mask m excludes (m != 1, 9)
  return m == 0 ? 6u : m <= 6 ? (uint32_t)(m - 1) : m == 7 ? 7u : 9u;
}
__device__ __forceinline__ uint32_t wm_pick(int m, uint32_t b1, uint32_t P1, uint32_t P2, uint32_t Pk) {
  if (m == 1) return Pk;
  if (m == 9) return P1;
  return b1 == wm_excl(m) ? P2 : P1;
}
#define WM_INIT 0x04440000u                 // b1 = b2 = kp = 4
template <int NF>
__device__ void cell_cost_multi(const uint16_t* D, int w, int h, int depth, int xt, int yt, int cx, int cy,
                                const double* ent, uint32_t* top, uint32_t* pk, double* out) {
  // top: this lane's word per column, [col][64 lanes]: value | b1 << 16 | b2 << 20 | kp << 24
  const int c = 1 << depth, half = c >> 1;
  const int tw = (w + xt - 1) / xt, th = (h + yt - 1) / yt;
  const int x0 = cx * tw, y0 = cy * th;
  for (int i = 0; i < tw; i++) top[i * 64] = WM_INIT | (cy ? D[(long)y0 * w + x0 + i - w] : (uint32_t)half);
  double cost[NF], pend[NF], cost1[4], pend1[4];
#pragma unroll
  for (int m = 0; m < NF; m++) { cost[m] = 0.0; pend[m] = 0.0; }
#pragma unroll
  for (int m = 0; m < 4; m++) { cost1[m] = 0.0; pend1[m] = 0.0; }
  bool have = false;
  for (int ym = 0; ym < th && y0 + ym < h; ym++) {
    uint32_t L, TL;
    if (cx) {
      L = D[(long)(y0 + ym) * w + x0 - 1];
      TL = (ym || cy) ? D[(long)(y0 + ym - 1) * w + x0 - 1] : (uint32_t)half;
    } else {
      L = TL = half;
    }
    const uint16_t* row = D + (long)(y0 + ym) * w + x0;
    const int vw = min(tw, w - x0);
    uint32_t lw = top[(tw - 1) * 64];                                  // the left candidates
    const bool a4 = ym == 0, b4first = !(ym > 0 && vw == tw);
    uint32_t vn = vw > 0 ? row[0] : 0u;
    for (int xm = 0; xm < vw; xm++) {
      const uint32_t v = vn;
      if (xm + 1 < vw) vn = row[xm + 1];
      const uint32_t wa = top[xm * 64];
      const int xr = xm + 1 == tw ? 0 : xm + 1;
      const uint32_t T = wa & 0xffffu, TR = top[xr * 64] & 0xffffu;
      Preds p;
      preds16(L, T, TL, TR, false, p);
      uint32_t k1 = 0xffffffffu, k2 = 0xffffffffu, kp = 0u;
#pragma unroll
      for (int k = 0; k < 16; k++) {
        // |v - p_k| by v_sad_u16 (values < 2^16: the high halves are 0)
        const uint32_t key = (__builtin_amdgcn_sad_u16(v, p.v[k], 0u) << 4) | (uint32_t)k;
        // k1 <= k2 always, so the new second smallest is the median of the three
        uint32_t k2n;
        asm("v_med3_u32 %0, %1, %2, %3" : "=v"(k2n) : "v"(k1), "v"(k2), "v"(key));
        k2 = k2n;
        k1 = min(k1, key);
        if (k == 1) kp = k1;                                            // the pair {0, 1}'s key
      }
      if (have) {
#pragma unroll
        for (int m = 0; m < NF; m++) cost[m] += pend[m];
#pragma unroll
        for (int m = 0; m < 4; m++) cost1[m] += pend1[m];
      }
      const uint32_t vc = v + (uint32_t)(half + c), cm = (uint32_t)(c - 1);
#pragma unroll
      for (int m = 0; m < 4; m++) {
        const uint32_t pkm = p.v[m == 0 ? 0 : m == 1 ? 1 : m == 2 ? 5 : 4];
        const uint32_t pa = a4 ? p.v[4] : pkm, pb = (xm == 0 && b4first) ? p.v[4] : pkm;
        pend1[m] = ent[(vc - midp(pa, pb)) & cm];
      }
      // the six picks through LDS: the 16 predictions as 8 dwords of u16 pairs, [pair][64 lanes]
      // (a lane's reads hit its own bank whatever the index), read back as dwords (one access
      // type for the location) and the half selected
#pragma unroll
      for (int k = 0; k < 8; k++) pk[k * 64] = p.v[2 * k] | (p.v[2 * k + 1] << 16);
      auto lpick = [&](uint32_t k) -> uint32_t {
        return __builtin_amdgcn_ubfe(pk[(k >> 1) * 64], (k & 1) * 16, 16);
      };
      const uint32_t a1 = (wa >> 16) & 15u, l1 = (lw >> 16) & 15u;
      const uint32_t PA1 = lpick(a1), PA2 = lpick((wa >> 20) & 15u), PAk = lpick((wa >> 24) & 15u);
      const uint32_t PB1 = lpick(l1), PB2 = lpick((lw >> 20) & 15u), PBk = lpick((lw >> 24) & 15u);
#pragma unroll
      for (int m = 0; m < NF; m++) {
        const uint32_t pr = midp(wm_pick(m, a1, PA1, PA2, PAk), wm_pick(m, l1, PB1, PB2, PBk));
        pend[m] = ent[(vc - pr) & cm];
      }
      lw = v | ((k1 & 15u) << 16) | ((k2 & 15u) << 20) | ((kp & 15u) << 24);
      top[xm * 64] = lw;
      have = true;
      TL = T;
      L = v;
    }
  }
  if (have) {
#pragma unroll
    for (int m = 0; m < NF; m++) cost[m] += pend[m];
#pragma unroll
    for (int m = 0; m < 4; m++) cost1[m] += pend1[m];
  }
#pragma unroll
  for (int m = 0; m < 4; m++) out[m] = cost1[m];
#pragma unroll
  for (int m = 0; m < NF; m++) out[4 + m] = cost[m];
}

// channelpredict_all (prediction.hpp:153-229) at one pixel, fully parallel: the best predictors
// it needs (row above, left neighbour / end of the row above) are recomputed from the originals
struct AllCtx {
  const uint16_t* D;
  int w, h, tw, th, xt, c, half;
  const uint16_t* plist;
  const uint16_t* ring;   // k_search's final pass (use_ring): original rows in LDS, row y at (y & rmask) << rsh
  bool use_ring;
  int rmask, rsh;
  __device__ __forceinline__ uint32_t px(int y, int x) const {
    return use_ring ? ring[((y & rmask) << rsh) + x] : D[(long)y * w + x];
  }
};

__device__ __forceinline__ void preds_all_at(const AllCtx& a, int x, int y, Preds& p) {
  const int w = a.w;
  const uint32_t L = x ? a.px(y, x - 1) : (uint32_t)a.half;
  const uint32_t T = y ? a.px(y - 1, x) : (uint32_t)a.half;
  const uint32_t TL = (x && y) ? a.px(y - 1, x - 1) : (uint32_t)a.half;
  uint32_t TR;
  if (w == 1) TR = T;                                        // top_row[0] not yet overwritten
  else if (x == w - 1) TR = a.px(y, 0);                // top_row[0]: this row's first value
  else TR = y ? a.px(y - 1, x + 1) : (uint32_t)a.half;
  preds16(L, T, TL, TR, true, p);
}

__device__ __forceinline__ uint32_t bp_all(const AllCtx& a, int x, int y) {
  if (y + 1 >= a.h) return 0;                                // last row keeps 0 (:214-216)
  Preds p;
  preds_all_at(a, x, y, p);
  return best_pred(a.px(y, x), p, a.plist[((y + 1) / a.th) * a.xt + x / a.tw], a.c);
}

__device__ __forceinline__ uint32_t resid_all(const AllCtx& a, int x, int y) {
  const uint32_t bA = y ? bp_all(a, x, y - 1) : 4u;
  const uint32_t bB = x ? bp_all(a, x - 1, y) : (y ? bp_all(a, a.w - 1, y - 1) : 4u);
  Preds p;
  preds_all_at(a, x, y, p);
  const uint32_t pr = midp(pick(p, bA), pick(p, bB));
  return ((uint32_t)((int)a.px(y, x) - (int)pr + a.half + a.c)) & (uint32_t)(a.c - 1);   // > 0: % c
}

// The mask costs of every searched plane: a lane per (mask, plane, cell) task, mask-major, so a
// wave's lanes share a mask (the one-predictor masks kMasks[0..3] walk without the predictor set)
// and all planes' walks run at once across the chip instead of one workgroup's tasks behind its
// slowest wave.  The full walk keeps the cell's top row and best predictors in LDS (8 KB per
// wave: ~120 VGPRs, four waves per SIMD).  ncmax: cells of the largest plane (host, from the tile
// size).
// Task kinds: at -s2..-s4 one task per (plane, cell) walks every mask at once (cell_cost_multi,
// k_search_walk_multi: its state is one LDS word per column, 42 x 64 lanes = 10.5 KB per wave);
// at -s1, whose one full mask walks faster alone, a task per mask (cell_cost_one / cell_cost).
__host__ __device__ inline bool walk_multi(int npred) { return npred == 5 || npred == 10 || npred == 14; }
__host__ __device__ inline int walk_kinds(int npred) { return walk_multi(npred) ? 1 : npred; }
#define WM_COLS 42
struct WalkTask {
  const uint16_t* D;
  double* ent;
  int w, h, depth, xt, yt, cell;
};
// task g of the (kind, plane, cell) space; false: nothing to walk
__device__ __forceinline__ bool walk_task(const EncodeJob& j, int npred, int ncmax, uint64_t g, uint32_t& m, WalkTask& k) {
  const uint32_t npl = (uint32_t)j.ntiles * HOH_NPLANE_S;
  m = (uint32_t)(g / ((uint64_t)npl * ncmax));
  if (m >= (uint32_t)walk_kinds(npred)) return false;
  const uint32_t rem = (uint32_t)(g % ((uint64_t)npl * ncmax)), pl = rem / ncmax, cell = rem % ncmax;
  const int t = (int)(pl / HOH_NPLANE_S), p = (int)(pl % HOH_NPLANE_S);
  const TileInfo ti = j.tiles[t];
  if (!plane_present(j, ti, p)) return false;
  k.w = ti.w; k.h = ti.h; k.depth = plane_depth(p);
  k.xt = (k.w + 39) / 40; k.yt = (k.h + 39) / 40;
  if (!(k.xt > 1 || k.yt > 1) || (int)cell >= k.xt * k.yt) return false;
  k.D = j.sym + fin_plane_off(j, t, p);
  k.ent = search_scr(j, (int)pl);
  k.cell = (int)cell;
  return true;
}
__global__ __launch_bounds__(64) void k_search_walk(EncodeJob j, int npred, int ncmax) {
  __shared__ uint16_t top[64][42];
  __shared__ uint8_t bp[64][44];
  const int lane = threadIdx.x;
  uint32_t m;
  WalkTask k;
  if (!walk_task(j, npred, ncmax, (uint64_t)blockIdx.x * 64 + lane, m, k)) return;
  const uint32_t mk = kMasks[m];
  const int cx = k.cell % k.xt, cy = k.cell / k.xt;
  k.ent[512 + k.cell * 14 + m] =
      m < 4 ? cell_cost_one(k.D, k.w, k.h, k.depth, k.xt, k.yt, cx, cy, (uint32_t)__builtin_ctz(mk), k.ent)
            : cell_cost(k.D, k.w, k.h, k.depth, k.xt, k.yt, cx, cy, mk, k.ent, top[lane], bp[lane]);
}
__global__ __launch_bounds__(64) void k_search_walk_multi(EncodeJob j, int npred, int ncmax) {
  __shared__ uint32_t top[WM_COLS * 64];
  __shared__ uint32_t pk[8 * 64];
  const int lane = threadIdx.x;
  uint32_t m;
  WalkTask k;
  if (!walk_task(j, npred, ncmax, (uint64_t)blockIdx.x * 64 + lane, m, k)) return;
  const int cx = k.cell % k.xt, cy = k.cell / k.xt;
  if (npred == 5) cell_cost_multi<1>(k.D, k.w, k.h, k.depth, k.xt, k.yt, cx, cy, k.ent, top + lane, pk + lane, k.ent + 512 + k.cell * 14);
  else if (npred == 10) cell_cost_multi<6>(k.D, k.w, k.h, k.depth, k.xt, k.yt, cx, cy, k.ent, top + lane, pk + lane, k.ent + 512 + k.cell * 14);
  else cell_cost_multi<10>(k.D, k.w, k.h, k.depth, k.xt, k.yt, cx, cy, k.ent, top + lane, pk + lane, k.ent + 512 + k.cell * 14);
}

// One workgroup per (tile, plane).  phase 0: the plane's data staged, the MED residuals'
// entropy weights to the scratch; then k_search_walk fills the mask costs; phase 1: the masks
// picked; pass 0 of -s>=3 then refines the weights and returns for a second walk, otherwise the
// final residuals and the predictor map follow.
__global__ __launch_bounds__(NT) void k_search(EncodeJob j, int phase, int pass) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sl_raw[];
  SearchLds& S = *(SearchLds*)sl_raw;
  const int t = blockIdx.x / HOH_NPLANE_S, p = blockIdx.x % HOH_NPLANE_S, tid = threadIdx.x;
  const TileInfo ti = j.tiles[t];
  PlaneInfo* pi = j.pinfo + (size_t)t * HOH_NPLANE_S + p;
  if (!plane_present(j, ti, p)) {
    if (tid == 0 && phase == 0) { PlaneInfo z; memset(&z, 0, sizeof(z)); *pi = z; }
    return;
  }
  const int w = ti.w, h = ti.h, depth = plane_depth(p), c = 1 << depth, half = c >> 1;
  const uint32_t npix = (uint32_t)w * h;
  uint16_t* D = j.sym + fin_plane_off(j, t, p);
  uint32_t* fh = j.hist + (size_t)(t * j.spt + KS_FIN + p) * 512;
  const uint32_t* mh = j.hist + (size_t)(t * j.spt + KS_MED + p) * 512;
  const int xt = (w + 39) / 40, yt = (h + 39) / 40;               // layer_encode.hpp:124-132, :150-151
  const bool grid = xt > 1 || yt > 1;
  double* ent = search_scr(j, t * HOH_NPLANE_S + p);
  const double* cost = ent + 512;
  const double* lg = nullptr;
  for (int k = 0; k < 4; k++) if (j.lg_n[k] == npix) lg = j.lg + j.lg_off[k];
  if (phase == 0) {
    if (!grid) {
      // no search: the layer keeps the MED residuals (00 00 00 10 header)
      const uint16_t* M = j.sym + med_plane_off(j, t, p);
      for (uint32_t q = tid; q < npix; q += NT) D[q] = M[q];
      for (int i = tid; i < 512; i += NT) fh[i] = mh[i];
      if (tid == 0) {
        PlaneInfo z; memset(&z, 0, sizeof(z));
        z.present = 1; z.depth = depth; z.fixed_len = 5;
        *pi = z;
      }
      return;
    }
    // the plane's data values, staged in the searched-residual slot (overwritten at the end)
    for (uint32_t q = tid; q < npix; q += NT) D[q] = (uint16_t)plane_value(j, ti, t, p, q);
    // entropy of the MED residuals over all pixels, freq = 1 + count (layer_encode.hpp:133-144)
    for (int i = tid; i < c; i += NT) ent[i] = lg[1 + mh[i]];
    return;
  }
  if (!grid) return;
  const int ncell = xt * yt, npred = j.speed * 5 < 14 ? j.speed * 5 : 14;
  const int tw = (w + xt - 1) / xt, th = (h + yt - 1) / yt;
  AllCtx a{D, w, h, tw, th, xt, c, half, S.plist, D, false, 3, 10};
  {
    for (int cell = tid; cell < ncell; cell += NT) {
      double best = 99999999999.0;                                // :177
      int bi = 0;
      for (int m = 0; m < npred; m++) {
        const double v = cost[cell * 14 + m];
        if (v < best) { best = v; bi = m; }
      }
      S.plist[cell] = kMasks[bi];
      S.pidx[cell] = (uint8_t)bi;
    }
    __syncthreads();
  }
  // channelpredict_all residuals over the staged data, rows from the last up.  Pass 0 of -s>=3
  // (refine, :215-231) only counts them: the entropy of those residuals, then a second walk.  The
  // final pass writes them in place: each row read completely before it is overwritten (reads
  // reach rows y-2..y only).
  // Each row's best predictors are computed once: bnext holds row y's (from the previous
  // iteration; the last row's are 0, :214-216), bcur gets row y - 1's, so a pixel costs one
  // bp_all and one predictor set instead of resid_all's two and three.  w <= 1024 (hoh_api).
  const bool refine = j.speed > 2 && pass == 0;
  uint8_t* bnext = S.brow[0];
  uint8_t* bcur = S.brow[1];
  for (int i = tid; i < w; i += NT) bnext[i] = 0;
  for (int i = tid; i < 512; i += NT) S.hist[i] = 0;
  if (w <= 256) {
    // Tiles up to 256 wide: bands of SB_R rows, two barriers a band.  A row's best predictors
    // depend on original pixels only, so a band's (rows y_lo - 1 .. yb - 1; row yb's from the
    // band before) are computed first, then all its residuals; the originals live in a 16-row LDS
    // ring (the plane is overwritten in place: a band reads rows y_lo - 2 .. yb, the next band's
    // new rows y_lo - SB_R - 2 .. y_lo - 3 are loaded meanwhile into other slots).
    constexpr int SB_R = 4;
    uint16_t* ring = &S.rows[0][0];                                   // [16][256]
    uint8_t* bpb = &S.brow[0][0];                                     // [SB_R + 1][256]
    a.ring = ring;
    a.use_ring = true;
    a.rmask = 15;
    a.rsh = 8;
    for (int r = max(0, h - SB_R - 2); r < h; r++)
      if (tid < w) ring[((r & 15) << 8) + tid] = D[(long)r * w + tid];
    uint32_t bkeep = 0;                                               // best predictor of (tid, yb): 0 in the last row
    __syncthreads();
    for (int yb = h - 1; yb >= 0; yb -= SB_R) {
      const int y_lo = max(0, yb - SB_R + 1), nr = yb - y_lo + 1;
      uint32_t nv[SB_R];
#pragma unroll
      for (int k = 0; k < SB_R; k++) {
        const int r = y_lo - SB_R - 2 + k;
        nv[k] = (r >= 0 && tid < w) ? D[(long)r * w + tid] : 0u;
      }
      // slot k: the best predictors of row y_lo - 1 + k (k = nr: row yb, kept from the band before)
      if (tid < w) {
        bpb[nr * 256 + tid] = (uint8_t)bkeep;
        for (int k = 0; k < nr; k++) {
          const int r = y_lo - 1 + k;
          if (r < 0) continue;
          Preds p;
          preds_all_at(a, tid, r, p);
          bpb[k * 256 + tid] = (uint8_t)best_pred(a.px(r, tid), p, a.plist[((r + 1) / th) * xt + tid / tw], c);
        }
      }
      __syncthreads();
      if (tid < w) {
        const int x = tid;
        for (int y = yb; y >= y_lo; y--) {
          const int k = y - y_lo + 1;                                  // row y's slot
          const uint32_t bA = y ? bpb[(k - 1) * 256 + x] : 4u;
          const uint32_t bB = x ? bpb[k * 256 + x - 1] : (y ? bpb[(k - 1) * 256 + w - 1] : 4u);
          Preds p;
          preds_all_at(a, x, y, p);
          const uint32_t pr = midp(pick(p, bA), pick(p, bB));
          const uint32_t r = ((uint32_t)((int)a.px(y, x) - (int)pr + half + c)) & (uint32_t)(c - 1);
          if (!refine) D[(long)y * w + x] = (uint16_t)r;
          atomicAdd(&S.hist[r], 1u);
        }
        bkeep = bpb[x];                                                // row y_lo - 1: the next band's yb
#pragma unroll
        for (int k = 0; k < SB_R; k++) {
          const int r = y_lo - SB_R - 2 + k;
          if (r >= 0) ring[((r & 15) << 8) + x] = (uint16_t)nv[k];
        }
      }
      __syncthreads();
    }
  } else {
  // the original rows in an LDS ring (the global plane is overwritten row by row): rows y, y - 1
  // and y - 2 are read at row y, row y - 3 is loaded meanwhile and lands in row y + 1's slot
  for (int k = 0; k < 3 && h - 1 - k >= 0; k++)
    for (int x = tid; x < w; x += NT) S.rows[(h - 1 - k) & 3][x] = D[(long)(h - 1 - k) * w + x];
  a.ring = &S.rows[0][0];
  a.use_ring = true;
  __syncthreads();
  // tiles up to NT wide (one pixel per thread): the predictor set row y - 1's best predictors were
  // computed from is kept (u16 pairs) for row y - 1's residuals in the next iteration
  const bool keep = w <= NT;
  uint32_t pc[8], pn[8];
  bool have = false;
  for (int y = h - 1; y >= 0; y--) {
    uint32_t nv[4];
    int n = 0;
    for (int x = tid; x < w && n < 4; x += NT) nv[n++] = y >= 3 ? D[(long)(y - 3) * w + x] : 0u;
    if (y > 0) {
      if (keep) {
        if (tid < w) {                                                 // bp_all(a, tid, y - 1)
          Preds p;
          preds_all_at(a, tid, y - 1, p);
#pragma unroll
          for (int k = 0; k < 8; k++) pn[k] = p.v[2 * k] | (p.v[2 * k + 1] << 16);
          bcur[tid] = y >= h ? 0 : (uint8_t)best_pred(a.px(y - 1, tid), p, a.plist[(y / th) * xt + tid / tw], c);
        }
      } else {
        for (int x = tid; x < w; x += NT) bcur[x] = (uint8_t)bp_all(a, x, y - 1);
      }
    }
    __syncthreads();
    n = 0;
    for (int x = tid; x < w && n < 4; x += NT) {                      // resid_all(a, x, y)
      const uint32_t bA = y ? bcur[x] : 4u;
      const uint32_t bB = x ? bnext[x - 1] : (y ? bcur[w - 1] : 4u);
      Preds p;
      if (keep && have) {
#pragma unroll
        for (int k = 0; k < 8; k++) { p.v[2 * k] = pc[k] & 0xffffu; p.v[2 * k + 1] = pc[k] >> 16; }
      } else {
        preds_all_at(a, x, y, p);
      }
      const uint32_t pr = midp(pick(p, bA), pick(p, bB));
      const uint32_t r = ((uint32_t)((int)a.px(y, x) - (int)pr + half + c)) & (uint32_t)(c - 1);
      // no barrier before these: the residuals read rows y .. y - 2 of the ring, and row y - 3
      // lands in row y + 1's slot (read last iteration, before the barrier that ended it)
      if (!refine) D[(long)y * w + x] = (uint16_t)r;
      atomicAdd(&S.hist[r], 1u);
      if (y >= 3) S.rows[(y - 3) & 3][x] = (uint16_t)nv[n];
      n++;
    }
    __syncthreads();
    uint8_t* const b = bnext;                                           // row y - 1 is next
    bnext = bcur;
    bcur = b;
#pragma unroll
    for (int k = 0; k < 8; k++) pc[k] = pn[k];
    have = keep && y > 0;
  }
  }
  if (refine) {
    for (int i = tid; i < c; i += NT) ent[i] = lg[1 + S.hist[i]];
    return;
  }
  for (int i = tid; i < 512; i += NT) fh[i] = S.hist[i];
  // predictor map: used masks and their order (:279-307)
  if (tid == 0) {
    uint32_t used = 0;
    for (int i = 0; i < ncell; i++) used |= 1u << S.pidx[i];
    uint32_t rank[14], k = 0;
    for (int m = 0; m < 14; m++) rank[m] = (used >> m) & 1 ? k++ : 0;
    uint16_t* ms = j.sym + map_sym_off(j, t, p);
    for (int i = 0; i < ncell; i++) ms[i] = (uint16_t)rank[S.pidx[i]];
    PlaneInfo z; memset(&z, 0, sizeof(z));
    z.present = 1; z.depth = depth; z.xt = xt; z.yt = yt;
    z.used = k; z.used_bits = used;
    z.fixed_len = 1 + 3 + 2 * k;
    *pi = z;
  }
}

// ---------------------------------------------------------------- plane-level entry points

// channelpredict_section (prediction.hpp:46-151) of one cell, one thread: the cell-local top row
// and best-predictor state live in the caller's scratch (the cell may be a whole plane)
__global__ void k_section_one(const uint16_t* D, int w, int h, int depth, int xt, int yt, int cx, int cy,
                              uint32_t mask, uint16_t* out, uint64_t* count, uint16_t* top, uint8_t* bp) {
  if (threadIdx.x || blockIdx.x) return;
  const int c = 1 << depth, half = c >> 1;
  const int tw = (w + xt - 1) / xt, th = (h + yt - 1) / yt;
  const int x0 = cx * tw, y0 = cy * th;
  for (int i = 0; i < tw; i++) {
    bp[i] = 4;
    top[i] = cy ? D[(long)y0 * w + x0 + i - w] : (uint16_t)half;
  }
  uint64_t k = 0;
  for (int ym = 0; ym < th && y0 + ym < h; ym++) {
    uint32_t L, TL;
    if (cx) {
      L = D[(long)(y0 + ym) * w + x0 - 1];
      TL = (ym || cy) ? D[(long)(y0 + ym - 1) * w + x0 - 1] : (uint32_t)half;
    } else {
      L = TL = half;
    }
    for (int xm = 0; xm < tw && x0 + xm < w; xm++) {
      const uint32_t v = D[(long)(y0 + ym) * w + x0 + xm];
      const uint32_t T = top[xm], TR = top[xm + 1 == tw ? 0 : xm + 1];
      Preds p;
      preds16(L, T, TL, TR, false, p);
      const uint32_t pr = midp(pick(p, bp[xm]), pick(p, bp[xm == 0 ? tw - 1 : xm - 1]));
      out[k++] = (uint16_t)(((int)v - (int)pr + half + c) % c);
      TL = T;
      top[xm] = (uint16_t)v;
      L = v;
      bp[xm] = (uint8_t)best_pred(v, p, mask, c);
    }
  }
  *count = k;
}

// channelpredict_all (prediction.hpp:153-229), one thread per pixel
__global__ __launch_bounds__(NT) void k_all_plane(const uint16_t* D, int w, int h, int depth, int xt, int yt,
                                                  const uint16_t* map, uint16_t* out) {
  const int c = 1 << depth;
  const AllCtx a{D, w, h, (w + xt - 1) / xt, (h + yt - 1) / yt, xt, c, c >> 1, map, D, false};
  const uint64_t n = (uint64_t)w * h;
  for (uint64_t q = (uint64_t)blockIdx.x * NT + threadIdx.x; q < n; q += (uint64_t)gridDim.x * NT) {
    const int y = (int)(q / (uint64_t)w), x = (int)(q - (uint64_t)y * w);
    out[q] = (uint16_t)resid_all(a, x, y);
  }
}

// unpredict_all (unprediction.hpp:6-91) with any predictor map: the exact inverse of
// channelpredict_all including LZ copies (LEMPEL_BACKREF).  Row y's first pixel needs the best
// predictor of row y-1's last pixel, so the recurrence is serial: one thread per plane.
__global__ void k_unpredict_all(const uint16_t* res, uint64_t nres, const uint16_t* backref, int w, int h,
                                int depth, int xt, int yt, const uint16_t* map, uint16_t* out,
                                uint16_t* top, uint8_t* bp, uint32_t* err) {
  if (threadIdx.x || blockIdx.x) return;
  const int c = 1 << depth, half = c >> 1;
  const int tw = (w + xt - 1) / xt, th = (h + yt - 1) / yt;
  for (int i = 0; i < w; i++) { bp[i] = 4; top[i] = (uint16_t)half; }
  uint64_t k = 0;
  for (int y = 0; y < h; y++) {
    uint32_t L = half, TL = half;
    for (int x = 0; x < w; x++) {
      const uint64_t loc = (uint64_t)y * w + x;
      const uint32_t T = top[x], TR = top[x + 1 == w ? 0 : x + 1];
      Preds p;
      preds16(L, T, TL, TR, true, p);
      uint32_t v;
      if (backref && backref[loc]) {
        if (backref[loc] > loc) { *err = 1; return; }
        v = out[loc - backref[loc]];
      } else {
        if (k >= nres) { *err = 1; return; }
        const uint32_t pr = midp(pick(p, bp[x]), pick(p, bp[x == 0 ? w - 1 : x - 1]));
        v = (uint32_t)((res[k++] - c - half + pr) & 0xffffu) % (uint32_t)c;   // :67-68 in uint16
      }
      out[loc] = (uint16_t)v;
      TL = T;
      top[x] = (uint16_t)v;
      L = v;
      bp[x] = y + 1 < h ? (uint8_t)best_pred(v, p, map[((y + 1) / th) * xt + x / tw], c) : (uint8_t)0;
    }
  }
  *err = 0;
}

// grid search of layer_encode.hpp:176-203 on a whole plane: costs per (cell, mask) ...
__global__ __launch_bounds__(NT) void k_search_costs(const uint16_t* D, int w, int h, int depth, int xt, int yt,
                                                     int npred, const double* ent, double* cost) {
  __shared__ uint16_t top[NT][40];
  __shared__ uint8_t bp[NT][40];
  const int k = blockIdx.x * NT + threadIdx.x;
  if (k >= xt * yt * npred) return;
  const int cell = k / npred, m = k % npred;
  cost[cell * 14 + m] = cell_cost(D, w, h, depth, xt, yt, cell % xt, cell / xt, kMasks[m], ent,
                                  top[threadIdx.x], bp[threadIdx.x]);
}

// ... and the first mask of least cost per cell (strict <, :196-200)
__global__ __launch_bounds__(NT) void k_search_pick(int ncell, int npred, const double* cost, uint16_t* plist,
                                                    uint8_t* pidx) {
  const int cell = blockIdx.x * NT + threadIdx.x;
  if (cell >= ncell) return;
  double best = 99999999999.0;
  int bi = 0;
  for (int m = 0; m < npred; m++) if (cost[cell * 14 + m] < best) { best = cost[cell * 14 + m]; bi = m; }
  plist[cell] = kMasks[bi];
  pidx[cell] = (uint8_t)bi;
}

void launch_section_one(const uint16_t* D, int w, int h, int depth, int xt, int yt, int cx, int cy, uint32_t mask,
                        uint16_t* out, uint64_t* count, uint16_t* top, uint8_t* bp, hipStream_t s) {
  hipLaunchKernelGGL(k_section_one, dim3(1), dim3(64), 0, s, D, w, h, depth, xt, yt, cx, cy, mask, out, count, top, bp);
}
void launch_all_plane(const uint16_t* D, int w, int h, int depth, int xt, int yt, const uint16_t* map, uint16_t* out,
                      hipStream_t s) {
  const uint64_t n = (uint64_t)w * h;
  const int blocks = (int)((n + NT - 1) / NT < 4096 ? (n + NT - 1) / NT : 4096);
  hipLaunchKernelGGL(k_all_plane, dim3(blocks > 0 ? blocks : 1), dim3(NT), 0, s, D, w, h, depth, xt, yt, map, out);
}
void launch_unpredict_all(const uint16_t* res, uint64_t nres, const uint16_t* backref, int w, int h, int depth,
                          int xt, int yt, const uint16_t* map, uint16_t* out, uint16_t* top, uint8_t* bp,
                          uint32_t* err, hipStream_t s) {
  hipLaunchKernelGGL(k_unpredict_all, dim3(1), dim3(64), 0, s, res, nres, backref, w, h, depth, xt, yt, map, out,
                     top, bp, err);
}
void launch_search_plane(const uint16_t* D, int w, int h, int depth, int xt, int yt, int npred, const double* ent,
                         double* cost, uint16_t* plist, uint8_t* pidx, hipStream_t s) {
  const int n = xt * yt * npred;
  hipLaunchKernelGGL(k_search_costs, dim3((n + NT - 1) / NT), dim3(NT), 0, s, D, w, h, depth, xt, yt, npred, ent, cost);
  hipLaunchKernelGGL(k_search_pick, dim3((xt * yt + NT - 1) / NT), dim3(NT), 0, s, xt * yt, npred, cost, plist, pidx);
}

// ---------------------------------------------------------------- LZ at seek distance 10..14

__device__ __forceinline__ uint32_t tile_px(const EncodeJob& j, const TileInfo& ti, uint32_t q) {
  const uint32_t y = q / (uint32_t)ti.w, x = q - y * (uint32_t)ti.w;
  const uint8_t* px = j.rgb + ((size_t)(ti.y0 + y) * j.W + ti.x0 + x) * 3;
  return px[0] | (px[1] << 8) | (px[2] << 16);
}

__device__ __forceinline__ uint32_t fp4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  uint32_t h = a * 0x9E3779B1u;
  h = (h ^ b) * 0x85EBCA77u;
  h = (h ^ c) * 0xC2B2AE3Du;
  h = (h ^ d) * 0x27D4EB2Fu;
  return (h ^ (h >> 15)) | 1u;
}

// fingerprint of the 4-pixel window starting at every position (0: fewer than 4 pixels left)
// Also the tile's pixels as u32 in tile raster order (tpx): k_lzscan's ring fills and run lengths
// read them as contiguous words instead of three bytes behind a division by the tile width.  And
// run8[q]: how many pixels from q on equal pixel q (1..254, 255 = at least 255), from a bitmap of
// the run ends over the chunk and the 259 positions after it (k_lzscan's run-length shortcut).
#define LZFP_AHEAD 260
#define LZFP_ROWS 16
__global__ __launch_bounds__(NT) void k_lzfp(EncodeJob j) {
  __shared__ uint32_t px[NT + LZFP_AHEAD];
  __shared__ uint64_t ends[(NT + LZFP_AHEAD + 63) / 64];
  __shared__ uint32_t fl[LZFP_ROWS][NT + 1];                      // 256-wide tiles: the block's rows' F
  const int t = blockIdx.y;
  const TileInfo ti = j.tiles[t];
  const uint32_t npix = (uint32_t)ti.w * ti.h, tid = threadIdx.x, lane = tid & 63;
  const uint32_t w = (uint32_t)ti.w, h = (uint32_t)ti.h;
  uint32_t* fo = j.fpb + (size_t)t * j.npix_cap;
  uint32_t* po = j.tpx + (size_t)t * j.npix_cap;
  uint32_t* ft = j.fpt + (size_t)t * j.npix_cap;
  uint8_t* ro = j.run8 + (size_t)t * j.npix_cap;
  constexpr uint32_t NP = NT + LZFP_AHEAD, NW = (NP + 63) / 64;
  // block b takes a contiguous range of chunks (of a 256-wide tile: rows [b*S, b*S + S)), so the
  // transposed fingerprints (k_lzscan's / k_lzvert's columns) leave as 4-word column pieces
  const uint32_t nch = (npix + NT - 1) / NT, S = (nch + gridDim.x - 1) / gridDim.x;
  const uint32_t ch0 = blockIdx.x * S, ch1 = min(nch, ch0 + S);
  const bool rows = w == NT && S <= LZFP_ROWS && (S & 3) == 0;
  for (uint32_t ch = ch0; ch < ch1; ch++) {
    const uint32_t c0 = ch * NT;
    // past the tile: a word no pixel has (pixels are 24-bit), so the tile's last run ends there
    for (uint32_t k = tid; k < NP; k += NT) px[k] = c0 + k < npix ? tile_px(j, ti, c0 + k) : 0xffffffffu;
    __syncthreads();
    for (uint32_t k0 = 0; k0 < NW * 64; k0 += NT) {
      const uint32_t k = k0 + tid;
      const uint64_t m = __ballot(k < NP && (k + 1 >= NP || px[k] != px[k + 1]));
      if (lane == 0 && (k >> 6) < NW) ends[k >> 6] = m;
    }
    __syncthreads();
    const uint32_t q = c0 + tid;
    if (q < npix) {
      const uint32_t f = q + 3 < npix ? fp4(px[tid], px[tid + 1], px[tid + 2], px[tid + 3]) : 0u;
      fo[q] = f;
      if (rows) fl[ch - ch0][tid] = f;
      else ft[(q % w) * h + q / w] = f;
      // the first run end at or after tid (at most 255 positions on)
      uint32_t e = 0xffffffffu;
      for (uint32_t wd = tid >> 6; wd < NW && wd <= ((tid + 255) >> 6); wd++) {
        uint64_t m = ends[wd];
        if (wd == (tid >> 6)) m &= ~0ull << (tid & 63);
        if (m) { e = wd * 64 + (uint32_t)(__ffsll((unsigned long long)m) - 1); break; }
      }
      // no end within 255 positions: 255 (e - tid + 1 would wrap to 0 at tid 0)
      const uint32_t r = e == 0xffffffffu ? 255u : e - tid + 1, r8 = r < 255 ? r : 255;
      ro[q] = (uint8_t)r8;
      po[q] = px[tid] | (r8 << 24);                                    // the pixel and its run, one gather
    }
    __syncthreads();
  }
  if (rows && ch0 < ch1) {
    // column x = tid, rows ch0 .. ch1 - 1: (ch1 - ch0) consecutive words of FT
    uint4* dst = (uint4*)(ft + (size_t)tid * h + ch0);
    for (uint32_t i = 0; i + 4 <= ch1 - ch0; i += 4)
      dst[i / 4] = make_uint4(fl[i][tid], fl[i + 1][tid], fl[i + 2][tid], fl[i + 3][tid]);
  }
}
// exact candidate screen: q can start a match of length >= 4 only if an equal window starts at
// q - b for some b <= min(limit, q), or at q - k*w with k*w <= 65536 (lz.hpp:35, :55); equal
// windows have equal fingerprints, so the screen never misses one.  Chunks of 256 positions in
// order, the last `limit` fingerprints in an LDS ring.
// The horizontal test is answered from LDS hash tables before any ring walk:
//  - three window tables (2048 slots each, three hashes of f): the latest position p < base whose
//    fingerprint hashed to the slot, (p + 1) << 8 | tag(f), by LDS atomic max (positions in the
//    high 24 bits, so the max is the latest; tiles hold < 2^24 pixels).  An occurrence of f in the
//    window updated all three slots, so one slot whose latest position is older than q - bm is an
//    exact no; a slot holding f's tag is a yes (an 8-bit tag collision only adds a candidate,
//    which k_lzscan measures and drops);
//  - two chunk tables (1024 slots each): the first position of the chunk per slot (atomic min);
//    a first position equal to q is an exact no for the chunk, an earlier one holding f a yes.
// Only a lane whose every slot is held by other fingerprints is walked: the wave walks each such
// lane's window together.  40 KB of LDS at -s1 (ring 8 KB, tables 24 + 8 KB): four tiles per CU.
// -s2..-s4 (windows of 2048..16384 fill the tables) take the global map below.
#define LZC_W 2048
#define LZC_C 1024
__device__ __forceinline__ uint32_t lzc_h(uint32_t f, int k) {
  return k == 0 ? (f >> 1) & (LZC_W - 1) : k == 1 ? (f >> 12) & (LZC_W - 1) : (f * 0x9E3779B1u) >> 21;
}
// Modes: LZC_WALK every lane walks its window (ring >= limit + NT); LZC_TAB the LDS window tables
// above (-s1); LZC_MAP (-s2..-s4, whose windows fill any LDS table) a per-tile open-addressing
// map in global memory of every fingerprint seen so far -> its latest position, (p + 1) << 8 |
// tag, linear probing from (f >> 1), at most half full, in the tab_gen buffer (k_tables writes
// it later).  Fingerprints whose slot chain and tag coincide share an entry holding the larger
// position, so "latest position older than q - bm" stays an exact no and only candidates are
// added.  One workgroup owns a tile's map: workgroup-scope CAS / max (performed in L2) and
// agent-scope loads, so no load is served from an L1 copy older than an atomic (a stale 0 or an
// older position would be a false no, a lost match), ordered between chunks by the barrier; the chunk's own positions come from the chunk tables (a walk of
// at most the chunk if they are unsure).
enum { LZC_WALK = 0, LZC_TAB = 1, LZC_MAP = 2 };
#ifndef LZC_MAP_LOAD_SCOPE
#define LZC_MAP_LOAD_SCOPE __HIP_MEMORY_SCOPE_AGENT                    // the map's loads: from L2 (below)
#endif
__device__ __forceinline__ uint32_t* lzc_map(const EncodeJob& j, int t) {
  return (uint32_t*)((char*)j.tab_gen + (size_t)t * TAB_TILE_BYTES + LZC_MAP_OFF);
}
// Vertical backs beyond the window (lz.hpp:54-74: q - k*w, limit < k*w <= min(65536, q)) for the
// positions k_lzcand left without a candidate, tiles whose every earlier row is in reach
// ((h - 1) * w <= 65536, w a multiple of 64 up to 256: 256^2 tiles).  A thread per column keeps
// a 4096-bit Bloom filter (three bits per fingerprint) of its column's rows up to y - kmin,
// kmin = limit / w + 1: a clear bit is an exact no.  A possible yes is settled by the whole wave
// on the transposed fingerprints (k_lzfp's FT: a column's rows are contiguous, 64 per load).  Row by
// row the wave of columns x .. x + 63 owns one candidate word; the rows' words are loaded eight
// rows ahead.  (k_lzcand walked sixteen rows a batch for every position without a candidate: 256
// loads for most positions of a noisy tile, 14 ms per natural 8192^2 image at -s1.)
#define LZV_WORDS 128
#define LZV_AHEAD 8
__host__ __device__ inline bool lzvert_ok(uint32_t w, uint32_t h) {
  return w >= 64 && w <= 256 && (w & 63) == 0 && (h - 1) * w <= 65536u;
}
__device__ __forceinline__ void lzv_bits(uint32_t f, uint32_t& a, uint32_t& b, uint32_t& c) {
  const uint32_t g = f * 0x9E3779B1u;
  a = g >> 20; b = (f ^ (f >> 15)) & 4095u; c = ((f >> 7) * 0x85EBCA6Bu) >> 20;
}
__global__ __launch_bounds__(64) void k_lzvert(EncodeJob j, int limit) {
  // one wave per 64 columns (32 KB: a 128 KB workgroup per tile waited for a whole CU's LDS
  // behind the concurrent predictor search)
  __shared__ uint32_t bl[LZV_WORDS][64];                          // [word][column]: conflict-free
  const int t = blockIdx.y, lane = threadIdx.x, x = blockIdx.x * 64 + lane;
  const TileInfo ti = j.tiles[t];
  const uint32_t w = ti.w, h = ti.h;
  if (!lzvert_ok(w, h) || (uint32_t)x >= w) return;                // whole waves (w % 64 == 0)
  for (int i = 0; i < LZV_WORDS; i++) bl[i][lane] = 0u;
  const uint32_t* F = j.fpb + (size_t)t * j.npix_cap;
  const uint32_t* FT = j.fpt + (size_t)t * j.npix_cap;
  uint64_t* cand = j.candbits + (size_t)t * (j.npix_cap / 64);
  const uint32_t kmin = (uint32_t)limit / w + 1;                  // rows y >= kmin only
  uint32_t added = 0;
  uint32_t fi[LZV_AHEAD], fq[LZV_AHEAD];
  uint64_t cw[LZV_AHEAD];
  auto load = [&](uint32_t y0) {
#pragma unroll
    for (int u = 0; u < LZV_AHEAD; u++) {
      const uint32_t y = y0 + u;
      fi[u] = y < h ? F[(y - kmin) * w + x] : 0u;
      fq[u] = y < h ? F[y * w + x] : 0u;
      cw[u] = y < h ? cand[(y * w + x) >> 6] : 0ull;
    }
  };
  if (kmin < h) load(kmin);
  for (uint32_t y0 = kmin; y0 < h; y0 += LZV_AHEAD) {
    uint32_t gi[LZV_AHEAD], gq[LZV_AHEAD];
    uint64_t gw[LZV_AHEAD];
#pragma unroll
    for (int u = 0; u < LZV_AHEAD; u++) { gi[u] = fi[u]; gq[u] = fq[u]; gw[u] = cw[u]; }
    if (y0 + LZV_AHEAD < h) load(y0 + LZV_AHEAD);
#pragma unroll
    for (int u = 0; u < LZV_AHEAD; u++) {
      const uint32_t y = y0 + u;
      if (y >= h) break;
      const uint32_t r = y - kmin, q = y * w + x, f = gq[u];
      uint32_t a, b, c;
      if (gi[u]) {                                                 // row r joins the filter
        lzv_bits(gi[u], a, b, c);
        bl[a >> 5][lane] |= 1u << (a & 31);
        bl[b >> 5][lane] |= 1u << (b & 31);
        bl[c >> 5][lane] |= 1u << (c & 31);
      }
      bool maybe = false;
      if (f && !((gw[u] >> (q & 63)) & 1)) {
        lzv_bits(f, a, b, c);
        maybe = ((bl[a >> 5][lane] >> (a & 31)) & (bl[b >> 5][lane] >> (b & 31)) & (bl[c >> 5][lane] >> (c & 31))) & 1;
      }
      // each possible yes: the wave reads the lane's column rows r, r - 1, .. 0, 64 per load
      bool hit = false;
      for (uint64_t um = __ballot(maybe); um; um &= um - 1) {
        const int l = __ffsll((unsigned long long)um) - 1;
        const uint32_t fl = __shfl(f, l), cl = (uint32_t)(x - lane + l) * h;
        bool found = false;
        for (int32_t r0 = (int32_t)r; r0 >= 0 && !found; r0 -= 64)
          found = __ballot(r0 - lane >= 0 && FT[cl + (uint32_t)(r0 - lane)] == fl) != 0;
        if (lane == l) hit = found;
      }
      const uint64_t m = __ballot(hit);
      if (lane == 0 && m) { cand[q >> 6] = gw[u] | m; added += (uint32_t)__popcll(m); }
    }
  }
  if (lane == 0 && added) atomicAdd(&j.tiles[t].ncand, added);
}

__global__ __launch_bounds__(NT) void k_lzcand(EncodeJob j, int limit, int ring, int mode, uint32_t mw, int lzc_nowalk) {
  extern __shared__ uint32_t fr[];
  uint32_t* ht = fr + ring;                                            // window tables (LZC_TAB)
  uint32_t* ct = ht + (mode == LZC_TAB ? 3 * LZC_W : 0);               // chunk tables (TAB, MAP)
  const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const TileInfo ti = j.tiles[t];
  const uint32_t npix = (uint32_t)ti.w * ti.h, w = ti.w;
  const uint32_t* F = j.fpb + (size_t)t * j.npix_cap;
  uint64_t* cand = j.candbits + (size_t)t * (j.npix_cap / 64);
  uint32_t* mp = lzc_map(j, t);
  const bool use_tab = mode != LZC_WALK;
  if (mode == LZC_TAB)
    for (uint32_t e = tid; e < 3 * LZC_W; e += NT) ht[e] = 0u;
  if (use_tab)
    for (uint32_t e = tid; e < 2 * LZC_C; e += NT) ct[e] = 0xffffffffu;
  if (mode == LZC_MAP)
    for (uint32_t e = tid; e < mw; e += NT) mp[e] = 0u;
  __syncthreads();
  uint32_t ncand = 0;
  for (uint32_t base = 0; base < npix; base += NT) {
    const uint32_t q = base + tid;
    const uint32_t f = q < npix ? F[q] : 0u;
    const uint32_t tag = f >> 24;
    const uint32_t hs0 = lzc_h(f, 0), hs1 = LZC_W + lzc_h(f, 1), hs2 = 2 * LZC_W + lzc_h(f, 2);
    const uint32_t cs0 = (f >> 1) & (LZC_C - 1), cs1 = LZC_C + ((f >> 12) & (LZC_C - 1));
    fr[q & (ring - 1)] = f;
    if (f && use_tab) {
      atomicMin(&ct[cs0], tid);
      atomicMin(&ct[cs1], tid);
    }
    __syncthreads();
    bool c = false, walk = f && !use_tab;
    const uint32_t bm = q < (uint32_t)limit ? q : (uint32_t)limit;
    if (f && use_tab) {
      // earlier in the chunk
      const uint32_t m0 = ct[cs0], m1 = ct[cs1];
      const bool first = m0 == (uint32_t)tid || m1 == (uint32_t)tid;
      c = (m0 < (uint32_t)tid && fr[(base + m0) & (ring - 1)] == f) ||
          (m1 < (uint32_t)tid && fr[(base + m1) & (ring - 1)] == f);
      walk = !first && !c;
      if (!c && mode == LZC_MAP) {
        // the latest earlier position of f (or of a fingerprint sharing its entry)
        for (uint32_t h = (f >> 1) & (mw - 1);; h = (h + 1) & (mw - 1)) {
          const uint32_t v = __hip_atomic_load(mp + h, __ATOMIC_RELAXED, LZC_MAP_LOAD_SCOPE);
          if (v == 0) break;
          if ((v & 0xffu) == tag) {
            c = q - ((v >> 8) - 1) <= bm;
            break;
          }
        }
      } else if (!c) {
        // in the window before the chunk
        bool none = false, yes = false;
        const uint32_t hw[3] = {ht[hs0], ht[hs1], ht[hs2]};
#pragma unroll
        for (int k = 0; k < 3; k++) {
          const uint32_t p1 = hw[k] >> 8;
          const bool recent = p1 && q - (p1 - 1) <= bm;
          none |= !recent;
          yes |= recent && (hw[k] & 0xffu) == tag;
        }
        c = yes && !none;
        walk = walk || (!none && !yes);
      }
    }
    // the uncertain lanes, one at a time by the whole wave: 64 window entries per LDS read
    // (consecutive addresses), a ballot per read, out at the first equal fingerprint.  With more
    // than 8 of them (the long windows of -s3/-s4 fill the tables) every lane walks its own
    // window instead, eight entries per LDS round trip.
    const uint32_t wb = mode == LZC_MAP ? min(bm, q - base) : bm;      // MAP: the chunk only
    if (lzc_nowalk && walk && !c) { c = true; walk = false; }          // knob LZC_NOWALK (measurement)
    const uint64_t um0 = __ballot(walk && !c);
    if (__popcll(um0) > 8) {
      for (uint32_t b0 = 1; walk && b0 <= wb && !c; b0 += 8) {
        uint32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = fr[(q - b0 - u) & (ring - 1)];
#pragma unroll
        for (int u = 0; u < 8; u++) c |= b0 + u <= wb && v[u] == f;
      }
    } else
    for (uint64_t um = um0; um; um &= um - 1) {
      const int l = __ffsll((unsigned long long)um) - 1;
      const uint32_t fl = __shfl(f, l), ql = __shfl(q, l), bl = __shfl(wb, l);
      bool hit = false;
      for (uint32_t b0 = 1; b0 <= bl && !hit; b0 += 64) {
        const uint32_t b = b0 + lane;
        hit = __ballot(b <= bl && fr[(ql - b) & (ring - 1)] == fl) != 0;
      }
      if (lane == l) c = hit;
    }
    if (f && !c && !lzvert_ok(w, ti.h)) {
      // vertical backs beyond the window (k_lzvert's tiles excepted): sixteen rows per batch of
      // (coalesced) global loads
      const uint32_t vlim = min(65536u, q);
      for (uint32_t b0 = (bm / w + 1) * w; b0 <= vlim && !c; b0 += 16 * w) {
        uint32_t v[16];
#pragma unroll
        for (int u = 0; u < 16; u++) v[u] = b0 + u * w <= vlim ? F[q - b0 - u * w] : 0u;
#pragma unroll
        for (int u = 0; u < 16; u++) c |= v[u] == f;
      }
    }
    const uint64_t word = __ballot(c);
    if (lane == 0 && q < npix) cand[q >> 6] = word;
    ncand += lane == 0 ? (uint32_t)__popcll(word) : 0u;
    __syncthreads();                                                   // every check has read the tables
    if (f && use_tab) {
      ct[cs0] = 0xffffffffu;
      ct[cs1] = 0xffffffffu;
      const uint32_t e = ((q + 1) << 8) | tag;
      if (mode == LZC_TAB) {
        atomicMax(&ht[hs0], e);
        atomicMax(&ht[hs1], e);
        atomicMax(&ht[hs2], e);
      } else {
        for (uint32_t h = (f >> 1) & (mw - 1);; h = (h + 1) & (mw - 1)) {
          uint32_t v = __hip_atomic_load(mp + h, __ATOMIC_RELAXED, LZC_MAP_LOAD_SCOPE);
          if (v == 0) {
            uint32_t z = 0;
            if (__hip_atomic_compare_exchange_strong(mp + h, &z, e, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP))
              break;
            v = z;                                                     // the winner's entry
          }
          if ((v & 0xffu) == tag) {
            __hip_atomic_fetch_max(mp + h, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            break;
          }
        }
      }
    }
    __syncthreads();
  }
  if (lane == 0 && ncand) atomicAdd(&j.tiles[t].ncand, ncand);
}

// LZ posting lists (-s2..-s4: windows of 2048..16384 positions).  Per tile, the positions sorted
// by a 16-bit hash of their window fingerprint, ascending inside a hash group: every position with
// the same fingerprint as q and before it is in q's group, before q, in descending order when
// walked back from q's rank -- so k_lzscan visits only equal-hash positions of q's window, back
// distances ascending, instead of every fingerprint of the window (lz.hpp:32-50 at seek 11..14).
// Two stable counting-sort passes (LSD, 8-bit digits) of the entries pos | hash << 16 |
// fingerprint << 32, one 1024-thread workgroup per tile (tiles strided over a grid of one
// workgroup per CU).  Both passes' digit counts come from one read of the fingerprints (LDS
// histograms); then each pass runs over chunks of LZSORT_C entries: a chunk is ranked in LDS (each
// wave a contiguous share of it, 64 at a time: ballot peers per digit, a wave-private running base
// per digit, one scan over (digit, wave)), staged in digit order, and leaves as one contiguous run
// per digit at the digit's running base -- whole lines, not one 8-byte store per line per wave
// (round 5 scattered straight from registers: 16 waves x 256 digits of open lines per tile, ~140 B
// of HBM traffic per position against ~28 stored).
// j.lzs_hmask is 0xffff; a knobs build can narrow it (LZS_HMASK) so that hash collisions are the rule
// (tools/scripts/r5_collide.sh: the files must not change)
__device__ __forceinline__ uint32_t lzs_hash(uint32_t f, uint32_t hm) { return ((f * 0x9E3779B1u) >> 16) & hm; }
// LZSORT_T threads per tile workgroup, chunks of LZSORT_C entries (a wave ranks LZSORT_C / (T / 64)
// of them).  Two shapes: 1024 / 4096 (one workgroup per CU) where the LZ stream is the longer one
// (-s1/-s2), 512 / 2048 at -s3/-s4, where the predictor search beside it is the longer one and
// gets half of each CU's waves back (natural 8192^2 -s4 31.6 -> 30.8 ms; at -s1 the 1024 shape is
// 1.6 ms faster: profiles/r06b/ab_lzsort_512.txt)
template <int LZSORT_T, int LZSORT_C>
__global__ __launch_bounds__(LZSORT_T) void k_lzsort(EncodeJob j, int limit) {
  constexpr int LZSORT_W = LZSORT_T / 64;
  constexpr int LZSORT_K = LZSORT_C / LZSORT_T;                  // groups of 64 per wave and chunk
  constexpr int LZSORT_RH = 32 * LZSORT_T;                       // positions whose ranks are built in LDS at a time (a word each)
  static_assert(LZSORT_C % LZSORT_T == 0, "whole groups per wave");
  // the sort's staging (a chunk's listed entries in digit order, then per wave its digit counts /
  // bases), later half a tile's ranks (k_lzscan's R)
  constexpr uint32_t UB = LZSORT_C + LZSORT_W * 128 > LZSORT_RH / 4 ? LZSORT_C + LZSORT_W * 128 : LZSORT_RH / 4;
  __shared__ __attribute__((aligned(16))) uint64_t ubuf[UB];
  uint64_t* buf = ubuf;
  uint32_t (*cnt)[256] = (uint32_t(*)[256])(ubuf + LZSORT_C);
  uint16_t* Rl = (uint16_t*)ubuf;
  __shared__ uint32_t hg[2][256];                                // per pass: digit counts, then running output bases
  __shared__ uint32_t cst[257];                                  // a chunk's digit starts in buf; [256]: its size
  __shared__ uint32_t wt[LZSORT_W];                              // scans: totals of the waves
  __shared__ uint32_t inner[65536 / 32];                         // flat positions inside a run (unlisted)
  __shared__ uint32_t cbit[65536 / 32];                          // the candidate screen (below)
  __shared__ uint32_t s_nl, s_ncand;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // this lane's digit group among the 64: the lanes with the same digit
  auto group = [&](bool valid, uint32_t d) -> uint64_t {
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; b++) {
      const uint64_t m = __ballot((d >> b) & 1);
      peers &= ((d >> b) & 1) ? m : ~m;
    }
    return peers;
  };
  auto wscan = [&](uint32_t v) -> uint32_t {                     // inclusive scan over the wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(v, o);
      if (lane >= o) v += u;
    }
    return v;
  };
  // tiles strided over the grid (a smaller grid keeps fewer tiles' scatter targets in L2 at once)
  for (int t = blockIdx.x; t < j.ntiles; t += gridDim.x) {
  __syncthreads();                                               // the previous tile done
  const TileInfo ti = j.tiles[t];
  const uint32_t n = (uint32_t)ti.w * ti.h;
  const uint32_t* F = j.fpb + (size_t)t * j.npix_cap;
  const uint32_t* TP = j.tpx + (size_t)t * j.npix_cap;
  const uint8_t* R8 = j.run8 + (size_t)t * j.npix_cap;
  // final order: one 8-byte entry per listed position, key (pos | hash << 16) low, fingerprint high
  uint64_t* SF = j.lzsf + (size_t)t * j.npix_cap;
  uint64_t* T = (uint64_t*)j.lzs + (size_t)t * j.npix_cap;       // after the first pass
  uint16_t* R = j.lzrank + (size_t)t * j.npix_cap;
  uint16_t* E = j.lzend + (size_t)t * j.npix_cap;
  const uint32_t hm = j.lzs_hmask;
  const uint64_t lt = (1ull << lane) - 1;
  // Flat positions (their window one colour: run8 >= 4) other than a run's first are not listed:
  // k_lzscan measures one representative per run from the run's start (its end in E).  They still
  // pass through the first pass, so that the second gives each the rank of its own run's start.
  // A flat position inside its run is a candidate at b = 1 (when it has a window: F != 0); the
  // listed ones are screened after the sort
  for (uint32_t c0 = 0; c0 < n; c0 += LZSORT_T) {
    const uint32_t i = c0 + tid;
    const bool in = i < n && i > 0 && R8[i] >= 4 && ((TP[i - 1] ^ TP[i]) & 0xffffffu) == 0;
    const uint64_t m = __ballot(in), mc = __ballot(in && F[i] != 0u);
    if (lane == 0) {
      inner[i >> 5] = (uint32_t)m; inner[(i >> 5) + 1] = (uint32_t)(m >> 32);
      cbit[i >> 5] = (uint32_t)mc; cbit[(i >> 5) + 1] = (uint32_t)(mc >> 32);
    }
  }
  if (tid < 512) hg[tid >> 8][tid & 255] = 0;
  if (tid == 0) s_ncand = 0;
  __syncthreads();
  auto is_inner = [&](uint32_t pos) -> bool { return (inner[pos >> 5] >> (pos & 31)) & 1; };
  // both passes' digit counts: every position for the first, the listed ones for the second
  for (uint32_t c0 = 0; c0 < n; c0 += LZSORT_T) {
    const uint32_t i = c0 + tid;
    const bool valid = i < n, listed = valid && !is_inner(i);
    const uint32_t h = valid ? lzs_hash(F[i], hm) : 0u, d0 = h & 255, d1 = h >> 8;
    const uint64_t g0 = group(valid, d0), g1 = group(listed, d1);
    if (valid && __popcll(g0 & lt) == 0) atomicAdd(&hg[0][d0], (uint32_t)__popcll(g0));
    if (listed && __popcll(g1 & lt) == 0) atomicAdd(&hg[1][d1], (uint32_t)__popcll(g1));
  }
  __syncthreads();
  {                                                              // -> each digit's first output slot
    const uint32_t hh = (uint32_t)tid >> 8;
    const uint32_t v = tid < 512 ? hg[hh][tid & 255] : 0u, incl = wscan(v);
    if (tid < 512 && lane == 63) wt[wv] = incl;
    __syncthreads();
    if (tid < 512) {
      uint32_t run = incl - v;
      for (int w = (int)hh * 4; w < wv; w++) run += wt[w];
      hg[hh][tid & 255] = run;
      if (tid == 511) s_nl = run + v;                            // listed positions
    }
  }
  for (int pass = 0; pass < 2; pass++) {
    const uint32_t sh = 16 + 8 * pass;
    uint64_t* out = pass ? SF : T;
    uint32_t* gb = hg[pass];
    for (uint32_t c0 = 0; c0 < n; c0 += LZSORT_C) {
      // this wave's share of the chunk: LZSORT_K groups of 64 consecutive entries
      const uint32_t b0 = c0 + (uint32_t)wv * (LZSORT_K * 64);
      uint64_t ent[LZSORT_K], lp[LZSORT_K];
      uint32_t dg[LZSORT_K];
      bool ls[LZSORT_K], vd[LZSORT_K];
#pragma unroll
      for (int k = 0; k < LZSORT_K; k++) {
        const uint32_t i = b0 + 64 * k + lane;
        vd[k] = i < n;
        uint64_t e = 0;
        if (vd[k]) {
          if (pass) e = T[i];
          else { const uint32_t f = F[i]; e = (uint64_t)f << 32 | (i | (lzs_hash(f, hm) << 16)); }
        }
        ent[k] = e;
        dg[k] = ((uint32_t)e >> sh) & 255;
        ls[k] = vd[k] && (!pass || !is_inner((uint32_t)e & 0xffffu));
      }
#pragma unroll
      for (int k = 0; k < 4; k++) cnt[wv][lane + 64 * k] = 0;    // each wave its own row
#pragma unroll
      for (int k = 0; k < LZSORT_K; k++) {
        lp[k] = group(vd[k], dg[k]) & __ballot(ls[k]);
        if (ls[k] && __popcll(lp[k] & lt) == 0) cnt[wv][dg[k]] += (uint32_t)__popcll(lp[k]);
      }
      __syncthreads();
      // the chunk's bases in buf: digits in order, the waves in order inside a digit (thread d < 256)
      {
        uint32_t c[LZSORT_W], tot = 0;
#pragma unroll
        for (int w = 0; w < LZSORT_W; w++) { c[w] = tid < 256 ? cnt[w][tid] : 0u; tot += c[w]; }
        const uint32_t incl = wscan(tot);
        if (tid < 256 && lane == 63) wt[wv] = incl;
        __syncthreads();
        if (tid < 256) {
          uint32_t run = incl - tot;
          for (int w = 0; w < wv; w++) run += wt[w];
          cst[tid] = run;
          if (tid == 255) cst[256] = run + tot;
#pragma unroll
          for (int w = 0; w < LZSORT_W; w++) { cnt[w][tid] = run; run += c[w]; }
        }
      }
      __syncthreads();
      // stage in digit order (stable: waves, groups, lanes in order)
#pragma unroll
      for (int k = 0; k < LZSORT_K; k++) {
        const uint32_t d = dg[k], o = cnt[wv][d] + (uint32_t)__popcll(lp[k] & lt);
        if (ls[k] && __popcll(lp[k] & lt) == 0) cnt[wv][d] = o + (uint32_t)__popcll(lp[k]);   // the group's first
        if (ls[k]) buf[o] = ent[k];
      }
      __syncthreads();
      // each digit's run of the chunk, contiguous at the digit's running base
      const uint32_t m = cst[256];
      for (uint32_t e = tid; e < m; e += LZSORT_T) {
        const uint64_t v = buf[e];
        const uint32_t d = ((uint32_t)v >> sh) & 255, o = gb[d] + (e - cst[d]);
        out[o] = v;
      }
      __syncthreads();
      if (tid < 256) gb[tid] += cst[tid + 1] - cst[tid];
    }
  }
  __syncthreads();
  // Ranks R (k_lzscan starts q's walk at R[q] - 1): a listed position's index in SF; a flat
  // position inside its run the last listed position before it in its group, which is its run's
  // start (every position between is inside the run, unlisted).  Built in LDS LZSORT_RH positions
  // at a time from SF (read coalesced) and written out in 16-B pieces (scattered u16 stores cost a
  // line each).  Run starts: thread i holds inner word i of the part; the last non-inner position
  // at or before each inner one comes from its own word or, by a max-scan over the words, from an
  // earlier word; before the part, from `carry` (the previous part's last run start's rank).
  {
    uint32_t carry = 0;
    for (uint32_t h0 = 0; h0 < n; h0 += LZSORT_RH) {
      const uint32_t hn = min((uint32_t)LZSORT_RH, n - h0);
      for (uint32_t i = tid; i < s_nl; i += LZSORT_T) {
        const uint32_t pos = (uint32_t)SF[i] & 0xffffu;
        if (pos - h0 < hn) Rl[pos - h0] = (uint16_t)i;
      }
      const uint32_t wb = 32 * (uint32_t)tid;
      const uint32_t iw = wb < hn ? inner[(h0 + wb) >> 5] : 0u;
      const uint32_t non = wb < hn ? ~iw : 0u;                   // non-inner (listed or past n) positions
      // inclusive max-scan of (last non-inner position + 1) over the words
      uint32_t lp = non ? wb + 32u - (uint32_t)__builtin_clz(non) : 0u;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(lp, o);
        if (lane >= o) lp = max(lp, u);
      }
      if (lane == 63) wt[wv] = lp;
      const uint32_t lprev = __shfl_up(lp, 1);
      __syncthreads();
      uint32_t ex = lane ? lprev : 0u, tot = 0;
#pragma unroll
      for (int w = 0; w < LZSORT_W; w++) {
        const uint32_t v = wt[w];
        if (w < wv) ex = max(ex, v);
        tot = max(tot, v);
      }
      const uint32_t before = ex ? (uint32_t)Rl[ex - 1] : carry;
      for (uint32_t m = iw; m; m &= m - 1) {
        const uint32_t b = (uint32_t)__builtin_ctz(m);
        const uint32_t nb = non & ((2u << b) - 1u);              // the word up to b (b = 31: all of it)
        Rl[wb + b] = nb ? Rl[wb + 31 - __builtin_clz(nb)] : (uint16_t)before;
      }
      carry = tot ? (uint32_t)Rl[tot - 1] : carry;
      __syncthreads();
      for (uint32_t e = 8 * (uint32_t)tid; e < hn; e += 8 * LZSORT_T) {
        if (e + 8 <= hn) *(uint4*)(R + h0 + e) = *(const uint4*)(Rl + e);
        else for (uint32_t i = e; i < hn; i++) R[h0 + i] = Rl[i];
      }
      __syncthreads();
    }
  }
  __syncthreads();
  // E = the last position of a listed run start's run (the position itself for every other
  // listed position).  (The fingerprints came through the sort beside the keys: k_lzscan's hit test
  // and the screen's walk read both with one 8-byte load.)
  const uint32_t nl = s_nl;
  for (uint32_t i = tid; i < nl; i += LZSORT_T) {
    const uint32_t p = (uint32_t)SF[i] & 0xffffu;
    uint32_t e = p;
    if (R8[p] >= 4) {
      while (R8[e] == 255) e += 254;                            // R8 saturates: e + 254 is in the run
      e += R8[e] - 1;
    }
    E[i] = (uint16_t)e;
  }
  __syncthreads();
  // The candidate screen (-s1..-s4, lz.hpp:37-42 at the seek window): a listed q is a horizontal
  // candidate iff an equal fingerprint starts at some b <= min(limit, q) -- walking back from q's
  // own entry over its hash group (the entries just before it here, read coalesced), a flat run
  // start seeing its colour's earlier runs in the window when the run's last listed position
  // (E - 3) is, stepping over its own run's start and hash collisions
  for (uint32_t iq = tid; iq < nl; iq += LZSORT_T) {
    const uint64_t vq = SF[iq];
    const uint32_t kq = (uint32_t)vq, q = kq & 0xffffu, f = (uint32_t)(vq >> 32);
    if (!f || q == 0) continue;
    const uint32_t bm = min(q, (uint32_t)limit), hq = kq >> 16;
    const bool flat = R8[q] >= 4;
    for (int32_t i = (int32_t)iq - 1; i >= 0; i--) {
      const uint64_t v = SF[i];
      const uint32_t e = (uint32_t)v, p = e & 0xffffu;
      if ((e >> 16) != hq) break;                                  // q's group starts after i
      const uint32_t en = flat ? (uint32_t)E[i] : p;
      const bool run = flat && en > p, own = run && en >= q;
      if (!own && q - (run ? en - 3u : p) > bm) break;             // older than the window
      if (!own && (uint32_t)(v >> 32) == f) { atomicOr(&cbit[q >> 5], 1u << (q & 31)); break; }
    }
  }
  __syncthreads();
  // every candidate word of the tile (k_lzvert then adds the vertical ones)
  uint64_t* cand = j.candbits + (size_t)t * (j.npix_cap / 64);
  uint32_t nc = 0;
  for (uint32_t w = tid; w < (n + 63) / 64; w += LZSORT_T) {
    const uint64_t word = (uint64_t)cbit[2 * w] | (uint64_t)cbit[2 * w + 1] << 32;
    cand[w] = word;
    nc += (uint32_t)__popcll(word);
  }
  if (nc) atomicAdd(&s_ncand, nc);
  __syncthreads();
  if (tid == 0 && s_ncand) atomicAdd(&j.tiles[t].ncand, s_ncand);
  }
}

#define LZS_KB 0x1ffffu      // k_lzscan keys: (L << 17) | (LZS_KB - b)
#define LZS_HB 16        // horizontal back-distance chunks of 64 whose fingerprints load at once
#define LZS_VB 4         // vertical chunks (k * w <= 65536: 256 rows of a 256-wide tile)
#define LZS_BITS 1024    // candidate words in LDS (tiles up to 65,536 pixels)
#ifndef LZS_SEG
#define LZS_SEG 4        // waves per tile (segment walks stitched as in k_lz); 8 measured: -s4 scan 12.1 -> 9.9 ms alone, the encode 41.5 -> 42.9 ms beside the search
#endif
// greedy scan (lz.hpp:32-95) over the candidates + the four LZ streams.
// Per candidate one batch of global loads (its fingerprint, 16 chunks of 64 horizontal back
// distances and the vertical ones) and then LDS only: the candidate bitmap is staged in LDS and

// the run lengths compare pixels from an LDS ring of the positions [q - limit, q + 260) (filled
// 64 positions at a time as the scan moves: each pixel read once per tile), sixteen positions per
// LDS round trip; vertical backs beyond the ring read the image.  rp = ring size (0: -s4, whose
// 16384-position window does not fit next to the other workgroups; pixels from the image).
// nseg waves per tile (LZS_SEG, each with its own pixel ring): the tile's walk
// is cut into segments walked at once and stitched by wave 0, exactly as k_lz does at -s0
// (segment matches packed into lzspec as two words: pos | (len - 4) << 16, back).
// OCC: waves per SIMD the register allocation is held to (0: the compiler's choice, 122 VGPRs,
// four workgroups per CU); the -s3/-s4 scan runs at five with 512-position rings (below)
template <int OCC>
__global__ __launch_bounds__(64 * LZS_SEG) __attribute__((amdgpu_waves_per_eu(OCC ? OCC : 1, OCC ? OCC : 10)))
void k_lzscan(EncodeJob j, int limit, int rp, int nseg_req, int hls) {
  // dynamic LDS: nseg rings of rp + 16 positions, then nseg hit lists of hls entries (a batch's
  // hits: 64 with posting lists, LZS_HB * 64 for the window walk)
  extern __shared__ uint32_t pring_all[];
  __shared__ uint64_t cb[LZS_BITS];
  __shared__ uint32_t vis[2 * LZS_BITS];                               // visited candidates
  __shared__ uint32_t s_cnt[LZS_SEG], s_exit[LZS_SEG];
  const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const TileInfo ti = j.tiles[t];
  const uint32_t npix = (uint32_t)ti.w * ti.h, nwords = (npix + 63) / 64, w = ti.w;
  const uint64_t* bits = j.candbits + (size_t)t * (j.npix_cap / 64);
  const uint32_t* F = j.fpb + (size_t)t * j.npix_cap;
  const uint32_t* FT = j.fpt + (size_t)t * j.npix_cap;
  const uint32_t th = (uint32_t)ti.h;
  const uint32_t* TP = j.tpx + (size_t)t * j.npix_cap;
  [[maybe_unused]] const uint8_t* R8 = j.run8 + (size_t)t * j.npix_cap;
  uint32_t pq_cur = 0, rq_cur = 0;                                     // pixel q and its run (measure)
  uint32_t* mt = j.matches + (size_t)t * 3 * (j.lz_cap + 1);
  int bonus = 0;                                                      // choh.cpp:139-154
  if (ti.colours != -1) {
    if (ti.colours <= 4) bonus = 32;
    else if (ti.colours <= 8) bonus = 20;
    else if (ti.colours <= 16) bonus = 10;
    else if (ti.colours <= 32) bonus = 2;
  }
  const uint32_t thr = 4 + bonus;
  const bool post = j.lzs != nullptr;                                  // posting lists (k_lzsort)
  const uint64_t* PSF = post ? j.lzsf + (size_t)t * j.npix_cap : nullptr;   // key | fingerprint << 32
  const uint16_t* PR = post ? j.lzrank + (size_t)t * j.npix_cap : nullptr;
  const uint16_t* PE = post ? j.lzend + (size_t)t * j.npix_cap : nullptr;
  const bool lds_bits = nwords <= LZS_BITS;
  const uint32_t nseg = (lds_bits && rp && nwords >= 4 * LZS_SEG && nseg_req > 1) ? (uint32_t)nseg_req : 1u;
  const uint32_t segcap = j.lz_cap / LZS_SEG;
  uint32_t* spec = j.lzspec + (size_t)t * 2 * j.lz_cap;
  auto seg_lo = [&](uint32_t s) { return s >= nseg ? npix : (nwords * s / nseg) * 64; };
  if (ti.ncand) {
    for (uint32_t i = tid; i < nwords; i += 64 * LZS_SEG) cb[i] = lds_bits ? bits[i] : 0;
    if (nseg > 1)
      for (uint32_t i = tid; i < 2 * nwords; i += 64 * LZS_SEG) vis[i] = 0;
  }
  __syncthreads();
  uint32_t* pring = pring_all + (size_t)(wv < (int)nseg ? wv : 0) * (uint32_t)(rp + 16);
  uint16_t* hl = (uint16_t*)(pring_all + (size_t)nseg_req * (rp ? rp + 16 : 1)) + (size_t)(wv < (int)nseg ? wv : 0) * hls;
  const uint32_t rmask = (uint32_t)rp - 1;
  // backs the ring serves: it holds [wend - rp, wend) with wend < q + 260 + 64, so q - b .. is in
  // it for b <= rp - 324 (and b <= limit); longer backs read the older side from the image
  const uint32_t reach = rp ? min((uint32_t)limit, (uint32_t)rp - 324u) : 0u;
  uint32_t wend = 0;
#ifdef HOH_DEBUG_READ
  // measurement builds: per-tile counters (EncodeJob::dbg; tools/scripts/lzscan_stats.py):
  // 0 measures, 1 posting batches, 2 hits measured, 3 ring runs, 4 image runs, 5 ring round trips,
  // 6 image round trips, 7 vertical runs, 8 measure cycles, 9 vertical cycles, 10 posting cycles,
  // 11 wave cycles, 12 matches, 13 stitch measures, 14 next_cand cycles
  auto dadd = [&](int k, uint32_t v) { if (j.dbg && lane == 0) atomicAdd(&j.dbg[(size_t)t * 64 + k], v); };
  const uint64_t t_wave0 = __builtin_amdgcn_s_memtime();
#define LZS_DBG(k, v) dadd(k, v)
#define LZS_T() __builtin_amdgcn_s_memtime()
#else
#define LZS_DBG(k, v) ((void)0)
#define LZS_T() 0ull
#endif
  auto fill_to = [&](uint32_t lo, uint32_t need) {
    if (lo > wend) wend = lo & ~63u;
    while (wend < need) {
      const uint32_t p = wend + (uint32_t)lane;
      const uint32_t v = TP[min(p, npix - 1)], e = p & rmask;              // unconditional load
      const uint32_t x = p < npix ? v & 0xffffffu : 0xff000000u;
      pring[e] = x;
      if (e < 16) pring[e + rp] = x;                                 // the mirror of entries 0..15
      wend += 64;
    }
    // the wave's own ring: its LDS accesses are ordered without a barrier
  };
  // run length of q against q - b (lz.hpp:37-45), at most 259
  auto runl = [&](uint32_t q, uint32_t b) -> uint32_t {
    const uint32_t lim = min(259u, npix - q);
    uint32_t L = 0;
    if (rp && b <= reach) {
      LZS_DBG(3, 1);
      for (;;) {
        LZS_DBG(5, 1);
        // sixteen positions per LDS round trip from two bases (the mirror spares every read its
        // wrap), the first unequal one by two select chains
        const uint32_t* pa = pring + ((q + L) & rmask);
        const uint32_t* pc = pring + ((q + L - b) & rmask);
        uint32_t a[16], c[16];
#pragma unroll
        for (int u = 0; u < 16; u++) { a[u] = pa[u]; c[u] = pc[u]; }
        uint32_t r0 = 8, r1 = 16;
#pragma unroll
        for (int u = 7; u >= 0; u--) {
          r1 = a[u + 8] != c[u + 8] ? (uint32_t)u + 8 : r1;
          r0 = a[u] != c[u] ? (uint32_t)u : r0;
        }
        const uint32_t run = r0 < 8 ? r0 : r1;
        L = min(L + run, lim);
        if (run < 16 || L >= lim) break;
      }
    } else {
      // backs beyond the ring (long ones, vertical ones past the window; every back without a
      // ring): the older side from the tile's pixel words, sixteen positions per round trip.
      // First the run lengths: both sides start with equal pixels c; where c's runs from q and from
      // q - b differ in length the copy ends at the shorter (the longer side still holds c where
      // the other has left it), so only equal runs (or runs of 255+) compare on, behind them.
      LZS_DBG(4, 1);
      const uint32_t wb = TP[q - b];                                   // pixel | run << 24
      if ((wb & 0xffffffu) != pq_cur) return 0u;
      const uint32_t rb = wb >> 24;
      if (rb != rq_cur) return min(min(rb, rq_cur), lim);
      L = min(rq_cur, lim);
      while (L < lim) {
        LZS_DBG(6, 1);
        uint32_t a[16], c[16];
#pragma unroll
        for (int u = 0; u < 16; u++) {
          const uint32_t p = min(q + L + (uint32_t)u, npix - 1);
          a[u] = rp ? pring[p & rmask] : TP[p] & 0xffffffu;
          c[u] = TP[p - b] & 0xffffffu;
        }
        uint32_t r0 = 8, r1 = 16;
#pragma unroll
        for (int u = 7; u >= 0; u--) {
          r1 = a[u + 8] != c[u + 8] ? (uint32_t)u + 8 : r1;
          r0 = a[u] != c[u] ? (uint32_t)u : r0;
        }
        const uint32_t run = r0 < 8 ? r0 : r1;
        L = min(L + run, lim);
        if (run < 16) break;
      }
    }
    return L;
  };
  // first candidate q >= pos (0xffffffff: none)
  auto next_cand = [&](uint32_t pos) -> uint32_t {
    if (pos >= npix) return 0xffffffffu;
    if (lds_bits) {                                   // usually in pos's own word
      const uint64_t wv2 = cb[pos >> 6] & (~0ull << (pos & 63));
      if (wv2) return (pos & ~63u) + (uint32_t)(__ffsll((unsigned long long)wv2) - 1);
    }
    for (uint32_t wi = pos >> 6; wi < nwords; wi += 64) {
      uint64_t w2 = (wi + lane < nwords) ? (lds_bits ? cb[wi + lane] : bits[wi + lane]) : 0;
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
  // (longest, back) at candidate q as the key (L << 17) | (LZS_KB - b)
  auto measure = [&](uint32_t q) -> uint32_t {
    [[maybe_unused]] const uint64_t tm0 = LZS_T();
    LZS_DBG(0, 1);
    const uint32_t wq = TP[q];
    pq_cur = wq & 0xffffffu;
    rq_cur = wq >> 24;
    const uint32_t bm = q < (uint32_t)limit ? q : (uint32_t)limit;
    const uint32_t kmax = min(65536u, q) / w;                         // vertical: k * w <= min(65536, q)
    const uint32_t yq = q / w, cbase = (q - yq * w) * th + yq;        // q's column in FT
    // one batch: f, the first 16 horizontal chunks, the vertical chunks
    const uint32_t f = F[q];
    uint32_t fv[LZS_HB], fw[LZS_VB];
#pragma unroll
    for (int c = 0; c < LZS_HB; c++) {
      const uint32_t b = 1 + 64 * c + lane;
      fv[c] = b <= bm && !post ? F[q - b] : 0u;
    }
    // what-if EXP & 16 (measurement, output invalid): no vertical search
    const uint32_t kmv = (j.exp & 16) ? 0u : kmax;
#pragma unroll
    for (int c = 0; c < LZS_VB; c++) {
      const uint32_t k = 1 + 64 * c + lane;
      fw[c] = k <= kmv && k * w > bm ? FT[cbase - k] : 0u;            // FT[x * h + y - k] = F[q - k * w]
    }
    if (rp) fill_to(q >= reach ? q - reach : 0u, q + 260);
    // horizontal: b = 1 .. min(limit, q), longest first, then the smallest b.  Each batch's hits
    // (equal fingerprints) are listed in LDS and measured 64 at a time; every hit is measured
    // (no stop at the first 259): the maximum key is the same, the smallest b of length 259
    // winning as in the reference's short circuit (lz.hpp:47-50).  A batch with a 259 ends the
    // walk.  Keys (L << 17) | (LZS_KB - b): L <= 259, b <= 65536 < LZS_KB.
    uint32_t mine = 0;
    bool done = false;
    [[maybe_unused]] const uint64_t tp0 = LZS_T();
    if (post) {
      // posting list: q's hash group walked back from q's rank, 64 positions a batch (back
      // distances ascending); the batch in which the group or the window ends is the last
      const uint32_t hq = lzs_hash(f, j.lzs_hmask);
      const uint64_t lt = (1ull << lane) - 1;
      // A flat q (its window one colour c) finds c's runs in its group by their starts only
      // (k_lzsort lists no other position of a flat run; PR[q] is its own run's start).  Of a run
      // [s, e] the copy from position p is min(e - p + 1, r) long when the lengths differ (r = q's
      // own run, capped), so p* = max(s, e - r + 1) is at least as long as any other p of the run
      // and nearer than the equally long ones: it is the run's one candidate (q - bm if p* is
      // older than the window).  q's own run gives b = 1 with length r.
      const bool flat = rq_cur >= 4;
      uint32_t rs = 0;
      if (flat) {
        uint32_t rq = rq_cur;
        if (rq == 255 && q + 255 < npix) {
          const uint32_t w2 = TP[q + 255];
          if ((w2 & 0xffffffu) == pq_cur) rq += w2 >> 24;
        }
        rs = min(rq, min(259u, npix - q));
        if ((TP[q - 1] & 0xffffffu) == pq_cur) {
          mine = (rs << 17) | (LZS_KB - 1u);
          done = rs >= min(259u, npix - q);                            // b = 1 at the cap: nothing beats it
        }
      }
      // the next batch's entries are loaded before this batch's hits are measured (prefetch)
      int32_t i0 = (int32_t)PR[q] - 1;
      uint32_t e_n = 0u, fe_n = ~f, en_n = 0u;
      if (i0 - lane >= 0) { const uint64_t v = PSF[i0 - lane]; e_n = (uint32_t)v; fe_n = (uint32_t)(v >> 32); if (flat) en_n = PE[i0 - lane]; }
      for (; i0 >= 0 && !done; i0 -= 64) {
        const int32_t i = i0 - lane;
        const uint32_t e = e_n, fe = fe_n, en = en_n;
        e_n = 0u; fe_n = ~f;
        if (i >= 64) { const uint64_t v = PSF[i - 64]; e_n = (uint32_t)v; fe_n = (uint32_t)(v >> 32); if (flat) en_n = PE[i - 64]; }
        const uint32_t p = e & 0xffffu;
        const bool run = flat && en > p;                               // a flat run's start
        // q's own run: PR[q] counts the listed positions before q in its group, which are its own
        // run's start and any hash-colliding ones after it (never a match: equal windows are flat)
        const bool own = run && en >= q;
        const uint32_t last = run ? en - 3u : p;                       // its last position in the group
        const bool inside = i >= 0 && (e >> 16) == hq && (own || q - last <= bm);
        const uint64_t inm = __ballot(inside);
        const bool hit = inside && !own && fe == f;
        const uint64_t m = __ballot(hit);
        uint32_t ps = p;
        if (run) ps = max(max(p, en + 1u - min(rs, en + 1u)), q - bm);
        if (hit) hl[__popcll(m & lt)] = (uint16_t)(q - ps);
        const uint32_t tot = (uint32_t)__popcll(m);
        LZS_DBG(1, 1);
        LZS_DBG(2, tot);
        bool top = false;
        for (uint32_t k = lane; k < tot; k += 64) {
          const uint32_t b = hl[k], L = runl(q, b);
          const uint32_t key = (L << 17) | (LZS_KB - b);
          if (key > mine) mine = key;
          top = top || L >= 259;
        }
        done = __ballot(top) != 0 || inm != ~0ull;
      }
      done = true;
    }
    for (uint32_t g0 = 1; g0 <= bm && !done; g0 += 64 * LZS_HB) {
      if (g0 > 1) {
#pragma unroll
        for (int c = 0; c < LZS_HB; c++) {
          const uint32_t b = g0 + 64 * c + lane;
          fv[c] = b <= bm ? F[q - b] : 0u;
        }
      }
      uint32_t tot = 0;
#pragma unroll
      for (int c = 0; c < LZS_HB; c++) {
        const bool hit = g0 + 64 * c + lane <= bm && fv[c] == f;
        const uint64_t m = __ballot(hit);
        if (hit)
          hl[tot + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] =
              (uint16_t)(g0 + 64 * c + lane);                          // b <= limit <= 16384
        tot += (uint32_t)__popcll(m);
      }
      bool top = false;
      for (uint32_t i = lane; i < tot; i += 64) {
        const uint32_t b = hl[i], L = runl(q, b);
        const uint32_t key = (L << 17) | (LZS_KB - b);
        if (key > mine) mine = key;
        top = top || L >= 259;
      }
      done = __ballot(top) != 0;
    }
    uint32_t best = wave_max_u32(mine);
#ifdef LZS_PRINTF
    if (lane == 0 && (q == 1 || q == 256 || q == 515))
      printf("lzscan t %d q %u: post %d rq %u pq %x R8[q+255] %u TP[q+255] %x best %u npix %u\n", t, q, (int)post,
             rq_cur, pq_cur, q + 255 < npix ? (uint32_t)R8[q + 255] : 999u, q + 255 < npix ? TP[q + 255] : 0u, best >> 17, npix);
#endif
    [[maybe_unused]] const uint64_t tv0 = LZS_T();
    LZS_DBG(10, (uint32_t)(tv0 - tp0));
    // vertical (lz.hpp:54-74): whole rows up to 65536 back, strictly longer only
    if ((best >> 17) < 259 && kmv) {
      uint32_t vmine = 0;
      auto vchunk = [&](uint32_t k, uint32_t fk) {
        const uint32_t b = k * w;
        // b <= bm was measured by the horizontal walk: not strictly longer there, skipped
        const bool hit = k <= kmax && b > bm && fk == f;
        if (!__ballot(hit)) return;
        if (hit) {
          const uint32_t key = (runl(q, b) << 17) | (LZS_KB - b);
          if (key > vmine) vmine = key;
        }
        LZS_DBG(7, (uint32_t)__popcll(__ballot(hit)));
      };
      uint32_t vh = 0;
#pragma unroll
      for (int c = 0; c < LZS_VB; c++) vh |= (uint32_t)(fw[c] == f) << c;
      for (uint32_t k0 = 1; k0 <= kmax; k0 += 64) {                   // beyond LZS_VB: narrow tiles
        const uint32_t k = k0 + lane, c = (k0 - 1) / 64;
        vchunk(k, c < LZS_VB ? ((vh >> c) & 1 ? f : ~f) : (k <= kmax ? F[q - k * w] : 0u));
      }
      const uint32_t vb = wave_max_u32(vmine);
      if ((vb >> 17) > (best >> 17)) best = vb;
    }
    LZS_DBG(9, (uint32_t)(LZS_T() - tv0));
    LZS_DBG(8, (uint32_t)(LZS_T() - tm0));
    return best;
  };
  uint32_t nm = 0;
  bool overflow = false;
  auto emit = [&](uint32_t q, uint32_t longest, uint32_t bb) {
    if (nm < j.lz_cap) {
      if (lane == 0) { mt[3 * nm] = q; mt[3 * nm + 1] = longest; mt[3 * nm + 2] = bb; }
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
      if (nseg > 1 && lane == 0) atomicOr(&vis[q >> 5], 1u << (q & 31));
      const uint32_t best = measure(q);
      const uint32_t longest = best >> 17, bb = LZS_KB - (best & LZS_KB);
      if (longest >= thr) {
        if (nseg == 1) emit(q, longest, bb);
        else if (cnt < segcap && lane == 0) {
          spec[2 * (wv * segcap + cnt)] = q | ((longest - 4) << 16);
          spec[2 * (wv * segcap + cnt) + 1] = bb;
        }
        cnt++;
        pos = q + longest;
      } else {
        pos = q + 1;
      }
    }
    if (lane == 0) { s_cnt[wv] = cnt; s_exit[wv] = max(pos, hi); }
    LZS_DBG(12, cnt);
    LZS_DBG(11, (uint32_t)(LZS_T() - t_wave0));
  }
  if (nseg > 1) {
    __syncthreads();
    if (wv) return;
    // ---- phase 2 (wave 0): stitch the segments (k_lz)
    uint32_t pos = 0;
    for (uint32_t s = 0; s < (ti.ncand ? nseg : 0u); s++) {
      const uint32_t hi = seg_lo(s + 1), cnt = s_cnt[s];
      if (cnt > segcap) { overflow = true; nm += cnt; continue; }     // cannot happen: lz_cap >= npix / 4 + 16
      uint32_t from = 0;
      bool conv = s == 0;
      if (s > 0) {
        while (pos < hi) {
          const uint32_t q = next_cand(pos);
          if (q >= hi) { pos = hi; break; }
          if ((vis[q >> 5] >> (q & 31)) & 1) { conv = true; pos = q; break; }
          LZS_DBG(13, 1);
          const uint32_t best = measure(q);
          const uint32_t longest = best >> 17, bb = LZS_KB - (best & LZS_KB);
          if (longest >= thr) { emit(q, longest, bb); pos = q + longest; }
          else pos = q + 1;
        }
        if (conv) {                                                   // first entry at or after pos
          from = cnt;
          for (uint32_t i0 = 0; i0 < cnt; i0 += 64) {
            const uint32_t i = i0 + lane;
            const uint64_t m = __ballot(i < cnt && (spec[2 * (s * segcap + i)] & 0xffffu) >= pos);
            if (m) { from = i0 + (uint32_t)(__ffsll((unsigned long long)m) - 1); break; }
          }
        }
      }
      if (conv) {
        for (uint32_t i = from + lane; i < cnt; i += 64) {
          const uint32_t e0 = spec[2 * (s * segcap + i)], e1 = spec[2 * (s * segcap + i) + 1], k = nm + (i - from);
          if (k < j.lz_cap) { mt[3 * k] = e0 & 0xffffu; mt[3 * k + 1] = (e0 >> 16) + 4; mt[3 * k + 2] = e1; }
        }
        nm += cnt - from;
        if (nm > j.lz_cap) overflow = true;
        pos = s_exit[s];
      }
    }
  } else if (wv) {
    return;
  }
  // streams (lz.hpp:75-95): future, length - 4, back % 256, back / 256 (as u8)
  uint16_t* lz0 = j.sym + lz_sym_off_s(j, t, 0);
  uint16_t* lz1 = j.sym + lz_sym_off_s(j, t, 1);
  uint16_t* lz2 = j.sym + lz_sym_off_s(j, t, 2);
  uint16_t* lz3 = j.sym + lz_sym_off_s(j, t, 3);
  uint32_t nf = 0, prev_end = 0;
  const uint32_t nmk = nm < j.lz_cap ? nm : j.lz_cap;
  for (uint32_t m = 0; m <= nmk; m++) {
    const bool tail = m == nmk;
    const uint32_t mpos = tail ? npix : mt[3 * m];
    const uint32_t g = mpos - prev_end, n255 = g / 255;
    if (nf + n255 + 1 > j.lz_cap) { overflow = true; break; }
    for (uint32_t k = lane; k < n255; k += 64) lz0[nf + k] = 255;
    nf += n255;
    if (!tail) {
      if (lane == 0) {
        lz0[nf] = (uint16_t)(g % 255);
        lz1[m] = (uint16_t)(mt[3 * m + 1] - 4);
        lz2[m] = (uint16_t)(mt[3 * m + 2] % 256);
        lz3[m] = (uint16_t)(uint8_t)(mt[3 * m + 2] / 256);
      }
      nf++;
      prev_end = mpos + mt[3 * m + 1];
    }
  }
  uint32_t nk = 0;
  for (uint32_t m = lane; m < nmk; m += 64) nk += mt[3 * m + 1];
  for (int o = 32; o > 0; o >>= 1) nk += __shfl_xor(nk, o);
  // only the fields this kernel owns: it runs on the side stream while k_rawmed / k_search read
  // the same TileInfo (flags through an atomic OR, never a whole-struct store)
  if (lane == 0) {
    if (overflow) atomicOr(&j.tiles[t].flags, (uint32_t)TF_OVERFLOW);
    j.tiles[t].nmatch = nm;
    j.tiles[t].nfut = nf;
    j.tiles[t].nclean = (overflow || !nmk) ? npix : npix - nk;
  }
}

// ---------------------------------------------------------------- stream set-up and choices

__global__ __launch_bounds__(128) void k_setup_s(EncodeJob j) {
  const int t = blockIdx.x, k = threadIdx.x;
  if (k >= SPT_S) return;
  const TileInfo ti = j.tiles[t];
  const uint32_t nclean = ti.nclean;
  const uint32_t nmk = ti.nmatch < j.lz_cap ? ti.nmatch : j.lz_cap;
  const uint32_t sid = t * SPT_S + k;
  StreamInfo st;
  memset(&st, 0, sizeof(st));
  st.mode = SM_EMPTY;
  if (k < KS_MED) {                                                   // LZ (lz.hpp:100-142)
    st.sym_off = lz_sym_off_s(j, t, k);
    st.slab_off = lz_slab_off_s(j, t, k);
    st.slab_cap = j.lz_cap + 8;
    st.n = k == 0 ? ti.nfut : nmk;
    st.range = 256;
    st.pb = 10;
    st.fast = 1;                                                      // k_tables decides
  } else {
    int p, kind;
    if (k < KS_FIN) { kind = KS_MED; p = k - KS_MED; }
    else if (k < KS_MAP) { kind = KS_FIN; p = k - KS_FIN; }
    else if (k < KS_VAR) { kind = KS_MAP; p = k - KS_MAP; }
    else { kind = KS_VAR; p = (k - KS_VAR) / 8; }
    const PlaneInfo pi = j.pinfo[(size_t)t * HOH_NPLANE_S + p];
    if (pi.present) {
      const uint32_t range = 1u << pi.depth;
      if (kind == KS_MED) {
        st.sym_off = med_plane_off(j, t, p);
        st.slab_off = plane_slab_off_s(j, t, p);
        st.slab_cap = j.npix_cap + 8;
        st.n = nclean; st.range = range; st.pb = 15; st.fast = 1;
        st.hist_src = sid + 1;
      } else if (kind == KS_MAP) {
        if (pi.xt) {
          st.sym_off = map_sym_off(j, t, p);
          st.slab_off = map_slab_off_s(j, t, p);
          st.slab_cap = HOH_MAPCAP + 8;
          st.n = pi.xt * pi.yt; st.range = pi.used; st.pb = 8;        // layer_encode.hpp:308-315
          st.fast = 1;
        }
      } else if (kind == KS_VAR) {
        st.sym_off = fin_plane_off(j, t, p);
        st.n = nclean; st.range = range; st.pb = kVarPb[(k - KS_VAR) % 8];
        st.sizeonly = 1; st.fast = 1;                                // k_tables decides
        st.hist_src = t * SPT_S + KS_FIN + p + 1;
      }
      // KS_FIN stays absent until k_choose_s activates it
    }
  }
  j.streams[sid] = st;
}

// The prob_bits ladder (layer_encode.hpp:326-398) needs a trial's exact size only where it can
// change the decision.  From k_tables' word bounds, per plane: t1 / t2 (prob_bits 16 / 15) when
// their order is uncertain; then, in each branch that can be taken, the trials whose lower bound
// is <= U = min(the depth bound, the branch trials' upper bounds).  U is at least the smallest
// value the ladder compares, so a trial above it can never be that minimum: if it comes before
// the minimum, whatever it sets is overwritten by the minimum's own update (strictly smaller),
// and after it, it updates nothing.  Such a trial is not encoded: its words are set to the lower
// bound (still above U, and on the certain side of a decided t1 / t2 order), sizeonly = 2.  The
// files are those of the full ladder.
__device__ __forceinline__ uint64_t trial_size(const StreamInfo& v, uint32_t words) {   // k_finalize's size
  const uint64_t rb = (uint64_t)words * 4, es = v.hdr_len + hoh_varint_len(rb) + rb;
  return v.expected_stored < es ? v.expected_stored : es;
}
__global__ __launch_bounds__(64) void k_prune_s(EncodeJob j) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= j.ntiles * HOH_NPLANE_S) return;
  const int t = i / HOH_NPLANE_S, p = i % HOH_NPLANE_S;
  const PlaneInfo pi = j.pinfo[i];
  if (!pi.present) return;
  const TileInfo ti = j.tiles[t];
  StreamInfo* v = j.streams + (size_t)t * SPT_S + KS_VAR + p * 8;
  uint64_t lo[8], hi[8];
  for (int k = 0; k < 8; k++) {
    if (v[k].mode != SM_RANS || !v[k].fast || v[k].err || v[k].sizeonly != 1 || v[k].whi < v[k].wlo || v[k].wlo < 2) {
      for (int a = 0; a < 8; a++)                                    // not a plain trial: keep them all
        j.trials[atomicAdd(j.ntrial, 1u)] = (uint32_t)(t * SPT_S + KS_VAR + p * 8 + a);
      return;
    }
    lo[k] = trial_size(v[k], v[k].wlo);
    hi[k] = trial_size(v[k], v[k].whi);
  }
  const uint64_t n = (uint64_t)ti.w * ti.h;
  const uint64_t dbound = (pi.depth * n + (pi.depth * n) % 8 + 1024) / 8;   // k_choose_s' first `possible`
  const bool surelyA = hi[0] < lo[1], surelyB = lo[0] >= hi[1];
  uint32_t need = (!surelyA && !surelyB) ? 3u : 0u;
  for (int br = 0; br < 2; br++) {
    if (br == 0 ? surelyB : surelyA) continue;                        // branch not taken
    const int ks[4] = {br, br ? 5 : 2, br ? 6 : 3, br ? 7 : 4};
    uint64_t U = dbound;
    for (int a = 0; a < 4; a++) U = hi[ks[a]] < U ? hi[ks[a]] : U;
    for (int a = 0; a < 4; a++)
      if (lo[ks[a]] <= U) need |= 1u << ks[a];
  }
  for (int k = 0; k < 8; k++) {
    if ((need >> k) & 1) {
      j.trials[atomicAdd(j.ntrial, 1u)] = (uint32_t)(t * SPT_S + KS_VAR + p * 8 + k);
      // a trial that can become the layer's final stream (k >= 2, k_choose_s) stores its words
      // in the trial pool when there is room: whi bounds them (k_tables; tests/
      // test_gpu_check_build.py), and the chain stops storing, never writes, past the slab
      if (k >= 2 && j.tpool_words) {
        const uint64_t cap = (uint64_t)v[k].whi + 64;
        const uint64_t o = atomicAdd(j.tpool_head, (unsigned long long)cap);
        if (o + cap <= j.tpool_words) {
          v[k].slab_off = j.tpool_off + o;
          v[k].slab_cap = (uint32_t)cap;
          v[k].sizeonly = 3;
        }
      }
    } else {
      v[k].sizeonly = 2; v[k].words = v[k].wlo;
    }
  }
#ifdef HOH_DEBUG_READ
  if (j.dbg) atomicAdd(&j.dbg[(size_t)t * 64 + 40 + __popc(need)], 1u);   // planes by trials kept (lzscan_stats.py)
#endif
}

// layer_encode.hpp:22, :115-120, :326-398 on the stream sizes
__global__ __launch_bounds__(64) void k_choose_s(EncodeJob j) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= j.ntiles * HOH_NPLANE_S) return;
  const int t = i / HOH_NPLANE_S, p = i % HOH_NPLANE_S;
  PlaneInfo pi = j.pinfo[i];
  if (!pi.present) return;
  const TileInfo ti = j.tiles[t];
  const StreamInfo* st = j.streams + (size_t)t * SPT_S;
  const uint64_t n = (uint64_t)ti.w * ti.h;
  uint64_t possible = (pi.depth * n + (pi.depth * n) % 8 + 1024) / 8;
  uint32_t valid = 0, fin = 0, fin_pb = 0, fin_k = 0;
  const uint64_t sm = st[KS_MED + p].size;
  if (sm < possible) { possible = sm; valid = 1; }
  const StreamInfo* v = st + KS_VAR + p * 8;
  const uint64_t t1 = v[0].size, t2 = v[1].size;
  if (t1 < t2) {
    if (t1 < possible) possible = t1;                                 // not swapped (Q14)
    for (int k = 2; k < 5; k++) if (v[k].size < possible) { possible = v[k].size; valid = 1; fin = 1; fin_pb = v[k].pb; fin_k = k; }
  } else {
    if (t2 < possible) possible = t2;
    for (int k = 5; k < 8; k++) if (v[k].size < possible) { possible = v[k].size; valid = 1; fin = 1; fin_pb = v[k].pb; fin_k = k; }
  }
  pi.possible = (uint32_t)possible;
  pi.valid = valid;
  pi.perm_final = fin;
  pi.size = pi.fixed_len + (pi.xt ? st[KS_MAP + p].size : 0) + (uint32_t)possible;
  pi.limit = pi.size;
  j.pinfo[i] = pi;
  if (fin) {
    StreamInfo f = v[0];
    f.pb = fin_pb;
    f.sizeonly = 0;
    f.slab_off = plane_slab_off_s(j, t, p);                          // the MED stream's slab: unused now
    f.slab_cap = j.npix_cap + 8;
    f.mode = SM_EMPTY; f.words = 0; f.size = 0; f.err = 0; f.fast = 1;   // k_tables decides
    const StreamInfo& w = v[fin_k];
    if (w.sizeonly == 3) {
      // the winning trial stored its words: the same symbols, prob_bits and table, so they are
      // this stream's words (the final chain launch skips it; k_tables rebuilds the header)
      f.slab_off = w.slab_off; f.slab_cap = w.slab_cap; f.words = w.words; f.widx_end = w.widx_end;
      f.sizeonly = 4;
    }
    j.streams[(size_t)t * SPT_S + KS_FIN + p] = f;
  }
}

// ---------------------------------------------------------------- tile layout and fixed bytes

// byte ranges of one layer in the file: [fixed header][map stream][permanent prefix], clipped to
// the layer's limit (the Q15 prefix of an indexed layer)
__device__ void place_layer(const EncodeJob& j, int t, int p, uint64_t off, uint32_t limit) {
  PlaneInfo& pi = j.pinfo[(size_t)t * HOH_NPLANE_S + p];
  StreamInfo* st = j.streams + (size_t)t * SPT_S;
  pi.out_off = off;
  pi.limit = limit;
  uint64_t o = pi.fixed_len;
  StreamInfo& mp = st[KS_MAP + p];
  if (pi.xt) {
    mp.out_off = off + o;
    if (o >= limit) mp.drop = 1;
    else if (o + mp.size > limit) mp.clip = (uint32_t)(limit - o);
    o += mp.size;
  }
  StreamInfo& pm = st[(pi.perm_final ? KS_FIN : KS_MED) + p];
  pm.out_off = off + o;
  const uint64_t want = pi.possible;
  const uint64_t room = limit > o ? limit - o : 0;
  const uint64_t keep = want < room ? want : room;
  if (keep == 0) pm.drop = 1;
  else pm.clip = (uint32_t)keep;
  st[(pi.perm_final ? KS_MED : KS_FIN) + p].drop = 1;
}

// One workgroup per file (k_layout's batch scheme): blockIdx.x = the image of a batch, its tiles
// [tb, te), its file at img * out_stride; else the one file / shard blob
__global__ __launch_bounds__(1024) void k_layout_s(EncodeJob j) {
  __shared__ uint64_t part[1024];
  __shared__ uint64_t tot_size, tot_vlen;
  const int tid = threadIdx.x, img = blockIdx.x;
  const int tb = j.nimg > 1 ? img * j.img_tiles : 0, te = j.nimg > 1 ? tb + j.img_tiles : j.ntiles;
  const uint64_t fbase = j.nimg > 1 ? (uint64_t)img * j.out_stride : 0;
  if (tid == 0) { tot_size = 0; tot_vlen = 0; }
  __syncthreads();
  for (int base = tb; base < te; base += 1024) {
    const int t = base + tid;
    uint64_t sz = 0, vl = 0;
    if (t < te) {
      TileInfo ti = j.tiles[t];
      StreamInfo* st = j.streams + (size_t)t * SPT_S;
      const PlaneInfo* pi = j.pinfo + (size_t)t * HOH_NPLANE_S;
      uint32_t bad = ti.flags & (TF_UNREPRODUCIBLE | TF_UNSUPPORTED | TF_OVERFLOW);
      for (int k = 0; k < SPT_S; k++) if (st[k].err) bad |= TF_OVERFLOW;
      const uint32_t lzb = 1 + st[0].size + st[1].size + st[2].size + st[3].size;   // lz.hpp:98-142
      uint64_t s64 = 2 + 1 + lzb;
      if (ti.flags & TF_GREY) {
        ti.mode = 0;                                              // bitimage (non-binary grey: flagged)
      } else {
        for (int p = 0; p < HOH_NPLANE_S; p++) if (pi[p].present && !pi[p].valid) bad |= TF_UNREPRODUCIBLE;
        const uint64_t L1 = pi[0].size, L2 = pi[1].size, L3 = pi[2].size;
        uint64_t best = L1 + L2 + L3 + lzb;                        // choh.cpp:295
        uint32_t mode = 128, ch1 = 0, c2 = 1, c3 = 2;
        if (pi[3].present && pi[3].size + 3ull * ti.colours + 1 + lzb < best) {   // :298-308
          best = pi[3].size + 3ull * ti.colours + 1 + lzb;
          mode = 127; ch1 = 3;
        }
        if (pi[4].present && pi[4].size + L1 + pi[5].size + lzb < best) {         // :309-325
          mode = 2; c2 = 4; c3 = 5;
        }
        if (ch1 == 3 && pi[3].size < L1) bad |= TF_UNREPRODUCIBLE;   // Q15 prefix past the layer
        ti.mode = mode;
        if (mode == 127) s64 += L1;
        else s64 += 1 + hoh_varint_len(L1) + hoh_varint_len(pi[c2].size) + L1 + pi[c2].size + pi[c3].size;
        ti.chmap = ch1 | (c2 << 4) | (c3 << 8);
      }
      if (bad) atomicOr(j.nimg > 1 ? j.img_err + img : j.gerr, j.nimg > 1 ? bad : bad << 8);
      ti.lz_bytes = lzb;
      ti.size = (uint32_t)s64;
      j.tiles[t] = ti;
      sz = s64;
      if (j.tile_sizes) j.tile_sizes[t] = (uint32_t)s64;
      if (j.write_table && t + 1 < te) vl = hoh_varint_len(s64);
    }
    if (sz) atomicAdd((unsigned long long*)&tot_size, (unsigned long long)sz);
    if (vl) atomicAdd((unsigned long long*)&tot_vlen, (unsigned long long)vl);
  }
  __syncthreads();
  const uint64_t first = j.prefix + tot_vlen;
  uint64_t carry_s = 0, carry_v = 0;
  for (int base = tb; base < te; base += 1024) {
    const int t = base + tid;
    uint64_t sz = 0, vl = 0;
    if (t < te) {
      sz = j.tiles[t].size;
      if (j.write_table && t + 1 < te) vl = hoh_varint_len(sz);
    }
    part[tid] = sz;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) { const uint64_t u = tid >= o ? part[tid - o] : 0; __syncthreads(); part[tid] += u; __syncthreads(); }
    const uint64_t es = part[tid] - sz, chunk_s = part[1023];
    __syncthreads();
    part[tid] = vl;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) { const uint64_t u = tid >= o ? part[tid - o] : 0; __syncthreads(); part[tid] += u; __syncthreads(); }
    const uint64_t ev = part[tid] - vl, chunk_v = part[1023];
    __syncthreads();
    if (t < te) {
      TileInfo ti = j.tiles[t];
      ti.off = fbase + first + carry_s + es;
      ti.pad = (uint32_t)(j.prefix + carry_v + ev);
      j.tiles[t] = ti;
      StreamInfo* st = j.streams + (size_t)t * SPT_S;
      uint64_t o = ti.off + 3 + 1;
      for (int k = 0; k < 4; k++) { st[k].out_off = o; o += st[k].size; }
      for (int p = 0; p < HOH_NPLANE_S; p++) {                  // everything not placed below is dropped
        st[KS_MED + p].drop = 1; st[KS_FIN + p].drop = 1; st[KS_MAP + p].drop = 1;
        for (int v = 0; v < 8; v++) st[KS_VAR + p * 8 + v].drop = 1;
      }
      if (!(ti.flags & TF_GREY)) {
        const PlaneInfo* pi = j.pinfo + (size_t)t * HOH_NPLANE_S;
        const uint32_t ch1 = ti.chmap & 15, c2 = (ti.chmap >> 4) & 15, c3 = (ti.chmap >> 8) & 15;
        const uint32_t L1 = pi[0].size;
        for (int k = KS_MED; k < KS_VAR; k++) st[k].drop = 0;
        if (ti.mode == 127) {
          place_layer(j, t, ch1, o, L1);
        } else {
          o += 1 + hoh_varint_len(L1) + hoh_varint_len(pi[c2].size);
          place_layer(j, t, ch1, o, L1);
          o += L1;
          place_layer(j, t, c2, o, pi[c2].size);
          o += pi[c2].size;
          place_layer(j, t, c3, o, pi[c3].size);
        }
        // layers that are not part of the tile
        for (int p = 0; p < HOH_NPLANE_S; p++) {
          if (p == (int)ch1 || (ti.mode != 127 && (p == (int)c2 || p == (int)c3))) continue;
          st[KS_MED + p].drop = 1; st[KS_FIN + p].drop = 1; st[KS_MAP + p].drop = 1;
        }
      }
    }
    carry_s += chunk_s;
    carry_v += chunk_v;
  }
  if (tid == 0) {
    if (j.nimg > 1) j.img_total[img] = first + tot_size;
    else *j.total = first + tot_size;
  }
}

// fixed bytes: tile framing (choh.cpp:115-116, :328, :351-356), LZ flags (lz.hpp:98) and every
// placed layer's header (layer_encode.hpp:57, :276-297 or :320-325), clipped to its limit
__global__ __launch_bounds__(64) void k_tilebytes_s(EncodeJob j) {
  const int t = blockIdx.x * 64 + threadIdx.x;
  if (t >= j.ntiles || !file_ok(j, t)) return;
  const TileInfo ti = j.tiles[t];
  uint8_t* o = j.out + ti.off;
  o[0] = 0; o[1] = 0;
  o[2] = (uint8_t)ti.mode;
  o[3] = 0x03;
  const int img = tile_img(j, t);
  const bool last = j.nimg > 1 ? (t + 1) % j.img_tiles == 0 : t + 1 == j.ntiles;
  if (j.write_table && !last) hoh_write_varint(j.out + (j.nimg > 1 ? (uint64_t)img * j.out_stride : 0), ti.pad, ti.size);
  if (ti.flags & TF_GREY) return;
  const PlaneInfo* pi = j.pinfo + (size_t)t * HOH_NPLANE_S;
  const uint32_t ch1 = ti.chmap & 15, c2 = (ti.chmap >> 4) & 15, c3 = (ti.chmap >> 8) & 15;
  if (ti.mode != 127) {
    uint32_t p = 3 + ti.lz_bytes;
    o[p++] = 0x24;
    p = hoh_write_varint(o, p, pi[0].size);
    p = hoh_write_varint(o, p, pi[c2].size);
  }
  const uint32_t layers[3] = {ch1, c2, c3};
  for (int k = 0; k < (ti.mode == 127 ? 1 : 3); k++) {
    const PlaneInfo& L = pi[layers[k]];
    uint8_t hb[32];
    uint32_t n = 0;
    hb[n++] = 0x10;
    if (L.xt) {
      hb[n++] = (uint8_t)(L.xt - 1);
      hb[n++] = (uint8_t)(L.yt - 1);
      hb[n++] = (uint8_t)L.used;
      for (int m = 0; m < 14; m++) {
        if (!((L.used_bits >> m) & 1)) continue;
        hb[n++] = (uint8_t)(kMasks[m] >> 8);
        hb[n++] = (uint8_t)(kMasks[m] & 255);
      }
    } else {
      hb[n++] = 0; hb[n++] = 0; hb[n++] = 0x00; hb[n++] = 0x10;
    }
    uint8_t* d = j.out + L.out_off;
    for (uint32_t i = 0; i < n && i < L.limit; i++) d[i] = hb[i];
  }
}

// ---------------------------------------------------------------- orchestration

static int ladder_prune() { return HOH_KNOB(LADDER_PRUNE, 1); }   // knob LADDER_PRUNE=0: every trial encoded
static int lzs_ring_max() { return HOH_KNOB(LZS_RING_MAX, 1024); }
static int lzs_seg() { const int n = HOH_KNOB(LZS_SEG, LZS_SEG); return n < 1 ? 1 : n > LZS_SEG ? LZS_SEG : n; }

void encode_speed_s(const EncodeJob& j, hipStream_t s, const SideStream& side, void (*mark)(void*, const char*), void* mc) {
  const int dist = j.speed == 1 ? 10 : j.speed == 2 ? 11 : j.speed == 3 ? 12 : 14;   // choh.cpp:125-137
  const int limit = 1 << dist;
  int ring = 1;
  while (ring < limit + NT) ring <<= 1;
  // The LZ screen and scan (k_lzfp, k_lzcand, k_lzscan: RGB -> fingerprints -> matches) share
  // nothing with the predictor search (RGB -> planes, residuals, histograms), so they run on the
  // context's side stream beside it; k_nuke (which compacts the searched planes) joins the two.
  // The search scratch and the LZ map lie in disjoint parts of each tile's tab_gen region.
  // a failed fork runs the LZ kernels on s itself (ordered), never unordered on the side stream
  // knob LZ_FORK=0: the LZ kernels on s itself (measurement)
  const int fork_ok = HOH_KNOB(LZ_FORK, 1);
  // k_lzfp before the fork at the speeds whose LZ stream is the longer (knob LZFP_FIRST: up to
  // that speed): alone it takes 0.6 ms, beside the predictor search's first kernels 2.6.  Natural
  // 8192^2 (profiles/r06b/ab_lzfp_first.txt): -s1 20.3 -> 18.9 ms, -s2 21.9 -> 20.4; at -s3 / -s4,
  // where the search stream is the longer, +0.4 / +-0
  const bool lzfp_first = j.speed <= HOH_KNOB(LZFP_FIRST, 2);
  if (lzfp_first) hipLaunchKernelGGL(k_lzfp, dim3(16, j.ntiles), dim3(NT), 0, s, j);
  const bool fork = fork_ok && side.s && side.fork && side.join && hipEventRecord(side.fork, s) == hipSuccess &&
                    hipStreamWaitEvent(side.s, side.fork, 0) == hipSuccess;
  hipStream_t sl = fork ? side.s : s;
  {
    if (!lzfp_first) hipLaunchKernelGGL(k_lzfp, dim3(16, j.ntiles), dim3(NT), 0, sl, j);
    // the hash tables pay at -s1's window (1024); the longer windows of -s2..-s4 fill them and
    // take the global map when a tile's (half-full) map fits its share of tab_gen
    uint32_t mw = 1;
    while (mw < 2u * (uint32_t)j.npix_cap) mw <<= 1;
    const int mode = limit <= 1024 ? LZC_TAB : (size_t)mw * 4 + LZC_MAP_OFF <= TAB_TILE_BYTES ? LZC_MAP : LZC_WALK;
    const int lring = mode == LZC_MAP ? 2 * NT : ring;
    const size_t lds = (size_t)(lring + (mode == LZC_TAB ? 3 * LZC_W : 0) + (mode != LZC_WALK ? 2 * LZC_C : 0)) * 4;
    if (j.lzs) {                      // posting lists: the screen is their first hit (k_lzsort's last loop)
      // one 1024-thread workgroup per CU striding over the tiles: against a workgroup per tile
      // (1024 in flight) the scatter targets of 4x fewer tiles share the L2s, the launch leaves
      // most of each CU to the predictor search beside it, and the natural 8192^2 encodes drop
      // by 1.4-1.7 ms at -s1..-s4 (k_lzsort 5.2 -> 3.7 ms at -s1; tools/scripts/r5_ab_lzsort.sh)
      const int sgk = HOH_KNOB(LZSORT_GRID, 0);                      // 0: the CU count
      const int sg = sgk > 0 ? sgk : j.cus > 0 ? j.cus : 256;
      const dim3 grid(sg > 0 && sg < j.ntiles ? sg : j.ntiles);
      if (j.speed >= HOH_KNOB(LZSORT_HALF_SPEED, 3)) hipLaunchKernelGGL((k_lzsort<512, 2048>), grid, dim3(512), 0, sl, j, limit);
      else hipLaunchKernelGGL((k_lzsort<1024, 4096>), grid, dim3(1024), 0, sl, j, limit);
    } else {
      hipLaunchKernelGGL(k_lzcand, dim3(j.ntiles), dim3(NT), lds, sl, j, limit, lring, mode, mw, HOH_KNOB(LZC_NOWALK, 0));
    }
    hipLaunchKernelGGL(k_lzvert, dim3(4, j.ntiles), dim3(64), 0, sl, j, limit);
    int rp = 1;
    while (rp < limit + 324) rp <<= 1;
    // Four segment walks per tile (stitched as in k_lz), each with a pixel ring of up to
    // lzs_ring_max() positions; the ring serves backs up to rp - 324, the rest (long backs of
    // -s3/-s4, vertical ones) read the image.  The scan waits on its loads, so workgroups per CU
    // (LDS) count for more than the ring's reach: at -s4 rings of 8192 positions (one workgroup
    // per CU) took 185 ms per natural 8192^2 encode, 2048 (three) 166 ms (round 4); with the run
    // walks of round 5, 1024-position rings (33 KB: four workgroups per CU, an 8192^2 image's
    // 1024 tiles in one round) against 2048: -s3 k_lzscan 16.3 -> 10.2 ms, -s4 18.9 -> 17.3.
    // knobs LZS_RING_MAX / LZS_SEG (measurement).
    // -s3/-s4 (windows of 8192 / 16384, most backs beyond any ring): 512-position rings and the
    // registers held to five waves per SIMD (25 KB: five workgroups per CU instead of four) --
    // natural -s4 37.5 -> 34.9 ms; at -s1 the 1024 rings stay (24.5 against 25.4 ms)
    const bool occ5 = j.speed >= HOH_KNOB(LZS_OCC_SPEED, 3);
    const int rmax = occ5 ? HOH_KNOB(LZS_RING_HI, 512) : lzs_ring_max();
    if (rp > rmax) rp = rmax;
    if (rp < (occ5 ? 512 : 1024)) rp = 0;
    const int nseg = rp ? lzs_seg() : 1;
    const int hls = j.lzs ? 64 : LZS_HB * 64;
    const size_t dyn = (size_t)nseg * (rp ? rp + 16 : 1) * 4 + (size_t)nseg * hls * 2;
    if (occ5) hipLaunchKernelGGL(k_lzscan<5>, dim3(j.ntiles), dim3(64 * LZS_SEG), dyn, sl, j, limit, rp, nseg, hls);
    else hipLaunchKernelGGL(k_lzscan<0>, dim3(j.ntiles), dim3(64 * LZS_SEG), dyn, sl, j, limit, rp, nseg, hls);
  }
  // the join: if its record fails, s waits for the whole side stream instead
  const bool joined = fork && hipEventRecord(side.join, sl) == hipSuccess;
  if (j.speed >= 3) hipLaunchKernelGGL(k_rawmed, dim3(j.ntiles), dim3(NT), 0, s, j);
  {
    const int npred = j.speed * 5 < 14 ? j.speed * 5 : 14;
    const int ncmax = ((j.tw + 39) / 40) * ((j.th + 39) / 40);
    const uint64_t ntask = (uint64_t)walk_kinds(npred) * j.ntiles * HOH_NPLANE_S * ncmax;
    const dim3 gs(j.ntiles * HOH_NPLANE_S), gw((unsigned)((ntask + 63) / 64));
    hipLaunchKernelGGL(k_search, gs, dim3(NT), sizeof(SearchLds), s, j, 0, 0);
    for (int pass = 0; pass < (j.speed > 2 ? 2 : 1); pass++) {
      if (walk_multi(npred)) hipLaunchKernelGGL(k_search_walk_multi, gw, dim3(64), 0, s, j, npred, ncmax);
      else hipLaunchKernelGGL(k_search_walk, gw, dim3(64), 0, s, j, npred, ncmax);
      hipLaunchKernelGGL(k_search, gs, dim3(NT), sizeof(SearchLds), s, j, 1, pass);
    }
  }
  mark(mc, "search");
  if (fork && (!joined || hipStreamWaitEvent(s, side.join, 0) != hipSuccess)) (void)hipStreamSynchronize(sl);
  launch_nuke(j, s);
  mark(mc, "lz");
  hipLaunchKernelGGL(k_setup_s, dim3(j.ntiles), dim3(128), 0, s, j);
  const int S = j.ntiles * SPT_S;
  launch_tables(j, S, s);
  EncodeJob jr = j;                        // the trial chains: the packed list, or every trial
  if (ladder_prune()) hipLaunchKernelGGL(k_prune_s, dim3((j.ntiles * HOH_NPLANE_S + 63) / 64), dim3(64), 0, s, j);
  else jr.trials = nullptr;
  mark(mc, "tables");
  // the MED planes' pb-15 encodes, the prob_bits ladder's trial encodes (size only) and the LZ /
  // predictor-map streams, all on the f64-quotient chain in one launch
  launch_rans_fast_s(jr, s, j.ntiles * 6, SidMap{3, KS_MED}, j.ntiles * 3, SidMap{3, KS_MED + 3},
                     j.ntiles * HOH_NPLANE_S * 8, SidMap{HOH_NPLANE_S * 8, KS_VAR}, j.ntiles * HOH_NPLANE_S * 8, S,
                     SidMap{0, 0}, S);
  launch_rans_gen(j, S, s);
  launch_finalize(j, S, s);
  mark(mc, "rans_enc");
  hipLaunchKernelGGL(k_choose_s, dim3((j.ntiles * HOH_NPLANE_S + 63) / 64), dim3(64), 0, s, j);
  const SidMap fin{HOH_NPLANE_S, KS_FIN};
  launch_tables(j, j.ntiles * HOH_NPLANE_S, s, fin);
  launch_rans_fast(j, j.ntiles * HOH_NPLANE_S, s, fin, j.ntiles * HOH_NPLANE_S, SidMap{0, 0}, 1);
  launch_rans_gen(j, j.ntiles * HOH_NPLANE_S, s, fin);
  launch_finalize(j, j.ntiles * HOH_NPLANE_S, s, fin);
  mark(mc, "rans_enc_final");
  hipLaunchKernelGGL(k_layout_s, dim3(j.nimg > 1 ? j.nimg : 1), dim3(1024), 0, s, j);
  hipLaunchKernelGGL(k_tilebytes_s, dim3((j.ntiles + 63) / 64), dim3(64), 0, s, j);
  launch_streambytes(j, S, s);
  mark(mc, "assemble");
}

// histogram of a u16 plane (entropy estimate of layer_encode.hpp:133-147)
__global__ __launch_bounds__(NT) void k_hist16(const uint16_t* in, uint64_t n, uint32_t* hist) {
  for (uint64_t q = (uint64_t)blockIdx.x * NT + threadIdx.x; q < n; q += (uint64_t)gridDim.x * NT)
    atomicAdd(&hist[in[q]], 1u);
}

void launch_hist16(const uint16_t* in, uint64_t n, uint32_t* hist, hipStream_t s) {
  const uint64_t b = (n + NT - 1) / NT;
  hipLaunchKernelGGL(k_hist16, dim3(b < 1024 ? (b ? (unsigned)b : 1u) : 1024u), dim3(NT), 0, s, in, n, hist);
}
