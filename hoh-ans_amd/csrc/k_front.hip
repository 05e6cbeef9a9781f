// Encoder front end, one workgroup per 256x256 tile (choh.cpp:464-500 tiles are independent):
//  * subtract-green (channel.hpp:73-79) + MED fast-path residuals for the three planes
//    (prediction.hpp:6-44), written to the residual arena, histograms in LDS;
//  * grey test (channel.hpp:21-31) and distinct-colour count capped at 257 (choh.cpp:17-46);
//  * LZ candidate detection for find_lz_rgb at -s0 (lz.hpp:32-53): a position is a candidate iff
//    some back distance b in [1, 64] gives a run of >= 4 equal RGB pixels.  The greedy selection
//    itself runs in k_lz.hip over the (sparse) candidate bitmap.
// Rows stream through an LDS ring of packed pixels so that every pixel is read from HBM once.
#include "hoh_internal.h"

#define RING 2048               // pixels; >= 4 rows of the widest tile (511) + 64
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

__global__ __launch_bounds__(NT) void k_front(EncodeJob j) {
  __shared__ uint32_t ring[RING];
  __shared__ uint64_t mring[RING];
  __shared__ uint32_t hist[3][512];
  __shared__ uint32_t hset[1024];
  __shared__ int s_ncol, s_notgrey, s_ncand;

  const int t = blockIdx.x, tid = threadIdx.x;
  const int gt = j.t0 + t;
  const int x0 = (gt % j.xt) * j.tw, y0 = (gt / j.xt) * j.th;
  const int w = min(j.tw, j.W - x0), h = min(j.th, j.H - y0);
  for (int i = tid; i < 3 * 512; i += NT) (&hist[0][0])[i] = 0;
  for (int i = tid; i < 1024; i += NT) hset[i] = 0xffffffffu;
  if (tid == 0) { s_ncol = 0; s_notgrey = 0; s_ncand = 0; }
  __syncthreads();

  uint16_t* res[3];
  for (int k = 0; k < 3; k++) res[k] = j.sym + (size_t)(t * 3 + k) * j.npix_cap;
  uint64_t* cand = j.candbits + (size_t)t * (j.npix_cap / 64);
  uint32_t tested = 0;
  int notgrey = 0, ncand = 0;

  for (int y = 0; y < h; y++) {
    const uint8_t* row = j.rgb + ((size_t)(y0 + y) * j.W + x0) * 3;
    for (int x = tid; x < w; x += NT) {
      uint32_t v = row[3 * x] | (row[3 * x + 1] << 8) | (row[3 * x + 2] << 16);
      ring[(y * w + x) & (RING - 1)] = v;
    }
    __syncthreads();
    for (int x = tid; x < w; x += NT) {
      const uint32_t q = (uint32_t)y * w + x;
      const uint32_t v = ring[q & (RING - 1)];
      const uint32_t pr = v & 255, pg = (v >> 8) & 255, pbb = v >> 16;
      notgrey |= (pr != pg) | (pr != pbb);
      // distinct colours, stop inserting past 256
      if (s_ncol <= 256) {
        uint32_t hsh = (v * 2654435761u) >> 22;
        for (int probe = 0; probe < 1024; probe++) {
          uint32_t old = atomicCAS(&hset[hsh], 0xffffffffu, v);
          if (old == 0xffffffffu) { atomicAdd(&s_ncol, 1); break; }
          if (old == v) break;
          hsh = (hsh + 1) & 1023;
        }
      }
      const bool hasL = x > 0, hasT = y > 0;
      const uint32_t vL = hasL ? ring[(q - 1) & (RING - 1)] : 0;
      const uint32_t vT = hasT ? ring[(q - w) & (RING - 1)] : 0;
      const uint32_t vTL = (hasL && hasT) ? ring[(q - w - 1) & (RING - 1)] : 0;
#pragma unroll
      for (int k = 0; k < 3; k++) {
        const int c = k ? 512 : 256, half = c / 2;
        uint16_t L = hasL ? (uint16_t)plane_val(vL, k) : (uint16_t)half;
        uint16_t T = hasT ? (uint16_t)plane_val(vT, k) : (uint16_t)half;
        uint16_t TL = (hasL && hasT) ? (uint16_t)plane_val(vTL, k) : (uint16_t)half;
        uint16_t p = med16(T, L, (uint16_t)(T + L - TL));
        uint32_t r = ((int)plane_val(v, k) - (int)p + half + c) & (c - 1);
        res[k][q] = (uint16_t)r;
        atomicAdd(&hist[k][r], 1u);
      }
      // LZ: bit b-1 set iff pixel q equals pixel q-b (lz.hpp:37-42)
      uint64_t m = 0;
      const uint32_t bmax = q < 64 ? q : 64;
      for (uint32_t b = 1; b <= bmax; b++) m |= (uint64_t)(ring[(q - b) & (RING - 1)] == v) << (b - 1);
      mring[q & (RING - 1)] = m;
    }
    __syncthreads();
    // candidates: a run of 4 at one back distance starting at q (needs q + 3 < npix)
    const uint32_t done = (uint32_t)(y + 1) * w;
    const uint32_t hi = done >= 3 ? done - 3 : 0;
    for (uint32_t q = tested + tid; q < hi; q += NT) {
      uint64_t a = mring[q & (RING - 1)] & mring[(q + 1) & (RING - 1)] & mring[(q + 2) & (RING - 1)] &
                   mring[(q + 3) & (RING - 1)];
      if (a) {
        atomicOr((unsigned long long*)&cand[q >> 6], 1ull << (q & 63));
        ncand++;
      }
    }
    if (hi > tested) tested = hi;
  }
  if (notgrey) atomicOr(&s_notgrey, 1);
  if (ncand) atomicAdd(&s_ncand, ncand);
  __syncthreads();
  for (int i = tid; i < 3 * 512; i += NT) {
    const int k = i / 512, s = i % 512;
    j.hist[(size_t)(t * SK_PER_TILE + SK_G + k) * 512 + s] = hist[k][s];
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

void launch_front(const EncodeJob& j, hipStream_t s) {
  hipLaunchKernelGGL(k_front, dim3(j.ntiles), dim3(NT), 0, s, j);
}
