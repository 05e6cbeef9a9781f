// Decoder kernels (dhoh.cpp:22-283 semantics with SURVEY Q1, Q9-Q12 fixed).
//  k_dtable:  the .hoh tile table (n-1 varints after the header) -> tile offsets, parsed in
//             parallel (terminator bytes + block prefix sums).
//  k_dparse:  one wave per tile walks the tile framing and its 6 entropy streams
//             (entropy_decoding.hpp:134-257): header varints, meta byte, frequency table
//             (clamped tables parsed in parallel: per-symbol field widths -> prefix sum ->
//             MSB-first field extraction), payload location; writes DecStream records, the
//             per-stream cumulative table and a 512-bucket slot->symbol table.
//  k_drans:   rANS decode (rans64.hpp:107-142).  With a side index: one workgroup per stream,
//             lane = 1024-symbol segment from the encoder's checkpoint, tables and payload in
//             LDS.  k_drans_wave: one wave per stream (no index).
//  k_dlz:     LZ streams -> match list (un_lz.hpp:150-170, Q11/Q12 handled).
//  k_dunpred_fast: MED inverse (prediction.hpp:26-41 inverted, every row, Q9 fixed) + inverse
//             subtract-green, one wave per tile, anti-diagonal wavefront over 64-row bands.
//  k_dunpred_lz: tiles with LZ copies, serial raster walk.
#include "hoh_dec.h"
#include "../../include/hoh_ans.h"
#include <string.h>
#include <stdlib.h>
#include <algorithm>
#include <type_traits>
#include <atomic>

extern std::atomic<uint64_t> g_device_allocs;   // hoh_api.cpp
#include <vector>
#include <mutex>
#include <chrono>
#include <stdio.h>

#define DSEG HOH_SEG

struct DecJob {
  const uint8_t* in;
  uint64_t size;
  int W, H, xt, yt, tw, th, ntiles;
  uint32_t npix_cap, lz_cap;
  uint32_t plane_cap;           // arena elements per tile-plane (flat or skewed layout + slack)
  uint64_t prefix;              // bytes before the tile table
  DecTile* tiles;
  DecStream* streams;
  uint32_t* cum;                // [stream][513]
  uint16_t* bsym;               // [stream][512] symbol at slot bucket*64 (prob_bits 15) / generic
  uint16_t* dsym;               // decoded symbols: planes [tile][3][plane_cap], LZ [tile][3][lz_cap]
  uint16_t* dplane;             // decoded planes of tiles with LZ matches [tile][3][npix_cap]
  uint32_t cum_stride;          // entries per stream in cum (>= range + 1)
  uint32_t* matches;            // [tile][lz_cap+1][4]: pixel index, length, back, nuked before
  int lzband;                   // rows per band of k_dunpred_lz (LDS-bound)
  int lzstage;                  // k_dunpred_lz stages each band's residuals in LDS
  uint32_t* lzt;                // tiles with LZ copies (w >= 64), appended by k_dlz; count in gerr[2];
                                //   then the chain tiles of the tile width [ntiles, 2 ntiles) (count
                                //   gerr[7]) and of the edge width [2 ntiles, 3 ntiles) (gerr[8])
  uint8_t* bmap;                // chain tiles: per-pixel back distance, [tile][th][pitch(tw)]
  uint32_t lz_xrow;             // copies reading the row above that make a tile a chain tile
  uint8_t* rgb;                 // output image
  uint32_t* gerr;
  const IndexStream* ix;        // optional side index
  const Checkpoint* ck;
  int nix;
  int t0;                       // global index of the first tile (shard decode)
  const uint32_t* tsizes;       // shard decode: tile byte sizes instead of the file's table
  int blk_ok;                   // plane_cap holds the blocked layout of a 256-wide tile
  int nimg, img_tiles;          // batch (hoh_decode_images_async): nimg files of img_tiles tiles, the
  uint64_t in_stride;           //   image their stack, file i at in + i * in_stride (nimg <= 1: one file)
  uint32_t exp;                 // measurement what-ifs (knob EXP, knob builds only; 0 in the product)
};

__device__ __forceinline__ uint64_t rd_varint(const uint8_t* b, uint64_t& p) {
  uint64_t b0 = b[p++];
  if (!(b0 & 0x80)) return b0;
  uint64_t b1 = b[p++];
  if (!(b1 & 0x80)) return ((b0 & 0x7f) << 7) + b1;
  uint64_t b2 = b[p++];
  return ((b0 & 0x7f) << 14) + ((b1 & 0x7f) << 7) + b2;
}

// MSB-first bit field at absolute bit position pos (the stuffer layout, varint.hpp:47-77)
__device__ __forceinline__ uint32_t get_bits(const uint8_t* b, uint64_t pos, uint32_t nb) {
  uint32_t v = 0;
  for (uint32_t i = 0; i < nb; i++) {
    const uint64_t q = pos + i;
    v = (v << 1) | ((b[q >> 3] >> (7 - (q & 7))) & 1);
  }
  return v;
}

// inclusive block-wide prefix sum (1024 threads); returns the block total through *total
__device__ uint64_t block_scan_1024(uint64_t v, uint64_t* wsum, uint64_t* total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t u = __shfl_up(v, o);
    if (lane >= o) v += u;
  }
  if (lane == 63) wsum[wv] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t run = 0;
    for (int i = 0; i < 16; i++) { const uint64_t x = wsum[i]; wsum[i] = run; run += x; }
    wsum[16] = run;
  }
  __syncthreads();
  v += wsum[wv];
  *total = wsum[16];
  __syncthreads();
  return v;
}

// Enqueue-only decodes have no host check between kernels: every kernel returns at once when an
// earlier kernel (or the header check) recorded an error.  Block-uniform: one read, one barrier
// (a block of the same kernel may set the word meanwhile).
__device__ __forceinline__ bool dec_abort(const DecJob& j) {
  __shared__ uint32_t g_abort;
  if (threadIdx.x == 0) g_abort = *(volatile const uint32_t*)j.gerr;
  __syncthreads();
  return g_abort != 0;
}

// the .hoh prefix the caller's W, H imply (async decode): magic .. tiling bytes, <= 16 bytes;
// a batch: every file's (one workgroup each)
__global__ void k_dhdr(DecJob j, uint64_t lo, uint64_t hi, int n) {
  const int i = threadIdx.x;
  if (i >= n) return;
  const uint64_t b = (uint64_t)blockIdx.x * j.in_stride + i;
  const uint8_t want = (uint8_t)((i < 8 ? lo >> (8 * i) : hi >> (8 * (i - 8))) & 255);
  if (b >= j.size || j.in[b] != want) atomicOr(j.gerr, 1u);
}

// Tile table (dhoh.cpp:42-65): n-1 varints after the header give tile sizes.  Parallel parse:
// a varint ends at a byte < 0x80, unless a run of >= 3 bytes >= 0x80 occurs (varint.hpp reads a
// third byte whole), in which case thread 0 re-parses serially.  Shard decode (tsizes set)
// takes the sizes from the caller instead.  Sizes are parked in tiles[i+1].off, then scanned.
// One workgroup per file: a batch's file blockIdx.x holds tiles [ib, ib + nt) at in_stride * it.
__global__ __launch_bounds__(1024) void k_dtable(DecJob j) {
  if (dec_abort(j)) return;
  __shared__ uint64_t wsum[17];
  __shared__ uint64_t tend;
  __shared__ int serial;
  const int tid = threadIdx.x;
  const bool batch = j.nimg > 1;
  const int ib = batch ? blockIdx.x * j.img_tiles : 0;
  const int nt = batch ? j.img_tiles : j.ntiles, nv = nt - 1;
  const uint64_t fb = batch ? (uint64_t)blockIdx.x * j.in_stride : 0;
  const uint64_t fend = batch ? min((uint64_t)j.size, fb + j.in_stride) : (uint64_t)j.size;
  DecTile* tiles = j.tiles + ib;
  for (int i = tid; i < nt; i += 1024) {
    DecTile t;
    const int g = j.t0 + ib + i;
    const int xo = (g % j.xt) * j.tw, yo = (g / j.xt) * j.th;
    t.x0 = xo; t.y0 = yo;
    t.w = min(j.tw, j.W - xo); t.h = min(j.th, j.H - yo);
    t.off = i == 0 ? 0 : (j.tsizes ? j.tsizes[ib + i - 1] : 0);
    t.mode = 0; t.nmatch = 0; t.err = 0; t.pad = 0;
    tiles[i] = t;
  }
  if (tid == 0) { tend = fb + j.prefix; serial = 0; }
  __syncthreads();
  if (!j.tsizes && nv > 0) {
    const uint64_t p0 = fb + j.prefix;
    const uint64_t end = min(fend, p0 + 3ull * nv);
    uint64_t cnt = 0;
    for (uint64_t base = p0; base < end && cnt < (uint64_t)nv; base += 1024) {
      const uint64_t pos = base + tid;
      const uint32_t b = pos < end ? j.in[pos] : 0xffu;
      const bool term = pos < end && b < 0x80;
      uint64_t tot;
      const uint64_t incl = block_scan_1024(term ? 1 : 0, wsum, &tot);
      const uint64_t idx = cnt + incl - 1;
      if (term && idx < (uint64_t)nv) {
        const bool b1 = pos >= p0 + 1 && j.in[pos - 1] >= 0x80;
        const bool b2 = b1 && pos >= p0 + 2 && j.in[pos - 2] >= 0x80;
        const bool b3 = b2 && pos >= p0 + 3 && j.in[pos - 3] >= 0x80;
        if (b3) serial = 1;
        uint64_t v = b;
        if (b2) v = ((uint64_t)(j.in[pos - 2] & 0x7f) << 14) + ((uint64_t)(j.in[pos - 1] & 0x7f) << 7) + b;
        else if (b1) v = ((uint64_t)(j.in[pos - 1] & 0x7f) << 7) + b;
        tiles[idx + 1].off = v;
        if (idx == (uint64_t)nv - 1) tend = pos + 1;
      }
      cnt += tot;
    }
    __syncthreads();
    if (cnt < (uint64_t)nv) serial = 1;
    __syncthreads();
    if (serial && tid == 0) {                       // exact varint.hpp:6-27 walk
      uint64_t p = p0;
      bool ok = true;
      for (int i = 0; i < nv; i++) {
        if (p + 3 > fend) { ok = false; break; }
        tiles[i + 1].off = rd_varint(j.in, p);
      }
      tend = p;
      if (!ok) atomicOr(j.gerr, 1u);
    }
  }
  __syncthreads();
  // exclusive offsets: tiles follow the table
  uint64_t carry = tend;
  for (int i0 = 0; i0 < nt; i0 += 1024) {
    const int i = i0 + tid;
    const uint64_t v = i < nt ? tiles[i].off : 0;
    uint64_t tot;
    const uint64_t incl = block_scan_1024(v, wsum, &tot);
    if (i < nt) tiles[i].off = carry + incl;     // tiles[0].off holds 0
    carry += tot;
  }
  __syncthreads();
  if (tid == 0 && tiles[nt - 1].off >= fend) atomicOr(j.gerr, 1u);
}

// parse one entropy stream starting at byte p (all lanes, uniform control flow)
__device__ bool parse_stream(const DecJob& j, uint64_t& p, int sid, uint64_t out_off, int lane) {
  DecStream d;
  memset(&d, 0, sizeof(d));
  d.ix = -1;
  d.out_off = out_off;
  if (p + 2 > j.size) return false;
  const uint64_t range = rd_varint(j.in, p) + 1;
  const uint64_t n = rd_varint(j.in, p);
  d.range = (uint32_t)range;
  d.n = (uint32_t)n;
  d.maxbits = hoh_bitlen(range - 1);
  if (n == 0) {
    d.mode = SM_EMPTY;
    if (lane == 0) j.streams[sid] = d;
    return true;
  }
  if (range + 1 > j.cum_stride || p >= j.size) return false;
  const uint8_t meta = j.in[p++];
  if (!(meta >> 7)) {                                    // stored
    d.mode = SM_STORED;
    d.payload_off = p;
    p += ((uint64_t)d.maxbits * n + 7) / 8;
    if (p > j.size) return false;
    if (lane == 0) j.streams[sid] = d;
    return true;
  }
  d.mode = SM_RANS;
  d.pb = (meta & 0x3c) >> 2;
  d.tsm = meta & 3;
  if (d.pb == 0 || (1u << d.pb) < range) return false;
  d.table_off = p;
  const uint64_t tb = p * 8;
  uint32_t* cum = j.cum + (size_t)sid * j.cum_stride;
  const uint32_t mb = d.maxbits;
  uint64_t bits = 0;
  if (d.tsm == 1) {
    for (uint32_t i = lane; i < range; i += 64) cum[i + 1] = get_bits(j.in, tb + (uint64_t)i * mb, mb);
    bits = (uint64_t)range * mb;
  } else if (d.tsm == 2) {
    const uint32_t cn = (d.pb - 1) / 4 + 2;
    uint32_t lower[8], upper[8];
    for (uint32_t i = 0; i < cn && i < 8; i++) {
      lower[i] = get_bits(j.in, tb + (uint64_t)(2 * i) * mb, mb);
      upper[i] = get_bits(j.in, tb + (uint64_t)(2 * i + 1) * mb, mb);
    }
    const uint64_t cb = tb + (uint64_t)2 * cn * mb;
    if (lower[0] == upper[0] && lower[0] < range) {
      // single-symbol stream: 2^pb overflowed its field at the encoder (Q6)
      uint32_t sb = cn >= 3 ? 4 * (cn - 1) : 4;
      if (sb > d.pb) sb = d.pb;
      for (uint32_t i = lane; i < range; i += 64) cum[i + 1] = i == lower[0] ? (1u << d.pb) : 0;
      bits = (uint64_t)2 * cn * mb + sb;
    } else {
      // field widths (entropy_decoding.hpp:219-234), prefix sum over contiguous lane chunks
      const uint32_t chunk = (uint32_t)((range + 63) / 64);
      const uint32_t c0 = lane * chunk, c1 = min((uint32_t)range, c0 + chunk);
      auto sbits = [&](uint32_t i) -> uint32_t {
        uint32_t sb = 0;
        if (lower[0] <= i && upper[0] >= i) sb = 1;
        if (lower[1] <= i && upper[1] >= i) sb = 4;
        for (uint32_t jj = 2; jj < cn; jj++) if (lower[jj] <= i && upper[jj] >= i) sb = 4 * jj;
        return sb > d.pb ? d.pb : sb;
      };
      uint32_t local = 0;
      for (uint32_t i = c0; i < c1; i++) local += sbits(i);
      uint32_t incl = local;
      for (int o = 1; o < 64; o <<= 1) {
        uint32_t u = __shfl_up(incl, o);
        if (lane >= o) incl += u;
      }
      uint64_t pos = cb + (incl - local);
      for (uint32_t i = c0; i < c1; i++) {
        const uint32_t sb = sbits(i);
        cum[i + 1] = get_bits(j.in, pos, sb);
        pos += sb;
      }
      bits = (uint64_t)2 * cn * mb + __shfl(incl, 63);
    }
  } else {
    return false;                                         // uniform / laplace tables: not written by choh
  }
  p += (bits + 7) / 8;
  __syncthreads();
  // cumulative (in place: cum[i+1] holds freq i)
  {
    const uint32_t chunk = (uint32_t)((range + 63) / 64);
    const uint32_t c0 = lane * chunk, c1 = min((uint32_t)range, c0 + chunk);
    uint32_t local = 0;
    for (uint32_t i = c0; i < c1; i++) local += cum[i + 1];
    uint32_t incl = local;
    for (int o = 1; o < 64; o <<= 1) {
      uint32_t u = __shfl_up(incl, o);
      if (lane >= o) incl += u;
    }
    uint32_t run = incl - local;
    for (uint32_t i = c0; i < c1; i++) { run += cum[i + 1]; cum[i + 1] = run; }
    if (lane == 0) cum[0] = 0;
    __syncthreads();
    if (cum[range] != (1u << d.pb)) return false;          // lossy raw table (Q4) or corrupt
  }
  // symbol at the start of every 2^(pb-9) slot bucket (512 buckets): only dec_run reads them, for
  // the streams no wave decoder takes (range > 512 or prob_bits > 15; never in a -s0 file).  The
  // binary searches over the global cum table cost k_dparse two thirds of its time when done for
  // every stream (0.19 ms alone, 0.53 ms per 8192^2 image under the bench's load).
  uint16_t* bs = j.bsym + (size_t)sid * 512;
  const uint32_t bshift = d.pb > 9 ? d.pb - 9 : 0;
  const uint32_t nbk = (range > 512 || d.pb > 15) ? 1u << (d.pb - bshift) : 0u;
  for (uint32_t b = lane; b < nbk; b += 64) {
    const uint32_t slot = b << bshift;
    uint32_t lo = 0, hi = (uint32_t)range;                 // cum[lo] <= slot < cum[hi]
    while (hi - lo > 1) { uint32_t mid = (lo + hi) / 2; if (cum[mid] <= slot) lo = mid; else hi = mid; }
    bs[b] = (uint16_t)lo;
  }
  const uint64_t data = rd_varint(j.in, p);
  if ((data & 3) || data < 8 || p + data > j.size) return false;
  d.payload_off = p;
  d.words = (uint32_t)(data / 4);
  p += data;                                              // Q1 fix: skip the payload
  if (lane == 0) {
    j.streams[sid] = d;
    if (j.gerr) atomicMax(j.gerr + 1, d.words);           // sizes the decoder's LDS payload stage
  }
  return true;
}

__global__ __launch_bounds__(64) void k_dparse(DecJob job) {
  if (dec_abort(job)) return;
  const int t = blockIdx.x, lane = threadIdx.x;
  // a batch: every bound check of this tile's framing and streams stops at its own file's end
  // (file i is [i * in_stride, (i + 1) * in_stride)), so a truncated file reads as corrupt instead
  // of running on into the next file's bytes
  DecJob j = job;
  if (j.nimg > 1) j.size = min(job.size, (uint64_t)(t / j.img_tiles + 1) * j.in_stride);
  DecTile ti = j.tiles[t];
  uint64_t p = ti.off;
  bool ok = p + 4 <= j.size;
  uint32_t err = 0;
  if (ok && (j.in[p] != 0 || j.in[p + 1] != 0)) { ok = false; err = 2; }   // nested tiling: unsupported
  if (ok) {
    p += 2;
    ti.mode = j.in[p++];
    if (ti.mode != 128) { ok = false; err = 2; }          // grey / bitimage / palette / rgb
  }
  if (ok) {
    const uint8_t lzt = j.in[p++];
    const size_t lzbase = (size_t)j.ntiles * 3 * j.plane_cap + (size_t)t * 3 * j.lz_cap;
    if (lzt != 0x03) { ok = false; err = 2; }
    for (int k = 0; k < 3 && ok; k++) ok = parse_stream(j, p, t * SK_PER_TILE + k, lzbase + (size_t)k * j.lz_cap, lane);
    if (ok && p + 1 < j.size && j.in[p] == 0x81 && j.in[p + 1] == 0x7f) { ok = false; err = 2; }  // 4th LZ stream (-s>=1)
  }
  if (ok) {
    if (j.in[p] != 0x24) ok = false;
    p++;
  }
  if (ok) {
    const uint64_t L1 = rd_varint(j.in, p), L2 = rd_varint(j.in, p);
    const uint64_t st[3] = {p, p + L1, p + L1 + L2};
    for (int k = 0; k < 3 && ok; k++) {
      uint64_t q = st[k];
      if (q + 5 > j.size || j.in[q] != 0x10 || j.in[q + 1] != 0 || j.in[q + 2] != 0 || j.in[q + 3] != 0 || j.in[q + 4] != 0x10) {
        ok = false; err = (q + 5 <= j.size && j.in[q] == 0x10) ? 2 : 1;   // -s>=1 predictor tiles: unsupported
        break;
      }
      q += 5;
      ok = parse_stream(j, q, t * SK_PER_TILE + 3 + k, (size_t)(t * 3 + k) * j.plane_cap, lane);
      const uint32_t depth = k ? 9 : 8;
      if (ok && j.streams[t * SK_PER_TILE + 3 + k].range != (1u << depth)) ok = false;
      // full-width tile plane without LZ copies: the blocked layout k_dunpred_fast reads
      if (ok && lane == 0 && ti.w == 256 && j.blk_ok &&
          j.streams[t * SK_PER_TILE + 3 + k].n == (uint32_t)ti.w * (uint32_t)ti.h)
        j.streams[t * SK_PER_TILE + 3 + k].blk = 1;
    }
  }
  if (!ok && !err) err = 1;
  if (lane == 0) {
    ti.err = err;
    j.tiles[t] = ti;
    if (err) atomicOr(j.gerr, err == 2 ? 2u : 1u);
  }
}

// match the decoder's streams to the side index by payload position
__global__ void k_dmatch(DecJob j, int nstreams) {
  if (dec_abort(j)) return;
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nstreams || s >= j.nix) return;
  DecStream d = j.streams[s];
  const IndexStream x = j.ix[s];
  if (d.mode == SM_RANS && x.mode == SM_RANS && x.payload_off == d.payload_off && x.n == d.n && x.words == d.words) {
    j.streams[s].ix = s;
  }
}

__device__ __forceinline__ uint32_t ld_u32_unaligned(const uint8_t* base, uint64_t off) {
  const uint64_t a = off & ~3ull;
  const uint32_t* w = (const uint32_t*)(base + a);
  const uint32_t lo = w[0];
  const uint32_t sh = (uint32_t)(off & 3);
  if (!sh) return lo;
  const uint32_t hi = w[1];
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// Blocked plane layout (residual planes of 256-wide tiles without LZ copies, DecStream.blk): row
// y = 64b + r of the tile, column x lives in band b at 8-element column block K = x/8 + ceil(r/8),
// block-major with the 64 rows of the band interleaved inside a block:
//   pos = b * BLK_BAND + (K * 64 + r) * 8 + x % 8.
// Skewing the blocks by ceil(r/8) makes the 8 columns k_dunpred_fast's lane r needs at step s
// (x = s - r .. s - r + 7) lie in blocks s/8 and s/8 + 1 for every lane, so each of its residual
// loads is one contiguous 1 KB (64 lanes x 16 B) instead of 64 scattered 16-B pieces; k_drans's
// thread for row r stores each 8-symbol block as 16 B next to its neighbour rows' (full lines).
#define BLK_NK 40                      // column blocks per band (32 + the skew of 8)
#define BLK_BAND (BLK_NK * 64 * 8)     // elements per band
__device__ __forceinline__ uint32_t blk_pos(uint32_t i) {
  const uint32_t y = i >> 8, x = i & 255, r = y & 63;
  return (y >> 6) * BLK_BAND + (((x >> 3) + ((r + 7) >> 3)) * 64 + r) * 8 + (x & 7);
}

struct OutCursor {
  uint16_t* out;
  uint32_t blk;
  __device__ OutCursor(uint16_t* o, uint32_t b, uint32_t) : out(o), blk(b) {}
  __device__ __forceinline__ void put(uint32_t i, uint16_t v) { out[blk ? blk_pos(i) : i] = v; }
};

// rANS decode (rans64.hpp:107-142) of symbols [s0, s1) of stream d from state x.  Payload words
// come from `words` (LDS-staged, word index wi) when non-null, else from the file (byte wp).
template <bool LDSW>
__device__ bool dec_run(const DecJob& j, const DecStream& d, const uint32_t* cum, const uint16_t* bs,
                        uint32_t bshift, const uint32_t* words, uint64_t x, uint64_t wp, uint64_t wend,
                        uint32_t s0, uint32_t s1, OutCursor oc, uint64_t* xend) {
  const uint32_t pb = d.pb, mask = (1u << pb) - 1, range = d.range;
  for (uint32_t i = s0; i < s1; i++) {
    const uint32_t slot = (uint32_t)x & mask;
    uint32_t s = bs[slot >> bshift];
    while (cum[s + 1] <= slot && s + 1 < range) s++;
    oc.put(i, (uint16_t)s);
    const uint32_t c = cum[s], f = cum[s + 1] - c;
    x = (uint64_t)f * (x >> pb) + (slot - c);                // Rans64DecAdvance
    if (x < (1ull << 31)) {
      if (wp >= wend) return false;
      x = (x << 32) | (LDSW ? words[wp] : ld_u32_unaligned(j.in, wp));
      wp += LDSW ? 1 : 4;
    }
  }
  *xend = x;
  return true;
}

#define DR_T 256      // threads per stream workgroup (lane = segment of HOH_SEG symbols)
#define DR_NB 1024    // 32-slot buckets (prob_bits <= 15)
#define DR_FIXED ((2 * DR_NB + 2 * 512) * 4)   // LDS bytes before the payload stage
#define DR_RW 16      // payload ring words per thread (ringed k_drans)
#define DR_SMEM (DR_FIXED + DR_RW * DR_T * 4 + 16)   // + the 4 wave totals of the table build (no static
                                                      // LDS: table offsets fold into the ds offsets)

__device__ __forceinline__ void dec_stored(const DecJob& j, int sid, const DecStream& d) {
  uint16_t* out = j.dsym + d.out_off;
  for (uint32_t i = threadIdx.x; i < d.n; i += blockDim.x) {
    const uint16_t v = (uint16_t)get_bits(j.in, d.payload_off * 8 + (uint64_t)i * d.maxbits, d.maxbits);
    out[d.blk ? blk_pos(i) : i] = v;
  }
}

// Exact slot -> symbol lookup in two LDS reads.  Symbols present in the table get a compact
// index k (ascending); per 32-slot bucket b: k0 = index of the symbol covering slot 32b and a
// mask with bit i set where a symbol starts at slot 32b + i (i > 0); per k: {f, c | sym << 16}.
// k(slot) = k0 + popcount(bits 1..slot&31 of the mask).  12 KB in all (a byte per slot was 32 KB).
struct DrTables {
  uint2* bk;    // [DR_NB] {start mask, k0}
  uint2* sy;    // [512]   {f, c | symbol << 16}
  __device__ __forceinline__ void lookup(uint32_t slot, uint32_t& sym, uint32_t& c, uint32_t& f) const {
    const uint2 e = bk[slot >> 5];
    const uint32_t k = e.y + __popc(__builtin_amdgcn_ubfe(e.x, 1, slot & 31));
    const uint2 t = sy[k];
    f = t.x;
    c = t.y & 0xffffu;
    sym = t.y >> 16;
  }
};

// One Rans64DecAdvance + renormalisation (rans64.hpp:107-142) on the split state (xh, xl) for
// prob_bits 7..15, in ~17 VALU operations: the bucket address straight from x, the popcount
// accumulating onto k0, x = f * (x >> pb) + (slot - c) as ONE v_mad_u64_u32
// f * lo32(x >> pb) + ((f * (xh >> pb)) << 32 | slot - c) (the 24-bit multiply is exact: f <= 2^15
// and xh >> pb < 2^24 because x < 2^63 and pb >= 7), the renorm select on the halves.
// bk / sy are LDS byte addresses; bmask = (mask >> 2) & ~7 turns x into the bucket's byte
// offset.  Returns the table word whose high half is the symbol.
// LDS loads by raw byte address (the kernel has no static LDS, so its dynamic area starts at 0):
// through the extern array every address carried an add of the array's link-time base
#ifdef __HIP_DEVICE_COMPILE__
// The raw-address accessors use may_alias types: one LDS location is written and read at
// different widths (u16 ring slots flushed as dwords, residual dwords read as u16), and with
// type-based alias analysis the compiler may otherwise move a load above a store of another type.
typedef uint16_t __attribute__((may_alias)) u16_ma;
typedef uint32_t __attribute__((may_alias)) u32_ma;
typedef uint2 __attribute__((may_alias)) u2_ma;
typedef uint4 __attribute__((may_alias)) u4_ma;
__device__ __forceinline__ uint2 lds_u2(uint32_t a) { return *(const __attribute__((address_space(3))) u2_ma*)(size_t)a; }
__device__ __forceinline__ uint32_t lds_u32(uint32_t a) { return *(const __attribute__((address_space(3))) u32_ma*)(size_t)a; }
__device__ __forceinline__ uint32_t lds_u16(uint32_t a) { return *(const __attribute__((address_space(3))) u16_ma*)(size_t)a; }
__device__ __forceinline__ void lds_st16(uint32_t a, uint32_t v) { *(__attribute__((address_space(3))) u16_ma*)(size_t)a = (uint16_t)v; }
__device__ __forceinline__ void lds_st2(uint32_t a, uint2 v) { *(__attribute__((address_space(3))) u2_ma*)(size_t)a = v; }
__device__ __forceinline__ void lds_st32(uint32_t a, uint32_t v) { *(__attribute__((address_space(3))) u32_ma*)(size_t)a = v; }
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) unsigned char*)p;
}
#else
__device__ uint32_t lds_addr(const void*);
__device__ void lds_st32(uint32_t, uint32_t);
__device__ uint2 lds_u2(uint32_t);
__device__ uint32_t lds_u32(uint32_t);
__device__ uint32_t lds_u16(uint32_t);
__device__ void lds_st16(uint32_t, uint32_t);
__device__ void lds_st2(uint32_t, uint2);
#endif

__device__ __forceinline__ uint32_t dstep(uint32_t bk, uint32_t sy, uint32_t bmask,
                                          uint32_t mask, uint32_t pb, uint32_t& xh, uint32_t& xl,
                                          uint32_t nw, uint32_t& wi) {
  const uint32_t slot = xl & mask;
  const uint2 e = lds_u2(bk + ((xl >> 2) & bmask));
  // v_bfe_u32 reads only bits [4:0] of its width operand: slot & 31 without the AND
  const uint32_t k = __popc(__builtin_amdgcn_ubfe(e.x, 1, slot)) + e.y;
  const uint2 t = lds_u2(sy + k * 8);
  const uint32_t d = slot - (t.y & 0xffffu);
  const uint32_t yl = __builtin_amdgcn_alignbit(xh, xl, pb);
  const uint64_t acc = ((uint64_t)__umul24(t.x, xh >> pb) << 32) | d;
  uint64_t x, co;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(x), "=s"(co) : "v"(t.x), "v"(yl), "v"(acc));
  const uint32_t nh = (uint32_t)(x >> 32), nl = (uint32_t)x;
  const bool r = x < (1ull << 31);
  xh = r ? nl : nh;
  xl = r ? nw : nl;
  wi += r;
  return t.y;
}

// Indexed decode (rans64.hpp:107-142): one 256-thread workgroup per stream, thread = segment of
// HOH_SEG symbols starting from the encoder's checkpoint.  LDS holds the lookup tables (12 KB) and
// a 16-word payload ring per thread (16 KB), refilled from the file 4 words a group ahead, so the
// per-symbol chain is LDS round trips only and five workgroups fit a CU (staging the whole payload
// needed a 40 KB stage and allowed three); the symbol stores are never awaited.
// Output is the flat plane: each thread stores its segment 16 symbols (32 B) at a time.
// k_drans's registers held to 4 waves per SIMD (128 VGPRs, was 129: three workgroups per CU
// where its 28 KB of LDS allows five; a 12-byte spill): batched decode 0.476 -> 0.459 ms/image,
// the headline pipeline +0.5 % (5 waves: 96 VGPRs, a 124-byte spill, 0.51 ms/image)
#ifndef DRANS_WPE
#define DRANS_WPE 4
#endif
#ifndef DR_LINE
#define DR_LINE 64    // symbols a thread stores at once (64: a whole 128-B line of its row)
#endif
#ifndef DUNF_WPE
#define DUNF_WPE 0
#endif
#if DRANS_WPE
#define DRANS_ATTR __attribute__((amdgpu_waves_per_eu(DRANS_WPE, DRANS_WPE)))
#else
#define DRANS_ATTR
#endif
#if DUNF_WPE
#define DUNF_ATTR __attribute__((amdgpu_waves_per_eu(DUNF_WPE, DUNF_WPE)))
#else
#define DUNF_ATTR
#endif
__global__ __launch_bounds__(DR_T) DRANS_ATTR void k_drans(DecJob j, int nstreams) {
  extern __shared__ __attribute__((aligned(16))) uint32_t dr_lds[];
  uint32_t* wtot = dr_lds + (DR_FIXED + DR_RW * DR_T * 4) / 4;
  // dec_abort through the dynamic area (read before the barrier that follows the table clear)
  if (threadIdx.x == 0) wtot[0] = *(volatile const uint32_t*)j.gerr;
  __syncthreads();
  if (wtot[0] || (j.exp & 32)) return;     // what-if EXP & 32 (measurement, output invalid): no rANS decode
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int sid = blockIdx.x;
  const DecStream d = j.streams[sid];
  if (d.mode == SM_STORED) { dec_stored(j, sid, d); return; }     // no separate launch
  if (d.mode != SM_RANS || d.range > 512 || d.pb > 15) return;
  const uint32_t pb = d.pb, M = 1u << pb, mask = M - 1, range = d.range;
  DrTables tb;
  tb.bk = (uint2*)dr_lds;                                     // 2 * DR_NB words
  tb.sy = (uint2*)(dr_lds + 2 * DR_NB);                       // 2 * 512 words
  uint32_t* pw = dr_lds + DR_FIXED / 4;                       // payload rings (DR_RW words per thread)
  uint32_t* cum_s = pw;                                       // range + 1 words, before the rings
  for (uint32_t i = tid; i <= range; i += DR_T) cum_s[i] = j.cum[(size_t)sid * j.cum_stride + i];
  const uint32_t nb = (M + 31) >> 5;
  for (uint32_t b = tid; b < nb; b += DR_T) tb.bk[b] = make_uint2(0, 0);
  __syncthreads();
  {
    // compact index of the symbols present: thread t owns symbols 2t, 2t+1 (range <= 512)
    const uint32_t s0 = 2 * tid, s1 = s0 + 1;
    const uint32_t a0 = s0 < range ? cum_s[s0] : 0, a1 = s0 < range ? cum_s[s0 + 1] : 0;
    const uint32_t a2 = s1 < range ? cum_s[s1 + 1] : 0;
    const uint32_t p0 = s0 < range && a1 > a0, p1 = s1 < range && a2 > a1;
    const uint32_t cnt = p0 + p1;
    uint32_t incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(incl, o);
      if (lane >= o) incl += t;
    }
    if (lane == 63) wtot[wv] = incl;
    __syncthreads();
    uint32_t k = incl - cnt;
    for (int q = 0; q < wv; q++) k += wtot[q];
    auto put = [&](uint32_t s, uint32_t c0, uint32_t c1, uint32_t kk) {
      tb.sy[kk] = make_uint2(c1 - c0, c0 | (s << 16));
      for (uint32_t b = (c0 + 31) >> 5; b <= (c1 - 1) >> 5; b++) tb.bk[b].y = kk;   // buckets it starts
      if (c0 & 31) atomicOr(&tb.bk[c0 >> 5].x, 1u << (c0 & 31));
    };
    if (p0) put(s0, a0, a1, k);
    if (p1) put(s1, a1, a2, k + p0);
  }
  __syncthreads();
  uint16_t* out = j.dsym + d.out_off;
  // generic decode of symbols [s0, s1) from state x (payload word wi of the stage, or the file)
  auto run = [&](uint64_t x, uint32_t wi, uint32_t s0, uint32_t s1, uint64_t* xe) -> bool {
    OutCursor oc(out, d.blk, s0);
    const uint64_t wend = (uint64_t)d.words;
    for (uint32_t i = s0; i < s1; i++) {
      const uint32_t slot = (uint32_t)x & mask;
      uint32_t sym, c, f;
      tb.lookup(slot, sym, c, f);
      oc.put(i, (uint16_t)sym);
      x = (uint64_t)f * (x >> pb) + (slot - c);             // Rans64DecAdvance
      if (x < (1ull << 31)) {
        if (wi >= wend) return false;
        x = (x << 32) | ld_u32_unaligned(j.in, d.payload_off + (uint64_t)wi * 4);
        wi++;
      }
    }
    *xe = x;
    return true;
  };
  if (d.ix < 0) {
    // no index for this stream: serial on thread 0
    if (tid == 0) {
      const uint64_t x = (uint64_t)ld_u32_unaligned(j.in, d.payload_off) | ((uint64_t)ld_u32_unaligned(j.in, d.payload_off + 4) << 32);
      uint64_t xe;
      if (!run(x, 2, 0, d.n, &xe) || xe != (1ull << 31)) atomicOr(j.gerr, 4u);
    }
    return;
  }
  const IndexStream xs = j.ix[d.ix];
  const uint32_t nseg = (d.n + DSEG - 1) / DSEG;
  bool bad = false;
  for (uint32_t sg0 = 0; sg0 < nseg; sg0 += DR_T) {
    const uint32_t sg = sg0 + tid;
    const bool act = sg < nseg;
    uint64_t x = 0, want = 1ull << 31;
    uint32_t wi = 0, s0 = 0, s1 = 0;
    if (act) {
      const Checkpoint c = j.ck[xs.ckpt_off + sg];
      x = (uint64_t)c.xl | ((uint64_t)c.xh << 32);
      wi = c.widx - xs.widx_end;
      s0 = sg * DSEG;
      s1 = min(d.n, s0 + DSEG);
      if (sg + 1 < nseg) { const Checkpoint c2 = j.ck[xs.ckpt_off + sg + 1]; want = (uint64_t)c2.xl | ((uint64_t)c2.xh << 32); }
    }
    if (act && s1 - s0 == DSEG && pb >= 7) {
      // Payload word k of the stream = bytes P+4k .. P+4k+3 of the file.  The lane's ring holds
      // words [fill-DR_RW, fill) in slots k % DR_RW (slot-major: lanes read consecutive banks).
      // A 16-symbol group reads at most 8 words (each symbol takes <= 15 bits, a renorm adds 32,
      // and the state stays in [2^31, 2^63)), so 8 words ready at a group's start suffice; the
      // next 4 are fetched one group ahead.
      uint32_t* rg = pw + tid;
      const uint64_t P = d.payload_off;
      const uint32_t al = (uint32_t)(P & 3);
      const uint64_t szal = j.size & ~3ull;
      uint32_t tailw = 0;
      for (uint64_t q = szal; q < j.size; q++) tailw |= (uint32_t)j.in[q] << (8 * (q & 3));
      // words k .. k+3 as the 5 file dwords that hold them (aligned when they land in the ring, so a
      // fetch issued a group ahead is not awaited at once: aligning it at issue put the load's
      // whole latency, and the line stores before it, in front of every group's steps)
      auto fetch5 = [&](uint32_t k, uint32_t* A) {
        const uint64_t a = (P & ~3ull) + (uint64_t)k * 4;
        if (a + 20 <= szal) {
          typedef uint32_t u4a __attribute__((ext_vector_type(4), aligned(4)));
          const u4a v = *(const u4a*)(j.in + a);
          A[0] = v.x; A[1] = v.y; A[2] = v.z; A[3] = v.w;
          A[4] = *(const uint32_t*)(j.in + a + 16);
        } else {
#pragma unroll
          for (int e = 0; e < 5; e++) {
            const uint64_t b = a + 4 * e;
            A[e] = b + 4 <= szal ? *(const uint32_t*)(j.in + b) : (b == szal ? tailw : 0u);
          }
        }
      };
      auto put4 = [&](uint32_t k, const uint32_t* A) {
#pragma unroll
        for (int e = 0; e < 4; e++) rg[((k + e) & (DR_RW - 1)) * DR_T] = __builtin_amdgcn_alignbyte(A[e + 1], A[e], al);
      };
      uint32_t fill = wi, pend[5];
      bool hp = true;                                        // pend holds words fill .. fill+3
      {
        uint32_t t0[5], t1[5];
        fetch5(fill, t0); fetch5(fill + 4, t1);
        put4(fill, t0); put4(fill + 4, t1);
        fill += 8;
        fetch5(fill, pend);                                  // lands at the first group
      }
      // LDS byte addresses (dynamic area at 0): tables at 0 and 2 * DR_NB * 4, this lane's ring
      // slot s at DR_FIXED + tid*4 + s*1024
      const uint32_t bmask = (mask >> 2) & ~7u, t4 = (uint32_t)tid * 4;
      uint32_t xh = (uint32_t)(x >> 32), xl = (uint32_t)x;
      // this thread's row r = sg (256-wide tile): flat, or blocked (blk_pos) in 16-B blocks
      uint4* o4 = d.blk ? (uint4*)(out + (sg >> 6) * BLK_BAND) + (sg & 63) + ((((sg & 63) + 7) >> 3) * 64)
                        : (uint4*)(out + s0);
      const uint32_t ostride = d.blk ? 64u : 1u;
      for (uint32_t g4 = 0; g4 < DSEG / DR_LINE; g4++) {
        uint32_t pk[DR_LINE / 2];                            // DR_LINE symbols of the lane's row
#pragma unroll
        for (int gi = 0; gi < DR_LINE / 16; gi++) {
          // land the words fetched a group ago (fill + 4 - wi <= DR_RW held when they were
          // issued, so no unread word is overwritten)
          if (hp) { put4(fill, pend); fill += 4; }
          while (fill - wi < 8) {                            // a lane that read fast: fetch now
            uint32_t t[5];
            fetch5(fill, t); put4(fill, t); fill += 4;
          }
          hp = fill + 4 - wi <= DR_RW;
          if (hp) fetch5(fill, pend);
#pragma unroll
          for (int u = 0; u < 16; u += 2) {
            const uint32_t w0 = lds_u32(DR_FIXED + (t4 | ((wi & (DR_RW - 1)) << 10)));
            const uint32_t a = dstep(0, 2 * DR_NB * 4, bmask, mask, pb, xh, xl, w0, wi);
            const uint32_t w1 = lds_u32(DR_FIXED + (t4 | ((wi & (DR_RW - 1)) << 10)));
            const uint32_t b = dstep(0, 2 * DR_NB * 4, bmask, mask, pb, xh, xl, w1, wi);
            pk[gi * 8 + u / 2] = __builtin_amdgcn_perm(b, a, 0x07060302u);   // the two high halves
          }
        }
        // the lane's whole 128-B line at once: 32-B pieces from 64 lanes 512 B apart left
        // partial lines for the memory side (WRITE_SIZE 1.6x the residual bytes)
#pragma unroll
        for (int e = 0; e < DR_LINE / 8; e++)
          o4[((DR_LINE / 8) * g4 + e) * ostride] = make_uint4(pk[4 * e], pk[4 * e + 1], pk[4 * e + 2], pk[4 * e + 3]);
      }
      if (xh != (uint32_t)(want >> 32) || xl != (uint32_t)want || wi > d.words) bad = true;
      continue;
    }
    if (!act) continue;
    uint64_t xe;
    if (!run(x, wi, s0, s1, &xe) || xe != want) bad = true;
  }
  if (bad) atomicOr(j.gerr, 4u);
}

// Serial decode of one whole stream by one wave (no index: a foreign .hoh, dhoh.cpp:297-396;
// or decode_entropy's single stream, entropy_decoding.hpp:268-276).  The chain itself is one
// lane's (rans64.hpp:107-142: each step needs the previous state), so the wave's other lanes
// keep its inputs and outputs off the chain: the lookup tables are built in LDS (DrTables, 12 KB:
// two dependent LDS reads per symbol instead of global ones), the payload is streamed into a
// 256-word LDS ring 64 words at a time (issued a group ahead, one coalesced load per lane), and
// each group's 64 symbols are staged in LDS and stored by all lanes (128 B per group).
#define DL_RING 256
#define DL_SMEM (2 * DR_NB * 4 + 2 * 512 * 4 + 513 * 4 + DL_RING * 4 + 64 * 2)
__device__ bool lane_decode(const DecJob& j, const DecStream& d, const uint32_t* cum_g, uint16_t* out,
                            unsigned char* smem) {
  const int lane = threadIdx.x;
  const uint32_t pb = d.pb, M = 1u << pb, mask = M - 1, range = d.range;
  DrTables tb;
  tb.bk = (uint2*)smem;
  tb.sy = (uint2*)(smem + 2 * DR_NB * 4);
  uint32_t* cum = (uint32_t*)(smem + 2 * DR_NB * 4 + 2 * 512 * 4);
  uint32_t* ring = cum + 513;
  uint16_t* ob = (uint16_t*)(ring + DL_RING);
  __shared__ uint32_t s_bad;
  for (uint32_t i = lane; i <= range; i += 64) cum[i] = cum_g[i];
  const uint32_t nb = (M + 31) >> 5;
  for (uint32_t b = lane; b < nb; b += 64) tb.bk[b] = make_uint2(0, 0);
  if (lane == 0) s_bad = 0;
  __syncthreads();
  {
    // compact index of the present symbols: lane l owns symbols 8l .. 8l+7 (range <= 512)
    uint32_t pres = 0;
#pragma unroll
    for (int e = 0; e < 8; e++) {
      const uint32_t sy = 8 * lane + e;
      if (sy < range && cum[sy + 1] > cum[sy]) pres |= 1u << e;
    }
    const uint32_t cnt = __popc(pres);
    uint32_t incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(incl, o);
      if (lane >= o) incl += t;
    }
    uint32_t k = incl - cnt;
    for (int e = 0; e < 8; e++) {
      if (!((pres >> e) & 1)) continue;
      const uint32_t sy = 8 * lane + e, c0 = cum[sy], c1 = cum[sy + 1];
      tb.sy[k] = make_uint2(c1 - c0, c0 | (sy << 16));
      for (uint32_t b = (c0 + 31) >> 5; b <= (c1 - 1) >> 5; b++) tb.bk[b].y = k;
      if (c0 & 31) atomicOr(&tb.bk[c0 >> 5].x, 1u << (c0 & 31));
      k++;
    }
  }
  // payload word k = bytes P + 4k .. P + 4k + 3 of the file (unaligned), 0 past the file
  const uint64_t P = d.payload_off, szal = j.size & ~3ull;
  const uint32_t al = (uint32_t)(P & 3), nw = d.words;
  auto word = [&](uint32_t k) -> uint32_t {
    if (k >= nw) return 0u;
    const uint64_t a = (P & ~3ull) + (uint64_t)k * 4;
    uint32_t lo = 0, hi = 0;
    for (int e = 0; e < 8; e++) {
      const uint64_t b = a + e;
      if (b < j.size) {
        const uint32_t v = j.in[b];
        if (e < 4) lo |= v << (8 * e); else hi |= v << (8 * (e - 4));
      }
    }
    if (a + 8 <= szal) { lo = *(const uint32_t*)(j.in + a); hi = *(const uint32_t*)(j.in + a + 4); }
    return __builtin_amdgcn_alignbyte(hi, lo, al);
  };
  uint32_t fill = 0;
  for (int r = 0; r < 2; r++) { ring[(fill + lane) & (DL_RING - 1)] = word(fill + lane); fill += 64; }
  __syncthreads();
  uint64_t x = (uint64_t)ring[0] | ((uint64_t)ring[1] << 32);
  uint32_t wi = 2;
  uint32_t pend = 0;
  bool hp = false;
  for (uint32_t g0 = 0; g0 < d.n; g0 += 64) {
    if (hp) { ring[(fill + lane) & (DL_RING - 1)] = pend; fill += 64; hp = false; }
    wi = __shfl(wi, 0);
    if (fill - wi < 128) { pend = word(fill + lane); hp = true; }   // lands next group
    __syncthreads();
    if (lane == 0) {
      const uint32_t g1 = min(d.n, g0 + 64);
      for (uint32_t i = g0; i < g1; i++) {
        const uint32_t nxt = ring[wi & (DL_RING - 1)];
        const uint32_t slot = (uint32_t)x & mask;
        uint32_t sym, c, f;
        tb.lookup(slot, sym, c, f);
        ob[i - g0] = (uint16_t)sym;
        x = (uint64_t)f * (x >> pb) + (slot - c);             // Rans64DecAdvance
        if (x < (1ull << 31)) { x = (x << 32) | nxt; wi++; }
      }
      if (wi > nw) s_bad = 1;
    }
    __syncthreads();
    if (g0 + lane < d.n) out[d.blk ? blk_pos(g0 + lane) : g0 + lane] = ob[lane];
  }
  __syncthreads();
  return lane != 0 || (!s_bad && x == (1ull << 31));
}

// streams k_drans_multi decodes (a chain lane each)
__device__ __forceinline__ bool multi_ok(const DecStream& d) {
  return d.mode == SM_RANS && d.range <= 512 && d.pb <= 15 && d.pb >= 7;
}

// Without an index: one wave per stream (lane_decode); streams outside its table format
// (range > 512 or prob_bits > 15, never in a -s0 file) fall back to one lane with global tables.
// With skip_multi the streams k_drans_multi takes are left to it.
__global__ __launch_bounds__(64) void k_drans_wave(DecJob j, int nstreams, int skip_multi) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dl_lds[];
  if (dec_abort(j)) return;
  const int sid = blockIdx.x;
  const DecStream d = j.streams[sid];
  if (d.mode != SM_RANS || (skip_multi && multi_ok(d))) return;
  uint16_t* out = j.dsym + d.out_off;
  if (d.range <= 512 && d.pb <= 15) {
    if (!lane_decode(j, d, j.cum + (size_t)sid * j.cum_stride, out, dl_lds)) atomicOr(j.gerr, 4u);
    return;
  }
  if (threadIdx.x) return;
  const uint64_t wend = d.payload_off + (uint64_t)d.words * 4;
  uint64_t x = (uint64_t)ld_u32_unaligned(j.in, d.payload_off) | ((uint64_t)ld_u32_unaligned(j.in, d.payload_off + 4) << 32);
  uint64_t xe;
  if (!dec_run<false>(j, d, j.cum + (size_t)sid * j.cum_stride, j.bsym + (size_t)sid * 512, d.pb > 9 ? d.pb - 9 : 0,
                      nullptr, x, d.payload_off + 8, wend, 0, d.n, OutCursor(out, 0, 0), &xe) || xe != (1ull << 31))
    atomicOr(j.gerr, 4u);
}

// ---------------------------------------------------------------- no index: many streams per wave
// A foreign .hoh (no side index) leaves one serial chain per stream (rans64.hpp:107-142,
// entropy_decoding.hpp:268-276).  k_drans_wave gives each stream a wave of its own and walks it on
// lane 0 (3,072 waves for an 8192^2 image, ~700 cycles per symbol with three of them per SIMD);
// k_drans_multi gives each chain a LANE: one wave decodes MS streams side by side, every chain
// lane with its own lookup tables in LDS (DrTables, 12 KB) and a 16-word payload ring refilled a
// 16-symbol group ahead exactly as k_drans's segment lanes do, so a step is dstep's ~17 VALU and
// two dependent LDS reads, and 64 decoded symbols leave the lane as one 128-B line (flat) or
// eight 16-B blocks (blocked layout).  Streams k_drans_multi takes: rANS, range <= 512,
// 7 <= prob_bits <= 15 (every plane and LZ stream choh writes); k_dmlist lists them.
// LDS map (byte addresses; no static LDS, so the dynamic area starts at 0): payload rings
// [0, 4 KB) (slot s of lane l at s * 256 + 4 l), the abort / count words at 4 KB, bucket table of
// chain m at 8 KB (m + 1) (8 KB aligned: its address is an OR), symbol table of chain m at
// 8 KB (MS + 1) + 4 KB m.
__host__ __device__ constexpr uint32_t dm_bk(int m) { return 8192u * (uint32_t)(m + 1); }
__host__ __device__ constexpr uint32_t dm_sy(int ms, int m) { return 8192u * (uint32_t)(ms + 1) + 4096u * (uint32_t)m; }
__host__ __device__ constexpr uint32_t dm_smem(int ms) { return dm_sy(ms, ms); }
#define DM_SCR 4096u
#define DM_MS 12

// the streams k_drans_multi decodes; the others stay with k_drans_wave.  Long streams
// (>= DM_LONG symbols: whole tile planes) are listed from the front (count in gerr[5]), short ones
// (LZ streams, compacted planes) from the back (count in gerr[6]), so the first rounds of
// k_drans_multi hold streams of similar length.
#define DM_LONG 16384
__global__ __launch_bounds__(256) void k_dmlist(DecJob j, int nstreams, uint32_t* list) {
  if (dec_abort(j)) return;
  const int s = blockIdx.x * blockDim.x + threadIdx.x, lane = threadIdx.x & 63;
  bool ok = false, lng = false;
  if (s < nstreams) {
    const DecStream d = j.streams[s];
    ok = multi_ok(d);
    lng = ok && d.n >= DM_LONG;
  }
  const uint64_t bl = __ballot(lng), bs = __ballot(ok && !lng), below = (1ull << lane) - 1;
  uint32_t base_l = 0, base_s = 0;
  if (lane == 0 && bl) base_l = atomicAdd(j.gerr + 5, (uint32_t)__popcll(bl));
  if (lane == 0 && bs) base_s = atomicAdd(j.gerr + 6, (uint32_t)__popcll(bs));
  base_l = __shfl(base_l, 0);
  base_s = __shfl(base_s, 0);
  if (lng) list[base_l + __popcll(bl & below)] = (uint32_t)s;
  else if (ok) list[nstreams - 1 - (base_s + __popcll(bs & below))] = (uint32_t)s;
}

// one decode step on chain lane tables at (bk, sy): dstep with the tables' bases ORed in
__device__ __forceinline__ uint32_t dstep_m(uint32_t bk, uint32_t sy, uint32_t bmask, uint32_t mask, uint32_t pb,
                                            uint32_t& xh, uint32_t& xl, uint32_t nw, uint32_t& wi) {
  const uint32_t slot = xl & mask;
  const uint2 e = lds_u2(((xl >> 2) & bmask) | bk);
  const uint32_t k = __popc(__builtin_amdgcn_ubfe(e.x, 1, slot)) + e.y;
  const uint2 t = lds_u2((k << 3) | sy);
  const uint32_t d = slot - (t.y & 0xffffu);
  const uint32_t yl = __builtin_amdgcn_alignbit(xh, xl, pb);
  const uint64_t acc = ((uint64_t)__umul24(t.x, xh >> pb) << 32) | d;
  uint64_t x, co;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(x), "=s"(co) : "v"(t.x), "v"(yl), "v"(acc));
  const uint32_t nh = (uint32_t)(x >> 32), nl = (uint32_t)x;
  const bool r = x < (1ull << 31);
  xh = r ? nl : nh;
  xl = r ? nw : nl;
  wi += r;
  return t.y;
}

// One chain lane: the whole stream d with its tables at LDS bytes (bkb, syb) and its payload
// ring in slots t4 + 256 s.  Payload words are fetched as raw dwords one 16-symbol group ahead and
// aligned when they land in the ring (aligning at the fetch made every fetch wait for its load).
template <class Step, class Look>
__device__ __forceinline__ bool dm_chain_t(const DecJob& j, const DecStream& d, Step step, Look look) {
  const uint32_t t4 = (uint32_t)threadIdx.x * 4;
  uint16_t* out = j.dsym + d.out_off;
  const uint32_t pb = d.pb, mask = (1u << pb) - 1;
  const uint64_t P = d.payload_off;
  const uint32_t al = (uint32_t)(P & 3);
  const uint64_t szal = j.size & ~3ull;
  uint32_t tailw = 0;
  for (uint64_t q = szal; q < j.size; q++) tailw |= (uint32_t)j.in[q] << (8 * (q & 3));
  auto fetch5 = [&](uint32_t kw, uint32_t* A) {              // raw dwords covering words kw .. kw+3
    const uint64_t a = (P & ~3ull) + (uint64_t)kw * 4;
    if (a + 20 <= szal) {
      typedef uint32_t u4a __attribute__((ext_vector_type(4), aligned(4)));
      const u4a v = *(const u4a*)(j.in + a);
      A[0] = v.x; A[1] = v.y; A[2] = v.z; A[3] = v.w;
      A[4] = *(const uint32_t*)(j.in + a + 16);
    } else {
#pragma unroll
      for (int e = 0; e < 5; e++) {
        const uint64_t b = a + 4 * e;
        A[e] = b + 4 <= szal ? *(const uint32_t*)(j.in + b) : (b == szal ? tailw : 0u);
      }
    }
  };
  auto put4 = [&](uint32_t kw, const uint32_t* A) {
#pragma unroll
    for (int e = 0; e < 4; e++)
      lds_st32(t4 | (((kw + e) & (DR_RW - 1)) << 8), __builtin_amdgcn_alignbyte(A[e + 1], A[e], al));
  };
  uint32_t wi = 2, xh, xl;
  {
    uint32_t A[5];
    fetch5(0, A);
    xl = __builtin_amdgcn_alignbyte(A[1], A[0], al);
    xh = __builtin_amdgcn_alignbyte(A[2], A[1], al);         // Rans64DecInit
  }
  const uint32_t ngrp = pb >= 7 ? d.n >> 6 : 0;
  if (ngrp) {
    uint32_t fill = wi, pend[5];
    bool hp = true;                                          // pend holds words fill .. fill+3
    {
      uint32_t a0[5], a1[5];
      fetch5(fill, a0); fetch5(fill + 4, a1);
      put4(fill, a0); put4(fill + 4, a1);
      fill += 8;
      fetch5(fill, pend);
    }
    for (uint32_t g = 0; g < ngrp; g++) {
      uint32_t pk[32];                                       // 64 symbols: one 128-B line
#pragma unroll
      for (int gi = 0; gi < 4; gi++) {
        if (hp) { put4(fill, pend); fill += 4; }
        while (fill - wi < 8) {
          uint32_t t[5];
          fetch5(fill, t); put4(fill, t); fill += 4;
        }
        hp = fill + 4 - wi <= DR_RW;
        if (hp) fetch5(fill, pend);
#pragma unroll
        for (int u = 0; u < 16; u += 2) {
          const uint32_t w0 = lds_u32(t4 | ((wi & (DR_RW - 1)) << 8));
          const uint32_t a = step(xh, xl, w0, wi);
          const uint32_t w1 = lds_u32(t4 | ((wi & (DR_RW - 1)) << 8));
          const uint32_t b = step(xh, xl, w1, wi);
          pk[gi * 8 + u / 2] = __builtin_amdgcn_perm(b, a, 0x07060302u);
        }
      }
      uint4* o4;
      uint32_t ostride;
      if (d.blk) {                                           // row r = g / 4, columns 64 (g % 4) ..
        const uint32_t r = g >> 2, rr = r & 63;
        o4 = (uint4*)(out + (r >> 6) * BLK_BAND) + rr + ((rr + 7) >> 3) * 64 + (g & 3) * 8 * 64;
        ostride = 64;
      } else {
        o4 = (uint4*)(out + (size_t)g * 64);
        ostride = 1;
      }
#pragma unroll
      for (int e = 0; e < 8; e++) o4[e * ostride] = make_uint4(pk[4 * e], pk[4 * e + 1], pk[4 * e + 2], pk[4 * e + 3]);
    }
  }
  // the last n % 64 symbols (or a whole stream with prob_bits < 7): one step at a time, payload
  // words from the file
  uint64_t x = ((uint64_t)xh << 32) | xl;
  OutCursor oc(out, d.blk, 0);
  for (uint32_t i = ngrp * 64; i < d.n; i++) {
    const uint32_t slot = (uint32_t)x & mask;
    uint32_t sym, c, f;
    look(slot, sym, c, f);
    oc.put(i, (uint16_t)sym);
    x = (uint64_t)f * (x >> pb) + (slot - c);                // Rans64DecAdvance
    if (x < (1ull << 31)) {
      if (wi >= d.words) return false;
      x = (x << 32) | ld_u32_unaligned(j.in, P + (uint64_t)wi * 4);
      wi++;
    }
  }
  return x == (1ull << 31) && wi <= d.words;
}

__device__ __forceinline__ bool dm_chain(const DecJob& j, const DecStream& d, uint32_t* dm_lds, uint32_t bkb,
                                         uint32_t syb) {
  const uint32_t pb = d.pb, mask = (1u << pb) - 1, bmask = (mask >> 2) & ~7u;
  DrTables tb;
  tb.bk = (uint2*)((unsigned char*)dm_lds + bkb);
  tb.sy = (uint2*)((unsigned char*)dm_lds + syb);
  return dm_chain_t(
      j, d,
      [&](uint32_t& xh, uint32_t& xl, uint32_t nw, uint32_t& wi) {
        return dstep_m(bkb, syb, bmask, mask, pb, xh, xl, nw, wi);
      },
      [&](uint32_t slot, uint32_t& sym, uint32_t& c, uint32_t& f) { tb.lookup(slot, sym, c, f); });
}

template <int MS>
__global__ __launch_bounds__(64) void k_drans_multi(DecJob j, const uint32_t* list, int nlist) {
  extern __shared__ __attribute__((aligned(16))) uint32_t dm_lds[];
  const int lane = threadIdx.x;
  uint32_t* scr = dm_lds + DM_SCR / 4;
  if (lane == 0) {
    scr[0] = *(volatile const uint32_t*)j.gerr;
    scr[1] = *(volatile const uint32_t*)(j.gerr + 5);
    scr[2] = *(volatile const uint32_t*)(j.gerr + 6);
  }
  __syncthreads();
  if (scr[0]) return;
  const uint32_t cl = scr[1], total = scr[1] + scr[2];
  // logical entry i: long streams from the front of the list, short ones from its back
  auto entry = [&](uint32_t i) -> uint32_t { return i < cl ? list[i] : list[nlist - 1 - (i - cl)]; };
  for (uint32_t base = blockIdx.x * MS; base < total; base += gridDim.x * MS) {
    const int ns = (int)min((uint32_t)MS, total - base);
    // lookup tables of every chain (the lane_decode construction, the whole wave per stream)
    for (int m = 0; m < ns; m++) {
      const DecStream d = j.streams[entry(base + m)];
      const uint32_t nb = ((1u << d.pb) + 31) >> 5;
      uint2* bk = (uint2*)((unsigned char*)dm_lds + dm_bk(m));
      for (uint32_t b = lane; b < nb; b += 64) bk[b] = make_uint2(0, 0);
    }
    __syncthreads();
    for (int m = 0; m < ns; m++) {
      const uint32_t sid = entry(base + m);
      const DecStream d = j.streams[sid];
      const uint32_t* cum = j.cum + (size_t)sid * j.cum_stride;
      uint2* bk = (uint2*)((unsigned char*)dm_lds + dm_bk(m));
      uint2* sy = (uint2*)((unsigned char*)dm_lds + dm_sy(MS, m));
      uint32_t pres = 0, cv[9];
#pragma unroll
      for (int e = 0; e < 9; e++) cv[e] = 8 * lane + e <= d.range ? cum[8 * lane + e] : 0;
#pragma unroll
      for (int e = 0; e < 8; e++)
        if (8 * lane + e < d.range && cv[e + 1] > cv[e]) pres |= 1u << e;
      const uint32_t c = __popc(pres);
      uint32_t incl = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(incl, o);
        if (lane >= o) incl += t;
      }
      uint32_t k = incl - c;
      for (int e = 0; e < 8; e++) {
        if (!((pres >> e) & 1)) continue;
        const uint32_t sv = 8 * lane + e, c0 = cv[e], c1 = cv[e + 1];
        sy[k] = make_uint2(c1 - c0, c0 | (sv << 16));
        for (uint32_t b = (c0 + 31) >> 5; b <= (c1 - 1) >> 5; b++) bk[b].y = k;
        if (c0 & 31) atomicOr(&bk[c0 >> 5].x, 1u << (c0 & 31));
        k++;
      }
    }
    __syncthreads();
    if (lane < ns && !dm_chain(j, j.streams[entry(base + lane)], dm_lds, dm_bk(lane), dm_sy(MS, lane)))
      atomicOr(j.gerr, 4u);
    __syncthreads();                                         // the tables are rebuilt next round
  }
}

// ---------------------------------------------------------------- no index: compact chain tables
// k_drans_lanes: a lane per chain like k_drans_multi, but with tables small enough that one
// workgroup holds up to 64 chains (k_drans_multi's 12 KB per chain made a workgroup a whole CU's
// LDS for 12 chains, 12 of 64 lanes busy, and one image's chains held every CU for 7 ms).
// Per chain (P = symbols present, in cum order):
//   B[b], b < 2^pb / 64: u16 index k0 of the symbol covering slot 64 b      (1 KB at prob_bits 15)
//   E[k], k < P + 3:     {c | symbol << 16, f}, then three sentinels c = 0xffff
// slot -> symbol: k0 = B[slot >> 6]; E[k0 .. k0 + 3] arrive in two ds_read2_b64; the covering
// entry is the last of them whose start c <= slot -- exact while at most three symbols start in
// (64 b, slot], i.e. everywhere but the rare-symbol tails, where the lane walks on entry by entry
// (the sentinels end every walk).  Synthetic tiles (P ~ 30-55): ~1.5 KB per chain; the worst case
// (P = 512) 5.1 KB.  (32-slot buckets walk less often but hold fewer chains per workgroup:
// measured slower in the pipeline, no faster alone.)
// Rounds are packed by table size before the launch (k_dlpack, one wave, greedy over the list in
// order: a round is the next entries -- at most 64 -- whose tables fit the LDS budget), and
// workgroup w takes rounds w, w + grid, ...: a round holds as many chains as fit and the grid keeps
// several images' chains resident at once.  (A first version claimed rounds from a device head by
// CAS at run time: hundreds of workgroups serialised on that one word before their first round.)
#define DL_BSH 6
#define DL_SCR 4096u             // abort word + list counts (payload rings below, [0, 4 KB))
#define DL_TAB 4160u             // first table byte
#define DL_NR 10                 // gerr word: rounds packed by k_dlpack

__host__ __device__ __forceinline__ uint32_t dl_nb(uint32_t pb) { return pb > DL_BSH ? 1u << (pb - DL_BSH) : 1u; }
__host__ __device__ __forceinline__ uint32_t dl_bytes(uint32_t pb, uint32_t npres) {
  return ((dl_nb(pb) * 2 + 7) & ~7u) + 8 * (npres + 3);
}

// every multi_ok stream's compact table size; one wave per stream
__global__ __launch_bounds__(64) void k_dlsize(DecJob j, uint32_t* tbytes) {
  if (dec_abort(j)) return;
  const int sid = blockIdx.x, lane = threadIdx.x;
  const DecStream d = j.streams[sid];
  if (!multi_ok(d)) return;
  const uint32_t* cum = j.cum + (size_t)sid * j.cum_stride;
  uint32_t cv[9], cnt = 0;
#pragma unroll
  for (int e = 0; e < 9; e++) cv[e] = 8 * lane + e <= d.range ? cum[8 * lane + e] : 0;
#pragma unroll
  for (int e = 0; e < 8; e++) cnt += (8 * lane + e < d.range && cv[e + 1] > cv[e]) ? 1u : 0u;
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if (lane == 0) tbytes[sid] = dl_bytes(d.pb, cnt);
}

// Greedy round packing over the multi list in k_drans_lanes' order (long streams from the front,
// short ones from the back): rounds[r] = first entry of round r, rounds[nr] = total, nr in
// gerr[DL_NR].  One wave; the sizes are staged in LDS 8192 at a time, 64 entries per step.
#define DLP_CH 8192
__global__ __launch_bounds__(64) void k_dlpack(DecJob j, const uint32_t* list, int nlist, const uint32_t* tbytes,
                                               uint32_t budget, uint32_t* rounds) {
  __shared__ uint32_t sz[DLP_CH];
  if (dec_abort(j)) return;
  const int lane = threadIdx.x;
  const uint32_t cl = *(volatile const uint32_t*)(j.gerr + 5), total = cl + *(volatile const uint32_t*)(j.gerr + 6);
  auto entry = [&](uint32_t i) -> uint32_t { return i < cl ? list[i] : list[nlist - 1 - (i - cl)]; };
  uint32_t nr = 0, p = 0;
  for (uint32_t c0 = 0; c0 < total; c0 += DLP_CH) {
    const uint32_t c1 = min(total, c0 + DLP_CH);
    for (uint32_t i = c0 + lane; i < c1; i += 64) sz[i - c0] = min(tbytes[entry(i)], budget + 1);
    __syncthreads();
    // rounds that start inside this chunk (a round may run past its end: sizes there are re-read)
    while (p < c1) {
      const uint32_t i = p + (uint32_t)lane;
      const uint32_t v = i < total ? (i < c1 ? sz[i - c0] : min(tbytes[entry(i)], budget + 1)) : budget + 1;
      uint32_t incl = v;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(incl, o);
        if (lane >= o) incl += u;
      }
      uint32_t n = (uint32_t)__popcll(__ballot(i < total && incl <= budget));
      if (n == 0) {                                          // cannot happen: budget >= dl_bytes(15, 512)
        if (lane == 0) atomicOr(j.gerr, 4u);
        return;
      }
      if (lane == 0) rounds[nr] = p;
      nr++;
      p += n;
    }
    __syncthreads();
  }
  if (lane == 0) {
    rounds[nr] = total;
    j.gerr[DL_NR] = nr;
  }
}

// one decode step on a compact table (B at byte Bb, E at byte Eb); returns the entry's low word
// (symbol in the high half)
__device__ __forceinline__ uint32_t dstep_l(uint32_t Bb, uint32_t Eb, uint32_t mask, uint32_t pb, uint32_t& xh,
                                           uint32_t& xl, uint32_t nw, uint32_t& wi) {
  const uint32_t slot = xl & mask;
  const uint32_t k0 = lds_u16(Bb + (__builtin_amdgcn_ubfe(xl, DL_BSH, pb - DL_BSH) << 1));
  const uint32_t ea = Eb + (k0 << 3);
  const uint2 e0 = lds_u2(ea), e1 = lds_u2(ea + 8), e2 = lds_u2(ea + 16), e3 = lds_u2(ea + 24);
  // the three compares are independent; the starts ascend, so the last one <= slot wins
  const bool s1 = (e1.x & 0xffffu) <= slot, s2 = (e2.x & 0xffffu) <= slot, s3 = (e3.x & 0xffffu) <= slot;
  uint2 t = s1 ? e1 : e0;
  t = s2 ? e2 : t;
  t = s3 ? e3 : t;
  if (s3) {                                                  // four or more starts: walk on (rare)
    for (uint32_t a = ea + 32;; a += 8) {
      const uint2 u = lds_u2(a);
      if ((u.x & 0xffffu) > slot) break;
      t = u;
    }
  }
  const uint32_t d = slot - (t.x & 0xffffu);
  const uint32_t yl = __builtin_amdgcn_alignbit(xh, xl, pb);
  const uint64_t acc = ((uint64_t)__umul24(t.y, xh >> pb) << 32) | d;
  uint64_t x, co;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(x), "=s"(co) : "v"(t.y), "v"(yl), "v"(acc));
  const uint32_t nh = (uint32_t)(x >> 32), nl = (uint32_t)x;
  const bool r = x < (1ull << 31);
  xh = r ? nl : nh;
  xl = r ? nw : nl;
  wi += r;
  return t.x;
}

__global__ __launch_bounds__(64) void k_drans_lanes(DecJob j, const uint32_t* list, int nlist, const uint32_t* tbytes,
                                                    uint32_t budget, const uint32_t* rounds) {
  extern __shared__ __attribute__((aligned(16))) uint32_t dm_lds[];
  const int lane = threadIdx.x;
  uint32_t* scr = dm_lds + DL_SCR / 4;
  if (lane == 0) {
    scr[0] = *(volatile const uint32_t*)j.gerr;
    scr[1] = *(volatile const uint32_t*)(j.gerr + 5);
    scr[2] = *(volatile const uint32_t*)(j.gerr + DL_NR);
  }
  __syncthreads();
  if (scr[0]) return;
  const uint32_t cl = scr[1], nr = scr[2];
  auto entry = [&](uint32_t i) -> uint32_t { return i < cl ? list[i] : list[nlist - 1 - (i - cl)]; };
  for (uint32_t r = blockIdx.x; r < nr; r += gridDim.x) {
    const uint32_t p = rounds[r], n = rounds[r + 1] - p;
    // this lane's table: the exclusive prefix of the round's sizes (lane m <-> chain m)
    const uint32_t sz = (uint32_t)lane < n ? tbytes[entry(p + lane)] : 0u;
    uint32_t incl = sz;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(incl, o);
      if (lane >= o) incl += u;
    }
    const uint32_t tb = DL_TAB + incl - sz;
    // tables of every chain of the round, the whole wave per stream
    for (uint32_t m = 0; m < n; m++) {
      const uint32_t sid = entry(p + m);
      const DecStream d = j.streams[sid];
      const uint32_t* cum = j.cum + (size_t)sid * j.cum_stride;
      const uint32_t Bb = __shfl(tb, (int)m), Eb = Bb + ((dl_nb(d.pb) * 2 + 7) & ~7u);
      uint32_t pres = 0, cv[9];
#pragma unroll
      for (int e = 0; e < 9; e++) cv[e] = 8 * lane + e <= d.range ? cum[8 * lane + e] : 0;
#pragma unroll
      for (int e = 0; e < 8; e++)
        if (8 * lane + e < d.range && cv[e + 1] > cv[e]) pres |= 1u << e;
      const uint32_t c = __popc(pres);
      uint32_t incl = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(incl, o);
        if (lane >= o) incl += t;
      }
      const uint32_t P = __shfl(incl, 63);
      uint32_t k = incl - c;
      for (int e = 0; e < 8; e++) {
        if (!((pres >> e) & 1)) continue;
        const uint32_t sv = 8 * lane + e, c0 = cv[e], c1 = cv[e + 1];
        lds_st2(Eb + 8 * k, make_uint2(c0 | (sv << 16), c1 - c0));
        for (uint32_t b = (c0 + (1u << DL_BSH) - 1) >> DL_BSH; b <= (c1 - 1) >> DL_BSH; b++) lds_st16(Bb + 2 * b, k);
        k++;
      }
      if (lane < 3) lds_st2(Eb + 8 * (P + lane), make_uint2(0xffffu, 0u));
    }
    __syncthreads();
    if ((uint32_t)lane < n) {
      const DecStream d = j.streams[entry(p + lane)];
      const uint32_t pb = d.pb, mask = (1u << pb) - 1, Bb = tb, Eb = tb + ((dl_nb(pb) * 2 + 7) & ~7u);
      const bool ok = dm_chain_t(
          j, d,
          [&](uint32_t& xh, uint32_t& xl, uint32_t nw, uint32_t& wi) { return dstep_l(Bb, Eb, mask, pb, xh, xl, nw, wi); },
          [&](uint32_t slot, uint32_t& sym, uint32_t& c, uint32_t& f) {
            uint32_t a = Eb + (lds_u16(Bb + ((slot >> DL_BSH) << 1)) << 3);
            uint2 t = lds_u2(a);
            for (;;) {
              const uint2 u = lds_u2(a + 8);
              if ((u.x & 0xffffu) > slot) break;
              t = u;
              a += 8;
            }
            sym = t.x >> 16;
            c = t.x & 0xffffu;
            f = t.y;
          });
      if (!ok) atomicOr(j.gerr, 4u);
    }
    __syncthreads();                                         // the tables are rebuilt next round
  }
}

// stored streams: MSB-first fixed-width fields (the no-index path; with an index k_drans's
// workgroup of the stream does this itself)
__global__ void k_dstored(DecJob j, int nstreams) {
  if (dec_abort(j)) return;
  const int sid = blockIdx.x;
  const DecStream d = j.streams[sid];
  if (d.mode != SM_STORED) return;
  dec_stored(j, sid, d);
}

// a tile with this many copies reading the row above is decoded as chains (the chain role of k_dunpred_lz)
#define LZ_XROW 16
// LZ streams -> matches (un_lz.hpp:150-170); one wave per tile, 64 future entries per step.
// Serially idx += fut[i], and a non-255 entry is a match (its length and back distance are the
// g-th entries of the other two streams, g = matches before it) that advances idx by L too: the
// positions are an inclusive prefix sum of v + L (uint32, wrapping like the serial walk), g a
// ballot count, `nuked` an exclusive prefix sum of L. Any bad match fails the tile (the serial
// walk stopped at the first one; the tile's error is the same).
__device__ __forceinline__ uint32_t wave_incl_u32(uint32_t x, uint32_t lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if (lane >= (uint32_t)o) x += y;
  }
  return x;
}

__global__ __launch_bounds__(64) void k_dlz(DecJob j) {
  if (dec_abort(j)) return;
  const int t = blockIdx.x;
  const uint32_t lane = threadIdx.x;
  DecTile ti = j.tiles[t];
  if (ti.err) return;
  const DecStream* st = j.streams + (size_t)t * SK_PER_TILE;
  const uint16_t* fut = j.dsym + st[0].out_off;
  const uint16_t* len = j.dsym + st[1].out_off;
  const uint16_t* bb = j.dsym + st[2].out_off;
  uint32_t* mt = j.matches + (size_t)t * 4 * (j.lz_cap + 1);
  const uint32_t npix = (uint32_t)ti.w * ti.h, w = (uint32_t)ti.w;
  const uint32_t nf = st[0].n, gcap = min(min(st[1].n, st[2].n), j.lz_cap);
  const uint64_t lt = (1ull << lane) - 1;
  uint32_t idx0 = 0, g0 = 0, nuked0 = 0, xrow = 0;
  bool bad = false;
  for (uint32_t i0 = 0; i0 < nf; i0 += 64) {
    const uint32_t i = i0 + lane;
    const uint32_t v = i < nf ? fut[i] : 0u;
    const bool m = i < nf && v != 255;
    const uint64_t mb = __ballot(m);
    const uint32_t g = g0 + (uint32_t)__popcll(mb & lt);
    uint32_t L = 0, back = 0;
    if (m) {
      if (g >= gcap) bad = true;
      else { L = (uint32_t)len[g] + 4; back = bb[g]; }
    }
    const uint32_t c = v + L;                                   // 255 entries: v = 255, L = 0
    const uint32_t ic = wave_incl_u32(c, lane), il = wave_incl_u32(L, lane);
    if (m && !bad) {
      const uint32_t idx = idx0 + ic - L;                       // the match's position
      if (back == 0 || back > idx || idx + L > npix) bad = true;
      else {
        *(uint4*)(mt + 4 * g) = make_uint4(idx, L, back, nuked0 + il - L);
        xrow += (idx % w) < back;                               // the copy reads the row above
      }
    }
    idx0 += __shfl(ic, 63);
    nuked0 += __shfl(il, 63);
    g0 += (uint32_t)__popcll(mb);
    if (__any(bad)) break;
  }
  bad = __any(bad) || idx0 > npix;
#pragma unroll
  for (int o = 32; o; o >>= 1) xrow += __shfl_xor(xrow, o);
  if (lane) return;
  ti.nmatch = g0;
  if (bad) { ti.err = 1; atomicOr(j.gerr, 1u); }
  j.tiles[t] = ti;
  // copies that keep reading the row above make the wavefront serial: such tiles (and every LZ
  // tile narrower than 64, whose copies reach two rows up) are chain tiles (the chain role of k_dunpred_lz),
  // listed by width class; the others are k_dunpred_lz's work list
  if (bad) return;
  if (!g0) {                                 // no copies: the planes must be whole (k_dunpred_fast)
    const uint32_t np = (uint32_t)ti.w * ti.h;
    if (st[3].n != np || st[4].n != np || st[5].n != np) { j.tiles[t].err = 1; atomicOr(j.gerr, 1u); }
    return;
  }
  if (xrow >= j.lz_xrow || ti.w < 64) {
    const int cls = ti.w == j.tw ? 1 : 2;
    j.lzt[(size_t)cls * j.ntiles + atomicAdd(j.gerr + 6 + cls, 1u)] = (uint32_t)t;
  } else {
    j.lzt[atomicAdd(j.gerr + 2, 1u)] = (uint32_t)t;
  }
}

__device__ __forceinline__ uint16_t dmed16(uint16_t a, uint16_t b, uint16_t c) {
  if (a > b) return b > c ? b : (c > a ? a : c);
  return b < c ? b : (c > a ? c : a);
}

// fast-path eligibility: no LZ copies and three complete (skewed) planes
__device__ __forceinline__ bool unpred_fast(const DecJob& j, int t, const DecTile& ti) {
  const DecStream* st = j.streams + (size_t)t * SK_PER_TILE + 3;
  const uint32_t np = (uint32_t)ti.w * ti.h;
  return ti.nmatch == 0 && st[0].n == np && st[1].n == np && st[2].n == np;
}

// lane r gets v of lane r-1; lane 0 gets `old` (DPP wave_shr:1, bound_ctrl off)
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v, uint32_t old) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xf, 0xf, false);
}

typedef unsigned short dus2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ dus2 as_d2(uint32_t v) { return __builtin_bit_cast(dus2, v); }
__device__ __forceinline__ uint32_t as_u32d(dus2 v) { return __builtin_bit_cast(uint32_t, v); }

__device__ __forceinline__ uint32_t med3u(uint32_t a, uint32_t b, uint32_t c) {
  return max(min(a, b), min(max(a, b), c));
}
// MED of plane values T, L, TL < 2^15 (prediction.hpp:21-28 computes the gradient T + L - TL in
// uint16 arithmetic): a negative gradient wraps to >= 2^16 - 2^15 in 16 bits and to >= 2^32 - 2^15
// in 32 bits, above max(T, L) either way, so the 32-bit wrap gives the same median without a mask
__device__ __forceinline__ uint32_t medp(uint32_t T, uint32_t L, uint32_t TL) { return med3u(T, L, T + L - TL); }

#define UP_P 8   // steps per residual group (one 16-B residual piece per lane and plane)
// LDS row of the output column ring: two halves of 64 columns x 3 B, each followed by a 4-byte pad
// (a pixel's dword store spills one byte past its slot: into the next column of its own half or
// into the pad, never into the other half, which may still wait for its flush), then a dummy
// slot for stores outside the tile; 99 dwords (odd: rows in different banks)
#define ORING_PITCH 396
#define OR_DUMMY 392
__device__ __forceinline__ uint32_t oring_col(uint32_t c) { return (c & 127u) * 3u + ((c >> 4) & 4u); }
// row above a band (k_dunpred_fast): entry x + LAST_OFF of lastG / lastRB holds column x
#define LAST_OFF 8
#define LAST_PAD 16
#define LAST_N(tw) ((((size_t)(tw)) + LAST_PAD + 7) & ~(size_t)7)   // entries of lastRB (16-B multiple)

typedef uint32_t u4h __attribute__((ext_vector_type(4), aligned(2)));

// 16-bit elements off .. off+7 of the 16 in w[0..7] (off lane-constant, 0..7): a 4-way select
// of the word pairs, then a funnel shift by a half word
__device__ __forceinline__ void win8(const uint32_t* w, uint32_t off, uint32_t* o) {
  const uint32_t q = off >> 1, sh = (off & 1) * 16;
  uint32_t sel[5];
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const uint32_t a0 = (q & 1) ? w[i + 1] : w[i];
    const uint32_t a1 = (q & 1) ? w[i + 3] : w[i + 2];
    sel[i] = (q & 2) ? a1 : a0;
  }
#pragma unroll
  for (int i = 0; i < 4; i++) o[i] = __builtin_amdgcn_alignbit(sel[i + 1], sel[i], sh);
}

// Wavefront MED inverse (prediction.hpp:26-41 inverted on every row, Q9 fixed) of the three
// planes of one tile + inverse subtract-green (channel.hpp:73-79), one wave per tile.
// Lane r owns row 64b + r of band b and decodes x = st - r at step st; T and TL come from lane
// r-1 through DPP (its values at steps st-1 and st-2); lane 0 takes T from the row above the band
// (LDS, read 8 columns at a time one group ahead by every lane at one broadcast address, so no
// step branches on the lane).  Before its first column a lane holds the edge value (128, or
// 256 | 256 << 16 for R'/B'), which makes L and TL right at x = 0 without selects.  The three
// planes are independent chains interleaved in one instruction stream; R' and B' (9-bit planes)
// travel as one packed pair R' | B' << 16 (the MED's uint16 gradient wrap, Q8, is the packed
// 16-bit wrap).  Residuals are read one window of 32 steps ahead: BLK (256-wide tiles, blk_pos)
// five 16-B blocks per plane, each load one contiguous 1 KB for the wave, the lane's 8 residuals
// of a group cut out of two blocks at its constant offset (win8); flat planes (other widths)
// four 16-B pieces per plane straight from the lane's 2-B aligned position (64 rows per load:
// the texture path's line rate made these loads half the kernel's time).  RGB goes to a
// 128-column LDS ring, one byte-aligned dword per pixel (a column outside the tile writes a
// dummy slot); each 64-column chunk leaves as coalesced row segments once all 64 rows have
// passed it.  (Storing each lane's 16-pixel window straight to its row as three 16-B pieces
// needs no ring but scatters every store over 64 rows: 1.5x slower.)  The band's last row goes to
// lastG / lastRB once per group from the lane that owns it.
template <bool BLK>
__device__ __forceinline__ void dunpred_fast_tile(const DecJob& j, const DecTile& ti, const uint16_t* plG,
                                                  unsigned char* lds) {
  uint8_t* ring = lds;                                        // [64][ORING_PITCH]
  uint32_t* lastRB = (uint32_t*)(lds + 64 * ORING_PITCH);     // R' | B' << 16 of the row above the band
  uint16_t* lastG = (uint16_t*)(lastRB + LAST_N(j.tw));
  const int lane = threadIdx.x;
  const int w = ti.w, h = ti.h, nst = w + 63;
  const size_t pitch = (size_t)j.W * 3;
  uint8_t* obase = j.rgb + ((size_t)ti.y0 * j.W + ti.x0) * 3;
  const uint16_t* plR = plG + j.plane_cap;
  const uint16_t* plB = plG + 2 * (size_t)j.plane_cap;
  const uint32_t KG = 128u, KRB = 0x01000100u;
  const bool dw_ok = ((pitch | ((size_t)ti.x0 * 3) | (size_t)j.rgb) & 3) == 0;
  const uint32_t orow = lds_addr(ring) + (uint32_t)lane * ORING_PITCH;   // LDS byte address
  int fr_row[3], fr_lds[3];
  size_t fr_glb[3];
#pragma unroll
  for (int q = 0; q < 3; q++) {
    const int e = lane + 64 * q, rr = e / 48, d = e - 48 * rr;
    fr_row[q] = rr; fr_lds[q] = rr * ORING_PITCH + 4 * d; fr_glb[q] = (size_t)rr * pitch + 4 * d;
  }
  for (int i = lane; i < w + LAST_PAD; i += 64) { lastRB[i] = KRB; lastG[i] = (uint16_t)KG; }   // row -1
  __syncthreads();
  for (int r0 = 0; r0 < h; r0 += 64) {
    const int y = r0 + lane;
    const int last = min(63, h - r0 - 1);
    const bool rowok = y < h;
    long F = (long)min(y, h - 1) * w - lane;                  // flat index of this lane at step 0
    if (F < 0) F = 0;                                          // rows past the tile: any residuals
    // flush chunk k (columns 64k .. 64k+63, all rows of the band) from the ring
    int flushed = 0;
    auto flush = [&](int k) {
      const int c0 = 64 * k, nc = min(64, w - c0), rows = last + 1;
      const uint8_t* src0 = ring + oring_col((uint32_t)c0);
      uint8_t* dst0 = obase + (size_t)r0 * pitch + (size_t)c0 * 3;
      if (dw_ok && nc == 64) {
        // 4 rows (192 dwords) per pass: lane l moves dwords l, l+64, l+128 of the block
        for (int rb = 0; rb < rows; rb += 4) {
#pragma unroll
          for (int q = 0; q < 3; q++)
            if (rb + fr_row[q] < rows)
              *(uint32_t*)(dst0 + (size_t)rb * pitch + fr_glb[q]) = *(const uint32_t*)(src0 + rb * ORING_PITCH + fr_lds[q]);
        }
      } else {
        const int nb = nc * 3;
        for (int e = lane; e < rows * nb; e += 64) {
          const int rr = e / nb, d = e - rr * nb;
          dst0[(size_t)rr * pitch + d] = src0[(size_t)rr * ORING_PITCH + d];
        }
      }
    };
    auto res = [&](const uint16_t* pl, int s0) -> u4h { return *(const u4h*)(pl + F + s0); };
    // the row above for lane 0: columns s0 .. s0+7 (past the row: not needed, not read)
    auto above = [&](int s0, uint4& ag0, uint4& ag1, uint4& arb0, uint4& arb1) {
      if (s0 < w) {
        const uint4* g = (const uint4*)(lastG + s0 + LAST_OFF);
        const uint4* rb = (const uint4*)(lastRB + s0 + LAST_OFF);
        const uint4 gg = g[0];
        ag0 = make_uint4(gg.x & 0xffffu, gg.x >> 16, gg.y & 0xffffu, gg.y >> 16);
        ag1 = make_uint4(gg.z & 0xffffu, gg.z >> 16, gg.w & 0xffffu, gg.w >> 16);
        arb0 = rb[0]; arb1 = rb[1];
      }
    };
    uint32_t cG = KG, cRB = KRB;           // this lane's values at the previous step (L)
    uint32_t pG = KG, pRB = KRB;           // T of the previous step (TL)
    // one group: steps s0 .. s0+7 with residuals (g, r, b); issues the residuals of group s0 + 24
    // into (gn, rn, bn) and the row above of group s0 + 8
    auto group = [&](int s0, const uint32_t (&qG)[4], const uint32_t (&qR)[4], const uint32_t (&qB)[4],
                     const uint4& ag0, const uint4& ag1, const uint4& arb0, const uint4& arb1,
                     uint4& ng0, uint4& ng1, uint4& nrb0, uint4& nrb1) {
      above(s0 + UP_P, ng0, ng1, nrb0, nrb1);
      const uint32_t oGs[8] = {ag0.x, ag0.y, ag0.z, ag0.w, ag1.x, ag1.y, ag1.z, ag1.w};
      const uint32_t oRBs[8] = {arb0.x, arb0.y, arb0.z, arb0.w, arb1.x, arb1.y, arb1.z, arb1.w};
      uint32_t keepG[UP_P], keepRB[UP_P];
#pragma unroll
      for (int u = 0; u < UP_P; u++) {
        const int x = s0 + u - lane;
        // G residual: the high half of the word is cut by the final & 255
        const uint32_t rG = (u & 1) ? qG[u >> 1] >> 16 : qG[u >> 1];
        // R' residual in the low half, B' in the high half: one byte permute
        const uint32_t rRB = __builtin_amdgcn_perm(qB[u >> 1], qR[u >> 1], (u & 1) ? 0x07060302u : 0x05040100u);
        const uint32_t TG = wave_shr1(cG, oGs[u]), TRB = wave_shr1(cRB, oRBs[u]);
        const uint32_t vG = (rG + medp(TG, cG, pG) + 128u) & 255u;
        const dus2 t2 = as_d2(TRB), l2 = as_d2(cRB);
        const dus2 g2 = t2 + l2 - as_d2(pRB);
        const dus2 m2 = __builtin_elementwise_max(__builtin_elementwise_min(t2, l2),
                                                  __builtin_elementwise_min(__builtin_elementwise_max(t2, l2), g2));
        const uint32_t vRB = as_u32d(as_d2(rRB) + m2 + (dus2)(256)) & 0x01ff01ffu;
        const bool pre = x < 0;
        pG = TG; pRB = TRB;
        cG = pre ? KG : vG;
        cRB = pre ? KRB : vRB;
        keepG[u] = cG; keepRB[u] = cRB;
        const uint32_t rb = vRB + vG * 0x10001u;      // R' + G | (B' + G) << 16, no carry across
        // R, G, B, 0 as one dword at the column's slot of the lane's ring row
        const uint32_t px = __builtin_amdgcn_perm(vG, rb, 0x0c020400u);
        const bool ok = rowok && (uint32_t)x < (uint32_t)w;
        uint32_t col = oring_col((uint32_t)x);
        asm volatile("" : "+v"(col));                  // computed by every lane: a select, not a branch
        lds_st32(orow + (ok ? col : (uint32_t)OR_DUMMY), px);
      }
      // the band's last row (its lane's values, edge values before column 0) for the next band
      const int x0 = s0 - lane;
      if (lane == last && x0 > -UP_P && x0 < w) {
#pragma unroll
        for (int u = 0; u < UP_P; u++) { lastG[x0 + u + LAST_OFF] = (uint16_t)keepG[u]; lastRB[x0 + u + LAST_OFF] = keepRB[u]; }
      }
      // columns < s0 + UP_P - 63 are complete in every row: flush whole 64-column chunks before
      // the ring slot is reused (column 64k + 128 arrives at step 64k + 128 at the earliest)
      const int done = s0 + UP_P - 63;
      while (64 * (flushed + 1) <= done && 64 * flushed < w) { flush(flushed); flushed++; }
    };
    // residuals of 32 steps per buffer (64 B of each plane per lane: four 16-B loads issued back
    // to back, so only the first misses the L1), loaded one window ahead; row-above values
    // alternate between two sets
    // Blocked planes: blocks s0/8 .. s0/8 + 4 of the lane's row (one contiguous 1 KB per load),
    // group g's 8 residuals start at element off = -lane & 7 of block s0/8 + g
    struct Win { uint4 g[5], r[5], b[5]; };
    const size_t bandoff = (size_t)(r0 >> 6) * BLK_BAND + (size_t)lane * 8;
    const uint32_t boff = (uint32_t)(-lane) & 7u;
    auto load = [&](Win& W, int s0) {
      if (BLK) {
#pragma unroll
        for (int k = 0; k < 5; k++) {
          const size_t e = bandoff + (size_t)min(s0 / 8 + k, BLK_NK - 1) * 512;
          W.g[k] = *(const uint4*)(plG + e); W.r[k] = *(const uint4*)(plR + e); W.b[k] = *(const uint4*)(plB + e);
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; k++) { const u4h v = res(plG, s0 + k * UP_P); W.g[k] = make_uint4(v.x, v.y, v.z, v.w); }
#pragma unroll
        for (int k = 0; k < 4; k++) { const u4h v = res(plR, s0 + k * UP_P); W.r[k] = make_uint4(v.x, v.y, v.z, v.w); }
#pragma unroll
        for (int k = 0; k < 4; k++) { const u4h v = res(plB, s0 + k * UP_P); W.b[k] = make_uint4(v.x, v.y, v.z, v.w); }
      }
    };
    auto words = [&](const uint4* c, int gi, uint32_t (&q)[4]) {
      if (BLK) {
        const uint32_t w8[8] = {c[gi].x, c[gi].y, c[gi].z, c[gi].w, c[gi + 1].x, c[gi + 1].y, c[gi + 1].z, c[gi + 1].w};
        win8(w8, boff, q);
      } else {
        q[0] = c[gi].x; q[1] = c[gi].y; q[2] = c[gi].z; q[3] = c[gi].w;
      }
    };
    auto window = [&](int s0, const Win& W, uint4* a, uint4* c) {
#pragma unroll
      for (int gi = 0; gi < 4; gi++) {
        uint32_t qG[4], qR[4], qB[4];
        words(W.g, gi, qG); words(W.r, gi, qR); words(W.b, gi, qB);
        if (gi & 1) group(s0 + gi * UP_P, qG, qR, qB, c[0], c[1], c[2], c[3], a[0], a[1], a[2], a[3]);
        else group(s0 + gi * UP_P, qG, qR, qB, a[0], a[1], a[2], a[3], c[0], c[1], c[2], c[3]);
      }
    };
    Win WA, WB;
    uint4 av[4] = {}, cv[4] = {};
    load(WA, 0);
    above(0, av[0], av[1], av[2], av[3]);
    for (int s0 = 0; s0 < nst; s0 += 8 * UP_P) {
      load(WB, s0 + 4 * UP_P);
      window(s0, WA, av, cv);
      if (s0 + 4 * UP_P >= nst) break;
      load(WA, s0 + 8 * UP_P);
      window(s0 + 4 * UP_P, WB, av, cv);
    }
    while (64 * flushed < w) { flush(flushed); flushed++; }
    __syncthreads();
  }
}

__global__ __launch_bounds__(64) DUNF_ATTR void k_dunpred_fast(DecJob j) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  if (dec_abort(j) || (j.exp & 64)) return;   // what-if EXP & 64 (measurement, output invalid)
  const int t = blockIdx.x;
  const DecTile ti = j.tiles[t];
  if (ti.err || !unpred_fast(j, t, ti)) return;
  const DecStream* st = j.streams + (size_t)t * SK_PER_TILE + 3;
  const uint16_t* pl = j.dsym + (size_t)(t * 3) * j.plane_cap;
  if (st[0].blk && st[1].blk && st[2].blk) dunpred_fast_tile<true>(j, ti, pl, lds);
  else dunpred_fast_tile<false>(j, ti, pl, lds);
}

// pixels of [0, i) covered by LZ copies (matches sorted by pixel index)
__device__ __forceinline__ uint32_t nuked_before(const uint32_t* mt, uint32_t nm, uint32_t i) {
  uint32_t lo = 0, hi = nm;                      // first match with idx >= i
  while (lo < hi) { const uint32_t mid = (lo + hi) / 2; if (mt[4 * mid] < i) lo = mid + 1; else hi = mid; }
  if (lo == 0) return 0;
  const uint32_t m = lo - 1;
  return mt[4 * m + 3] + min(mt[4 * m + 1], i - mt[4 * m]);
}

#define PK_HALF (128u | (256u << 8) | (256u << 17))

// packed (G:8 | R':9 | B':9) MED inverse of one pixel
__device__ __forceinline__ uint32_t unpred_px(uint32_t T, uint32_t L, uint32_t TL, uint32_t r) {
  const uint32_t tg = T & 255, lg = L & 255, ag = TL & 255;
  const uint32_t tr = (T >> 8) & 511, lr = (L >> 8) & 511, ar = (TL >> 8) & 511;
  const uint32_t tb = T >> 17, lb = L >> 17, ab = TL >> 17;
  const uint32_t g = ((r & 255) + medp(tg, lg, ag) + 128u) & 255u;
  const uint32_t rr = (((r >> 8) & 511) + medp(tr, lr, ar) + 256u) & 511u;
  const uint32_t bb = ((r >> 17) + medp(tb, lb, ab) + 256u) & 511u;
  return g | (rr << 8) | (bb << 17);
}

// Tiles with LZ copies (lz.hpp at -s0: back distance 1..64 pixels in raster order, so a copy
// at the start of a row can read the end of the row above, which a fixed-skew wavefront has not
// produced yet).  Dynamic wavefront, one wave per tile: lane r owns row r0+r of a band and
// advances its own column counter when (a) the lane above has passed the column (T, TL) and
// (b) a copy's source pixel is done.  Decoded pixels (packed G/R'/B') live in LDS rows
// [row above band | band rows]; the band's residuals (a contiguous range, residuals skip
// copied pixels) are staged in LDS first.  Needs w >= 64 (copies reach at most one row up).
// A small persistent grid walks the list of LZ tiles k_dlz built (a launch over every tile
// would dispatch ~1000 idle workgroups that each need the 66 KB band).
__device__ __forceinline__ void dunpred_lz_tile(const DecJob& j, int t, uint32_t* lz_lds, int BR);

// Launched twice per decode (the LZ tile count is only known on the device): `many` = 0 runs
// when at most LZ_FEW tiles have copies (LZ_FEW workers, 64-row bands: the fewest steps per
// tile), `many` = 1 otherwise (a worker per tile, 32-row bands in 33 KB: four per CU, so the
// tiles of a natural image, many of them nearly serial, run at once).
#define LZ_FEW 256
template <bool FULL, int CH_R>
__device__ void chain_tiles(const DecJob& j, int cls, uint32_t blk);
template <int CH_R>
__device__ void chain_full(const DecJob& j, int cls, uint32_t blk);

// Workgroups [0, wgrid) take the wavefront tiles; the ones after them the chain tiles (ga
// workgroups per width class, class 2 only when the edge column is narrower), so both run in
// the same launch, concurrently, without a second stream.  No static LDS: the chain code
// addresses the dynamic area from 0.
template <int CH_R>
__global__ __launch_bounds__(64) void k_dunpred_lz(DecJob j, int br, int many, int wgrid, int ga, int full1, int full2) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lz_lds[];
  if (*(volatile const uint32_t*)j.gerr) return;                      // one load per wave: uniform
  const uint32_t cnt = *(volatile const uint32_t*)(j.gerr + 2);
  if ((cnt > LZ_FEW) != (many != 0)) return;
  // the chain workgroups come first in the grid: they are the launch's long pole (a serial walk
  // per tile plane), and behind ~1000 wavefront workgroups they waited for free CUs
  const uint32_t nch = gridDim.x - (uint32_t)wgrid;
#ifdef DEC_DBG
  // per workgroup {start, end} (s_memrealtime, 100 MHz) at the tail of the bmap buffer
  uint32_t* dbg = (uint32_t*)(j.bmap + (size_t)j.ntiles * j.th * ((j.tw + 15) & ~15) + 16) + (many ? 8192 : 0);
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
#endif
  if (blockIdx.x < nch) {
    __builtin_amdgcn_s_setprio(3);                                     // issue ahead of the wavefront waves
    const uint32_t ci = blockIdx.x;
    const int cls = ci < (uint32_t)ga ? 1 : 2;
    const uint32_t blk = ci - (cls - 1) * ga;
    if (cls == 1 ? full1 : full2) chain_full<CH_R>(j, cls, blk);
    else chain_tiles<false, CH_R>(j, cls, blk);
#ifdef DEC_DBG
    if (threadIdx.x == 0 && blockIdx.x < 4096) { dbg[2 * blockIdx.x] = (uint32_t)t0; dbg[2 * blockIdx.x + 1] = (uint32_t)__builtin_amdgcn_s_memrealtime(); }
#endif
    return;
  }
  for (uint32_t i = blockIdx.x - nch; i < cnt; i += wgrid) {
    dunpred_lz_tile(j, (int)j.lzt[i], lz_lds, br);
    __syncthreads();
  }
#ifdef DEC_DBG
  if (threadIdx.x == 0 && blockIdx.x < 4096) { dbg[2 * blockIdx.x] = (uint32_t)t0; dbg[2 * blockIdx.x + 1] = (uint32_t)__builtin_amdgcn_s_memrealtime(); }
#endif
}


__device__ __forceinline__ void dunpred_lz_tile(const DecJob& j, int t, uint32_t* lz_lds, int BR) {
  const DecTile ti = j.tiles[t];
  if (ti.err || unpred_fast(j, t, ti) || ti.w < 64) return;
  const int lane = threadIdx.x;
  const int w = ti.w, h = ti.h;
  uint32_t* band = lz_lds;                                   // (BR+1) rows x w
  uint32_t* stage = band + (size_t)(BR + 1) * w;             // BR rows x w packed residuals (lzstage)
  const DecStream* st = j.streams + (size_t)t * SK_PER_TILE + 3;
  const uint32_t* mt = j.matches + (size_t)t * 4 * (j.lz_cap + 1);
  const uint32_t nm = ti.nmatch, npix = (uint32_t)w * h;
  const uint32_t n = st[0].n;
  if (st[1].n != n || st[2].n != n || nuked_before(mt, nm, npix) + n != npix) {
    if (lane == 0) atomicOr(j.gerr, 1u);
    return;
  }
  const uint16_t* resG = j.dsym + (size_t)(t * 3) * j.plane_cap;
  const uint16_t* resR = resG + j.plane_cap;
  const uint16_t* resB = resR + j.plane_cap;
  uint8_t* obase = j.rgb + ((size_t)ti.y0 * j.W + ti.x0) * 3;
  bool bad = false;
  for (int r0 = 0; r0 < h; r0 += BR) {
    const int r1 = min(h, r0 + BR);
    const uint32_t kb0 = (uint32_t)r0 * w - nuked_before(mt, nm, (uint32_t)r0 * w);
    const uint32_t kb1 = (uint32_t)r1 * w - nuked_before(mt, nm, (uint32_t)r1 * w);
    __syncthreads();
    // the band's residuals (one contiguous range of the compacted planes) packed into LDS with
    // coalesced loads: the wavefront then waits on LDS, not on a global load per pixel
    if (j.lzstage)
      for (uint32_t i = (uint32_t)lane; i < kb1 - kb0; i += 64)
        stage[i] = resG[kb0 + i] | ((uint32_t)resR[kb0 + i] << 8) | ((uint32_t)resB[kb0 + i] << 17);
    __syncthreads();
    const int y = r0 + lane;
    const bool act = lane < BR && y < h;
    uint32_t prog = act ? 0u : (uint32_t)w;
    uint32_t nuk = act ? nuked_before(mt, nm, (uint32_t)y * w) : 0u;
    uint32_t m = 0;                                          // first match ending after row start
    if (act) {
      uint32_t lo = 0, hi = nm;
      while (lo < hi) { const uint32_t mid = (lo + hi) / 2; if (mt[4 * mid] + mt[4 * mid + 1] <= (uint32_t)y * w) lo = mid + 1; else hi = mid; }
      m = lo;
    }
    uint32_t midx = 0xffffffffu, mlen = 0, mback = 0;
    if (m < nm) { midx = mt[4 * m]; mlen = mt[4 * m + 1]; mback = mt[4 * m + 2]; }
    // the next match, loaded one match ahead (its latency hides behind the current one)
    uint32_t nidx = 0xffffffffu, nlen = 0, nback = 0;
    if (m + 1 < nm) { nidx = mt[4 * m + 4]; nlen = mt[4 * m + 5]; nback = mt[4 * m + 6]; }
    uint32_t left = PK_HALF;
    const uint32_t rowbase = (uint32_t)y * w;
    // the lane's next residual (index rowbase - nuked-before-row), loaded one use ahead so the
    // dependent loop never waits on memory for it
    auto ldres = [&](uint32_t k) -> uint32_t {
      if (j.lzstage) {
        if (kb1 == kb0) return 0u;
        return stage[min(max(k, kb0), kb1 - 1) - kb0];
      }
      const uint32_t kk = k < kb1 ? k : (kb1 ? kb1 - 1 : 0);
      return resG[kk] | ((uint32_t)resR[kk] << 8) | ((uint32_t)resB[kk] << 17);
    };
    uint32_t kcur = rowbase - nuk;
    uint32_t rcur = act ? ldres(kcur) : 0u;
    uint32_t* myrow = band + (size_t)(lane + 1) * w;
    const uint32_t* uprow = band + (size_t)lane * w;
    while (__any(prog < (uint32_t)w)) {
      const uint32_t above = wave_shr1(prog, (uint32_t)w);
      if (prog < (uint32_t)w) {
        const uint32_t x = prog, i = rowbase + x;
        if (m < nm && midx + mlen <= i) {
          m++;
          if (m < nm && nidx + nlen > i) {               // the usual case: the prefetched match
            midx = nidx; mlen = nlen; mback = nback;
          } else {
            while (m < nm && mt[4 * m] + mt[4 * m + 1] <= i) m++;
            midx = 0xffffffffu;
            if (m < nm) { midx = mt[4 * m]; mlen = mt[4 * m + 1]; mback = mt[4 * m + 2]; }
          }
          nidx = 0xffffffffu;
          if (m + 1 < nm) { nidx = mt[4 * m + 4]; nlen = mt[4 * m + 5]; nback = mt[4 * m + 6]; }
        }
        const bool copy = m < nm && midx <= i;
        bool ready = above > x;
        uint32_t src = 0;
        if (copy) {
          src = i - mback;
          if (src < rowbase) {
            if (src + (uint32_t)w < rowbase) { bad = true; src = rowbase; }   // two rows up: w < 64 only
            else ready = above > src + (uint32_t)w - rowbase;
          }
        }
        if (ready) {
          uint32_t v;
          if (copy) {
            v = src >= rowbase ? myrow[src - rowbase] : uprow[src + w - rowbase];
            nuk++;
          } else {
            const uint32_t T = y == 0 ? PK_HALF : uprow[x];
            const uint32_t TL = (y == 0 || x == 0) ? PK_HALF : uprow[x - 1];
            const uint32_t L = x == 0 ? PK_HALF : left;
            const uint32_t k = i - nuk;
            uint32_t r = 0;
            if (k < kb0 || k >= kb1 || k != kcur) bad = true;
            else r = rcur;
            kcur = k + 1;
            rcur = ldres(kcur);
            v = unpred_px(T, L, TL, r);
          }
          myrow[x] = v;
          left = v;
          prog++;
        }
      }
    }
    __syncthreads();
    // the band's RGB rows leave from LDS as coalesced row segments (lanes = consecutive pixels)
    for (int rr = 0; rr < r1 - r0; rr++) {
      const uint32_t* brow = band + (size_t)(rr + 1) * w;
      uint8_t* orow = obase + (size_t)(r0 + rr) * j.W * 3;
      for (int x = lane; x < w; x += 64) {
        const uint32_t v = brow[x], G = v & 255;
        uint8_t* o = orow + (size_t)x * 3;
        o[0] = (uint8_t)(((v >> 8) & 511) + G); o[1] = (uint8_t)G; o[2] = (uint8_t)((v >> 17) + G);
      }
    }
    const int lastrow = r1 - r0;                            // LDS row of the band's last image row
    for (int x = lane; x < w; x += 64) band[x] = band[(size_t)lastrow * w + x];
    __syncthreads();
  }
  if (bad) atomicOr(j.gerr, 1u);
}


// ---------------------------------------------------------------- LZ tiles as chains
// A copy at a row's start that reads the end of the row above serialises a tile's rows (the
// reference's raster order, un_lz.hpp:150-170 + unprediction.hpp:35-89): a tile with many of
// them has no wavefront parallelism left, only its three planes, whose MED chains (L -> value ->
// L) are independent once the copies are known.  the chain role of k_dunpred_lz gives each (tile, plane) a LANE
// (21 tiles per wave, lanes 3q + p) and walks the tile in raster order, one pixel per step for
// every lane at once: the wave's tiles share a width, so the pixel index, the row loop and the
// ring addresses are wave-uniform and a row starts with L = TL = half without a per-step select.
// Per step and lane: the back distance from the tile's byte map (16 columns per load, one block
// ahead), the copy source and T from a per-lane LDS ring of the last R values (R >= 2w, filled
// with half first: row 0 reads half for T and TL), the residual from a 64-entry per-lane LDS ring
// refilled 16 at a time a block ahead, MED, the select, the ring store and one u16 store of the
// plane value (k_dcompose turns the three planes into RGB).
__device__ __forceinline__ uint32_t bm_pitch(uint32_t w) { return (w + 15) & ~15u; }

// per-pixel back distance of the chain tiles (0: predicted pixel), rows padded to 16 bytes
// A small grid strides over both chain lists (an image without chain tiles dispatches little).
__device__ __forceinline__ void backmap_tile(const DecJob& j, int t);
__global__ __launch_bounds__(256) void k_dbackmap(DecJob j) {
  if (dec_abort(j)) return;
  const uint32_t n1 = *(volatile const uint32_t*)(j.gerr + 7), n2 = *(volatile const uint32_t*)(j.gerr + 8);
  for (uint32_t e = blockIdx.x; e < n1 + n2; e += gridDim.x) {
    backmap_tile(j, (int)(e < n1 ? j.lzt[(size_t)j.ntiles + e] : j.lzt[(size_t)2 * j.ntiles + e - n1]));
    __syncthreads();
  }
}

__device__ __forceinline__ void backmap_tile(const DecJob& j, int t) {
  const DecTile ti = j.tiles[t];
  const uint32_t w = ti.w, pitch = bm_pitch(w), tp = bm_pitch(j.tw);
  uint8_t* bm = j.bmap + (size_t)t * j.th * tp;
  uint4* b4 = (uint4*)bm;
  for (uint32_t q = threadIdx.x; q < (uint32_t)ti.h * pitch / 16; q += 256) b4[q] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  const uint32_t* mt = j.matches + (size_t)t * 4 * (j.lz_cap + 1);
  for (uint32_t m = threadIdx.x; m < ti.nmatch; m += 256) {
    const uint4 v = *(const uint4*)(mt + 4 * m);                        // idx, length, back
    for (uint32_t q = v.x; q < v.x + v.y; q++) bm[(q / w) * pitch + q % w] = (uint8_t)v.z;
  }
}

#ifdef __HIP_DEVICE_COMPILE__
__device__ __forceinline__ uint4 lds_u4(uint32_t a) { return *(const __attribute__((address_space(3))) u4_ma*)(size_t)a; }
__device__ __forceinline__ void lds_st4(uint32_t a, uint4 v) { *(__attribute__((address_space(3))) u4_ma*)(size_t)a = v; }
#else
__device__ uint4 lds_u4(uint32_t);
__device__ void lds_st4(uint32_t, uint4);
#endif

// LDS map (byte addresses; no static LDS): value rings of CH_R u16 at lane * CH_VS, residual
// rings of 64 entries + a mirror of entries 0..15 (a block's 16 entries k.. are always
// contiguous) at CH_RES_OFF + lane * CH_QS, the abort word last.  The lane strides are an odd number of dwords:
// the lanes' rings start on different banks, so the wave's same-offset accesses (T, the ring
// store, every step) are conflict-free (a 2 KB stride put all 63 lanes on one bank).
// CH_T tiles per wave (lanes 3q + p < 3 CH_T): 35 KB of LDS with R = 512, so the launch
// co-resides with the other kernels of images in flight (21 tiles needed 137 KB, a whole CU's).
#define CH_T 10
#define CH_L (3 * CH_T)
#define CH_QS 164
__host__ __device__ constexpr uint32_t ch_vs(int R) { return (uint32_t)R * 2 + 4; }
__host__ __device__ constexpr uint32_t ch_res_off(int R) { return CH_L * ch_vs(R); }
__host__ __device__ constexpr uint32_t ch_scr(int R) { return ch_res_off(R) + CH_L * CH_QS; }
__host__ __device__ constexpr uint32_t ch_smem(int R) { return ch_scr(R) + 16; }

// Chain tiles whose width is a multiple of 16 (every 256-wide tile): k_dexpand has already
// put each pixel's residual + half into the output plane itself (copies: anything), so a step
// takes its residual from the block's 32 bytes in registers (one SDWA add) instead of a
// residual ring indexed by a running symbol count, and the block's values overwrite the
// residuals it consumed.  16-pixel blocks never straddle a row; their ring slots are contiguous
// (constant ds offsets); the next step's LDS reads (T, the copy source) are issued before the
// current step's arithmetic.
template <int CH_R>
__device__ void chain_full(const DecJob& j, int cls, uint32_t blk) {
  const uint32_t lane = threadIdx.x, q = lane / 3, p = lane - 3 * q;
  const uint32_t base = blk * CH_T, cnt = *(volatile const uint32_t*)(j.gerr + 6 + cls);
  if (base >= cnt) return;
  const bool act = lane < CH_L && base + q < cnt;
  const int t = (int)j.lzt[(size_t)cls * j.ntiles + base + (act ? q : 0)];
  const DecTile ti = j.tiles[t];
  const uint32_t w = __builtin_amdgcn_readfirstlane(ti.w);             // one width per wave
  const uint32_t h = act ? (uint32_t)ti.h : 0u;
  uint32_t hmax = h;
#pragma unroll
  for (int o = 32; o; o >>= 1) hmax = max(hmax, (uint32_t)__shfl_xor(hmax, o));
  if (lane >= CH_L) return;                                            // no rings for these lanes
  const uint32_t c = p ? 512u : 256u, half = c >> 1, cm = c - 1;
  uint16_t* outp = j.dplane + (size_t)(t * 3 + p) * j.npix_cap;
  const uint4* e4 = (const uint4*)outp;
  const uint32_t pitch = bm_pitch(w), npix = w * (h ? h : 1u);
  const uint8_t* bm = j.bmap + (size_t)t * j.th * bm_pitch(j.tw);
  const uint32_t rb = lane * ch_vs(CH_R);                              // this lane's value ring
  for (uint32_t e = 0; e < CH_R; e += 2) lds_st32(rb + 2 * e, half | (half << 16));
  uint4 bnext = *(const uint4*)bm;                                     // row 0, columns 0..15
  uint4 en0 = e4[0], en1 = e4[1];                                      // block 0's residuals
  for (uint32_t y = 0; y < hmax; y++) {
    uint32_t L = half, Tp = half;                                      // row start: L = TL = half
    const bool live = y < h;
    for (uint32_t x0 = 0; x0 < w; x0 += 16) {
      const uint32_t i0 = y * w + x0;
      const uint4 bcur = bnext, ec0 = en0, ec1 = en1;
      {
        const uint32_t ny = x0 + 16 < w ? y : y + 1, nx = x0 + 16 < w ? x0 + 16 : 0;
        const bool more = live && ny < h;
        bnext = more ? *(const uint4*)(bm + (size_t)ny * pitch + nx) : make_uint4(0, 0, 0, 0);
        const uint32_t nb = more ? (i0 + 16) / 8 : 0u;                 // (block i0 + 16 < npix)
        en0 = e4[nb]; en1 = e4[nb + 1];
      }
      if (!live) continue;
      const uint32_t bw[4] = {bcur.x, bcur.y, bcur.z, bcur.w};
      const uint32_t rw[8] = {ec0.x, ec0.y, ec0.z, ec0.w, ec1.x, ec1.y, ec1.z, ec1.w};
      const uint32_t pos0 = i0 & (CH_R - 1);
      const uint32_t tA = rb + 2 * ((pos0 - w) & (CH_R - 1));          // T of step u at tA + 2u
      const uint32_t wA = rb + 2 * pos0;                               // this block's slots
      auto block = [&](auto nowrap_c) {
        constexpr bool NOWRAP = decltype(nowrap_c)::value;
        auto srcA = [&](int u, uint32_t b) -> uint32_t {
          // (wA - 2b) + 2u: the constant part goes to the read's offset field (the empty asm keeps
          // the compiler from reassociating it back into a per-step add)
          if (NOWRAP) {
            uint32_t sb = wA - 2 * b;
            asm("" : "+v"(sb));
            return sb + 2 * u;
          }
          return rb + 2 * ((pos0 + (uint32_t)u - b) & (CH_R - 1));
        };
        // step 0 reads its copy source after every earlier write, so even b = 1 comes from the
        // ring (at a row's start that is the end of the row above, not L = half)
        uint32_t b = bw[0] & 255u;
        uint32_t T = lds_u16(tA), vC = lds_u16(srcA(0, b ? b : 1));
#pragma unroll
        for (int u = 0; u < 16; u++) {
          uint32_t bn = 0, Tn = 0, vCn = 0;
          if (u < 15) {
            bn = (bw[(u + 1) >> 2] >> (8 * ((u + 1) & 3))) & 255u;
            Tn = lds_u16(tA + 2 * (u + 1));
            vCn = lds_u16(srcA(u + 1, bn));
          }
          const uint32_t r = (rw[u >> 1] >> (16 * (u & 1))) & 0xffffu;   // residual + half
          uint32_t vm = (r + medp(T, L, Tp)) & cm, vc = (u > 0 && b == 1) ? L : vC;
          // both values, then a select: left to itself the compiler branches around the MED
          asm volatile("" : "+v"(vm), "+v"(vc));
          const uint32_t v = b ? vc : vm;
          lds_st16(wA + 2 * u, v);
          Tp = T;
          L = v;
          b = bn; T = Tn; vC = vCn;
        }
      };
      if (pos0 >= 256) block(std::true_type{});                         // i - b >= 1 for every b <= 255
      else block(std::false_type{});
      // the block's 16 values over its residuals (two 16-byte stores)
      uint32_t d[8];
#pragma unroll
      for (int e = 0; e < 8; e++) d[e] = lds_u32(wA + 4 * e);
      uint4* o4 = (uint4*)(outp + i0);
      o4[0] = make_uint4(d[0], d[1], d[2], d[3]);
      o4[1] = make_uint4(d[4], d[5], d[6], d[7]);
    }
  }
  (void)npix;
}

// k_dexpand: each FULL chain tile's three residual streams spread to their pixels (+ half) in the
// output planes, copies skipped (bmap != 0); the streams' lengths are checked against the count
// of non-copy pixels.  One workgroup per tile, 1024 pixels per pass: four per thread (a row never
// splits a thread's four: w % 16 == 0), wave prefix counts by ballots, the waves' totals in LDS.
__global__ __launch_bounds__(256) void k_dexpand(DecJob j, int full1, int full2) {
  if (dec_abort(j)) return;
  __shared__ uint32_t wtot[4];
  const uint32_t n1 = *(volatile const uint32_t*)(j.gerr + 7), n2 = *(volatile const uint32_t*)(j.gerr + 8);
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (uint32_t e = blockIdx.x; e < n1 + n2; e += gridDim.x) {
    const bool c1 = e < n1;
    if (!(c1 ? full1 : full2)) continue;
    const int t = (int)(c1 ? j.lzt[(size_t)j.ntiles + e] : j.lzt[(size_t)2 * j.ntiles + e - n1]);
    const DecTile ti = j.tiles[t];
    const uint32_t w = ti.w, npix = w * ti.h, pitch = bm_pitch(w);
    const uint8_t* bm = j.bmap + (size_t)t * j.th * bm_pitch(j.tw);
    const uint16_t* r0 = j.dsym + (size_t)(t * 3) * j.plane_cap;
    const uint16_t* r1 = r0 + j.plane_cap;
    const uint16_t* r2 = r1 + j.plane_cap;
    uint16_t* o0 = j.dplane + (size_t)(t * 3) * j.npix_cap;
    uint16_t* o1 = o0 + j.npix_cap;
    uint16_t* o2 = o1 + j.npix_cap;
    // eight pixels per thread and pass (never split by a row: w % 16 == 0); the next pass's map
    // bytes are loaded before this pass's residual gathers
    auto mapw = [&](uint32_t i) -> uint2 {
      if (i >= npix) return make_uint2(0x01010101u, 0x01010101u);      // no pixel: "copies"
      const uint32_t y = i / w, x = i - y * w;
      return *(const uint2*)(bm + (size_t)y * pitch + x);
    };
    uint32_t kb = 0;
    uint2 mnext = mapw(8 * tid);
    for (uint32_t i0 = 0; i0 < npix; i0 += 2048) {
      const uint32_t i = i0 + 8 * tid;
      const uint2 m = mnext;
      mnext = mapw(i + 2048);
      uint32_t f = 0;
#pragma unroll
      for (int u = 0; u < 8; u++) f |= ((((u < 4 ? m.x : m.y) >> (8 * (u & 3))) & 255u) == 0 ? 1u : 0u) << u;
      const uint32_t n = __popc(f);
      // exclusive prefix of n over the wave (four bit planes of n by ballot), then over the waves
      uint32_t ex = 0, wt = 0;
#pragma unroll
      for (int bit = 0; bit < 4; bit++) {
        const uint64_t bl = __ballot((n >> bit) & 1);
        ex += __builtin_amdgcn_mbcnt_hi((uint32_t)(bl >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bl, 0u)) << bit;
        wt += (uint32_t)__popcll(bl) << bit;
      }
      if (lane == 0) wtot[wv] = wt;
      __syncthreads();
      uint32_t k = kb + ex, tot = 0;
#pragma unroll
      for (int v = 0; v < 4; v++) { const uint32_t x = wtot[v]; if ((uint32_t)v < wv) k += x; tot += x; }
      __syncthreads();
      if (i < npix) {
        uint32_t a[4] = {0, 0, 0, 0}, bq[4] = {0, 0, 0, 0}, cq[4] = {0, 0, 0, 0};   // u16 pairs per plane
#pragma unroll
        for (int u = 0; u < 8; u++) {
          uint32_t g = 0, rr = 0, bb = 0;
          if ((f >> u) & 1) { g = r0[k] + 128u; rr = r1[k] + 256u; bb = r2[k] + 256u; k++; }
          a[u >> 1] |= g << (16 * (u & 1));
          bq[u >> 1] |= rr << (16 * (u & 1));
          cq[u >> 1] |= bb << (16 * (u & 1));
        }
        *(uint4*)(o0 + i) = make_uint4(a[0], a[1], a[2], a[3]);
        *(uint4*)(o1 + i) = make_uint4(bq[0], bq[1], bq[2], bq[3]);
        *(uint4*)(o2 + i) = make_uint4(cq[0], cq[1], cq[2], cq[3]);
      }
      kb += tot;
    }
    if (tid < 3 && kb != j.streams[t * SK_PER_TILE + 3 + tid].n) atomicOr(j.gerr, 1u);
  }
}

// FULL: the wave's width is a multiple of 16, so 16-pixel blocks never straddle a row, their
// ring slots are contiguous (constant ds offsets) and every block flushes its 16 values to the
// plane with two 16-byte stores.  Within a block the next step's LDS reads (T, the copy source,
// both candidate residuals) are issued before the current step's arithmetic, so the chain waits
// on its VALU operations, not on LDS round trips.
// Workgroup `blk` of the chain tiles of width class cls (called from k_dunpred_lz, whose launch
// has at least ch_smem(CH_R) bytes of dynamic LDS starting at address 0).
template <bool FULL, int CH_R>
__device__ void chain_tiles(const DecJob& j, int cls, uint32_t blk) {
  const uint32_t lane = threadIdx.x, q = lane / 3, p = lane - 3 * q;
  const uint32_t base = blk * CH_T, cnt = *(volatile const uint32_t*)(j.gerr + 6 + cls);
  if (base >= cnt) return;
  const bool act = lane < CH_L && base + q < cnt;
  const int t = (int)j.lzt[(size_t)cls * j.ntiles + base + (act ? q : 0)];
  const DecTile ti = j.tiles[t];
  const uint32_t w = __builtin_amdgcn_readfirstlane(ti.w);             // one width per wave
  const uint32_t h = act ? (uint32_t)ti.h : 0u;
  uint32_t hmax = h;
#pragma unroll
  for (int o = 32; o; o >>= 1) hmax = max(hmax, (uint32_t)__shfl_xor(hmax, o));
  if (lane >= CH_L) return;                                            // no rings for these lanes
  const uint32_t c = p ? 512u : 256u, half = c >> 1, cm = c - 1;
  const DecStream st = j.streams[t * SK_PER_TILE + 3 + p];
  const uint16_t* res = j.dsym + (size_t)(t * 3 + p) * j.plane_cap;
  uint16_t* outp = j.dplane + (size_t)(t * 3 + p) * j.npix_cap;
  const uint32_t pitch = bm_pitch(w);
  const uint8_t* bm = j.bmap + (size_t)t * j.th * bm_pitch(j.tw);
  const uint32_t rb = lane * ch_vs(CH_R), qb = ch_res_off(CH_R) + lane * CH_QS;   // this lane's rings
  for (uint32_t e = 0; e < CH_R; e += 2) lds_st32(rb + 2 * e, half | (half << 16));
  // 16 residuals (two 16-byte loads) into ring entries s0 .. s0 + 15 as dwords
  auto land16 = [&](uint32_t s0, const uint4& a, const uint4& b4) {
    const uint32_t v[8] = {a.x, a.y, a.z, a.w, b4.x, b4.y, b4.z, b4.w};
#pragma unroll
    for (int e = 0; e < 8; e++) lds_st32(qb + 2 * s0 + 4 * e, v[e]);
    if (s0 == 0) {                                                     // the mirror (entries 64..79)
#pragma unroll
      for (int e = 0; e < 8; e++) lds_st32(qb + 128 + 4 * e, v[e]);
    }
  };
  // residual ring: entries [k, kfill) resident, the next 16 in flight (pend) when hp
  uint32_t k = 0, kfill = 32;
  uint4 pend0, pend1;
  {
    const uint4* r4 = (const uint4*)res;
    land16(0, r4[0], r4[1]);
    land16(16, r4[2], r4[3]);
    pend0 = r4[4]; pend1 = r4[5];
  }
  bool hp = true;
  uint4 bnext = *(const uint4*)bm;                                     // row 0, columns 0..15
  for (uint32_t y = 0; y < hmax; y++) {
    uint32_t L = half, Tp = half;                                      // row start: L = TL = half
    const bool live = y < h;
    for (uint32_t x0 = 0; x0 < w; x0 += 16) {
      const uint4 bcur = bnext;
      {
        const uint32_t ny = x0 + 16 < w ? y : y + 1, nx = x0 + 16 < w ? x0 + 16 : 0;
        bnext = live && ny < h ? *(const uint4*)(bm + (size_t)ny * pitch + nx) : make_uint4(0, 0, 0, 0);
      }
      if (!live) continue;
      if (hp) {                                                        // land the residuals fetched a block ago
        land16(kfill & 63, pend0, pend1);
        kfill += 16;
      }
      hp = kfill + 16 - k <= 64;
      if (hp) {
        const uint4* r4 = (const uint4*)(res + kfill);
        pend0 = r4[0]; pend1 = r4[1];
      }
      const uint32_t i0 = y * w + x0;
      const uint32_t bw[4] = {bcur.x, bcur.y, bcur.z, bcur.w};
      if (FULL) {
        const uint32_t pos0 = i0 & (CH_R - 1);
        const uint32_t tA = rb + 2 * ((pos0 - w) & (CH_R - 1));        // T of step u at tA + 2u
        const uint32_t wA = rb + 2 * pos0;                             // this block's slots
        // the 16 steps, specialised on whether a copy source can wrap around the ring (b <= 255).
        // The block's residuals are ring entries k .. k + 15, contiguous thanks to the mirror: the
        // next step's entry is known from the byte map alone (d counts this block's non-copy
        // steps), so every read of step u + 1 is issued before step u's arithmetic.  A copy with
        // b <= 1 reads a harmless slot of its own ring (b = 0 uses the MED value, b = 1 uses L).
        auto block = [&](auto nowrap_c) {
          constexpr bool NOWRAP = decltype(nowrap_c)::value;
          auto srcA = [&](int u, uint32_t b) -> uint32_t {
            return NOWRAP ? wA + 2 * u - 2 * b : rb + 2 * ((pos0 + (uint32_t)u - b) & (CH_R - 1));
          };
          const uint32_t qk = qb + 2 * (k & 63);
          uint32_t d = 0;
          // step 0 reads its copy source after every earlier write, so even b = 1 comes from the
          // ring (at a row's start that is the end of the row above, not L = half)
          uint32_t b = bw[0] & 255u;
          uint32_t T = lds_u16(tA), vC = lds_u16(srcA(0, b ? b : 1)), r = lds_u16(qk);
#pragma unroll
          for (int u = 0; u < 16; u++) {
            const uint32_t dn = d + (b == 0 ? 1u : 0u);
            uint32_t bn = 0, Tn = 0, vCn = 0, rn = 0;
            if (u < 15) {
              bn = (bw[(u + 1) >> 2] >> (8 * ((u + 1) & 3))) & 255u;
              Tn = lds_u16(tA + 2 * (u + 1));
              vCn = lds_u16(srcA(u + 1, bn));
              rn = lds_u16(qk + 2 * dn);
            }
            const uint32_t pr = medp(T, L, Tp);
            uint32_t vm = (r + pr + half) & cm, vc = (u > 0 && b == 1) ? L : vC;
            // both values, then a select: left to itself the compiler branches around the MED
            // (exec-mask juggling on every step of a divergent wave)
            asm volatile("" : "+v"(vm), "+v"(vc));
            const uint32_t v = b ? vc : vm;
            lds_st16(wA + 2 * u, v);
            Tp = T;
            L = v;
            b = bn; T = Tn; vC = vCn; r = rn; d = dn;
          }
          k += d;
        };
        if (pos0 >= 256) block(std::true_type{});                       // i - b >= 1 for every b <= 255
        else block(std::false_type{});
        // the block's 16 values to the plane (two 16-byte stores)
        uint32_t d[8];
#pragma unroll
        for (int e = 0; e < 8; e++) d[e] = lds_u32(wA + 4 * e);
        uint4* o4 = (uint4*)(outp + i0);
        o4[0] = make_uint4(d[0], d[1], d[2], d[3]);
        o4[1] = make_uint4(d[4], d[5], d[6], d[7]);
      } else {
#pragma unroll
        for (int u = 0; u < 16; u++) {
          if (x0 + u < w) {
            const uint32_t i = i0 + u;
            const uint32_t b = (bw[u >> 2] >> (8 * (u & 3))) & 255u;
            const uint32_t vC = lds_u16(rb + 2 * ((i - b) & (CH_R - 1)));
            const uint32_t T = lds_u16(rb + 2 * ((i - w) & (CH_R - 1)));
            const uint32_t r = lds_u16(qb + 2 * (k & 63));
            const uint32_t pr = medp(T, L, Tp);
            const uint32_t vm = (r + pr + half) & cm;
            const uint32_t v = b ? vC : vm;
            k += b ? 0u : 1u;
            lds_st16(rb + 2 * (i & (CH_R - 1)), v);
            outp[i] = (uint16_t)v;
            Tp = T;
            L = v;
          }
        }
      }
    }
  }
  if (act && k != st.n) atomicOr(j.gerr, 1u);
}

// RGB of the chain tiles from their three decoded planes (inverse subtract-green)
__device__ __forceinline__ void compose_tile(const DecJob& j, int t);
__global__ __launch_bounds__(256) void k_dcompose(DecJob j) {
  if (dec_abort(j)) return;
  const uint32_t n1 = *(volatile const uint32_t*)(j.gerr + 7), n2 = *(volatile const uint32_t*)(j.gerr + 8);
  for (uint32_t e = blockIdx.x; e < n1 + n2; e += gridDim.x)
    compose_tile(j, (int)(e < n1 ? j.lzt[(size_t)j.ntiles + e] : j.lzt[(size_t)2 * j.ntiles + e - n1]));
}

__device__ __forceinline__ void compose_tile(const DecJob& j, int t) {
  const DecTile ti = j.tiles[t];
  const uint16_t* G = j.dplane + (size_t)(t * 3) * j.npix_cap;
  const uint16_t* Rp = G + j.npix_cap;
  const uint16_t* Bp = Rp + j.npix_cap;
  const uint32_t w = ti.w, npix = w * ti.h;
  if ((w & 15) == 0 && (j.W & 15) == 0 && (ti.x0 & 15) == 0 && ((uintptr_t)j.rgb & 15) == 0) {
    // 16 pixels per thread: 32 B of each plane in, 48 B of RGB out as three 16-B stores (the
    // plane offsets are multiples of 64 values, the RGB rows and groups 16-B aligned)
    for (uint32_t i0 = threadIdx.x * 16; i0 < npix; i0 += 256 * 16) {
      const uint32_t yy = i0 / w, xx = i0 - yy * w;
      const uint4* g4 = (const uint4*)(G + i0);
      const uint4* r4 = (const uint4*)(Rp + i0);
      const uint4* b4 = (const uint4*)(Bp + i0);
      const uint4 ga = g4[0], gb = g4[1], ra = r4[0], rb = r4[1], ba = b4[0], bb = b4[1];
      const uint32_t gw[8] = {ga.x, ga.y, ga.z, ga.w, gb.x, gb.y, gb.z, gb.w};
      const uint32_t rw[8] = {ra.x, ra.y, ra.z, ra.w, rb.x, rb.y, rb.z, rb.w};
      const uint32_t bw[8] = {ba.x, ba.y, ba.z, ba.w, bb.x, bb.y, bb.z, bb.w};
      uint32_t px[16];                                  // 0x00BBGGRR
#pragma unroll
      for (int m = 0; m < 16; m++) {
        const uint32_t sh = 16 * (m & 1);
        const uint32_t g = (gw[m >> 1] >> sh) & 0xffffu;
        const uint32_t r = ((rw[m >> 1] >> sh) + g) & 255u, b = ((bw[m >> 1] >> sh) + g) & 255u;   // -256: mod 256
        px[m] = r | (g << 8) | (b << 16);
      }
      uint32_t o[12];
#pragma unroll
      for (int k = 0; k < 12; k++) {
        uint32_t d = 0;
#pragma unroll
        for (int c = 0; c < 4; c++) {
          const int mb = 4 * k + c;
          d |= ((px[mb / 3] >> (8 * (mb % 3))) & 255u) << (8 * c);
        }
        o[k] = d;
      }
      uint4* out = (uint4*)(j.rgb + ((size_t)(ti.y0 + yy) * j.W + ti.x0 + xx) * 3);
      out[0] = make_uint4(o[0], o[1], o[2], o[3]);
      out[1] = make_uint4(o[4], o[5], o[6], o[7]);
      out[2] = make_uint4(o[8], o[9], o[10], o[11]);
    }
    return;
  }
  for (uint32_t i = threadIdx.x; i < npix; i += 256) {
    const uint32_t yy = i / w, xx = i - yy * w;
    uint8_t* o = j.rgb + ((size_t)(ti.y0 + yy) * j.W + ti.x0 + xx) * 3;
    const uint32_t g = G[i];
    o[0] = (uint8_t)(Rp[i] + g - 256); o[1] = (uint8_t)g; o[2] = (uint8_t)(Bp[i] + g - 256);
  }
}

// ---------------------------------------------------------------- host side

static int dbuf(DecWork& w, int k, size_t bytes, void** p) {
  if (bytes == 0) bytes = 16;
  if (w.sizes[k] < bytes) {
    if (w.bufs[k]) (void)hipFree(w.bufs[k]);
    w.bufs[k] = nullptr;
    w.sizes[k] = 0;
    if (hipMalloc(&w.bufs[k], bytes) != hipSuccess) return 3;
    g_device_allocs.fetch_add(1, std::memory_order_relaxed);
    w.sizes[k] = bytes;
  }
  *p = w.bufs[k];
  return 0;
}

struct AsyncDec {              // enqueue-only decode: expected header bytes and the status slot
  uint64_t hdr[2];
  int hl;
  uint64_t* status;
  uint64_t bytes;               // the status size word on success
};
static int decode_run(hoh_ctx* c, DecJob& j, const hoh_index* idx, hipStream_t s, const AsyncDec* as = nullptr);
void launch_status_dec(const uint32_t* gerr, uint64_t bytes, uint64_t* out, hipStream_t s, int n = 1);

int decode_image_impl(hoh_ctx* c, const uint8_t* d_in, size_t size, uint8_t* d_rgb, size_t cap, int* Wp, int* Hp,
                      const hoh_index* idx, hipStream_t s) {
  // header (host copy of the first bytes: W, H decide every launch size)
  uint8_t hb[16] = {0};
  const size_t hn = size < 16 ? size : 16;
  if (hipMemcpyAsync(hb, d_in, hn, hipMemcpyDeviceToHost, s) != hipSuccess) return 3;
  if (hipStreamSynchronize(s) != hipSuccess) return 3;
  if (hn < 8 || hb[0] != 153 || hb[1] != 72 || hb[2] != 79 || hb[3] != 72) return 7;
  if (hb[4] != 2 || hb[5] != 8) return 6;
  uint64_t p = 6;
  auto rv = [&](uint64_t& v) {
    uint64_t b0 = hb[p++];
    if (!(b0 & 0x80)) { v = b0; return; }
    uint64_t b1 = hb[p++];
    if (!(b1 & 0x80)) { v = ((b0 & 0x7f) << 7) + b1; return; }
    uint64_t b2 = hb[p++];
    v = ((b0 & 0x7f) << 14) + ((b1 & 0x7f) << 7) + b2;
  };
  uint64_t wv, hv;
  rv(wv); rv(hv);
  const int W = (int)wv + 1, H = (int)hv + 1;
  *Wp = W; *Hp = H;
  if ((size_t)W * H * 3 > cap) return 2;
  DecJob j;
  memset(&j, 0, sizeof(j));
  j.W = W; j.H = H;
  if (!((W >= 512 || H >= 512) && W >= 256 && H >= 256)) return 6;   // header-only files (Q13)
  j.xt = W / 256; j.yt = H / 256;
  j.tw = (W + j.xt - 1) / j.xt; j.th = (H + j.yt - 1) / j.yt;
  if (p + 2 > size || hb[p] != (uint8_t)(j.xt - 1) || hb[p + 1] != (uint8_t)(j.yt - 1)) return 7;
  j.prefix = p + 2;
  j.ntiles = j.xt * j.yt;
  j.in = d_in;
  j.size = size;
  j.rgb = d_rgb;
  return decode_run(c, j, idx, s);
}

// enqueue-only decode of a W x H file (the caller knows the dimensions; the header is checked on
// the device); {status, W*H*3} land in d_status
int decode_image_async_impl(hoh_ctx* c, const uint8_t* d_in, size_t size, int W, int H, uint8_t* d_rgb, size_t cap,
                            const hoh_index* idx, uint64_t* d_status, hipStream_t s) {
  if (!((W >= 512 || H >= 512) && W >= 256 && H >= 256)) return 6;   // header-only files: sync call
  if ((size_t)W * H * 3 > cap) return 2;
  DecJob j;
  memset(&j, 0, sizeof(j));
  j.W = W; j.H = H;
  j.xt = W / 256; j.yt = H / 256;
  j.tw = (W + j.xt - 1) / j.xt; j.th = (H + j.yt - 1) / j.yt;
  uint8_t hb[16];
  int p = 0;
  hb[p++] = 153; hb[p++] = 72; hb[p++] = 79; hb[p++] = 72; hb[p++] = 2; hb[p++] = 8;   // choh.cpp:437-446
  for (uint32_t v : {(uint32_t)W - 1, (uint32_t)H - 1}) p = (int)hoh_write_varint(hb, (uint32_t)p, v);
  hb[p++] = (uint8_t)(j.xt - 1);
  hb[p++] = (uint8_t)(j.yt - 1);
  AsyncDec as;
  as.hdr[0] = as.hdr[1] = 0;
  for (int i = 0; i < p; i++) as.hdr[i / 8] |= (uint64_t)hb[i] << (8 * (i % 8));
  as.hl = p;
  as.status = d_status;
  as.bytes = (uint64_t)W * H * 3;
  j.prefix = (uint64_t)p;
  j.ntiles = j.xt * j.yt;
  j.in = d_in;
  j.size = size;
  j.rgb = d_rgb;
  return decode_run(c, j, idx, s, &as);
}

// enqueue-only decode of n W x H files at d_in + i * stride into n contiguous images (their stack:
// one job, every kernel over all n files' tiles); {status, W*H*3} per image in d_status
int decode_images_async_impl(hoh_ctx* c, int n, const uint8_t* d_in, size_t stride, int W, int H, uint8_t* d_rgb,
                             const hoh_index* idx, uint64_t* d_status, hipStream_t s) {
  if (!((W >= 512 || H >= 512) && W >= 256 && H >= 256)) return 6;
  const size_t img = (size_t)W * H * 3;
  if (n == 1 || !batch_stacks(W, H)) {
    if (idx && n > 1) return 6;
    for (int i = 0; i < n; i++) {
      const int r = decode_image_async_impl(c, d_in + i * stride, stride, W, H, d_rgb + i * img, img, idx,
                                            d_status + 2 * i, s);
      if (r) return r;
    }
    return 0;
  }
  if ((int64_t)H * n > (1ll << 30)) return 1;
  DecJob j;
  memset(&j, 0, sizeof(j));
  j.xt = W / 256; j.yt = H / 256;
  j.tw = (W + j.xt - 1) / j.xt; j.th = (H + j.yt - 1) / j.yt;
  uint8_t hb[16];
  int p = 0;
  hb[p++] = 153; hb[p++] = 72; hb[p++] = 79; hb[p++] = 72; hb[p++] = 2; hb[p++] = 8;   // choh.cpp:437-446
  for (uint32_t v : {(uint32_t)W - 1, (uint32_t)H - 1}) p = (int)hoh_write_varint(hb, (uint32_t)p, v);
  hb[p++] = (uint8_t)(j.xt - 1);
  hb[p++] = (uint8_t)(j.yt - 1);
  AsyncDec as;
  as.hdr[0] = as.hdr[1] = 0;
  for (int i = 0; i < p; i++) as.hdr[i / 8] |= (uint64_t)hb[i] << (8 * (i % 8));
  as.hl = p;
  as.status = d_status;
  as.bytes = (uint64_t)img;
  j.W = W; j.H = H * n;                           // the stack
  j.yt *= n;
  j.prefix = (uint64_t)p;
  j.ntiles = j.xt * j.yt;
  j.nimg = n;
  j.img_tiles = j.ntiles / n;
  j.in_stride = stride;
  j.in = d_in;
  j.size = (uint64_t)n * stride;
  j.rgb = d_rgb;
  return decode_run(c, j, idx, s, &as);
}

// shard decode: tiles [t0, t0+ntiles) of a W x H image, their bytes concatenated in d_blob
int decode_tiles_impl(hoh_ctx* c, const uint8_t* d_blob, size_t size, int W, int H, int t0, int ntiles,
                      const uint32_t* h_sizes, uint8_t* d_rgb, const hoh_index* idx, hipStream_t s) {
  DecJob j;
  memset(&j, 0, sizeof(j));
  j.W = W; j.H = H;
  if (!((W >= 512 || H >= 512) && W >= 256 && H >= 256)) return 6;
  j.xt = W / 256; j.yt = H / 256;
  j.tw = (W + j.xt - 1) / j.xt; j.th = (H + j.yt - 1) / j.yt;
  if (t0 < 0 || ntiles <= 0 || t0 + ntiles > j.xt * j.yt) return 1;
  j.t0 = t0;
  j.ntiles = ntiles;
  j.prefix = 0;
  j.in = d_blob;
  j.size = size;
  j.rgb = d_rgb;
  uint64_t tot = 0;
  for (int i = 0; i < ntiles; i++) tot += h_sizes[i];
  if (tot > size) return 7;
  DecWork& w = ctx_dec(c);
  void* q;
  int e;
  if ((e = dbuf(w, 12, (size_t)ntiles * 4, &q))) return e;
  if (hipMemcpyAsync(q, h_sizes, (size_t)ntiles * 4, hipMemcpyHostToDevice, s) != hipSuccess) return 3;
  j.tsizes = (const uint32_t*)q;
  return decode_run(c, j, idx, s);
}

// enqueue-only shard decode: the tile sizes stay on the device (as the encoder wrote them), so
// nothing waits on the host; {status, tile pixels * 3} land in d_status
int decode_tiles_async_impl(hoh_ctx* c, const uint8_t* d_blob, size_t size, int W, int H, int t0, int ntiles,
                            const uint32_t* d_sizes, uint8_t* d_rgb, const hoh_index* idx, uint64_t* d_status,
                            hipStream_t s) {
  DecJob j;
  memset(&j, 0, sizeof(j));
  j.W = W; j.H = H;
  if (!((W >= 512 || H >= 512) && W >= 256 && H >= 256)) return 6;
  j.xt = W / 256; j.yt = H / 256;
  j.tw = (W + j.xt - 1) / j.xt; j.th = (H + j.yt - 1) / j.yt;
  if (t0 < 0 || ntiles <= 0 || t0 + ntiles > j.xt * j.yt) return 1;
  j.t0 = t0;
  j.ntiles = ntiles;
  j.prefix = 0;
  j.in = d_blob;
  j.size = size;
  j.rgb = d_rgb;
  j.tsizes = d_sizes;
  AsyncDec as;
  as.hdr[0] = as.hdr[1] = 0;
  as.hl = 0;                                      // a blob has no header to check
  as.status = d_status;
  as.bytes = 0;
  for (int i = 0; i < ntiles; i++) {
    const int g = t0 + i, xo = (g % j.xt) * j.tw, yo = (g / j.xt) * j.th;
    as.bytes += (uint64_t)std::min(j.tw, W - xo) * std::min(j.th, H - yo) * 3;
  }
  return decode_run(c, j, idx, s, &as);
}

// enqueue-only decode of n shards (tiles [t0, t0+ntiles) of n W x H images): blob i at
// d_blob + i * stride, its tile sizes at d_sizes + i * ntiles (device), band i's RGB at
// d_rgb + i * W * rows * 3.  Whole 256-row tile bands stack into one W x (n * rows) job (one
// dtable workgroup per blob), as decode_images_async_impl stacks whole files; otherwise the
// shards run one after another.  {status, band RGB bytes} per shard in d_status.
int decode_tiles_images_async_impl(hoh_ctx* c, int n, const uint8_t* d_blob, size_t stride, int W, int H, int t0,
                                   int ntiles, const uint32_t* d_sizes, uint8_t* d_rgb, const hoh_index* idx,
                                   uint64_t* d_status, hipStream_t s) {
  if (!((W >= 512 || H >= 512) && W >= 256 && H >= 256)) return 6;
  const int xt = W / 256, yt = H / 256, th = (H + yt - 1) / yt;
  if (t0 < 0 || ntiles <= 0 || t0 + ntiles > xt * yt || t0 % xt || ntiles % xt) return 1;
  const int y0 = (t0 / xt) * th, rows = std::min(H, (t0 + ntiles) / xt * th) - y0;
  const size_t band = (size_t)W * rows * 3;
  if (n == 1 || !batch_stacks(W, H)) {
    if (idx && n > 1) return 6;
    for (int i = 0; i < n; i++) {
      const int r = decode_tiles_async_impl(c, d_blob + i * stride, stride, W, H, t0, ntiles, d_sizes + (size_t)i * ntiles,
                                            d_rgb + i * band - (size_t)y0 * W * 3, idx, d_status + 2 * i, s);
      if (r) return r;
    }
    return 0;
  }
  if ((int64_t)rows * n > (1ll << 30) || (int64_t)ntiles * n > (1 << 24)) return 1;
  DecJob j;
  memset(&j, 0, sizeof(j));
  j.W = W; j.H = rows * n;                        // the stack of the n bands
  j.xt = xt; j.yt = rows * n / 256;
  j.tw = (W + xt - 1) / xt; j.th = 256;
  j.t0 = 0;
  j.ntiles = ntiles * n;
  j.nimg = n;
  j.img_tiles = ntiles;
  j.in_stride = stride;
  j.prefix = 0;
  j.in = d_blob;
  j.size = (uint64_t)n * stride;
  j.rgb = d_rgb;
  j.tsizes = d_sizes;
  AsyncDec as;
  as.hdr[0] = as.hdr[1] = 0;
  as.hl = 0;                                      // blobs have no header to check
  as.status = d_status;
  as.bytes = (uint64_t)band;
  return decode_run(c, j, idx, s, &as);
}

// copies reading the row above that make an LZ tile a chain tile (knobs LZ_XROW, LZ_XROW_BATCH).
// A batch decodes many images' LZ tiles at once, and there the raster chains (less work per tile
// than the dynamic wavefront) pay from 2 such copies on: natural 8192^2 -s0 pipeline 50.1 -> 53.5
// GB/s, while one image alone keeps 16 (its wavefront tiles finish sooner: 5.43 against 5.55 ms;
// profiles/r06b/xrow_sweep.txt)
static uint32_t lz_xrow(bool batch) {
  return batch ? (uint32_t)HOH_KNOB(LZ_XROW_BATCH, 2) : (uint32_t)HOH_KNOB(LZ_XROW, LZ_XROW);
}

// No-index chain kernel choice (hoh_ctx_set_option HOH_OPT_NOIX_DECODER, default adaptive).
// k_drans_multi (12 chains per CU, full tables) has the shorter step (~260 cycles against
// k_drans_lanes' ~400) but holds a whole CU per 12 chains; k_drans_lanes packs up to 64 chains per
// workgroup into compact tables and fills the device when several decodes run at once.  So an
// adaptive decode that has the device to itself takes k_drans_multi, one that finds another
// context's no-index chain kernel still in flight, or whose plane chains need more than one round
// of k_drans_multi (batches, 16384^2), takes k_drans_lanes.  HOH_NOIX_WAVE: one wave per stream
// (k_drans_wave, the round-2 decoder).

// Contexts' completion events per device, to count the no-index decodes in flight beside this one.
static std::mutex g_noix_mu;
static std::vector<DecWork*> g_noix;

void noix_release(DecWork& w) {
  if (!w.noix_ev) return;
  {
    std::lock_guard<std::mutex> g(g_noix_mu);
    g_noix.erase(std::remove(g_noix.begin(), g_noix.end(), &w), g_noix.end());
  }
  (void)hipEventDestroy(w.noix_ev);
  w.noix_ev = nullptr;
  w.noix_dev = -1;
}

// Another context's no-index decode issued this recently (knob NOIX_WINDOW_MS) counts as
// concurrent traffic even when its chain kernel has finished (a pipeline's decodes leave gaps
// between kernels; one k_drans_multi among them takes every CU's LDS for its 7 ms)
static int64_t noix_window_us() { return (int64_t)HOH_KNOB(NOIX_WINDOW_MS, 20) * 1000; }

// 1 if another context on this device issued a no-index decode within the window or its chain
// kernel has not finished (hipEventQuery only: nothing waits); registers w on first use and stamps
// its issue time.  A failure to create the event reads as busy.
static int noix_busy(DecWork& w, int dev) {
  const int64_t now = std::chrono::duration_cast<std::chrono::microseconds>(
                          std::chrono::steady_clock::now().time_since_epoch()).count();
  if (!w.noix_ev) {
    if (hipEventCreateWithFlags(&w.noix_ev, hipEventDisableTiming) != hipSuccess) { w.noix_ev = nullptr; return 1; }
    w.noix_dev = dev;
    std::lock_guard<std::mutex> g(g_noix_mu);
    g_noix.push_back(&w);
  }
  std::lock_guard<std::mutex> g(g_noix_mu);
  w.noix_t = now;
  for (DecWork* o : g_noix)
    if (o != &w && o->noix_dev == dev &&
        (now - o->noix_t < noix_window_us() || hipEventQuery(o->noix_ev) == hipErrorNotReady)) return 1;
  return 0;
}
// k_drans_lanes: LDS table budget per workgroup (knob DL_BUDGET_KB, >= the 5.1 KB worst-case
// table) and workgroups per CU (knob DL_WG)
// (no-index pipeline, 4 contexts x batches of 8: 20 KB x 4 68.8 GB/s, 32 x 4 75.1, 48 x 3 78.6,
// 64 x 2 73.7, 80 x 2 62.2; profiles/r06b/noix_pipeline_lds_budget_sweep.txt)
static uint32_t dl_budget() {
  const uint32_t kb = (uint32_t)HOH_KNOB(DL_BUDGET_KB, 48);
  return std::max<uint32_t>(std::min<uint32_t>(kb, 150u) * 1024u, dl_bytes(15, 512));
}
static int dl_wg_per_cu() { return std::max(1, HOH_KNOB(DL_WG, 3)); }

static int decode_run(hoh_ctx* c, DecJob& j, const hoh_index* idx, hipStream_t s, const AsyncDec* as) {
  j.exp = (uint32_t)HOH_KNOB(EXP, 0);
  j.npix_cap = (uint32_t)(((size_t)j.tw * j.th + 63) / 64 * 64);
  j.lz_cap = (uint32_t)((j.npix_cap / 4 + j.npix_cap / 255 + 16 + 7) / 8 * 8);
  {
    // flat planes + slack for k_dunpred_fast's residual reads three groups past a row's end
    j.plane_cap = (uint32_t)(((size_t)j.npix_cap + 8 * UP_P + 128 + 63) / 64 * 64);
    // 256-wide tiles: room for the blocked layout (its reads stay inside the tile's bands)
    j.blk_ok = j.tw == 256;
    if (j.blk_ok) j.plane_cap = std::max<uint32_t>(j.plane_cap, (uint32_t)(((size_t)j.th + 63) / 64 * BLK_BAND));
  }
  const int S = j.ntiles * SK_PER_TILE;
  DecWork& w = ctx_dec(c);
  void* q;
  int e;
  if ((e = dbuf(w, 0, (size_t)j.ntiles * sizeof(DecTile), &q))) return e; j.tiles = (DecTile*)q;
  if ((e = dbuf(w, 1, (size_t)S * sizeof(DecStream), &q))) return e; j.streams = (DecStream*)q;
  j.cum_stride = 513;
  if ((e = dbuf(w, 2, (size_t)S * 513 * 4, &q))) return e; j.cum = (uint32_t*)q;
  if ((e = dbuf(w, 3, (size_t)S * 512 * 2, &q))) return e; j.bsym = (uint16_t*)q;
  if ((e = dbuf(w, 4, ((size_t)j.ntiles * 3 * j.plane_cap + (size_t)j.ntiles * 3 * j.lz_cap) * 2, &q))) return e; j.dsym = (uint16_t*)q;
  if ((e = dbuf(w, 5, (size_t)j.ntiles * 4 * (j.lz_cap + 1) * 4, &q))) return e; j.matches = (uint32_t*)q;
  if ((e = dbuf(w, 6, 64, &q))) return e; j.gerr = (uint32_t*)q;
  if ((e = dbuf(w, 7, (size_t)j.ntiles * 3 * j.npix_cap * 2, &q))) return e; j.dplane = (uint16_t*)q;
  if ((e = dbuf(w, 14, (size_t)j.ntiles * 3 * 4, &q))) return e; j.lzt = (uint32_t*)q;
#ifdef DEC_DBG
  if ((e = dbuf(w, 15, (size_t)j.ntiles * j.th * ((j.tw + 15) & ~15) + 16 + (1 << 16), &q))) return e; j.bmap = (uint8_t*)q;
#else
  if ((e = dbuf(w, 15, (size_t)j.ntiles * j.th * ((j.tw + 15) & ~15) + 16, &q))) return e; j.bmap = (uint8_t*)q;
#endif
  j.lz_xrow = lz_xrow(j.nimg > 1);
  if (idx) {                                   // a batch's index serves that batch's layout only
    uint64_t st = 0;
    const int ni = index_batch(idx, &st);
    if (ni != (j.nimg > 1 ? j.nimg : 1) || (ni > 1 && st != j.in_stride)) return 1;
  }
  j.ix = index_streams(idx);
  j.ck = index_ckpts(idx);
  j.nix = index_nstreams(idx);
  const int indexed = j.ix && j.nix == S;
  if (hipMemsetAsync(j.gerr, 0, 64, s) != hipSuccess) return 3;
  if (hipMemsetAsync(j.streams, 0, (size_t)S * sizeof(DecStream), s) != hipSuccess) return 3;
  ctx_mark(c, s, "start", as == nullptr);
  const int nfile = j.nimg > 1 ? j.nimg : 1;
  if (as && as->hl) hipLaunchKernelGGL(k_dhdr, dim3(nfile), dim3(64), 0, s, j, as->hdr[0], as->hdr[1], as->hl);
  hipLaunchKernelGGL(k_dtable, dim3(nfile), dim3(1024), 0, s, j);
  ctx_mark(c, s, "dtable", false);
  hipLaunchKernelGGL(k_dparse, dim3(j.ntiles), dim3(64), 0, s, j);
  ctx_mark(c, s, "dparse", false);
  if (indexed) {
    hipLaunchKernelGGL(k_dmatch, dim3((S + 255) / 256), dim3(256), 0, s, j, S);
    hipLaunchKernelGGL(k_drans, dim3(S), dim3(DR_T), DR_SMEM, s, j, S);
  } else if (ctx_noix(c) == HOH_NOIX_WAVE) {                  // the one-wave-per-stream decoder alone
    hipLaunchKernelGGL(k_drans_wave, dim3(S), dim3(64), DL_SMEM, s, j, S, 0);
  } else {
    // every plane / LZ stream: a chain lane of k_drans_multi or k_drans_lanes (noix_multi above);
    // anything else: k_drans_wave
    void* q2;
    if ((e = dbuf(w, 13, (size_t)S * 12 + 8, &q2))) return e;
    uint32_t* mlist = (uint32_t*)q2;
    uint32_t* tbytes = mlist + S;
    uint32_t* rounds = tbytes + S;                           // S + 1 words
    hipLaunchKernelGGL(k_dmlist, dim3((S + 255) / 256), dim3(256), 0, s, j, S, mlist);
    const int pin = ctx_noix(c);
    // k_drans_multi only while the plane chains fit one round of it (12 per CU: one 8192^2 image);
    // a batch of eight took 8 rounds, 50 ms, where k_drans_lanes takes two (profiles/r06b/noix_pipeline_prof.txt)
    const bool one_round = 3 * j.ntiles <= DM_MS * ctx_cus(c);
    const bool multi = pin == HOH_NOIX_MULTI || (pin != HOH_NOIX_LANES && one_round && !noix_busy(w, ctx_device(c)));
    if (multi) {
      // one workgroup per CU (its LDS is a whole CU's), rounds of DM_MS streams per workgroup
      const int nmax = std::min(S, 6 * j.ntiles);
      const int grid = std::min((nmax + DM_MS - 1) / DM_MS, ctx_cus(c));
      hipLaunchKernelGGL(k_drans_multi<DM_MS>, dim3(grid), dim3(64), dm_smem(DM_MS), s, j, (const uint32_t*)mlist, S);
    } else {
      hipLaunchKernelGGL(k_dlsize, dim3(S), dim3(64), 0, s, j, tbytes);
      const uint32_t budget = dl_budget();
      hipLaunchKernelGGL(k_dlpack, dim3(1), dim3(64), 0, s, j, (const uint32_t*)mlist, S, (const uint32_t*)tbytes, budget,
                         rounds);
      const int grid = std::min(S, dl_wg_per_cu() * ctx_cus(c));
      hipLaunchKernelGGL(k_drans_lanes, dim3(grid), dim3(64), DL_TAB + budget, s, j, (const uint32_t*)mlist, S,
                         (const uint32_t*)tbytes, budget, (const uint32_t*)rounds);
    }
    if (w.noix_ev) (void)hipEventRecord(w.noix_ev, s);
    hipLaunchKernelGGL(k_drans_wave, dim3(S), dim3(64), DL_SMEM, s, j, S, 1);
  }
  ctx_mark(c, s, "drans", false);
  if (!indexed) hipLaunchKernelGGL(k_dstored, dim3(S), dim3(256), 0, s, j, S);
  hipLaunchKernelGGL(k_dlz, dim3(j.ntiles), dim3(64), 0, s, j);
  ctx_mark(c, s, "dlz", false);
  // chain tiles: their back-distance maps (the chains themselves run inside k_dunpred_lz)
  const int gsmall = std::min(j.ntiles, 256);
  hipLaunchKernelGGL(k_dbackmap, dim3(gsmall), dim3(256), 0, s, j);
  {
    const int we = j.W - (j.xt - 1) * j.tw;
    hipLaunchKernelGGL(k_dexpand, dim3(j.ntiles), dim3(256), 0, s, j, j.tw % 16 == 0 ? 1 : 0, we % 16 == 0 ? 1 : 0);
  }
  hipLaunchKernelGGL(k_dunpred_fast, dim3(j.ntiles), dim3(64), (size_t)64 * ORING_PITCH + 6 * LAST_N(j.tw), s, j);
  {
    // On natural images most tiles hold copies, and a copy at a row's start that reads the end of
    // the row above turns the wavefront into raster order (such a tile is nearly serial), so the
    // tiles themselves are the parallelism; with few LZ tiles, 64-row bands take fewer steps.
    const size_t rowb = (size_t)j.tw * 4, lds = 160 * 1024;
    j.lzstage = 0;
    const int br_few = (int)std::min<size_t>(64, lds / rowb - 2);
    const int br_many = (int)std::min<size_t>(32, lds / rowb - 2);
    j.lzband = br_few;
    // + the chain tiles' workgroups (ring R >= 2w: row 0 reads T / TL from the initial half values)
    const int we = j.W - (j.xt - 1) * j.tw;                             // the edge column's width
    const int ga = (j.ntiles + CH_T - 1) / CH_T, gc = ga * (we != j.tw ? 2 : 1);
    const bool r512 = 2 * j.tw <= 512;
    const size_t cl = r512 ? ch_smem(512) : ch_smem(1024);
    const int wf = std::min(j.ntiles, LZ_FEW), full1 = j.tw % 16 == 0, full2 = we % 16 == 0;
    auto launch = [&](int grid, size_t band, int br, int many) {
      const size_t l = std::max(band, cl);
      if (r512) hipLaunchKernelGGL(k_dunpred_lz<512>, dim3(grid + gc), dim3(64), l, s, j, br, many, grid, ga, full1, full2);
      else hipLaunchKernelGGL(k_dunpred_lz<1024>, dim3(grid + gc), dim3(64), l, s, j, br, many, grid, ga, full1, full2);
    };
    launch(wf, (size_t)(br_few + 1) * rowb, br_few, 0);
    // the wavefront workgroups stride over the LZ tile list, so more of them than the CUs hold
    // at once (their LDS bands: ~4 per CU) buy nothing; a grid of one per tile dispatched ~8,000
    // workgroups per batch of eight 8192^2 images even when no tile has copies (knob LZ_WG_PER_CU)
    const int wcap = HOH_KNOB(LZ_WG_PER_CU, 4) * ctx_cus(c);
    if (j.ntiles > LZ_FEW) launch(wcap > 0 && wcap < j.ntiles ? wcap : j.ntiles, (size_t)(br_many + 1) * rowb, br_many, 1);
    hipLaunchKernelGGL(k_dcompose, dim3(gsmall), dim3(256), 0, s, j);   // the chain tiles' RGB
  }
  ctx_mark(c, s, "dunpred", false);
  if (hipGetLastError() != hipSuccess) return 3;
  if (as) {
    launch_status_dec(j.gerr, as->bytes, as->status, s, j.nimg > 1 ? j.nimg : 1);
    return hipGetLastError() == hipSuccess ? 0 : 3;
  }
  uint64_t* pin = ctx_pinned(c);
  if (hipMemcpyAsync(pin, j.gerr, 8, hipMemcpyDeviceToHost, s) != hipSuccess) return 3;
  if (hipStreamSynchronize(s) != hipSuccess) return 3;
  const uint32_t ge = (uint32_t)pin[0];
  if (ge & 2) return 6;
  if (ge) return 7;
  return 0;
}

// ---------------------------------------------------------------- single stream (decode_entropy)

__global__ __launch_bounds__(64) void k_dstream(DecJob j, uint64_t bp, uint64_t* res) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dl_lds[];
  const int lane = threadIdx.x;
  uint64_t p = bp;
  const bool ok = parse_stream(j, p, 0, 0, lane);
  __syncthreads();
  if (!ok) { if (lane == 0) res[0] = 1; return; }
  const DecStream d = j.streams[0];
  if (d.mode == SM_RANS && d.range <= 512 && d.pb <= 15) {      // the whole wave (lane_decode)
    const bool good = lane_decode(j, d, j.cum, j.dsym, dl_lds);
    if (lane == 0) { res[0] = good ? 0 : 1; res[1] = d.n; res[2] = p; }
    return;
  }
  if (lane != 0) return;
  res[1] = d.n;
  if (d.mode == SM_RANS) {
    const uint64_t wend = d.payload_off + (uint64_t)d.words * 4;
    uint64_t x = (uint64_t)ld_u32_unaligned(j.in, d.payload_off) | ((uint64_t)ld_u32_unaligned(j.in, d.payload_off + 4) << 32);
    uint64_t xe;
    if (!dec_run<false>(j, d, j.cum, j.bsym, d.pb > 9 ? d.pb - 9 : 0, nullptr, x, d.payload_off + 8, wend, 0, d.n,
                        OutCursor(j.dsym, 0, 0), &xe) || xe != (1ull << 31)) {
      res[0] = 1;
      return;
    }
  } else if (d.mode == SM_STORED) {
    for (uint32_t i = 0; i < d.n; i++) j.dsym[i] = (uint16_t)get_bits(j.in, d.payload_off * 8 + (uint64_t)i * d.maxbits, d.maxbits);
  }
  res[0] = 0;
  res[2] = p;
}

// decode one stream of `in` (device, size bytes) at byte pointer bp into d_out (device)
int decode_stream_impl(hoh_ctx* c, const uint8_t* d_in, size_t size, size_t* bp, uint16_t* d_out, size_t cap,
                       size_t* n, hipStream_t s) {
  DecJob j;
  memset(&j, 0, sizeof(j));
  DecWork& w = ctx_dec(c);
  void* q;
  int e;
  j.in = d_in;
  j.size = size;
  j.cum_stride = 4097;
  if ((e = dbuf(w, 8, sizeof(DecStream), &q))) return e; j.streams = (DecStream*)q;
  if ((e = dbuf(w, 9, 4097 * 4, &q))) return e; j.cum = (uint32_t*)q;
  if ((e = dbuf(w, 10, 512 * 2, &q))) return e; j.bsym = (uint16_t*)q;
  if ((e = dbuf(w, 11, 64, &q))) return e;
  uint64_t* res = (uint64_t*)q;
  j.dsym = d_out;
  // the symbol count must fit: peek happens on the host (hoh_entropy_count) before the call
  hipLaunchKernelGGL(k_dstream, dim3(1), dim3(64), DL_SMEM, s, j, (uint64_t)*bp, res);
  if (hipGetLastError() != hipSuccess) return 3;
  uint64_t* pin = ctx_pinned(c);
  if (hipMemcpyAsync(pin, res, 24, hipMemcpyDeviceToHost, s) != hipSuccess) return 3;
  if (hipStreamSynchronize(s) != hipSuccess) return 3;
  if (pin[0]) return 7;
  if (pin[1] > cap) return 2;
  *n = (size_t)pin[1];
  *bp = (size_t)pin[2];
  return 0;
}
