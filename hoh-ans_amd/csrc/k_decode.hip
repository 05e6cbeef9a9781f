// Decoder kernels (dhoh.cpp:22-283 semantics with SURVEY Q1, Q9-Q12 fixed).
//  k_dtable: the .hoh tile table (n-1 varints after the header) -> tile offsets.
//  k_dparse: one wave per tile walks the tile framing and its 6 entropy streams
//            (entropy_decoding.hpp:134-257): header varints, meta byte, frequency table
//            (clamped tables parsed in parallel: per-symbol field widths -> prefix sum ->
//            MSB-first field extraction), payload location; writes DecStream records, the
//            per-stream cumulative table and a 64-slot bucket table for symbol lookup.
//  k_drans:  rANS decode (rans64.hpp:107-142).  With a side index: one lane per 1024-symbol
//            segment starting from the encoder's checkpoint; without: one lane per stream.
//  k_dlz:    LZ streams -> match list (un_lz.hpp:150-170, Q11/Q12 handled).
//  k_dunpred: MED inverse (prediction.hpp:26-41 inverted, every row, Q9 fixed), LZ copies and
//            inverse subtract-green, one workgroup per tile, three waves (one per plane) running
//            an anti-diagonal wavefront over 64-row bands.
#include "hoh_dec.h"
#include <string.h>

#define DSEG HOH_SEG

struct DecJob {
  const uint8_t* in;
  uint64_t size;
  int W, H, xt, yt, tw, th, ntiles;
  uint32_t npix_cap, lz_cap;
  uint64_t prefix;              // bytes before the tile table
  DecTile* tiles;
  DecStream* streams;
  uint32_t* cum;                // [stream][513]
  uint16_t* bsym;               // [stream][512] symbol at slot bucket*64 (prob_bits 15) / generic
  uint16_t* dsym;               // decoded symbols: planes [tile][3][npix_cap], LZ [tile][3][lz_cap]
  uint16_t* dplane;             // decoded planes of tiles with LZ matches [tile][3][npix_cap]
  uint32_t cum_stride;          // entries per stream in cum (>= range + 1)
  int band;                     // rows per wavefront band (<= 64, LDS-bound)
  uint32_t* matches;            // [tile][lz_cap][3]
  uint8_t* rgb;                 // output image
  uint32_t* gerr;
  const IndexStream* ix;        // optional side index
  const Checkpoint* ck;
  int nix;
  int t0;                       // global index of the first tile (shard decode)
  const uint32_t* tsizes;       // shard decode: tile byte sizes instead of the file's table
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

__global__ void k_dtable(DecJob j) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint64_t p = j.prefix;
  uint64_t off = 0;
  for (int i = 0; i < j.ntiles; i++) {
    DecTile t;
    const int g = j.t0 + i;
    const int xo = (g % j.xt) * j.tw, yo = (g / j.xt) * j.th;
    t.x0 = xo; t.y0 = yo;
    t.w = min(j.tw, j.W - xo); t.h = min(j.th, j.H - yo);
    t.off = off;               // relative to the first tile, fixed below
    t.mode = 0; t.nmatch = 0; t.err = 0; t.pad = 0;
    j.tiles[i] = t;
    if (i + 1 < j.ntiles) {
      if (j.tsizes) { off += j.tsizes[i]; continue; }
      if (p + 3 > j.size) { atomicOr(j.gerr, 1u); return; }
      off += rd_varint(j.in, p);
    }
  }
  for (int i = 0; i < j.ntiles; i++) j.tiles[i].off += p;   // tiles follow the table (dhoh.cpp:42-65)
  if (j.tiles[j.ntiles - 1].off >= j.size) atomicOr(j.gerr, 1u);
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
  // symbol at the start of every 2^(pb-9) slot bucket (512 buckets)
  uint16_t* bs = j.bsym + (size_t)sid * 512;
  const uint32_t bshift = d.pb > 9 ? d.pb - 9 : 0;
  const uint32_t nbk = 1u << (d.pb - bshift);
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
  if (lane == 0) j.streams[sid] = d;
  return true;
}

__global__ __launch_bounds__(64) void k_dparse(DecJob j) {
  const int t = blockIdx.x, lane = threadIdx.x;
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
    const size_t lzbase = (size_t)j.ntiles * 3 * j.npix_cap + (size_t)t * 3 * j.lz_cap;
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
      ok = parse_stream(j, q, t * SK_PER_TILE + 3 + k, (size_t)(t * 3 + k) * j.npix_cap, lane);
      const uint32_t depth = k ? 9 : 8;
      if (ok && j.streams[t * SK_PER_TILE + 3 + k].range != (1u << depth)) ok = false;
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

// rANS decode of [s0, s1) of stream d from state x, word cursor wp (byte offset of next word)
__device__ bool dec_run(const DecJob& j, const DecStream& d, const uint32_t* cum, const uint16_t* bs,
                        uint64_t x, uint64_t wp, uint64_t wend, uint32_t s0, uint32_t s1, uint16_t* out,
                        uint64_t* xend) {
  const uint32_t pb = d.pb, mask = (1u << pb) - 1;
  const uint32_t bshift = pb > 9 ? pb - 9 : 0;
  for (uint32_t i = s0; i < s1; i++) {
    const uint32_t slot = (uint32_t)x & mask;
    uint32_t s = bs[slot >> bshift];
    while (cum[s + 1] <= slot) s++;
    out[i] = (uint16_t)s;
    const uint32_t c = cum[s], f = cum[s + 1] - c;
    x = (uint64_t)f * (x >> pb) + (slot - c);                // Rans64DecAdvance
    if (x < (1ull << 31)) {
      if (wp + 4 > wend) return false;
      x = (x << 32) | ld_u32_unaligned(j.in, wp);
      wp += 4;
    }
  }
  *xend = x;
  return true;
}

// grid: with index -> one workgroup (64 lanes) per stream, lane = segment (strided);
//       without    -> 64 streams per workgroup, one lane each.
__global__ __launch_bounds__(64) void k_drans(DecJob j, int nstreams, int indexed) {
  __shared__ uint32_t cum_s[513];
  __shared__ uint16_t bs_s[512];
  const int lane = threadIdx.x;
  if (indexed) {
    const int sid = blockIdx.x;
    const DecStream d = j.streams[sid];
    if (d.mode != SM_RANS || d.range > 512) return;
    for (uint32_t i = lane; i <= d.range; i += 64) cum_s[i] = j.cum[(size_t)sid * j.cum_stride + i];
    for (uint32_t i = lane; i < 512; i += 64) bs_s[i] = j.bsym[(size_t)sid * 512 + i];
    __syncthreads();
    const uint64_t wend = d.payload_off + (uint64_t)d.words * 4;
    uint16_t* out = j.dsym + d.out_off;
    if (d.ix < 0) {
      // no index for this stream: serial on lane 0
      if (lane == 0) {
        uint64_t x = (uint64_t)ld_u32_unaligned(j.in, d.payload_off) | ((uint64_t)ld_u32_unaligned(j.in, d.payload_off + 4) << 32);
        uint64_t xe;
        if (!dec_run(j, d, cum_s, bs_s, x, d.payload_off + 8, wend, 0, d.n, out, &xe) || xe != (1ull << 31)) atomicOr(j.gerr, 4u);
      }
      return;
    }
    const IndexStream xs = j.ix[d.ix];
    const uint32_t nseg = (d.n + DSEG - 1) / DSEG;
    for (uint32_t sg = lane; sg < nseg; sg += 64) {
      const Checkpoint c = j.ck[xs.ckpt_off + sg];
      const uint64_t x = (uint64_t)c.xl | ((uint64_t)c.xh << 32);
      const uint64_t wp = d.payload_off + (uint64_t)(c.widx - xs.widx_end) * 4;
      const uint32_t s0 = sg * DSEG, s1 = min(d.n, s0 + DSEG);
      uint64_t xe;
      bool ok = dec_run(j, d, cum_s, bs_s, x, wp, wend, s0, s1, out, &xe);
      uint64_t want = 1ull << 31;
      if (sg + 1 < nseg) { const Checkpoint c2 = j.ck[xs.ckpt_off + sg + 1]; want = (uint64_t)c2.xl | ((uint64_t)c2.xh << 32); }
      if (!ok || xe != want) atomicOr(j.gerr, 4u);
    }
    return;
  }
  const int sid = blockIdx.x * 64 + lane;
  if (sid >= nstreams) return;
  const DecStream d = j.streams[sid];
  if (d.mode != SM_RANS) return;
  const uint64_t wend = d.payload_off + (uint64_t)d.words * 4;
  uint64_t x = (uint64_t)ld_u32_unaligned(j.in, d.payload_off) | ((uint64_t)ld_u32_unaligned(j.in, d.payload_off + 4) << 32);
  uint64_t xe;
  if (!dec_run(j, d, j.cum + (size_t)sid * j.cum_stride, j.bsym + (size_t)sid * 512, x, d.payload_off + 8, wend, 0, d.n,
               j.dsym + d.out_off, &xe) || xe != (1ull << 31))
    atomicOr(j.gerr, 4u);
}

// stored streams: MSB-first fixed-width fields
__global__ void k_dstored(DecJob j, int nstreams) {
  const int sid = blockIdx.x;
  const DecStream d = j.streams[sid];
  if (d.mode != SM_STORED) return;
  uint16_t* out = j.dsym + d.out_off;
  for (uint32_t i = threadIdx.x; i < d.n; i += blockDim.x)
    out[i] = (uint16_t)get_bits(j.in, d.payload_off * 8 + (uint64_t)i * d.maxbits, d.maxbits);
}

// LZ streams -> matches (un_lz.hpp:150-170); one lane per tile
__global__ void k_dlz(DecJob j) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= j.ntiles) return;
  DecTile ti = j.tiles[t];
  if (ti.err) return;
  const DecStream* st = j.streams + (size_t)t * SK_PER_TILE;
  const uint16_t* fut = j.dsym + st[0].out_off;
  const uint16_t* len = j.dsym + st[1].out_off;
  const uint16_t* bb = j.dsym + st[2].out_off;
  uint32_t* mt = j.matches + (size_t)t * 3 * (j.lz_cap + 1);
  const uint32_t npix = (uint32_t)ti.w * ti.h;
  uint32_t idx = 0, g = 0, nm = 0;
  bool bad = false;
  for (uint32_t i = 0; i < st[0].n; i++) {
    const uint32_t v = fut[i];
    if (v == 255) { idx += 255; continue; }
    idx += v;
    if (g >= st[1].n || g >= st[2].n || nm >= j.lz_cap) { bad = true; break; }
    const uint32_t L = len[g] + 4, back = bb[g];
    g++;
    if (back == 0 || back > idx || idx + L > npix) { bad = true; break; }
    mt[3 * nm] = idx; mt[3 * nm + 1] = L; mt[3 * nm + 2] = back;
    nm++;
    idx += L;
  }
  if (idx > npix) bad = true;
  ti.nmatch = nm;
  if (bad) { ti.err = 1; atomicOr(j.gerr, 1u); }
  j.tiles[t] = ti;
}

__device__ __forceinline__ uint16_t dmed16(uint16_t a, uint16_t b, uint16_t c) {
  if (a > b) return b > c ? b : (c > a ? a : c);
  return b < c ? b : (c > a ? c : a);
}

// Tiles without LZ matches: wavefront.  Each of 3 waves decodes one plane; a band of 64 rows is
// swept along anti-diagonals (lane = row in band, step t decodes x = t - lane), T/TL come from
// the lane above via DPP-free __shfl_up of the previous step, row -1 of a band from LDS.
// Tiles with matches (rare) use a serial raster loop per plane (LZ copies can point up-right).
#define BAND 64
__global__ __launch_bounds__(192) void k_dunpred(DecJob j) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int t = blockIdx.x;
  const DecTile ti = j.tiles[t];
  if (ti.err) return;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int w = ti.w, h = ti.h;
  const int depth = wv ? 9 : 8, c = 1 << depth, half = c / 2;
  const int BR = j.band;
  uint16_t* band = (uint16_t*)lds + (size_t)wv * BR * w;         // decoded band of this plane
  uint16_t* prevrow = (uint16_t*)lds + (size_t)3 * BR * w + (size_t)wv * w;
  const uint16_t* res = j.dsym + (size_t)(t * 3 + wv) * j.npix_cap;
  const DecStream d = j.streams[t * SK_PER_TILE + 3 + wv];
  if (ti.nmatch == 0) {
    if (d.n != (uint32_t)(w * h)) { if (threadIdx.x == 0) atomicOr(j.gerr, 1u); return; }
    for (int r0 = 0; r0 < h; r0 += BR) {
      const int y = r0 + lane;
      const bool act = y < h && lane < BR;
      uint32_t cur = 0, prev = 0;        // this lane's value at steps t-1 and t-2
      for (int st = 0; st < w + j.band - 1; st++) {
        const int x = st - lane;
        // values of the lane above at steps st-1 (x, y-1) and st-2 (x-1, y-1)
        const uint32_t up1 = __shfl_up(cur, 1), up2 = __shfl_up(prev, 1);
        if (act && x >= 0 && x < w) {
          uint16_t T, TL;
          if (y == 0) { T = half; TL = half; }
          else if (lane == 0) { T = prevrow[x]; TL = x ? prevrow[x - 1] : (uint16_t)half; }
          else { T = (uint16_t)up1; TL = x ? (uint16_t)up2 : (uint16_t)half; }
          const uint16_t L = x ? (uint16_t)cur : (uint16_t)half;
          const uint16_t p = dmed16(T, L, (uint16_t)(T + L - TL));
          const uint16_t v = (uint16_t)((res[(size_t)y * w + x] + p - half + c) & (c - 1));
          band[lane * w + x] = v;
          prev = cur;
          cur = v;
        }
      }
      __syncthreads();
      // row r0+63 (or the last row) becomes row -1 of the next band
      const int last = min(BR, h - r0) - 1;
      for (int x = lane; x < w; x += 64) prevrow[x] = band[last * w + x];
      // inverse subtract-green for this band once all three planes are done
      uint16_t* bG = (uint16_t*)lds;
      uint16_t* bR = bG + BR * w;
      uint16_t* bB = bR + BR * w;
      const int rows = last + 1;
      for (int i = threadIdx.x; i < rows * w; i += 192) {
        const int yy = i / w, xx = i % w;
        const uint16_t G = bG[i], R = bR[i], B = bB[i];
        uint8_t* o = j.rgb + ((size_t)(ti.y0 + r0 + yy) * j.W + ti.x0 + xx) * 3;
        o[0] = (uint8_t)(R + G - 256); o[1] = (uint8_t)G; o[2] = (uint8_t)(B + G - 256);
      }
      __syncthreads();
    }
    return;
  }
  // serial path (tiles with LZ matches): lane 0 of each wave walks its plane in raster order
  const uint32_t* mt = j.matches + (size_t)t * 3 * (j.lz_cap + 1);
  uint16_t* plane = j.dplane + (size_t)(t * 3 + wv) * j.npix_cap;
  if (lane == 0) {
    uint32_t k = 0, m = 0, nm = ti.nmatch;   // residuals are consumed by the non-matched pixels
    for (int y = 0; y < h; y++) {
      for (int x = 0; x < w; x++) {
        const uint32_t i = (uint32_t)y * w + x;
        while (m < nm && mt[3 * m] + mt[3 * m + 1] <= i) m++;
        uint16_t v;
        if (m < nm && mt[3 * m] <= i) {
          v = plane[i - mt[3 * m + 2]];
        } else {
          const uint16_t r = res[k++];
          const uint16_t L = x ? plane[i - 1] : (uint16_t)half;
          const uint16_t T = y ? plane[i - w] : (uint16_t)half;
          const uint16_t TL = (x && y) ? plane[i - w - 1] : (uint16_t)half;
          const uint16_t p = dmed16(T, L, (uint16_t)(T + L - TL));
          v = (uint16_t)((r + p - half + c) & (c - 1));
        }
        plane[i] = v;
      }
    }
    if (k != d.n) atomicOr(j.gerr, 1u);
  }
  __syncthreads();
  const uint16_t* G = j.dplane + (size_t)(t * 3) * j.npix_cap;
  const uint16_t* R = G + j.npix_cap;
  const uint16_t* B = R + j.npix_cap;
  for (int i = threadIdx.x; i < w * h; i += 192) {
    const int yy = i / w, xx = i % w;
    uint8_t* o = j.rgb + ((size_t)(ti.y0 + yy) * j.W + ti.x0 + xx) * 3;
    o[0] = (uint8_t)(R[i] + G[i] - 256); o[1] = (uint8_t)G[i]; o[2] = (uint8_t)(B[i] + G[i] - 256);
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
    w.sizes[k] = bytes;
  }
  *p = w.bufs[k];
  return 0;
}

static int decode_run(hoh_ctx* c, DecJob& j, const hoh_index* idx, hipStream_t s);

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

static int decode_run(hoh_ctx* c, DecJob& j, const hoh_index* idx, hipStream_t s) {
  j.npix_cap = (uint32_t)(((size_t)j.tw * j.th + 63) / 64 * 64);
  j.lz_cap = (uint32_t)((j.npix_cap / 4 + j.npix_cap / 255 + 16 + 7) / 8 * 8);
  const int S = j.ntiles * SK_PER_TILE;
  DecWork& w = ctx_dec(c);
  void* q;
  int e;
  if ((e = dbuf(w, 0, (size_t)j.ntiles * sizeof(DecTile), &q))) return e; j.tiles = (DecTile*)q;
  if ((e = dbuf(w, 1, (size_t)S * sizeof(DecStream), &q))) return e; j.streams = (DecStream*)q;
  j.cum_stride = 513;
  if ((e = dbuf(w, 2, (size_t)S * 513 * 4, &q))) return e; j.cum = (uint32_t*)q;
  if ((e = dbuf(w, 3, (size_t)S * 512 * 2, &q))) return e; j.bsym = (uint16_t*)q;
  if ((e = dbuf(w, 4, ((size_t)j.ntiles * 3 * j.npix_cap + (size_t)j.ntiles * 3 * j.lz_cap) * 2, &q))) return e; j.dsym = (uint16_t*)q;
  if ((e = dbuf(w, 5, (size_t)j.ntiles * 3 * (j.lz_cap + 1) * 4, &q))) return e; j.matches = (uint32_t*)q;
  if ((e = dbuf(w, 6, 64, &q))) return e; j.gerr = (uint32_t*)q;
  if ((e = dbuf(w, 7, (size_t)j.ntiles * 3 * j.npix_cap * 2, &q))) return e; j.dplane = (uint16_t*)q;
  j.ix = index_streams(idx);
  j.ck = index_ckpts(idx);
  j.nix = index_nstreams(idx);
  const int indexed = j.ix && j.nix == S;
  if (hipMemsetAsync(j.gerr, 0, 64, s) != hipSuccess) return 3;
  if (hipMemsetAsync(j.streams, 0, (size_t)S * sizeof(DecStream), s) != hipSuccess) return 3;
  ctx_mark(c, s, "start", true);
  hipLaunchKernelGGL(k_dtable, dim3(1), dim3(64), 0, s, j);
  ctx_mark(c, s, "dtable", false);
  hipLaunchKernelGGL(k_dparse, dim3(j.ntiles), dim3(64), 0, s, j);
  ctx_mark(c, s, "dparse", false);
  if (indexed) {
    hipLaunchKernelGGL(k_dmatch, dim3((S + 255) / 256), dim3(256), 0, s, j, S);
    hipLaunchKernelGGL(k_drans, dim3(S), dim3(64), 0, s, j, S, 1);
  } else {
    hipLaunchKernelGGL(k_drans, dim3((S + 63) / 64), dim3(64), 0, s, j, S, 0);
  }
  ctx_mark(c, s, "drans", false);
  hipLaunchKernelGGL(k_dstored, dim3(S), dim3(256), 0, s, j, S);
  hipLaunchKernelGGL(k_dlz, dim3((j.ntiles + 63) / 64), dim3(64), 0, s, j);
  ctx_mark(c, s, "dlz", false);
  j.band = BAND;
  while (j.band > 1 && (size_t)3 * j.band * j.tw * 2 + (size_t)3 * j.tw * 2 > 160 * 1024) j.band /= 2;
  const size_t lds = (size_t)3 * j.band * j.tw * 2 + (size_t)3 * j.tw * 2;
  hipLaunchKernelGGL(k_dunpred, dim3(j.ntiles), dim3(192), lds, s, j);
  ctx_mark(c, s, "dunpred", false);
  if (hipGetLastError() != hipSuccess) return 3;
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
  const int lane = threadIdx.x;
  uint64_t p = bp;
  const bool ok = parse_stream(j, p, 0, 0, lane);
  __syncthreads();
  if (lane != 0) return;
  if (!ok) { res[0] = 1; return; }
  const DecStream d = j.streams[0];
  res[1] = d.n;
  if (d.mode == SM_RANS) {
    const uint64_t wend = d.payload_off + (uint64_t)d.words * 4;
    uint64_t x = (uint64_t)ld_u32_unaligned(j.in, d.payload_off) | ((uint64_t)ld_u32_unaligned(j.in, d.payload_off + 4) << 32);
    uint64_t xe;
    if (!dec_run(j, d, j.cum, j.bsym, x, d.payload_off + 8, wend, 0, d.n, j.dsym, &xe) || xe != (1ull << 31)) {
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
  hipLaunchKernelGGL(k_dstream, dim3(1), dim3(64), 0, s, j, (uint64_t)*bp, res);
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
