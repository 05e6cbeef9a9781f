// Internal definitions shared by the HIP kernels and the host orchestration of libhohgpu.
// Device code is written for gfx950 (wave64, 160 KiB LDS per CU).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <stdlib.h>

// Measurement knobs (A/B runs of tools/scripts only).  The product library has one schedule: a
// knob is its compile-time default.  A library built with -DHOH_KNOBS (`make KNOBS=1`, or
// tools/scripts/mkvar.sh ... -DHOH_KNOBS) reads HOH_<name> from the environment once per site.
#ifdef HOH_KNOBS
static inline int hoh_knob_env(const char* name, int def) { const char* e = getenv(name); return e ? atoi(e) : def; }
#define HOH_KNOB(name, def) ([] { static const int v_ = hoh_knob_env("HOH_" #name, (def)); return v_; }())
#else
#define HOH_KNOB(name, def) (def)
#endif

#define HOH_WAVE 64
#define HOH_HDR_CAP 1600          // bytes reserved per stream for varints + meta + table
#define HOH_FAST_RANGE 512        // LDS-table fast encoder handles range <= 512 at prob_bits 15
// entries per stream of the fast encoder's table (a skew of 2-16 entries against the L1 sets
// measured no different: profiles/r06/ab_chain_placement_and_table_skew.txt)
#ifndef HOH_FAST_STRIDE
#define HOH_FAST_STRIDE HOH_FAST_RANGE
#endif
#define HOH_SEG 256               // decode checkpoint spacing (symbols)
#define HOH_MAX_TILE_W 65535
#define HOH_LZ_WINDOW 64          // -s0 seek distance 6 -> 1 << 6 pixels back (choh.cpp:125, lz.hpp:20)

// stream kinds inside a tile (stream id = tile * SK_PER_TILE + kind); SK_I is the indexed
// (palette) plane that competes with the three sub-green planes (choh.cpp:298-308)
enum { SK_LZ_FUTURE = 0, SK_LZ_LENGTH = 1, SK_LZ_BACKBY = 2, SK_G = 3, SK_R = 4, SK_B = 5, SK_I = 6,
       SK_PER_TILE = 7 };

// -s1..-s4 stream kinds (stream id = tile * SPT_S + kind).  Planes p: 0 G, 1 R', 2 B' (sub-green),
// 3 indexed (palette candidates), 4 R, 5 B (plain, -s>=3 RGB mode, choh.cpp:265-293)
enum { KS_LZ = 0,          // 4 LZ streams (lz.hpp:100-142, backby2 at distance > 8)
       KS_MED = 4,         // + p: MED fast-path residuals at prob_bits 15 (layer_encode.hpp:106-120)
       KS_FIN = 10,        // + p: searched residuals at the winning prob_bits (full encode)
       KS_MAP = 16,        // + p: predictor map stream (layer_encode.hpp:308-317)
       KS_VAR = 22,        // + p * 8 + v: searched residuals, size-only, prob_bits kVarPb[v]
       SPT_S = 70 };
#define HOH_NPLANE_S 6
#define HOH_MAPCAP 176     // cells of the 40-px grid: ceil(511 / 40)^2 = 169, rounded to 8

struct PlaneInfo {         // one -s>=1 layer (layer_encode.hpp:11-412)
  uint32_t present;
  uint32_t depth;
  uint32_t xt, yt;         // predictor grid (0 = no grid: 00 00 00 10 header)
  uint32_t used;           // distinct masks used
  uint32_t used_bits;      // bit j: stock mask j used
  uint32_t fixed_len;      // 0x10 + fixed header bytes before the map stream
  uint32_t possible;       // bytes of the permanent buffer that reach the layer
  uint32_t perm_final;     // 1: the permanent buffer is the KS_FIN stream, 0: KS_MED (prefix)
  uint32_t valid;          // 0: permanent holds uninitialised bytes
  uint32_t size;           // layer bytes
  uint32_t limit;          // bytes of this layer that reach the tile (Q15 prefix), else size
  uint64_t out_off;        // file offset of the layer
};

// stream coding modes (entropy_encoding.hpp)
enum { SM_EMPTY = 0, SM_RANS = 1, SM_STORED = 2 };

// tile flags
enum {
  TF_GREY = 1,            // R == G == B everywhere (channel.hpp:21-31)
  TF_BINARY = 2,          // grey with <= 2 values -> bitimage mode 0, no plane data
  TF_PALETTE_CAND = 4,    // <= 256 colours: palette_encode competes (choh.cpp:298-308)
  TF_UNREPRODUCIBLE = 8,  // the reference copies uninitialised bytes for this tile
  TF_UNSUPPORTED = 16,
  TF_OVERFLOW = 32        // an internal capacity was exceeded
};

struct StreamInfo {
  uint64_t sym_off;       // element offset of the symbols in the u16 symbol arena (16-B aligned)
  uint64_t slab_off;      // word offset of this stream's rANS slab
  uint64_t out_off;       // byte offset of the stream in the output buffer
  uint32_t n;             // symbol count
  uint32_t range;         // alphabet size
  uint32_t pb;            // prob_bits (scale bits)
  uint32_t slab_cap;      // words available in the slab
  uint32_t hdr_len;       // varint(range-1) varint(n) meta table  (rANS form)
  uint32_t vlen;          // bytes of the two header varints
  uint32_t maxbits;       // bits of (range - 1)
  uint32_t words;         // rANS words including the 2 flush words
  uint32_t widx_end;      // final slab index of the first payload word
  uint32_t mode;          // SM_*
  uint32_t size;          // final coded bytes of the stream
  uint32_t err;           // nonzero: error code
  uint64_t expected_stored;
  uint32_t fast;          // encoded by the LDS-table fast kernel
  uint32_t ckpt_off;      // index of the first checkpoint of this stream
  uint32_t drop;          // coded but not part of the file (losing colour mode)
  uint32_t clip;          // nonzero: only the first clip bytes go to the file (Q15 prefix)
  uint32_t sizeonly;      // rANS state chain only: words counted, none stored (2: pruned, words = wlo;
                          //   3: a kept trial that stores its words in the trial pool; 4: the
                          //   layer's final stream whose words a stored trial already holds)
  uint32_t hist_src;      // 0: count the symbols; k + 1: the histogram of stream k
  uint32_t wlo, whi;      // size-only trials: bounds on words (k_tables, from the code length)
};

struct TileInfo {
  int32_t x0, y0, w, h;   // tile rectangle inside the image
  int32_t colours;        // distinct colours (<= 256) or -1 (choh.cpp:17-46)
  uint32_t flags;         // TF_*
  uint32_t nmatch;        // LZ matches taken
  uint32_t ncand;         // LZ candidate positions
  uint32_t size;          // tile bytes
  uint32_t lz_bytes;      // 1 + the three LZ stream sizes
  uint64_t off;           // output byte offset of the tile
  uint32_t mode;          // internal colour mode byte (128 sub-green, 127 indexed, 0 bitimage)
  uint32_t pad;           // layout: byte offset of this tile's size varint
  uint32_t nclean;        // -s>=1: pixels outside LZ copies
  uint32_t nfut;          // -s>=1: symbols of the LZ "future" stream
  uint32_t chmap;         // -s>=1: layers of channels 1..3 (plane index, 4 bits each)
  uint32_t pad2;
};

struct Checkpoint {       // encoder state after coding symbol k*HOH_SEG == decoder state before it
  uint32_t xl, xh;
  uint32_t widx;          // slab index of the next word the decoder reads
  uint32_t pad;
};

struct EncFast {          // fast encoder symbol (16 B): quotient by exact f64 reciprocal
  double inv;             // 1/f rounded up by two ulps
  uint32_t f;
  uint32_t c;             // cumulative start
};

struct EncGen {           // generic encoder symbol: rans64.hpp Rans64EncSymbol layout
  uint64_t rcp;
  uint32_t freq, bias, cmpl, shift;
};

#ifdef __HIPCC__
// maximum over the 64 lanes (every lane active), in registers: DPP within rows of 16 (xor 1,
// xor 2, half mirror, mirror), then the four row maxima by readlane (a __shfl_xor tree is 6
// dependent LDS permute round trips per call; the scan calls this once per candidate)
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xf, 0xf, false));
  const uint32_t a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
  const uint32_t c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
  return max(max(a, b), max(c, d));
}

#endif

__host__ __device__ inline uint32_t hoh_varint_len(uint64_t v) {
  return v < (1u << 7) ? 1u : v < (1u << 14) ? 2u : v < (1u << 21) ? 3u : 0u;   // varint.hpp:29-45 (Q2)
}

__host__ __device__ inline uint32_t hoh_write_varint(uint8_t* b, uint32_t loc, uint64_t v) {
  if (v < (1u << 7)) {
    b[loc++] = (uint8_t)v;
  } else if (v < (1u << 14)) {
    b[loc++] = (uint8_t)((v >> 7) + 128);
    b[loc++] = (uint8_t)(v % 128);
  } else if (v < (1u << 21)) {
    b[loc++] = (uint8_t)((v >> 14) + 128);
    b[loc++] = (uint8_t)(((v >> 7) % 128) + 128);
    b[loc++] = (uint8_t)(v % 128);
  }
  return loc;
}

__host__ __device__ inline uint32_t hoh_bitlen(uint64_t v) {
  uint32_t b = 0;
  for (; v; v >>= 1) b++;
  return b;
}

// ---------------------------------------------------------------- kernel launch declarations

struct EncodeJob {
  // image
  const uint8_t* rgb;
  int W, H;
  int xt, yt, tw, th;     // tiling (choh.cpp:454-461)
  int t0, ntiles;         // tiles [t0, t0 + ntiles) of the image are coded
  uint32_t npix_cap;      // max pixels of one tile (per-plane stride of the residual arena)
  uint32_t lz_cap;        // symbols per LZ stream slot
  int speed;              // cruncher_mode (-sN)
  int spt;                // streams per tile: SK_PER_TILE (-s0) or SPT_S
  // arenas
  uint16_t* sym;          // residual planes + LZ symbols
  uint32_t* hist;         // [stream][512]
  uint64_t* candbits;     // [tile][npix_cap/64] LZ candidate bitmap
  uint32_t* matches;      // [tile][lz_cap] packed (pos, len, back) triples (3 words each)
  uint32_t* lzspec;       // [tile][lz_cap] k_lz's segment walks: pos | (len - 4) << 16 | (back - 1) << 24
  uint32_t* palette;      // [tile][256] colours in first-occurrence order (palette tiles)
  int32_t* ncol;          // [tile] distinct colours (<= 256) or -1 (k_colours)
  uint8_t* idx8;          // -s>=1: [tile][npix_cap] palette indices (the indexed plane's data)
  uint32_t* fpb;          // -s>=1: [tile][npix_cap] 4-pixel window fingerprints (LZ)
  uint32_t* tpx;          // -s>=1: [tile][npix_cap] the tile's pixels in tile raster order (LZ): rgb | run8 << 24
  uint32_t* fpt;          // -s>=1: [tile][npix_cap] the fingerprints transposed, FT[x * h + y] (k_lzfp)
  uint8_t* run8;          // -s>=1: [tile][npix_cap] length of the run of equal pixels from each position
                          //   (tile raster order, 1..254 exact, 255 = at least 255)
  uint32_t* lzs;          // -s>=1, tiles <= 65536 px: [tile][npix_cap] k_lzsort's first-pass entries (u64); null: no
                          //   posting lists.  The lists themselves are lzsf: positions grouped by
                          //   hash16(fingerprint), ascending inside a group
  uint16_t* lzrank;       //   [tile][npix_cap] index of each position in lzsf (flat run-inner positions: their run start's)
  uint32_t lzs_hmask;     //   the posting hash's mask (0xffff; knob LZS_HMASK in measurement builds)
  int cus;                // compute units of the device (k_lzsort's grid: one tile workgroup per CU; k_nuke's)
  uint16_t* lzend;        //   [tile][npix_cap] per lzsf entry: the last position of a flat run start's run, else the position
  uint64_t* lzsf;         //   [tile][npix_cap] the listed positions in order: key (pos | hash << 16) | fingerprint << 32
  PlaneInfo* pinfo;       // -s>=1: [tile][6]
  uint32_t* trials;       // -s>=1 with ladder pruning: the sids of the trials k_prune_s keeps (else null)
  uint32_t* ntrial;       // their count (zeroed per encode)
  const double* lg;       // -s>=1: -log2(k / n) for k = 0..n+1, one table per tile pixel count
  uint32_t lg_n[4];
  uint64_t lg_off[4];
  StreamInfo* streams;    // [ntiles * SK_PER_TILE]
  TileInfo* tiles;        // [ntiles]
  uint8_t* hdr;           // [stream][HOH_HDR_CAP]
  EncFast* tab_fast;      // [stream][HOH_FAST_STRIDE]
  int tab_wide;           // tab_fast passes 4 GB: the chains address each lane's table through 64 bits
  EncGen* tab_gen;        // [stream][gen_stride] (generic streams)
  uint32_t gen_stride;    // entries per stream in tab_gen (>= range)
  uint32_t hdr_cap;       // bytes per stream in hdr
  uint32_t* slabs;        // rANS words
  uint64_t slab_words;    // words in slabs (bounds of the encoder's indexed stores; 0 = unchecked)
  Checkpoint* ckpt;
  uint32_t* gerr;         // global error word
  uint32_t* dbg;          // measurement builds only (HOH_DEBUG_READ): [tile][64] counters, else null
  uint32_t exp;           // measurement what-ifs (knob EXP, knob builds only; 0 in the product): output invalid
  // -s>=1: the ladder trials k_prune_s keeps that could win the layer (KS_VAR + p*8 + 2..7) store
  // their words in a pool of the slab arena (sizeonly 3), so the winner is not encoded a second
  // time: words [tpool_off, tpool_off + tpool_words) of slabs, bump-allocated through *tpool_head
  uint64_t tpool_off, tpool_words;
  unsigned long long* tpool_head;
  uint64_t* total;        // total bytes of the tile blob
  uint32_t* tile_sizes;   // out: per tile bytes (may be null)
  uint8_t* out;           // output: [prefix bytes][tile size table][tiles]
  uint64_t cap;
  uint64_t prefix;        // bytes before the tile size table (file header, written by the host)
  int write_table;        // write the n-1 tile size varints (a whole .hoh); 0 for a shard blob
  // batch of images (hoh_encode_images_async): the job's image is the stack of nimg images of one
  // shape (their tile rows follow each other), and each image's tiles form a file of their own
  int nimg;               // images (1: one image or shard)
  int img_tiles;          // tiles per image
  uint64_t out_stride;    // bytes from one image's file to the next in out
  uint64_t* img_total;    // [nimg] each file's bytes (nimg > 1; else *total)
  uint32_t* img_err;      // [nimg] TF_* flags of each image's tiles (nimg > 1; else in gerr)
};

// A batch stacks when the image is tiled (choh.cpp:454-461) with tile rows of exactly 256: then
// n images one after another in memory are the tiles of the n*H image (whose tiling is the same
// 256-row grid), tile row for tile row.
inline int batch_stacks(int W, int H) { return (W >= 512 || H >= 512) && W >= 256 && H >= 256 && H % 256 == 0; }

// the image of tile t and the base of its file in out
__host__ __device__ inline int tile_img(const EncodeJob& j, int t) { return j.nimg > 1 ? t / j.img_tiles : 0; }
// a batch image's file is written only when it fits its stride and none of its tiles failed
__device__ __forceinline__ bool file_ok(const EncodeJob& j, int t) {
  if (*j.gerr) return false;
  if (j.nimg <= 1) return *j.total <= j.cap;
  const int img = tile_img(j, t);
  return j.img_total[img] <= j.out_stride && !j.img_err[img];
}

// arena offsets (elements / words): [tile][3] planes, [tile][3] LZ streams, [tile] indexed plane
__host__ __device__ inline size_t idx_plane_off(const EncodeJob& j, int t) {
  return (size_t)j.ntiles * 3 * (j.npix_cap + j.lz_cap) + (size_t)t * j.npix_cap;
}
__host__ __device__ inline size_t idx_slab_off(const EncodeJob& j, int t) {
  return (size_t)j.ntiles * 3 * (j.npix_cap + 8 + j.lz_cap + 8) + (size_t)t * (j.npix_cap + 8);
}

// MED residual plane p of tile t and the kind of its stream / histogram
__host__ __device__ inline size_t med_plane_off(const EncodeJob& j, int t, int p) {
  if (j.speed == 0) return p < 3 ? (size_t)(t * 3 + p) * j.npix_cap : idx_plane_off(j, t);
  return (size_t)(t * HOH_NPLANE_S + p) * j.npix_cap;
}
__host__ __device__ inline int med_kind(const EncodeJob& j, int p) { return (j.speed == 0 ? SK_G : KS_MED) + p; }

// -s>=1 arenas: sym = [t][6] MED | [t][6] searched | [t][4][lz_cap] LZ | [t][6][MAPCAP] maps;
// slabs = [t][6] planes | [t][4] LZ | [t][6] maps
__host__ __device__ inline size_t fin_plane_off(const EncodeJob& j, int t, int p) {
  return (size_t)j.ntiles * HOH_NPLANE_S * j.npix_cap + (size_t)(t * HOH_NPLANE_S + p) * j.npix_cap;
}
__host__ __device__ inline size_t lz_sym_off_s(const EncodeJob& j, int t, int k) {
  return (size_t)j.ntiles * 2 * HOH_NPLANE_S * j.npix_cap + (size_t)(t * 4 + k) * j.lz_cap;
}
__host__ __device__ inline size_t map_sym_off(const EncodeJob& j, int t, int p) {
  return (size_t)j.ntiles * (2 * HOH_NPLANE_S * (size_t)j.npix_cap + 4 * (size_t)j.lz_cap) +
         (size_t)(t * HOH_NPLANE_S + p) * HOH_MAPCAP;
}
__host__ __device__ inline size_t sym_total_s(int ntiles, uint32_t npix_cap, uint32_t lz_cap) {
  return (size_t)ntiles * (2 * HOH_NPLANE_S * (size_t)npix_cap + 4 * (size_t)lz_cap + HOH_NPLANE_S * HOH_MAPCAP);
}
__host__ __device__ inline size_t plane_slab_off_s(const EncodeJob& j, int t, int p) {
  return (size_t)(t * HOH_NPLANE_S + p) * (j.npix_cap + 8);
}
__host__ __device__ inline size_t lz_slab_off_s(const EncodeJob& j, int t, int k) {
  return (size_t)j.ntiles * HOH_NPLANE_S * (j.npix_cap + 8) + (size_t)(t * 4 + k) * (j.lz_cap + 8);
}
__host__ __device__ inline size_t map_slab_off_s(const EncodeJob& j, int t, int p) {
  return (size_t)j.ntiles * (HOH_NPLANE_S * ((size_t)j.npix_cap + 8) + 4 * ((size_t)j.lz_cap + 8)) +
         (size_t)(t * HOH_NPLANE_S + p) * (HOH_MAPCAP + 8);
}
__host__ __device__ inline size_t slab_total_s(int ntiles, uint32_t npix_cap, uint32_t lz_cap) {
  return (size_t)ntiles * (HOH_NPLANE_S * ((size_t)npix_cap + 8) + 4 * ((size_t)lz_cap + 8) + HOH_NPLANE_S * (HOH_MAPCAP + 8));
}

// stream subsets: sid(i) = (i / per) * spt + base + i % per (per == 0: sid = i)
struct SidMap { int per, base; };
__host__ __device__ inline int map_sid(const SidMap& m, int spt, int i) {
  return m.per ? (i / m.per) * spt + m.base + i % m.per : i;
}

void launch_front(const EncodeJob& j, hipStream_t s);
void launch_palette(const EncodeJob& j, hipStream_t s);
void launch_lz(const EncodeJob& j, hipStream_t s);
void launch_tables(const EncodeJob& j, int nstreams, hipStream_t s, SidMap m = SidMap{0, 0});
// kind 0: prob_bits-15 streams; 1: any prob_bits 7..19; 2: the same, size-only trial encodes
void launch_rans_fast(const EncodeJob& j, int nplane, hipStream_t s, SidMap a, int na, SidMap b, int kind = 0);
void launch_rans_fast_s(const EncodeJob& j, hipStream_t s, int np0, SidMap a0, int na0, SidMap b0, int np2, SidMap a2,
                        int na2, int np1, SidMap a1, int na1);
void launch_rans_fast01(const EncodeJob& j, hipStream_t s, int np0, SidMap a0, int na0, SidMap b0, int np1, SidMap a1,
                        int na1, SidMap b1);
void launch_rans_gen(const EncodeJob& j, int nstreams, hipStream_t s, SidMap m = SidMap{0, 0});
void launch_finalize(const EncodeJob& j, int nstreams, hipStream_t s, SidMap m = SidMap{0, 0});
void launch_nuke(const EncodeJob& j, hipStream_t s);
struct SideStream {        // a context's second stream for work that forks off the main one
  hipStream_t s = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
};
void encode_speed_s(const EncodeJob& j, hipStream_t s, const SideStream& side, void (*mark)(void*, const char*), void* mctx);
void launch_layout(const EncodeJob& j, hipStream_t s);
void launch_assemble(const EncodeJob& j, int nstreams, hipStream_t s);
void launch_streambytes(const EncodeJob& j, int nstreams, hipStream_t s);
