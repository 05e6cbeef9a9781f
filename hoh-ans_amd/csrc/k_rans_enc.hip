// rANS encoders (rans64.hpp:65-103, :262-278; entropy_encoding.hpp:206-238).
//
// Bit-exactness forces one serial coder state per stream (the reference never interleaves), so
// the encoder is a chain of 65,536 dependent steps per 256x256 tile plane, and one wave issues
// one instruction every ~6 cycles: the chain's length is its instruction count.  The fast
// kernel therefore spends all its effort on instructions per step:
//  * one stream per lane, 64 streams per wave; the symbol tables (16-B entries: 1/f as
//    f64, f, c) are gathered from global memory (L2-resident, ~8 KB per stream) one 8-symbol
//    block ahead through 32-bit offsets from one scalar base (two symbol offsets per packed
//    16-bit shift);
//  * the quotient floor(x/f) of the reciprocal step is computed exactly with two f64
//    multiplications by 1/f rounded up one ulp (the high word first, then remainder*2^32 +
//    low word, both < 2^53: exact floors), which is mathematically identical to the Alverson
//    reciprocal of Rans64EncPutSymbol; the new low word is x_lo + c + ql*(2^15 - f);
//  * each step writes its speculative output word to an LDS window and adds the renorm decision
//    to a bit mask (one add-with-carry); once per 32 steps only the emitted words are copied to
//    the slab.  (Storing every speculative word straight to the slab at the next output slot
//    removes the mask and the flush loop but costs a scattered 64-lane store per step: measured
//    40% slower.)
// The generic kernel (LZ streams, other prob_bits) is the reference reciprocal step verbatim.
// Both record decode checkpoints every HOH_SEG symbols (Recoil-style side index; the .hoh bytes
// are unaffected).
#include "hoh_internal.h"

#include <algorithm>
#include <cstdlib>
#include <atomic>

#define WIN 32
// lane row pitch of the LDS window in dwords: odd, so the 64 lanes' writes of one step fall in 64
// different banks (a 32-dword pitch put every lane in one of two banks: a 32-way conflict per write)
#ifndef WIN_PITCH
#define WIN_PITCH (WIN + 1)
#endif
typedef unsigned short us2 __attribute__((ext_vector_type(2)));

// plane index -> stream: [0, na) through map a, then map b (e.g. the sub-green planes of every
// tile first, the rarely present indexed planes after them, so idle lanes share few waves)
__device__ __forceinline__ uint32_t plane_sid(int pi, int spt, SidMap a, int na, SidMap b) {
  return pi < na ? map_sid(a, spt, pi) : map_sid(b, spt, pi - na);
}

// byte offsets (from the table base) of the entries of 8 packed u16 symbols
__device__ __forceinline__ void offs8(uint32_t* o, uint4 w, uint32_t base) {
  const uint32_t d[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t t = __builtin_bit_cast(uint32_t, __builtin_bit_cast(us2, d[k]) << (us2)(4));
    uint32_t lo;
    asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:DWORD"
        : "=v"(lo) : "v"(t), "v"(base));        // base + low half: one instruction
    o[2 * k] = lo;
    o[2 * k + 1] = base + (t >> 16);
  }
}

__device__ __forceinline__ EncFast ent(const char* tb, uint32_t off) { return *(const EncFast*)(tb + off); }

__device__ __forceinline__ void lookup8(EncFast* e, uint4 sy, const char* tb, uint32_t base) {
  uint32_t o[8];
  offs8(o, sy, base);
#pragma unroll
  for (int k = 0; k < 8; ++k) e[k] = ent(tb, o[k]);
}

struct Coder {
  uint32_t xh, xl, mask, slot;
  uint32_t widx;
  uint32_t* slab;
  uint32_t* win;
  uint32_t lost;          // trials (KIND 3): words not written (size-only lanes: all of them;
                          //   storing lanes: any past the slab's start), counted
  bool keep;              // trials (KIND 3): this lane stores its words
};

// copy the window's emitted words to the slab (backwards, rans64 order); GUARD (stored ladder
// trials, whose slab is sized by the word bound): a word that would land before the slab's start
// is counted in c.lost instead of written
template <bool GUARD = false>
__device__ __forceinline__ void flush_win(Coder& c) {
  uint32_t m = c.mask;
  const uint32_t shift = WIN - c.slot;
  while (m) {
    const uint32_t t = __builtin_clz(m) - shift;
    if (!GUARD || (c.keep && c.widx)) c.slab[--c.widx] = c.win[t];
    else c.lost++;
    m &= ~(0x80000000u >> (t + shift));
  }
  c.mask = 0;
  c.slot = 0;
}

// one step, prob_bits 15 (x_max = f << 48): the low word goes to the LDS window speculatively,
// the renormalisation decision into the mask
__device__ __forceinline__ void step15(Coder& c, const EncFast& e) {
  c.win[c.slot] = c.xl;
  const uint32_t f = e.f;
  // emit = x >= x_max, i.e. (x_hi >> 16) >= f; (nh, nl) = emit ? (0, x_hi) : (x_hi, x_lo); the
  // decision is shifted into the mask by an add-with-carry of the compare itself: 4 instructions
  uint32_t nh, nl;
  uint64_t co;                               // the add-with-carry's own carry-out (unused)
  asm("v_cmp_ge_u32_sdwa vcc, %[xh], %[f] src0_sel:WORD_1 src1_sel:DWORD\n\t"
      "v_addc_co_u32_e64 %[m], %[co], %[m], %[m], vcc\n\t"
      "v_cndmask_b32_e64 %[nh], %[xh], 0, vcc\n\t"
      "v_cndmask_b32_e32 %[nl], %[xl], %[xh], vcc"
      : [nh] "=&v"(nh), [nl] "=&v"(nl), [m] "+v"(c.mask), [co] "=&s"(co)
      : [xh] "v"(c.xh), [xl] "v"(c.xl), [f] "v"(f)
      : "vcc");
  // No int<->f64 conversion on the chain (they issue at half the f64 rate): the kernel runs with
  // f64 rounding toward zero (k_rans_fast sets MODE), so fma(m, inv, 2^52) = 2^52 + floor(m*inv)
  // exactly for every m*inv < 2^52, and its low word IS the quotient; integers m < 2^52 enter
  // f64 as the bit pattern {m_lo, 0x43300000 | m_hi} = 2^52 + m, minus 2^52 (exact).
  //   qh = floor(nh / f)               (nh < 2^31)
  //   rh = nh - qh*f                   (qh < 2^16, f <= 2^15: one 24-bit multiply)
  //   ql = floor((rh*2^32 + nl) / f)   (< 2^32)
  // The quotients equal the Alverson reciprocal's: inv = RN(1/f) + 1 ulp, so 1/f <= inv <=
  // (1/f)(1 + 1.5 * 2^-52): m*inv >= m/f, and m*inv - m/f < 2^32 * 1.5 * 2^-52 < 1/f for
  // m/f < 2^32 and f <= 2^19, so m*inv stays below floor(m/f) + 1 (m/f <= floor + 1 - 1/f).
  const double two52 = 4503599627370496.0;
  const double nhd = __builtin_bit_cast(double, ((uint64_t)0x43300000u << 32) | nh) - two52;
  const uint32_t qh = (uint32_t)__builtin_bit_cast(uint64_t, __builtin_fma(nhd, e.inv, two52));
  const uint32_t rh = nh - __umul24(qh, f);
  const double n2d = __builtin_bit_cast(double, ((uint64_t)(0x43300000u | rh) << 32) | nl) - two52;
  const uint32_t ql = (uint32_t)__builtin_bit_cast(uint64_t, __builtin_fma(n2d, e.inv, two52));
  c.xl = nl + e.c + ql * (32768u - f);
  c.xh = __builtin_amdgcn_alignbit(qh, ql, 17);
  c.slot++;
}

// Any prob_bits 7..19 (LZ streams at 10, predictor maps at 8, the -s>=1 ladder 12..19,
// layer_encode.hpp:326-391, lz.hpp:100-142): the same quotients with
// x_max = f << (63 - pb) tested as x_hi >= f << (31 - pb) (exact: f << (31 - pb) <= 2^31), the
// low word nl + c + ql * (2^pb - f) and the high word (q * 2^pb) >> 32 = alignbit(qh, ql, 32 - pb).
// The f64 floors stay exact for every f <= 2^19 (step15's bound: the quotients are < 2^32).
// Size-only encodes (SO: the ladder's trial streams) only count the emitted words.
struct PbShape {
  uint32_t sh, M, a32;       // 31 - pb, 2^pb, 32 - pb
};

template <bool SO>
__device__ __forceinline__ void stepg(Coder& c, const EncFast& e, const PbShape& g) {
  if (!SO) c.win[c.slot] = c.xl;
  const uint32_t f = e.f, fs = f << g.sh;
  uint32_t nh, nl;
  uint64_t co;
  if (SO) {
    asm("v_cmp_ge_u32_e32 vcc, %[xh], %[fs]\n\t"
        "v_addc_co_u32_e64 %[m], %[co], %[m], 0, vcc\n\t"
        "v_cndmask_b32_e64 %[nh], %[xh], 0, vcc\n\t"
        "v_cndmask_b32_e32 %[nl], %[xl], %[xh], vcc"
        : [nh] "=&v"(nh), [nl] "=&v"(nl), [m] "+v"(c.mask), [co] "=&s"(co)
        : [xh] "v"(c.xh), [xl] "v"(c.xl), [fs] "v"(fs)
        : "vcc");
  } else {
    asm("v_cmp_ge_u32_e32 vcc, %[xh], %[fs]\n\t"
        "v_addc_co_u32_e64 %[m], %[co], %[m], %[m], vcc\n\t"
        "v_cndmask_b32_e64 %[nh], %[xh], 0, vcc\n\t"
        "v_cndmask_b32_e32 %[nl], %[xl], %[xh], vcc"
        : [nh] "=&v"(nh), [nl] "=&v"(nl), [m] "+v"(c.mask), [co] "=&s"(co)
        : [xh] "v"(c.xh), [xl] "v"(c.xl), [fs] "v"(fs)
        : "vcc");
  }
  const double two52 = 4503599627370496.0;
  const double nhd = __builtin_bit_cast(double, ((uint64_t)0x43300000u << 32) | nh) - two52;
  const uint32_t qh = (uint32_t)__builtin_bit_cast(uint64_t, __builtin_fma(nhd, e.inv, two52));
  const uint32_t rh = nh - __umul24(qh, f);
  const double n2d = __builtin_bit_cast(double, ((uint64_t)(0x43300000u | rh) << 32) | nl) - two52;
  const uint32_t ql = (uint32_t)__builtin_bit_cast(uint64_t, __builtin_fma(n2d, e.inv, two52));
  c.xl = nl + e.c + ql * (g.M - f);
  c.xh = __builtin_amdgcn_alignbit(qh, ql, g.a32);
  if (!SO) c.slot++;
}

// KIND 0: prob_bits 15 (step15); 1: any prob_bits 12..19; 2: the same, size only; 3: the ladder
// trials of one launch (KIND 1's steps; a lane stores its words when its trial holds a pool slab,
// sizeonly 3, and only counts them otherwise -- one instruction stream for both kinds of lane)
template <int KIND>
__device__ __forceinline__ void stepk(Coder& c, const EncFast& e, const PbShape& g) {
  if (KIND == 0) step15(c, e);
  else stepg<KIND == 2>(c, e, g);
}

__device__ __forceinline__ void ckpt(const Coder& c, Checkpoint* ck, uint32_t k) {
  if (!ck) return;                          // no side index for this job
  Checkpoint p;
  p.xl = c.xl; p.xh = c.xh; p.widx = c.widx - __popc(c.mask); p.pad = 0;
  ck[k] = p;
}

template <int KIND, bool WIDE>
__device__ __forceinline__ void rans_fast_run(const EncodeJob& j, uint32_t sid, const StreamInfo& st);

// One lane per stream, 64 streams per wave, one wave per workgroup: block blk of a launch.
// WIDE: each lane's table through its own 64-bit address (jobs whose tables pass 4 GB: batched
// -s>=1 encodes); otherwise 32-bit offsets from one scalar base (the -s0 chains)
template <int KIND, bool WIDE = false>
__device__ __forceinline__ void rans_fast_body(const EncodeJob& j, int nplane, SidMap ma, int na, SidMap mb, int blk) {
  const int lane = threadIdx.x & 63;
  // the chain is the critical path of an image: win issue arbitration against co-resident waves
#ifndef CHAIN_PRIO
#define CHAIN_PRIO 3
#endif
  __builtin_amdgcn_s_setprio(CHAIN_PRIO);
  // f64 rounding toward zero (MODE.FP_ROUND[3:2] = 3) for step15's floor-by-fma, this wave only.
  // Set in asm so the compiler's mode tracking does not restore round-to-nearest before its own
  // f64 instructions: the only other f64 operations here are the exact 2^52 subtractions.
  asm volatile("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 2, 2), 3");
  const int pi = blk * 64 + lane;
  if (pi >= nplane) return;
  uint32_t sid;
  if (KIND == 2 && j.trials) {             // the ladder trials k_prune_s kept, packed
    if ((uint32_t)pi >= *j.ntrial) return;
    sid = j.trials[pi];
  } else {
    sid = plane_sid(pi, j.spt, ma, na, mb);
  }
  StreamInfo st = j.streams[sid];
  if (!st.fast || st.mode != SM_RANS || st.err || st.n == 0) return;
  // another launch's stream: KIND 0 real pb-15 encodes, 1 real encodes at other prob_bits, 2 every
  // size-only trial
  if ((KIND == 2) != (st.sizeonly != 0) || (KIND != 2 && (KIND == 0) != (st.pb == 15))) return;
  if (st.sizeonly == 2) return;            // pruned trial (k_prune_s): its words are set
  // trials: the storing chain for every lane when the pool is on (storing and counting lanes share
  // a wave: two kinds of chain in one wave would run one after the other)
  if (KIND == 2 && j.tpool_words) rans_fast_run<3, WIDE>(j, sid, st);
  else rans_fast_run<KIND, WIDE>(j, sid, st);
}

template <int KIND, bool WIDE>
__device__ __forceinline__ void rans_fast_run(const EncodeJob& j, uint32_t sid, const StreamInfo& st) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  constexpr bool GUARD = KIND == 3;
  const int lane = threadIdx.x & 63;
  const uint32_t n = st.n;
  const PbShape g{31u - st.pb, 1u << st.pb, 32u - st.pb};
  // what-if EXP & 1 (measurement, output invalid): the 64 lanes' tables of block 0 for every
  // wave, so every table gather hits L2
  const uint32_t tsid = (j.exp & 1) ? (uint32_t)lane : sid;
  const char* tb = (const char*)j.tab_fast + (WIDE ? (size_t)tsid * (HOH_FAST_STRIDE * sizeof(EncFast)) : 0);
  const uint32_t tbase = WIDE ? 0u : tsid * (uint32_t)(HOH_FAST_STRIDE * sizeof(EncFast));
  Coder c;
  c.xh = 0; c.xl = 1u << 31; c.mask = 0; c.slot = 0; c.lost = 0;
  c.keep = !GUARD || st.sizeonly == 3;
  const uint32_t cap = c.keep ? st.slab_cap : 0u;
  c.slab = j.slabs + (c.keep ? st.slab_off : 0);
  c.widx = cap;
  c.win = (uint32_t*)(lds + threadIdx.x * WIN_PITCH * 4);
  Checkpoint* ck = j.ckpt ? j.ckpt + st.ckpt_off : nullptr;
  const uint16_t* sp = j.sym + st.sym_off;
  // prologue: the top n % 32 symbols one at a time (descending); the rest is whole windows
  const uint32_t r = n & 31, nb = (n - r) / 8;   // nb 8-symbol blocks, a multiple of 4
  for (uint32_t i = n; i > n - r; i--) stepk<KIND>(c, ent(tb, tbase + (uint32_t)sp[i - 1] * 16u), g);
  if (KIND != 2) flush_win<GUARD>(c);
  if (((nb * 8) % HOH_SEG) == 0 && nb * 8 < n) ckpt(c, ck, nb * 8 / HOH_SEG);
  if (nb) {
    // table entries gathered 16 steps ahead (two 8-symbol blocks per buffer): with several images
    // in flight the 8 KB-per-stream tables live in MALL/HBM rather than L2, and an 8-step lead
    // left the chain waiting on the gather (15 % of its time even alone; four 8-entry buffers
    // 24 steps ahead, or unconditional gathers past the stream's start, measured slower)
    const uint4* sp4 = (const uint4*)sp;
    const int np = (int)nb / 2;                    // pairs of blocks, even
    EncFast eA[16], eB[16];
    auto syms = [&](int p, uint4& hi, uint4& lo) { hi = sp4[2 * p + 1]; lo = sp4[2 * p]; };
    auto look = [&](EncFast* e, const uint4& hi, const uint4& lo) {
      lookup8(e, hi, tb, tbase);
      lookup8(e + 8, lo, tb, tbase);
    };
    auto run = [&](const EncFast* e, int p) {
#pragma unroll
      for (int k = 7; k >= 0; --k) stepk<KIND>(c, e[k], g);
      if (((2 * p + 1) & (HOH_SEG / 8 - 1)) == 0) ckpt(c, ck, (uint32_t)(2 * p + 1) * 8 / HOH_SEG);
#pragma unroll
      for (int k = 7; k >= 0; --k) stepk<KIND>(c, e[8 + k], g);
      if (((2 * p) & (HOH_SEG / 8 - 1)) == 0) ckpt(c, ck, (uint32_t)(2 * p) * 8 / HOH_SEG);
    };
    uint4 h, l;
    syms(np - 1, h, l); look(eA, h, l);
    syms(np - 2, h, l); look(eB, h, l);
    if (np >= 3) syms(np - 3, h, l);
    for (int p = np - 1; p >= 1; p -= 2) {
      // entering: eA = pair p, eB = pair p-1 (in flight), {h, l} = symbols of pair p-2
      run(eA, p);
      if (p >= 2) { look(eA, h, l); if (p >= 3) syms(p - 3, h, l); }
      run(eB, p - 1);
      if (p >= 3) { look(eB, h, l); if (p >= 4) syms(p - 4, h, l); }
      if (KIND != 2) flush_win<GUARD>(c);
    }
  }
  if (KIND == 2) {                         // size only: the emitted words + the two flushed ones
    j.streams[sid].words = c.mask + 2;
    j.streams[sid].widx_end = 0;
    return;
  }
  flush_win<GUARD>(c);
  if (GUARD && (!c.keep || c.lost || c.widx < 2)) {
    // a counting lane, or a storing one whose bound failed (counted only: its winner is encoded
    // again); the emitted words + the two flushed ones
    j.streams[sid].words = cap - c.widx + c.lost + 2;
    j.streams[sid].widx_end = 0;
    if (c.keep) j.streams[sid].sizeonly = 1;
    return;
  }
  c.slab[--c.widx] = c.xh;                 // Rans64EncFlush: lo at the lower address
  c.slab[--c.widx] = c.xl;
  j.streams[sid].words = cap - c.widx;
  j.streams[sid].widx_end = c.widx;
}

template <int KIND, bool WIDE>
__global__ __launch_bounds__(64) void k_rans_fast(EncodeJob j, int nplane, SidMap ma, int na, SidMap mb, int nblk,
                                                  int rot) {
  // the grid covers every CU; the working blocks are a window rotated per launch so that the
  // chains of images in flight land on different CUs instead of sharing the first ones
  const int blk = (int)((blockIdx.x + gridDim.x - rot) % gridDim.x);
  if (blk < nblk) rans_fast_body<KIND, WIDE>(j, nplane, ma, na, mb, blk);
}

// The pb-15 plane chains and, in otherwise idle blocks of the same chip-wide grid, the LZ
// streams (prob_bits 10): one launch, so the short LZ chains run beside the long ones instead of
// after them (-0.2 ms per image encoded alone).
#ifndef CHAIN_WAVES
#define CHAIN_WAVES 1
#endif
__global__ __launch_bounds__(64 * CHAIN_WAVES) void k_rans_fast01(EncodeJob j, int np0, SidMap a0, int na0, SidMap b0,
                                                                  int nblk0, int np1, SidMap a1, int na1, SidMap b1,
                                                                  int nblk1, int rot) {
  const int blk = (int)((blockIdx.x + gridDim.x - rot) % gridDim.x) * CHAIN_WAVES + (int)(threadIdx.x >> 6);
  if (blk < nblk0) rans_fast_body<0>(j, np0, a0, na0, b0, blk);
  else if (blk - nblk0 < nblk1) rans_fast_body<1>(j, np1, a1, na1, b1, blk - nblk0);
}

// -s>=1: the real pb-15 encodes (KIND 0), every size-only trial of the prob_bits ladder (KIND 2)
// and the other real encodes (KIND 1: LZ / predictor-map streams) are independent, so they share
// one launch: an image waits for one chain length instead of three.  One chain per SIMD (a 40 KB
// request per one-wave workgroup: four per CU), the long chains first in the grid.
// WIDE only for jobs whose tables pass 4 GB (j.tab_wide); otherwise 32-bit offsets from one base,
// as the -s0 chain (one instruction per two gathers' addresses instead of two per gather)
template <bool WIDE>
__global__ __launch_bounds__(64) void k_rans_fast_s(EncodeJob j, int np0, SidMap a0, int na0, SidMap b0, int nblk0,
                                                    int np2, SidMap a2, int na2, int nblk2,
                                                    int np1, SidMap a1, int na1, int nblk1) {
  const int blk = (int)blockIdx.x;
  if (blk < nblk0) rans_fast_body<0, WIDE>(j, np0, a0, na0, b0, blk);
  else if (blk - nblk0 < nblk2) rans_fast_body<2, WIDE>(j, np2, a2, na2, SidMap{0, 0}, blk - nblk0);
  else if (blk - nblk0 - nblk2 < nblk1) rans_fast_body<1, WIDE>(j, np1, a1, na1, SidMap{0, 0}, blk - nblk0 - nblk2);
}

// Generic: one lane per stream, rans64.hpp:262-278 verbatim (64x64 high product).
__global__ __launch_bounds__(64) void k_rans_gen(EncodeJob j, int nstreams, SidMap sm) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= nstreams) return;
  const int sid = map_sid(sm, j.spt, i);
  StreamInfo st = j.streams[sid];
  if (st.fast || st.mode != SM_RANS || st.err || st.n == 0 || st.sizeonly == 2) return;
  const uint16_t* sp = j.sym + st.sym_off;
  const EncGen* tab = j.tab_gen + (size_t)sid * j.gen_stride;
  uint32_t* slab = j.slabs + st.slab_off;
  Checkpoint* ck = j.ckpt ? j.ckpt + st.ckpt_off : nullptr;
  uint32_t widx = st.slab_cap;
  const uint32_t pb = st.pb;
  const bool so = st.sizeonly;                  // size-only: count the words, store nothing
  const bool ckp = !so && ck != nullptr;
  uint64_t x = 1ull << 31;
  auto step = [&](const EncGen& g, uint32_t i) {           // symbol i - 1
    const uint64_t x_max = (((1ull << 31) >> pb) << 32) * g.freq;
    if (x >= x_max) {
      --widx;
      if (!so) slab[widx] = (uint32_t)x;
      x >>= 32;
    }
    const uint64_t q = __umul64hi(x, g.rcp) >> g.shift;
    x = x + g.bias + q * g.cmpl;
    if (ckp && ((i - 1) % HOH_SEG) == 0) {
      Checkpoint p;
      p.xl = (uint32_t)x; p.xh = (uint32_t)(x >> 32); p.widx = widx; p.pad = 0;
      ck[(i - 1) / HOH_SEG] = p;
    }
  };
  // the top n % 8 symbols one at a time, then 8-symbol blocks whose symbols and table entries
  // are gathered one block ahead (two buffers), so the chain waits on no load
  uint32_t k = st.n;
  for (; k > (st.n & ~7u); k--) step(tab[sp[k - 1]], k);
  if (k) {
    EncGen ga[8], gb[8];
    auto fetch = [&](EncGen* g, uint32_t top) {           // symbols top-1 .. top-8
      uint32_t sy[8];
#pragma unroll
      for (int u = 0; u < 8; u++) sy[u] = sp[top - 1 - u];
#pragma unroll
      for (int u = 0; u < 8; u++) g[u] = tab[sy[u]];
    };
    auto run = [&](const EncGen* g, uint32_t top) {
#pragma unroll
      for (int u = 0; u < 8; u++) step(g[u], top - u);
    };
    fetch(ga, k);
    for (;;) {
      fetch(gb, k > 8 ? k - 8 : 8);                      // unconditional (a conditional load would
      run(ga, k);                                         // make the compiler wait at the join)
      k -= 8;
      if (!k) break;
      fetch(ga, k > 8 ? k - 8 : 8);
      run(gb, k);
      k -= 8;
      if (!k) break;
    }
  }
  widx -= 2;
  if (!so) { slab[widx + 1] = (uint32_t)(x >> 32); slab[widx] = (uint32_t)x; }
  j.streams[sid].words = st.slab_cap - widx;
  j.streams[sid].widx_end = widx;
}

static std::atomic<unsigned> g_rot{0};

// LDS requested per chain workgroup (isolation: at most 160 / this many chains per CU; knob
// CHAIN_LDS_KB), never less than the lanes' output windows (WIN_PITCH dwords per lane)
#ifndef CHAIN_LDS_DEF
#define CHAIN_LDS_DEF (CHAIN_WAVES == 1 ? 56 : 81)
#endif
static size_t chain_lds(int waves = 1) {
  const int kb = HOH_KNOB(CHAIN_LDS_KB, CHAIN_LDS_DEF);
  const size_t want = (size_t)(kb > 160 ? 160 : kb) * 1024, win = (size_t)WIN_PITCH * 4 * 64 * waves;
  return want < win ? win : want;
}

void launch_rans_fast01(const EncodeJob& j, hipStream_t s, int np0, SidMap a0, int na0, SidMap b0, int np1, SidMap a1,
                        int na1, SidMap b1) {
  const int nblk0 = (np0 + 63) / 64, nblk1 = (np1 + 63) / 64;
  const int nwg = (nblk0 + nblk1 + CHAIN_WAVES - 1) / CHAIN_WAVES;
  const int grid = std::max(nwg, 1024 / CHAIN_WAVES);
  const int rot = (int)((g_rot.fetch_add(1) * 8u * (unsigned)((nwg + 7) / 8)) % (unsigned)grid);
  hipLaunchKernelGGL(k_rans_fast01, dim3(grid), dim3(64 * CHAIN_WAVES), chain_lds(CHAIN_WAVES), s, j, np0, a0, na0, b0,
                     nblk0, np1, a1, na1, b1, nblk1, rot);
}

void launch_rans_fast(const EncodeJob& j, int nplane, hipStream_t s, SidMap a, int na, SidMap b, int kind) {
  if (nplane <= 0) return;
  // The chain is issue-bound, so two chains on one SIMD run at half speed, and a launch ends with
  // its slowest chain; more than two chains per CU also slow each other.  One chain wave per
  // workgroup with a 56 KB LDS request (8 KB are used) caps the chains at two per CU and, alone,
  // spreads an image's 48 chains over 48 CUs.  The grid covers the chip with a per-launch rotation
  // so that the chains of images in flight land on different CUs.  (Measured alternatives:
  // docs/EXPERIMENTS.md §4.)
  const int nblk = (nplane + 63) / 64;
  // KIND 1 (LZ / map streams, the ladder's winners): short or few chains, no chip-wide grid
  const int grid = (nblk >= 1024 || kind == 1) ? nblk : 1024;
  const int rot = grid == nblk ? 0 : (int)((g_rot.fetch_add(1) * 8u * (unsigned)((nblk + 7) / 8)) % (unsigned)grid);
  const bool w = j.tab_wide != 0;
  if (kind == 0) {
    if (w) hipLaunchKernelGGL((k_rans_fast<0, true>), dim3(grid), dim3(64), chain_lds(), s, j, nplane, a, na, b, nblk, rot);
    else hipLaunchKernelGGL((k_rans_fast<0, false>), dim3(grid), dim3(64), chain_lds(), s, j, nplane, a, na, b, nblk, rot);
  } else if (kind == 1) {   // short or few chains (LZ / map streams, the ladder's winners): the window only
    if (w) hipLaunchKernelGGL((k_rans_fast<1, true>), dim3(grid), dim3(64), WIN_PITCH * 4 * 64, s, j, nplane, a, na, b, nblk, rot);
    else hipLaunchKernelGGL((k_rans_fast<1, false>), dim3(grid), dim3(64), WIN_PITCH * 4 * 64, s, j, nplane, a, na, b, nblk, rot);
  } else {   // size-only trial encodes: no window; one chain per SIMD (40 KB), all at once
    if (w) hipLaunchKernelGGL((k_rans_fast<2, true>), dim3(grid), dim3(64), 40 * 1024, s, j, nplane, a, na, b, nblk, rot);
    else hipLaunchKernelGGL((k_rans_fast<2, false>), dim3(grid), dim3(64), 40 * 1024, s, j, nplane, a, na, b, nblk, rot);
  }
}

void launch_rans_fast_s(const EncodeJob& j, hipStream_t s, int np0, SidMap a0, int na0, SidMap b0, int np2, SidMap a2,
                        int na2, int np1, SidMap a1, int na1) {
  const int nblk0 = (np0 + 63) / 64, nblk2 = (np2 + 63) / 64, nblk1 = (np1 + 63) / 64;
  if (nblk0 + nblk2 + nblk1 == 0) return;
  static_assert(WIN_PITCH * 4 * 64 <= 40 * 1024, "the window fits the 40 KB request");
  // LDS request per chain workgroup (chains per CU; knob CHAIN_S_LDS_KB)
  const size_t lds = (size_t)std::max(40, std::min(160, HOH_KNOB(CHAIN_S_LDS_KB, 40))) * 1024;
  if (j.tab_wide)
    hipLaunchKernelGGL((k_rans_fast_s<true>), dim3(nblk0 + nblk2 + nblk1), dim3(64), lds, s, j, np0, a0, na0, b0, nblk0,
                       np2, a2, na2, nblk2, np1, a1, na1, nblk1);
  else
    hipLaunchKernelGGL((k_rans_fast_s<false>), dim3(nblk0 + nblk2 + nblk1), dim3(64), lds, s, j, np0, a0, na0, b0, nblk0,
                       np2, a2, na2, nblk2, np1, a1, na1, nblk1);
}

void launch_rans_gen(const EncodeJob& j, int nstreams, hipStream_t s, SidMap m) {
  if (nstreams <= 0) return;
  hipLaunchKernelGGL(k_rans_gen, dim3((nstreams + 63) / 64), dim3(64), 0, s, j, nstreams, m);
}
