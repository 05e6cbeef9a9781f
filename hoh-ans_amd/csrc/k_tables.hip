// Per-stream table construction, one wave per stream (entropy_encoding.hpp:19-216):
//  histogram -> normalize_freqs (stattools.hpp:13-70, wave-parallel steal search with the
//  reference's "first strictly smallest freq > 1" rule) -> clamp scan and expected sizes
//  (entropy_encoding.hpp:45-122, with the reference's 32-bit / size_t wrap arithmetic) ->
//  serialised header + frequency table (MSB-first stuffer with the reference's unmasked
//  overflow, varint.hpp:47-77) -> encoder symbol tables for the rANS kernels.
#include "hoh_internal.h"

#define MAXR 4096

struct Sink { uint8_t* b; uint32_t loc; uint32_t rem; uint32_t br; };

// stuffer (varint.hpp:47-77) without recursion: a field wider than the free bits and than 8
// is split into a top part and 8-bit bottoms exactly as the recursive calls do
__device__ void stuff_base(Sink& s, uint32_t v, uint32_t bits) {
  if (bits < s.br) {
    s.rem = (uint8_t)(s.rem + (uint8_t)(v << (s.br - bits)));
    s.br -= bits;
  } else if (bits == s.br) {
    s.b[s.loc++] = (uint8_t)(s.rem + (uint8_t)v);
    s.rem = 0;
    s.br = 8;
  } else {
    s.b[s.loc++] = (uint8_t)(s.rem + (uint8_t)(v >> (bits - s.br)));
    s.br = 8 - (bits - s.br);
    s.rem = (uint8_t)((v << s.br) % 256);
  }
}

__device__ void stuff(Sink& s, uint32_t v, uint32_t bits) {
  uint32_t pend[4];
  int np = 0;
  while (bits > s.br && bits > 8 && np < 4) {
    pend[np++] = v % 256;
    v >>= 8;
    bits -= 8;
  }
  stuff_base(s, v, bits);
  while (np > 0) stuff_base(s, pend[--np], 8);
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
  for (int o = 32; o > 0; o >>= 1) {
    uint64_t u = __shfl_xor(v, o);
    v = u < v ? u : v;
  }
  return v;
}

__global__ __launch_bounds__(64) void k_tables(EncodeJob j, SidMap sm) {
  extern __shared__ uint32_t tb_lds[];             // fr[gen_stride] | cum[gen_stride + 1]
  uint32_t* fr = tb_lds;
  uint32_t* cum = tb_lds + j.gen_stride;
  __shared__ uint32_t s_err;
  const int s = map_sid(sm, j.spt, blockIdx.x), lane = threadIdx.x;
  StreamInfo st = j.streams[s];
  uint8_t* hd = j.hdr + (size_t)s * j.hdr_cap;
  if (st.range == 0) {                     // absent stream (bitimage tile)
    if (lane == 0) { st.size = 0; st.hdr_len = 0; st.mode = SM_EMPTY; j.streams[s] = st; }
    return;
  }
  const uint32_t range = st.range, n = st.n, pb = st.pb;
  uint32_t vlen = hoh_write_varint(hd, 0, range - 1);
  vlen = hoh_write_varint(hd, vlen, n);
  if (n == 0) {                            // entropy_encoding.hpp:19-23
    if (lane == 0) { st.vlen = st.hdr_len = st.size = vlen; st.mode = SM_EMPTY; st.fast = 0; j.streams[s] = st; }
    return;
  }
  if (pb == 0 || pb > 31 || range > MAXR || range > j.gen_stride || ((uint64_t)1 << pb) < range) {
    if (lane == 0) { st.err = 1; j.streams[s] = st; atomicOr(j.gerr, 1u); }
    return;
  }
  if (lane == 0) s_err = 0;
  for (uint32_t i = lane; i < range; i += 64) fr[i] = 0;
  __syncthreads();
  const uint16_t* sy = j.sym + st.sym_off;
  if (j.hist && st.hist_src) {
    for (uint32_t i = lane; i < range; i += 64) fr[i] = j.hist[(size_t)(st.hist_src - 1) * 512 + i];
  } else {
    for (uint32_t i = lane; i < n; i += 64) {
      uint32_t v = sy[i];
      if (v < range) atomicAdd(&fr[v], 1u); else s_err = 1;
    }
  }
  __syncthreads();
  if (s_err) {
    if (lane == 0) { st.err = 2; j.streams[s] = st; atomicOr(j.gerr, 2u); }
    return;
  }
  // ---- normalize_freqs: cumulative (wave scan over contiguous chunks)
  const uint32_t chunk = (range + 63) / 64;
  const uint32_t c0 = lane * chunk, c1 = min(range, c0 + chunk);
  uint32_t local = 0;
  for (uint32_t i = c0; i < c1; i++) local += fr[i];
  uint32_t incl = local;
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t u = __shfl_up(incl, o);
    if (lane >= o) incl += u;
  }
  uint32_t run = incl - local;
  for (uint32_t i = c0; i < c1; i++) { run += fr[i]; cum[i + 1] = run; }
  if (lane == 0) cum[0] = 0;
  __syncthreads();
  const uint32_t total = cum[range];
  const uint32_t target = 1u << pb;
  for (uint32_t i = 1 + lane; i <= range; i += 64) cum[i] = (uint32_t)(((uint64_t)target * cum[i]) / total);
  __syncthreads();
  // Symbols scaled to zero width steal one slot each (stattools.hpp:28-58).  The reference fixes
  // them in index order, each time from the first symbol of smallest width > 1; stealing never
  // touches a zero-width symbol and leaves the victim the unique smallest until it reaches width
  // 1, so the candidates (width > 1) are drained in (width, index) order, each giving width - 1
  // slots.  All Z steals are therefore placed at once: every candidate below a threshold width
  // m* drops to 1, the first q of width m* (by index) too, the next one gives rem slots, where
  // the threshold follows from the per-width capacities.  Widths then rebuild cum by a scan.
  uint32_t Z = 0;
  for (uint32_t base = 0; base < range; base += 64) {
    const uint32_t i0 = base + lane;
    Z += __popcll(__ballot(i0 < range && fr[i0] && cum[i0 + 1] == cum[i0]));
  }
  if (Z) {
    uint32_t R = Z, mprev = 1, mstar = 0, q = 0, rem = 0;
    for (;;) {
      uint32_t m = ~0u;
      for (uint32_t i = lane; i < range; i += 64) {
        const uint32_t w = cum[i + 1] - cum[i];
        if (w > mprev && w < m) m = w;
      }
      for (int o = 32; o > 0; o >>= 1) { const uint32_t u = __shfl_xor(m, o); m = u < m ? u : m; }
      if (m == ~0u) { if (lane == 0) s_err = 3; break; }        // nothing left to steal from
      uint32_t c = 0;
      for (uint32_t base = 0; base < range; base += 64) {
        const uint32_t i0 = base + lane;
        c += __popcll(__ballot(i0 < range && cum[i0 + 1] - cum[i0] == m));
      }
      if ((uint64_t)c * (m - 1) >= R) { mstar = m; q = R / (m - 1); rem = R % (m - 1); break; }
      R -= c * (m - 1);
      mprev = m;
    }
    __syncthreads();
    if (!s_err) {
      // final widths into fr (fr[i] > 0 still marks presence for the zero test)
      uint32_t rank = 0;                                     // width-m* symbols before this chunk
      for (uint32_t base = 0; base < range; base += 64) {
        const uint32_t i0 = base + lane;
        const uint32_t w = i0 < range ? cum[i0 + 1] - cum[i0] : 0;
        const bool atm = i0 < range && w == mstar;
        const uint64_t bm = __ballot(atm);
        const uint32_t r = rank + __popcll(bm & ((1ull << lane) - 1));
        rank += __popcll(bm);
        uint32_t nw = w;
        if (i0 < range) {
          if (fr[i0] && w == 0) nw = 1;
          else if (w > 1 && w < mstar) nw = 1;
          else if (atm) nw = r < q ? 1 : (r == q ? w - rem : w);
        }
        __syncthreads();
        if (i0 < range) fr[i0] = nw;
      }
      __syncthreads();
      // cum = exclusive scan of the final widths
      const uint32_t ch = (range + 63) / 64;
      const uint32_t a0 = lane * ch, a1 = min(range, a0 + ch);
      uint32_t loc = 0;
      for (uint32_t i = a0; i < a1; i++) loc += fr[i];
      uint32_t inc = loc;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(inc, o);
        if (lane >= o) inc += u;
      }
      uint32_t run2 = inc - loc;
      __syncthreads();
      for (uint32_t i = a0; i < a1; i++) { run2 += fr[i]; cum[i + 1] = run2; }
    }
  }
  __syncthreads();
  if (s_err) {
    if (lane == 0) { st.err = 3; j.streams[s] = st; atomicOr(j.gerr, 4u); }
    return;
  }
  for (uint32_t i = lane; i < range; i += 64) fr[i] = cum[i + 1] - cum[i];
  __syncthreads();
  // Size-only trials of the prob_bits ladder: bounds on the words the chain will count, from the
  // code length I = sum count * log2(2^pb / f) (k_prune_s skips the trials whose bounds cannot
  // change the ladder's decision).  Rans64 keeps x in [2^31, 2^63): a step multiplies x by
  // 2^pb / f within a factor 1 +- d, d = 2^(pb - 31) (|x' - x 2^pb / f| < 2^pb and x / f >=
  // 2^(31 - pb)), a renormalisation loses at most a factor 1 - d, so log2(x) + 32 * emits is
  // 31 + I + e with -3nd < e < 1.5nd (|log2(1 +- d)| < 1.5d for d <= 2^-12).  The final
  // log2(x) in [31, 63) leaves (I + e - 32) / 32 < emits < (I + e) / 32; one bit more either
  // side covers the f64 sum.  words = emits + the two flush words.
  uint32_t wlo = 0, whi = 0;
  if (st.sizeonly && j.hist && st.hist_src) {
    double part = 0.0;
    for (uint32_t i = lane; i < range; i += 64) {
      const uint32_t cnt = j.hist[(size_t)(st.hist_src - 1) * 512 + i];
      if (cnt && fr[i]) part += (double)cnt * ((double)pb - log2((double)fr[i]));
    }
    for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
    const double d = ldexp(1.0, (int)pb - 31), slack = 1.0 + 1e-9 * part;
    const double lo = (part - 3.0 * n * d - slack - 32.0) / 32.0, hi = (part + 1.5 * n * d + slack) / 32.0;
    wlo = lo > 0.0 ? (uint32_t)floor(lo) + 2u : 2u;
    whi = (uint32_t)floor(hi) + 1u + 2u;
  }
  // ---- encoder symbol tables.  The f64-quotient chain (k_rans_fast) takes prob_bits 7..19 with
  // range <= 512 (7: its 24-bit multiply of the high quotient; 19: its floors' exactness bound,
  // k_rans_enc.hip step15)
  const bool fast = pb >= 7 && pb <= 19 && range <= HOH_FAST_RANGE && st.fast;
  for (uint32_t i = lane; i < (fast ? (uint32_t)HOH_FAST_RANGE : range); i += 64) {
    const uint32_t f = i < range ? fr[i] : 0, c = i < range ? cum[i] : 0;
    if (fast) {
      EncFast e;
      if (f) {
        double inv = 1.0 / (double)f;
        unsigned long long b = __double_as_longlong(inv);
        e.inv = __longlong_as_double((long long)(b + 1));   // RN(1/f) + 1 ulp >= 1/f
      } else {
        e.inv = 1.0;
      }
      e.f = f ? f : 1;
      e.c = c;
      j.tab_fast[(size_t)s * HOH_FAST_STRIDE + i] = e;
    } else {
      EncGen g;                                           // rans64.hpp:167-247
      g.freq = f;
      g.cmpl = (1u << pb) - f;
      if (f < 2) {
        g.rcp = ~0ull; g.shift = 0; g.bias = c + (1u << pb) - 1;
      } else {
        uint32_t shift = 0;
        while (f > (1u << shift)) shift++;
        uint64_t x0 = f - 1, x1 = 1ull << (shift + 31);
        uint64_t t1 = x1 / f;
        x0 += (x1 % f) << 32;
        uint64_t t0 = x0 / f;
        g.rcp = t0 + (t1 << 32); g.shift = shift - 1; g.bias = c;
      }
      j.tab_gen[(size_t)s * j.gen_stride + i] = g;
    }
  }
  // ---- header + table bytes (entropy_encoding.hpp:43-200).  Lane 0 runs the clamp scans
  // (they stop at the first frequency needing prob_bits bits, so they are short); the fields are
  // then written by the whole wave when every value fits its field (the stuffer's unmasked
  // overflow cannot occur), else by lane 0 with the exact serial stuffer.
  __shared__ uint16_t s_lower[16], s_upper[16];
  __shared__ uint32_t s_mode;
  const uint32_t maxbits = hoh_bitlen(range - 1);
  const uint64_t expected_stored = vlen + 1 + ((uint64_t)maxbits * n + 8 - 1) / 8;
  const uint64_t expected_raw = ((uint64_t)pb * range + 8 - 1) / 8;
  const uint32_t cn32 = (pb - 1) / 4 + 2;
  const uint32_t cn = (uint8_t)cn32;
  // first and last present symbols: the clamp scans below do nothing over the absent symbols at
  // either end (size_bits stays 0, nothing is added), so they start there (the residual planes
  // of an image have ~100+ absent symbols at each end, ~2/3 of the serial scan steps)
  uint32_t first = range, lastnz = 0;
  for (uint32_t base = 0; base < range; base += 64) {
    const uint32_t i0 = base + lane;
    const uint64_t bm = __ballot(i0 < range && fr[i0] != 0);
    if (bm) {
      if (first == range) first = base + (uint32_t)__builtin_ctzll(bm);
      lastnz = base + 63 - (uint32_t)__builtin_clzll(bm);
    }
  }
  if (first == range) { first = 0; lastnz = range - 1; }
  // The clamp scans (entropy_encoding.hpp:48-122), wave-parallel.  The serial scan only ever raises
  // size_bits (0 -> 1 -> 4 -> 8 -> ...), so after symbol i it is level(max of the frequencies
  // scanned so far), lower[idx] is the first symbol whose frequency reaches the idx-th raise's
  // threshold (1, 2, 16, 256, ...), and the scan stops at the first symbol whose level reaches pb.
  // Each 64-symbol chunk: a prefix max, the levels, one ballot for the stop and one per raise.
  auto level = [&](uint32_t m) -> uint32_t {        // smallest of 0, 1, 4, 8, 12, ... with m < 2^s
    const uint32_t bl = m ? 32u - __builtin_clz(m) : 0u;
    return bl <= 1 ? bl : 4u * ((bl + 3) / 4);
  };
  auto nraise = [&](uint32_t sb) -> uint32_t { return sb == 0 ? 0u : sb == 1 ? 1u : sb / 4 + 1; };
  auto thr = [&](uint32_t idx) -> uint32_t { return idx == 0 ? 1u : idx == 1 ? 2u : 1u << (4 * (idx - 1)); };
  const uint32_t ncl = cn < 16 ? cn : 16u;
  // one direction: dir = +1 from `from` up to range - 1, dir = -1 from `from` down to 0.  Returns
  // the sum of the levels up to the stop (pb at the stop); sets the stop position (range / 0, as
  // the serial loop leaves it, if the scan never stops), the final size_bits, the maximum
  // frequency scanned (stop symbol included: it decides how many raises happened) and the first
  // crossing of every raise threshold.
  auto scan = [&](int dir, uint32_t from, uint32_t* cross, uint32_t& stop, uint32_t& sbf, uint32_t& mx) -> uint64_t {
    uint64_t sum = 0;
    uint32_t carry = 0, found = 0;
    for (uint32_t c = 0;; c++) {
      const int64_t ii = (int64_t)from + dir * (int64_t)(64 * c + lane);
      const bool valid = ii >= 0 && ii < (int64_t)range;
      if (!__ballot(valid)) break;
      const uint32_t v = valid ? fr[(uint32_t)ii] : 0u;
      uint32_t m = v;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(m, o);
        if (lane >= o) m = max(m, u);
      }
      m = max(m, carry);
      const uint32_t sl = level(m);
#pragma unroll
      for (uint32_t idx = 0; idx < 16; idx++) {              // constant indices: cross stays in registers
        if (idx >= ncl || ((found >> idx) & 1)) continue;
        const uint64_t b = __ballot(valid && v >= thr(idx));
        if (b) {
          cross[idx] = (uint32_t)((int64_t)from + dir * (int64_t)(64 * c + __builtin_ctzll(b)));
          found |= 1u << idx;
        }
      }
      const uint64_t hb = __ballot(valid && sl >= pb);
      const uint32_t k = hb ? (uint32_t)__builtin_ctzll(hb) : 64u;
      uint32_t part = valid && (uint32_t)lane < k ? sl : 0u;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
      sum += part;
      if (hb) {
        stop = (uint32_t)((int64_t)from + dir * (int64_t)(64 * c + k));
        sum += pb;
        sbf = pb;
        mx = __shfl(m, (int)k);
        return sum;
      }
      carry = __shfl(m, 63);
    }
    stop = dir > 0 ? range : 0u;
    sbf = level(carry);
    mx = carry;
    return sum;
  };
  uint32_t lo_x[16] = {0}, up_x[16] = {0}, climb, climb2, sbf1, sbf2, mf, mb;
  const uint64_t s1 = scan(1, first, lo_x, climb, sbf1, mf);
  const uint64_t s2 = scan(-1, lastnz, up_x, climb2, sbf2, mb);
  if (lane == 0) {
    uint64_t exp_cl = (uint64_t)(uint32_t)((uint32_t)(2 * ((int)maxbits - 1)) * cn32);
    exp_cl += (uint64_t)(uint32_t)(pb * 2);
    exp_cl += s1 + s2;
    const uint32_t nf = nraise(level(mf)), nb = nraise(level(mb));
#pragma unroll
    for (uint32_t i = 0; i < 16; i++) {
      s_lower[i] = (uint16_t)(i < ncl ? (i < nf ? lo_x[i] : range - 1) : 0u);
      s_upper[i] = (uint16_t)(i < ncl && i < nb ? up_x[i] : 0u);
    }
    exp_cl += (uint64_t)sbf2 * ((uint64_t)climb2 - (uint64_t)climb - 1);     // size_t wrap (Q5)
    exp_cl = (exp_cl + 8 - 1) / 8;
    const bool raw = expected_raw < exp_cl;
    hd[vlen] = (uint8_t)((1u << 7) + (pb << 2) + (raw ? 1 : 2));
    s_mode = raw ? 1 : 2;
  }
  __syncthreads();
  const bool raw = s_mode == 1;
  auto sbits = [&](uint32_t i) -> uint32_t {                           // entropy_encoding.hpp:176-190
    uint32_t sb = 0;
    if (s_lower[0] <= i && s_upper[0] >= i) sb = 1;
    if (s_lower[1] <= i && s_upper[1] >= i) sb = 4;
    for (uint32_t jj = 2; jj < cn && jj < 16; jj++)
      if (s_lower[jj] <= i && s_upper[jj] >= i) sb = 4 * jj;
    return sb > pb ? pb : sb;
  };
  const uint32_t chunk2 = (range + 63) / 64;
  const uint32_t d0 = lane * chunk2, d1 = min(range, d0 + chunk2);
  bool fits = !raw;
  uint32_t mybits = 0;
  if (!raw)
    for (uint32_t i = d0; i < d1; i++) {
      const uint32_t sb = sbits(i);
      if (fr[i] >> sb) fits = false;
      mybits += sb;
    }
  uint32_t loc;
  if (__ballot(!fits) == 0) {
    // parallel writer: fields MSB-first into an LDS bit buffer (cum is free now), then copied
    uint32_t* bb = cum;
    const uint32_t head = 2 * cn * maxbits;
    uint32_t incl = mybits;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(incl, o);
      if (lane >= o) incl += u;
    }
    const uint32_t total = head + __shfl(incl, 63);
    const uint32_t nbytes = (total + 7) / 8;
    for (uint32_t w = lane; w < (nbytes + 3) / 4; w += 64) bb[w] = 0;
    __syncthreads();
    auto put = [&](uint32_t pos, uint32_t v, uint32_t nb) {
      if (!nb || !v) return;
      const uint32_t off = pos & 7;
      const uint32_t al = v << (32 - off - nb);                       // big-endian window at byte pos/8
      for (uint32_t k = 0; k < 4; k++) {
        const uint32_t byte = (al >> (24 - 8 * k)) & 255u;
        if (byte) {
          const uint32_t bi = (pos >> 3) + k;
          atomicOr(&bb[bi >> 2], byte << (8 * (bi & 3)));
        }
      }
    };
    if (lane < 2 * (int)cn) put((uint32_t)lane * maxbits, (lane & 1) ? s_upper[lane >> 1] : s_lower[lane >> 1], maxbits);
    uint32_t pos = head + incl - mybits;
    for (uint32_t i = d0; i < d1; i++) {
      const uint32_t sb = sbits(i);
      put(pos, fr[i], sb);
      pos += sb;
    }
    __syncthreads();
    const uint8_t* bs = (const uint8_t*)bb;
    for (uint32_t k = lane; k < nbytes; k += 64) hd[vlen + 1 + k] = bs[k];
    loc = vlen + 1 + nbytes;
  } else {
    if (lane != 0) return;
    Sink sk{hd, vlen + 1, 0, 8};
    if (raw) {
      for (uint32_t i = 0; i < range; i++) stuff(sk, fr[i], maxbits);
    } else {
      for (uint32_t i = 0; i < cn; i++) {
        stuff(sk, s_lower[i], maxbits);
        stuff(sk, s_upper[i], maxbits);
      }
      for (uint32_t i = 0; i < range; i++) stuff(sk, fr[i], sbits(i));
    }
    if (sk.br != 8) hd[sk.loc++] = (uint8_t)sk.rem;
    loc = sk.loc;
  }
  if (lane != 0) return;
  st.vlen = vlen;
  st.hdr_len = loc;
  st.maxbits = maxbits;
  st.expected_stored = expected_stored;
  st.fast = fast ? 1 : 0;
  st.mode = SM_RANS;
  st.wlo = wlo;
  st.whi = whi;
  j.streams[s] = st;
}

void launch_tables(const EncodeJob& j, int nstreams, hipStream_t s, SidMap m) {
  // LDS sized to the job's largest alphabet (512 for images): many streams per CU at once, so
  // the serial header writer of each runs concurrently with the others
  if (nstreams <= 0) return;
  hipLaunchKernelGGL(k_tables, dim3(nstreams), dim3(64), (size_t)(2 * j.gen_stride + 1) * 4, s, j, m);
}
