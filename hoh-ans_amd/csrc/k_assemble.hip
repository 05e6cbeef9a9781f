// Stream finalisation, tile layout and byte assembly of the tile blob.
//  finalize: rANS vs stored decision (entropy_encoding.hpp:244-267) and final stream sizes;
//  layout:   tile sizes (choh.cpp:328-366 framing), exclusive scan -> tile and stream offsets;
//  assemble: every stream writes header+table, varint(rANS bytes) and its little-endian payload
//            words at its (unaligned) byte offset, or its MSB-first stored bits; one thread per
//            tile writes the fixed framing bytes.
#include "hoh_internal.h"

__global__ __launch_bounds__(64) void k_finalize(EncodeJob j, int nstreams, SidMap sm) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= nstreams) return;
  const int s = map_sid(sm, j.spt, i);
  StreamInfo st = j.streams[s];
  if (st.err) return;
  if (st.mode == SM_RANS) {
    const uint64_t rb = (uint64_t)st.words * 4;
    const uint64_t es = st.hdr_len + hoh_varint_len(rb) + rb;
    if (st.expected_stored < es) {
      st.mode = SM_STORED;
      st.size = (uint32_t)st.expected_stored;
    } else {
      st.size = (uint32_t)es;
    }
    if (st.words > st.slab_cap && !st.sizeonly) { st.err = 9; atomicOr(j.gerr, 8u); }
  }
  j.streams[s] = st;
}

// single workgroup: tile sizes, then two scans (tile bytes and, when the job writes the .hoh
// tile table, the varint lengths of all but the last tile size, choh.cpp:496-498)
__device__ uint64_t block_excl_scan(uint64_t v, uint64_t* part, int tid) {
  part[tid] = v;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    uint64_t u = tid >= o ? part[tid - o] : 0;
    __syncthreads();
    part[tid] += u;
    __syncthreads();
  }
  const uint64_t incl = part[tid];
  __syncthreads();
  return incl - v;
}

// One workgroup per file: blockIdx.x = the image of a batch (its tiles [tb, te), its file at
// img * out_stride), else the one file / shard blob.
__global__ __launch_bounds__(1024) void k_layout(EncodeJob j) {
  __shared__ uint64_t part[1024];
  __shared__ uint64_t tot_size, tot_vlen;
  const int tid = threadIdx.x, img = blockIdx.x;
  const int tb = j.nimg > 1 ? img * j.img_tiles : 0, te = j.nimg > 1 ? tb + j.img_tiles : j.ntiles;
  const uint64_t fbase = j.nimg > 1 ? (uint64_t)img * j.out_stride : 0;
  if (tid == 0) { tot_size = 0; tot_vlen = 0; }
  __syncthreads();
  // pass 1: tile sizes and the table length
  for (int base = tb; base < te; base += 1024) {
    const int t = base + tid;
    uint64_t sz = 0, vl = 0;
    if (t < te) {
      TileInfo ti = j.tiles[t];
      const StreamInfo* st = j.streams + (size_t)t * j.spt;
      uint32_t bad = ti.flags & (TF_UNREPRODUCIBLE | TF_UNSUPPORTED | TF_OVERFLOW);
      for (int k = 0; k < j.spt; k++) if (st[k].err) bad |= TF_OVERFLOW;
      const uint32_t lzb = 1 + st[0].size + st[1].size + st[2].size;   // lz.hpp:98 + 3 streams
      uint64_t s64 = 2 + 1 + lzb;                                        // choh.cpp:115-116, :328-331
      if (ti.mode == 128 || ti.mode == 127) {
        const uint32_t L1 = 5 + st[3].size, L2 = 5 + st[4].size, L3 = 5 + st[5].size;
        ti.mode = 128;
        if (!(ti.flags & TF_GREY) && (ti.flags & TF_PALETTE_CAND)) {
          // palette_encode (choh.cpp:90-99) vs sub-green (:295-308): the indexed layer wins when
          // layer + 3 * colours + 1 < G + R' + B' layers; the tile then carries channel_size1
          // (the GREEN layer's size) bytes of the indexed layer and no palette (Q15)
          const uint64_t Li = 5 + (uint64_t)st[SK_I].size;
          if (Li + 3 * (uint64_t)ti.colours + 1 < (uint64_t)L1 + L2 + L3) {
            ti.mode = 127;
            if (Li < L1) bad |= TF_UNREPRODUCIBLE;                       // prefix runs past the layer
          }
        }
        if (ti.mode == 128) s64 += 1 + hoh_varint_len(L1) + hoh_varint_len(L2) + L1 + L2 + L3;   // :352-363
        else s64 += L1;                                                  // :335-338
      }
      if (bad) atomicOr(j.nimg > 1 ? j.img_err + img : j.gerr, j.nimg > 1 ? bad : (uint32_t)bad << 8);
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
  // pass 2: offsets
  uint64_t carry_s = 0, carry_v = 0;
  for (int base = tb; base < te; base += 1024) {
    const int t = base + tid;
    uint64_t sz = 0, vl = 0;
    if (t < te) {
      sz = j.tiles[t].size;
      if (j.write_table && t + 1 < te) vl = hoh_varint_len(sz);
    }
    const uint64_t es = block_excl_scan(sz, part, tid);
    const uint64_t chunk_s = part[1023];
    __syncthreads();
    const uint64_t ev = block_excl_scan(vl, part, tid);
    const uint64_t chunk_v = part[1023];
    __syncthreads();
    if (t < te) {
      TileInfo ti = j.tiles[t];
      ti.off = fbase + first + carry_s + es;
      ti.pad = (uint32_t)(j.prefix + carry_v + ev);     // where this tile's size varint goes (in its file)
      j.tiles[t] = ti;
      StreamInfo* st = j.streams + (size_t)t * j.spt;
      uint64_t o = ti.off + 3 + 1;
      for (int k = 0; k < 3; k++) { st[k].out_off = o; o += st[k].size; }
      if (ti.mode == 128) {
        const uint32_t L1 = 5 + st[3].size, L2 = 5 + st[4].size;
        o += 1 + hoh_varint_len(L1) + hoh_varint_len(L2);
        for (int k = 3; k < 6; k++) { st[k].out_off = o + 5; o += 5 + st[k].size; }
        st[SK_I].drop = 1;
      } else if (ti.mode == 127) {
        for (int k = 3; k < 6; k++) st[k].drop = 1;
        st[SK_I].out_off = o + 5;
        st[SK_I].clip = st[3].size;
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

__global__ __launch_bounds__(64) void k_tilebytes(EncodeJob j) {
  const int t = blockIdx.x * 64 + threadIdx.x;
  if (t >= j.ntiles || !file_ok(j, t)) return;
  const TileInfo ti = j.tiles[t];
  const StreamInfo* st = j.streams + (size_t)t * j.spt;
  uint8_t* o = j.out + ti.off;
  o[0] = 0; o[1] = 0;                                  // 1x1 inner tiling (choh.cpp:115-116)
  o[2] = (uint8_t)ti.mode;                             // internal colour mode (:328)
  o[3] = 0x03;                                         // LZ flags (lz.hpp:98)
  const int img = tile_img(j, t);
  const bool last = j.nimg > 1 ? (t + 1) % j.img_tiles == 0 : t + 1 == j.ntiles;
  if (j.write_table && !last)                          // choh.cpp:496-498
    hoh_write_varint(j.out + (j.nimg > 1 ? (uint64_t)img * j.out_stride : 0), ti.pad, ti.size);
  if (ti.mode == 127) {                                // indexed layer header (layer_encode.hpp:57, :320-325)
    uint8_t* q = o + 3 + ti.lz_bytes;
    q[0] = 0x10; q[1] = 0; q[2] = 0; q[3] = 0x00; q[4] = 0x10;
  }
  if (ti.mode == 128) {
    uint32_t p = 3 + ti.lz_bytes;
    o[p++] = 0x24;                                     // channel order G R B (:352)
    const uint32_t L1 = 5 + st[3].size, L2 = 5 + st[4].size;
    p = hoh_write_varint(o, p, L1);
    p = hoh_write_varint(o, p, L2);
    for (int k = 3; k < 6; k++) {                      // layer_encode.hpp:57, :320-325
      uint8_t* q = j.out + st[k].out_off - 5;
      q[0] = 0x10; q[1] = 0; q[2] = 0; q[3] = 0x00; q[4] = 0x10;
    }
  }
}

__global__ __launch_bounds__(256) void k_streambytes(EncodeJob j) {
  const int s = blockIdx.x, tid = threadIdx.x;
  if (!file_ok(j, s / j.spt)) return;
  const StreamInfo st = j.streams[s];
  if (st.range == 0 || st.drop) return;
  uint8_t* o = j.out + st.out_off;
  const uint8_t* hd = j.hdr + (size_t)s * j.hdr_cap;
  const uint64_t lim = st.clip ? st.clip : ~0ull;   // bytes of the stream that reach the file
  if (st.mode == SM_EMPTY) {
    for (uint32_t i = tid; i < st.vlen && i < lim; i += 256) o[i] = hd[i];
    return;
  }
  if (st.mode == SM_RANS) {
    const uint64_t rb = (uint64_t)st.words * 4;
    const uint32_t vl = hoh_varint_len(rb);
    for (uint32_t i = tid; i < st.hdr_len && i < lim; i += 256) o[i] = hd[i];
    if (tid == 0) {
      uint8_t v[3];
      const uint32_t n = hoh_write_varint(v, 0, rb);
      for (uint32_t k = 0; k < n; k++) if (st.hdr_len + k < lim) o[st.hdr_len + k] = v[k];
    }
    const uint64_t p0 = st.hdr_len + vl;
    uint8_t* pay = o + p0;
    const uint32_t* w = j.slabs + st.slab_off + st.widx_end;
    if (p0 + 4ull * st.words <= lim) {
      for (uint32_t i = tid; i < st.words; i += 256) {
        const uint32_t v = w[i];
        pay[4 * i] = (uint8_t)v; pay[4 * i + 1] = (uint8_t)(v >> 8);
        pay[4 * i + 2] = (uint8_t)(v >> 16); pay[4 * i + 3] = (uint8_t)(v >> 24);
      }
    } else {
      for (uint64_t b = tid; p0 + b < lim && b < 4ull * st.words; b += 256)
        pay[b] = (uint8_t)(w[b / 4] >> (8 * (b % 4)));
    }
    return;
  }
  // stored: varint(range-1) varint(n) 0x00, then n symbols of maxbits bits, MSB first
  for (uint32_t i = tid; i < st.vlen && i < lim; i += 256) o[i] = hd[i];
  if (tid == 0 && st.vlen < lim) o[st.vlen] = 0;
  uint8_t* pay = o + st.vlen + 1;
  const uint16_t* sy = j.sym + st.sym_off;
  const uint32_t mb = st.maxbits;
  uint64_t nbytes = ((uint64_t)mb * st.n + 7) / 8;
  if (st.vlen + 1 + nbytes > lim) nbytes = lim > st.vlen + 1 ? lim - st.vlen - 1 : 0;
  for (uint64_t k = tid; k < nbytes; k += 256) {
    uint32_t byte = 0;
    for (int bit = 0; bit < 8; bit++) {
      const uint64_t g = k * 8 + bit;
      uint32_t b = 0;
      if (g < (uint64_t)mb * st.n) {
        const uint64_t i = g / mb;
        const uint32_t within = (uint32_t)(g % mb);
        b = (sy[i] >> (mb - 1 - within)) & 1;
      }
      byte = (byte << 1) | b;
    }
    pay[k] = (uint8_t)byte;
  }
}

void launch_finalize(const EncodeJob& j, int nstreams, hipStream_t s, SidMap m) {
  if (nstreams <= 0) return;
  hipLaunchKernelGGL(k_finalize, dim3((nstreams + 63) / 64), dim3(64), 0, s, j, nstreams, m);
}

void launch_layout(const EncodeJob& j, hipStream_t s) {
  hipLaunchKernelGGL(k_layout, dim3(j.nimg > 1 ? j.nimg : 1), dim3(1024), 0, s, j);
}

void launch_assemble(const EncodeJob& j, int nstreams, hipStream_t s) {
  hipLaunchKernelGGL(k_tilebytes, dim3((j.ntiles + 63) / 64), dim3(64), 0, s, j);
  hipLaunchKernelGGL(k_streambytes, dim3(nstreams), dim3(256), 0, s, j);
}

void launch_streambytes(const EncodeJob& j, int nstreams, hipStream_t s) {
  hipLaunchKernelGGL(k_streambytes, dim3(nstreams), dim3(256), 0, s, j);
}
