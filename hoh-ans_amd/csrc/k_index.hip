// Decode side index capture (see include/hoh_ans.h, hoh_index): per stream, where its payload
// sits in the .hoh and the encoder checkpoints every HOH_SEG symbols.
#include "hoh_dec.h"

__global__ void k_index_capture(EncodeJob j, IndexStream* is, size_t per, int nstreams) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nstreams) return;
  const StreamInfo st = j.streams[s];
  IndexStream x;
  x.n = st.n;
  x.mode = st.mode;
  x.widx_end = st.widx_end;
  x.ckpt_off = (uint32_t)((size_t)s * per);       // the encoder's own checkpoint layout
  x.words = st.words;
  x.pad = 0;
  x.payload_off = st.out_off + st.hdr_len + hoh_varint_len((uint64_t)st.words * 4);
  is[s] = x;
}

void launch_index_capture(const EncodeJob& j, IndexStream* is, size_t per, hipStream_t s) {
  const int S = j.ntiles * SK_PER_TILE;
  hipLaunchKernelGGL(k_index_capture, dim3((S + 255) / 256), dim3(256), 0, s, j, is, per, S);
}

void dec_free(DecWork& w) {
  noix_release(w);
  for (int i = 0; i < 16; i++) {
    if (w.bufs[i]) (void)hipFree(w.bufs[i]);
    w.bufs[i] = nullptr;
    w.sizes[i] = 0;
  }
}
