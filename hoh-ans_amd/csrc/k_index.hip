// Decode side index capture (see include/hoh_ans.h, hoh_index): per stream, where its payload
// sits in the .hoh and the encoder checkpoints every HOH_SEG symbols.
#include "hoh_dec.h"

__global__ void k_index_capture(EncodeJob j, IndexStream* is, Checkpoint* ck, size_t per) {
  const int s = blockIdx.x;
  const StreamInfo st = j.streams[s];
  if (threadIdx.x == 0) {
    IndexStream x;
    x.n = st.n;
    x.mode = st.mode;
    x.widx_end = st.widx_end;
    x.ckpt_off = (uint32_t)((size_t)s * per);
    x.words = st.words;
    x.pad = 0;
    x.payload_off = st.out_off + st.hdr_len + hoh_varint_len((uint64_t)st.words * 4);
    is[s] = x;
  }
  const uint32_t nck = st.mode == SM_RANS ? (st.n + HOH_SEG - 1) / HOH_SEG : 0;
  for (uint32_t k = threadIdx.x; k < nck; k += blockDim.x) ck[(size_t)s * per + k] = j.ckpt[st.ckpt_off + k];
}

void launch_index_capture(const EncodeJob& j, IndexStream* is, Checkpoint* ck, size_t per, hipStream_t s) {
  hipLaunchKernelGGL(k_index_capture, dim3(j.ntiles * SK_PER_TILE), dim3(64), 0, s, j, is, ck, per);
}

void dec_free(DecWork& w) {
  for (int i = 0; i < 16; i++) {
    if (w.bufs[i]) (void)hipFree(w.bufs[i]);
    w.bufs[i] = nullptr;
    w.sizes[i] = 0;
  }
}
