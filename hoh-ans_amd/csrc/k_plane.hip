// Plane-level kernels behind the reference's per-plane functions (layer_encode.hpp:11,
// prediction.hpp:6, unprediction.hpp:6, channel.hpp:73) for callers that drive single planes.
#include "hoh_internal.h"

__device__ __forceinline__ uint16_t pmed16(uint16_t a, uint16_t b, uint16_t c) {
  if (a > b) return b > c ? b : (c > a ? a : c);
  return b < c ? b : (c > a ? c : a);
}

// channelpredict_fastpath (prediction.hpp:6-44): every residual depends on originals only
__global__ void k_predict(const uint16_t* d, int w, int h, int depth, uint16_t* out) {
  const int c = 1 << depth, half = c / 2;
  const size_t n = (size_t)w * h;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int x = (int)(i % w), y = (int)(i / w);
    const uint16_t L = x ? d[i - 1] : (uint16_t)half;
    const uint16_t T = y ? d[i - w] : (uint16_t)half;
    const uint16_t TL = (x && y) ? d[i - w - 1] : (uint16_t)half;
    const uint16_t p = pmed16(T, L, (uint16_t)(T + L - TL));
    out[i] = (uint16_t)(((int)d[i] - (int)p + half + c) & (c - 1));
  }
}

// MED inverse with LZ back-references, serial raster order (unprediction.hpp:35-89 with the
// fast-path predictor on every row: SURVEY Q9 fixed)
__global__ void k_unpredict_serial(const uint16_t* res, size_t nres, const uint16_t* br, int w, int h, int depth,
                                   uint16_t* o, uint32_t* err) {
  if (threadIdx.x || blockIdx.x) return;
  const int c = 1 << depth, half = c / 2;
  size_t k = 0;
  for (int y = 0; y < h; y++) {
    for (int x = 0; x < w; x++) {
      const size_t i = (size_t)y * w + x;
      if (br && br[i]) {
        if (br[i] > i) { *err = 1; return; }
        o[i] = o[i - br[i]];
        continue;
      }
      if (k >= nres) { *err = 1; return; }
      const uint16_t L = x ? o[i - 1] : (uint16_t)half;
      const uint16_t T = y ? o[i - w] : (uint16_t)half;
      const uint16_t TL = (x && y) ? o[i - w - 1] : (uint16_t)half;
      const uint16_t p = pmed16(T, L, (uint16_t)(T + L - TL));
      o[i] = (uint16_t)((res[k++] + p - half + c) & (c - 1));
    }
  }
  *err = (k == nres) ? 0 : 1;
}

// subtract_green (channel.hpp:73-79) and inverse
__global__ void k_green(const uint8_t* s, size_t n, uint16_t* G, uint16_t* R, uint16_t* B) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    G[i] = s[3 * i + 1];
    R[i] = (uint16_t)((int)s[3 * i] - (int)s[3 * i + 1] + 256);
    B[i] = (uint16_t)((int)s[3 * i + 2] - (int)s[3 * i + 1] + 256);
  }
}

__global__ void k_addgreen(const uint16_t* G, const uint16_t* R, const uint16_t* B, size_t n, uint8_t* o) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    o[3 * i + 1] = (uint8_t)G[i];
    o[3 * i] = (uint8_t)(R[i] + G[i] - 256);
    o[3 * i + 2] = (uint8_t)(B[i] + G[i] - 256);
  }
}

// keep residuals of non-nuked pixels (layer_encode.hpp:93-99); one workgroup, in order
__global__ __launch_bounds__(1024) void k_compact(const uint16_t* in, const uint8_t* nuke, size_t n, uint16_t* out,
                                                  uint64_t* count) {
  __shared__ uint32_t part[1024];
  __shared__ uint64_t carry;
  const int tid = threadIdx.x;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (size_t base = 0; base < n; base += 1024) {
    const size_t i = base + tid;
    const uint32_t keep = (i < n && (!nuke || !nuke[i])) ? 1 : 0;
    part[tid] = keep;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
      uint32_t v = tid >= o ? part[tid - o] : 0;
      __syncthreads();
      part[tid] += v;
      __syncthreads();
    }
    if (keep) out[carry + part[tid] - 1] = in[i];
    __syncthreads();
    if (tid == 0) carry += part[1023];
    __syncthreads();
  }
  if (tid == 0) *count = carry;
}

void launch_predict(const uint16_t* d, int w, int h, int depth, uint16_t* out, hipStream_t s) {
  hipLaunchKernelGGL(k_predict, dim3(1024), dim3(256), 0, s, d, w, h, depth, out);
}
void launch_unpredict_serial(const uint16_t* res, size_t nres, const uint16_t* br, int w, int h, int depth,
                             uint16_t* o, uint32_t* err, hipStream_t s) {
  hipLaunchKernelGGL(k_unpredict_serial, dim3(1), dim3(1), 0, s, res, nres, br, w, h, depth, o, err);
}
void launch_green(const uint8_t* rgb, size_t n, uint16_t* G, uint16_t* R, uint16_t* B, hipStream_t s) {
  hipLaunchKernelGGL(k_green, dim3(1024), dim3(256), 0, s, rgb, n, G, R, B);
}
void launch_addgreen(const uint16_t* G, const uint16_t* R, const uint16_t* B, size_t n, uint8_t* o, hipStream_t s) {
  hipLaunchKernelGGL(k_addgreen, dim3(1024), dim3(256), 0, s, G, R, B, n, o);
}
void launch_compact(const uint16_t* in, const uint8_t* nuke, size_t n, uint16_t* out, uint64_t* count, hipStream_t s) {
  hipLaunchKernelGGL(k_compact, dim3(1), dim3(1024), 0, s, in, nuke, n, out, count);
}
