// Utility kernels: deterministic synthetic RGB (same integer formula as hoh_ans/synth.py).
#include "hoh_internal.h"

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void k_synth(uint8_t* rgb, int W, int H, int y0, uint64_t salt, int noise) {
  const size_t total = (size_t)W * H * 3;
  const int A[3] = {37, 53, 29}, B[3] = {23, 31, 47}, O[3] = {10, 80, 160};
  const uint64_t k = (uint64_t)noise + 1;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % 3);
    const size_t px = i / 3;
    const long long x = (long long)(px % W), y = (long long)(px / W) + y0;
    const uint64_t gi = ((uint64_t)y * W + (uint64_t)x) * 3 + c;
    const long long base = (((A[c] * x + B[c] * y) >> 8) + O[c]) & 255;
    const uint64_t h = splitmix64(salt + gi);
    const long long nz = (long long)(h % k) + (long long)((h >> 16) % k) - noise;
    long long v = base + nz;
    v = v < 0 ? 0 : v > 255 ? 255 : v;
    rgb[i] = (uint8_t)v;
  }
}

// rows [y0, y0 + H) of the global synthetic image of width W
void launch_synth(uint8_t* rgb, int W, int H, int y0, uint64_t seed, int noise, hipStream_t s) {
  const uint64_t salt = seed * 0x100000001B3ull;
  hipLaunchKernelGGL(k_synth, dim3(4096), dim3(256), 0, s, rgb, W, H, y0, salt, noise);
}

// ---- enqueue-only API support (hoh_*_async): results are written by the stream, not read back

// up to 16 bytes from kernel arguments into device memory (the .hoh header of an async encode;
// a batch: one copy per file, blockIdx.x * stride apart)
__global__ void k_put_bytes(uint8_t* dst, uint64_t lo, uint64_t hi, int n, uint64_t stride) {
  const int i = threadIdx.x;
  if (i < n) dst[blockIdx.x * stride + i] = (uint8_t)((i < 8 ? lo >> (8 * i) : hi >> (8 * (i - 8))) & 255);
}

// encoder status word -> {HOH status code, file bytes}: the mapping of encode_tiles_impl's
// host epilogue (hoh_api.cpp), evaluated on the device
__global__ void k_status_enc(const uint32_t* gerr, const uint64_t* total, uint64_t cap, uint64_t* out) {
  if (threadIdx.x) return;
  const uint32_t g = gerr[0];
  const uint64_t t = total[0];
  uint64_t code = 0;
  if (g) {
    const uint32_t tf = g >> 8;
    code = (tf & TF_UNREPRODUCIBLE) ? 5 : (tf & TF_UNSUPPORTED) ? 6 : (g & 2) ? 4 : 3;
  } else if (t > cap) {
    code = 2;
  }
  out[0] = code;
  out[1] = t;
}

// a batch: {code, file bytes} per image; the job's error word fails every image, an image's
// tile flags and its stride only its own
__global__ void k_status_enc_batch(const uint32_t* gerr, const uint64_t* img_total, const uint32_t* img_err,
                                   uint64_t stride, uint64_t* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t g = gerr[0], tf = img_err[i];
  const uint64_t t = img_total[i];
  uint64_t code = 0;
  if (g) code = (g & 2) ? 4 : 3;
  else if (tf) code = (tf & TF_UNREPRODUCIBLE) ? 5 : (tf & TF_UNSUPPORTED) ? 6 : 3;
  else if (t > stride) code = 2;
  out[2 * i] = code;
  out[2 * i + 1] = t;
}

// decoder error word -> {HOH status code, decoded bytes} (decode_run's epilogue)
// (a batch of n decodes: one {code, bytes} per image, the job's error word for all)
__global__ void k_status_dec(const uint32_t* gerr, uint64_t bytes, uint64_t* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t g = gerr[0];
  out[2 * i] = g ? ((g & 2) ? 6 : 7) : 0;
  out[2 * i + 1] = g ? 0 : bytes;
}

void launch_put_bytes(uint8_t* dst, const uint8_t* b, int n, hipStream_t s, int copies, uint64_t stride) {
  uint64_t w[2] = {0, 0};
  for (int i = 0; i < n && i < 16; i++) w[i / 8] |= (uint64_t)b[i] << (8 * (i % 8));
  hipLaunchKernelGGL(k_put_bytes, dim3(copies), dim3(64), 0, s, dst, w[0], w[1], n, stride);
}

void launch_status_enc_batch(const uint32_t* gerr, const uint64_t* img_total, const uint32_t* img_err,
                             uint64_t stride, uint64_t* out, int n, hipStream_t s) {
  hipLaunchKernelGGL(k_status_enc_batch, dim3((n + 63) / 64), dim3(64), 0, s, gerr, img_total, img_err, stride, out, n);
}

void launch_status_enc(const uint32_t* gerr, const uint64_t* total, uint64_t cap, uint64_t* out, hipStream_t s) {
  hipLaunchKernelGGL(k_status_enc, dim3(1), dim3(64), 0, s, gerr, total, cap, out);
}

void launch_status_dec(const uint32_t* gerr, uint64_t bytes, uint64_t* out, hipStream_t s, int n) {
  hipLaunchKernelGGL(k_status_dec, dim3((n + 63) / 64), dim3(64), 0, s, gerr, bytes, out, n);
}

// ---- natural-statistic synthetic RGB (hoh_ans/natural.py, the same integer formula) ----------

__device__ __forceinline__ uint64_t nat_h(uint64_t salt, uint64_t k, uint64_t a, uint64_t b) {
  return splitmix64(salt + (k << 48) + (a << 24) + b);
}

// bilinear value noise on a 2^lg grid, node values h(k, gx, gy) & m
__device__ __forceinline__ long long nat_vnoise(uint64_t salt, int k, int lg, uint64_t m, long long x, long long y) {
  const long long S = 1ll << lg;
  const uint64_t gx = (uint64_t)(x >> lg), gy = (uint64_t)(y >> lg);
  const long long fx = x & (S - 1), fy = y & (S - 1);
  const long long v00 = (long long)(nat_h(salt, k, gx, gy) & m), v10 = (long long)(nat_h(salt, k, gx + 1, gy) & m);
  const long long v01 = (long long)(nat_h(salt, k, gx, gy + 1) & m), v11 = (long long)(nat_h(salt, k, gx + 1, gy + 1) & m);
  const long long top = v00 * (S - fx) + v10 * fx, bot = v01 * (S - fx) + v11 * fx;
  return (top * (S - fy) + bot * fy) >> (2 * lg);
}

__global__ void k_natural(uint8_t* rgb, int W, int rows, int y0, uint64_t salt) {
  const size_t total = (size_t)W * rows;
  for (size_t px = (size_t)blockIdx.x * blockDim.x + threadIdx.x; px < total; px += (size_t)gridDim.x * blockDim.x) {
    const long long x = (long long)(px % W), y = (long long)(px / W) + y0;
    const long long R = nat_vnoise(salt, 1, 7, 1023, x, y) + nat_vnoise(salt, 2, 4, 127, x, y);
    const uint64_t rk = nat_h(salt, 3, (uint64_t)(R >> 6), (uint64_t)(((x >> 9) << 12) | (y >> 9)));
    const long long Lf = 2 * nat_vnoise(salt, 4, 8, 255, x, y) + nat_vnoise(salt, 5, 6, 255, x, y) +
                         nat_vnoise(salt, 6, 3, 63, x, y);
    const long long L = (Lf * 79) >> 8;
    const long long T = nat_vnoise(salt, 8, 2, 63, x, y) - 32;
    const uint64_t hp = nat_h(salt, 7, (uint64_t)x, (uint64_t)y);
    auto u = [](uint64_t v, int s, uint64_t m) { return (long long)((v >> s) & m); };
    const long long t = u(rk, 0, 7), base = u(rk, 8, 255);
    long long chR = u(rk, 16, 63) - 32;
    if (chR == 0) chR = 9;
    const long long ch[3] = {chR, 0, u(rk, 22, 63) - 32};
    const long long gain = u(rk, 28, 7), sx = u(rk, 32, 63) - 32, sy = u(rk, 38, 63) - 32;
    const long long nl = u(hp, 0, 7) + u(hp, 3, 7) - 7, nb = u(hp, 16, 63) - 32;
#pragma unroll
    for (int c = 0; c < 3; c++) {
      const long long nc = u(hp, 6 + 2 * c, 3) == 0 ? u(hp, 12 + c, 1) * 2 - 1 : 0;
      long long v = base + ch[c];
      if (t == 0) {
      } else if (t <= 3) {
        v += (((L - 128) * gain) >> 2) + nl + nc;
      } else if (t <= 5) {
        v += T + (nb >> 1) + nc;
      } else if (t == 6) {
        v += (((x & 511) * sx + (y & 511) * sy) >> 7) + (nl >> 1);
      } else {
        v += 48 * (((x >> 2) + (y >> 2)) & 1);
      }
      v = v < 0 ? 0 : v > 255 ? 255 : v;
      rgb[px * 3 + c] = (uint8_t)v;
    }
  }
}

void launch_natural(uint8_t* rgb, int W, int rows, int y0, uint64_t seed, hipStream_t s) {
  const uint64_t salt = seed * 0xD6E8FEB86659FD93ull;
  hipLaunchKernelGGL(k_natural, dim3(4096), dim3(256), 0, s, rgb, W, rows, y0, salt);
}
