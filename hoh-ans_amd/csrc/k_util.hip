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
