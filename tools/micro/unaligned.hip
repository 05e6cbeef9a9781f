// Does gfx950 (as configured by ROCm) honour misaligned addresses on global_load_dwordx4 and on
// LDS dword / b128 accesses?  Prints OK / MISMATCH per case.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
typedef uint32_t u4a __attribute__((ext_vector_type(4), aligned(2)));
typedef uint32_t u1a __attribute__((aligned(1)));
__global__ void k(const uint8_t* in, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t s[1024];
  const int l = threadIdx.x;
  for (int i = l; i < 1024; i += 64) s[i] = (uint8_t)(i * 7 + 3);
  __syncthreads();
  // global: 16 B from byte offset 2*l + 2 (2-byte aligned)
  const u4a v = *(const u4a*)(in + 2 * l + 2);
  out[l * 8 + 0] = v.x; out[l * 8 + 1] = v.y; out[l * 8 + 2] = v.z; out[l * 8 + 3] = v.w;
  // LDS dword read at byte offset 3*l + 1, then dword write at byte offset 3*l + 513
  uint32_t r;
  const uint32_t a = (uint32_t)(size_t)(__attribute__((address_space(3))) uint8_t*)(s + 3 * l + 1);
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(a) : "memory");
  out[l * 8 + 4] = r;
  __syncthreads();
  if (l == 5) asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" :: "v"(a), "v"(0xa1b2c3d4u) : "memory");
  __syncthreads();
  out[l * 8 + 5] = *(volatile const uint32_t*)(s + 4 * l);
  out[l * 8 + 6] = 0; out[l * 8 + 7] = 0;
}
int main() {
  uint8_t h[4096]; for (int i = 0; i < 4096; i++) h[i] = (uint8_t)(i * 13 + 1);
  uint8_t* din; uint32_t* dout; CK(hipMalloc(&din, 4096)); CK(hipMalloc(&dout, 64 * 32));
  CK(hipMemcpy(din, h, 4096, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, din, dout);
  CK(hipDeviceSynchronize());
  uint32_t o[64 * 8]; CK(hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost));
  uint8_t s[1024]; for (int i = 0; i < 1024; i++) s[i] = (uint8_t)(i * 7 + 3);
  int bad_g = 0, bad_r = 0, bad_w = 0;
  for (int l = 0; l < 64; l++) {
    for (int e = 0; e < 4; e++) { uint32_t w; memcpy(&w, h + 2 * l + 2 + 4 * e, 4); bad_g += o[l * 8 + e] != w; }
    uint32_t w; memcpy(&w, s + 3 * l + 1, 4); bad_r += o[l * 8 + 4] != w;
  }
  uint32_t x = 0xa1b2c3d4u; memcpy(s + 16, &x, 4);
  for (int l = 0; l < 64; l++) { uint32_t w; memcpy(&w, s + 4 * l, 4); bad_w += o[l * 8 + 5] != w; }
  printf("global dwordx4 at 2-B alignment: %s\n", bad_g ? "MISMATCH" : "OK");
  printf("LDS dword read at 1-B alignment: %s\n", bad_r ? "MISMATCH" : "OK");
  printf("LDS dword write at 1-B alignment: %s\n", bad_w ? "MISMATCH" : "OK");
  return 0;
}
