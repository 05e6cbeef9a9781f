// Launch cost of a workgroup that exits at once, by dynamic LDS request (tools/micro/README.md):
// grid G one-wave workgroups, each reading one word and returning.  Prints us per launch.
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ __launch_bounds__(64) void k_exit(const unsigned* g, int many) {
  extern __shared__ unsigned lds[];
  if ((*(volatile const unsigned*)g > 256u) != (many != 0)) return;
  lds[threadIdx.x] = threadIdx.x;
}
__global__ __launch_bounds__(256) void k_busy(unsigned* o, int n) {
  unsigned v = threadIdx.x;
  for (int i = 0; i < n; i++) v = v * 1664525u + 1013904223u;
  o[blockIdx.x * 256 + threadIdx.x] = v;
}
int main() {
  unsigned* g; unsigned* o;
  hipMalloc(&g, 64); hipMemset(g, 0, 64);
  hipMalloc(&o, 1 << 24);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const size_t lds[] = {0, 16384, 32768, 65536, 68096, 98304, 131072, 155648};
  const int grids[] = {359, 1127};
  for (int gi = 0; gi < 2; gi++)
    for (size_t L : lds) {
      for (int prior = 0; prior < 2; prior++) {
        float best = 1e9;
        for (int r = 0; r < 8; r++) {
          if (prior) hipLaunchKernelGGL(k_busy, dim3(1024), dim3(256), 0, 0, o, 20000);
          hipEventRecord(a, 0);
          hipLaunchKernelGGL(k_exit, dim3(grids[gi]), dim3(64), L, 0, g, 0);
          hipEventRecord(b, 0);
          hipEventSynchronize(b);
          float ms; hipEventElapsedTime(&ms, a, b);
          if (ms < best) best = ms;
        }
        printf("grid %5d lds %6zu B after %s: %8.1f us\n", grids[gi], L, prior ? "busy kernel" : "idle     ", best * 1e3);
      }
    }
  return 0;
}
