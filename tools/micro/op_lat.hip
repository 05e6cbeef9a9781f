// Micro-benchmark: dependent-chain latency and single-wave issue cost of the VALU ops a
// rans64 step is built from, on gfx950 (one wave per CU, s_memtime around the chain).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

#define REP16(X) X X X X X X X X X X X X X X X X
#define REP64(X) REP16(X) REP16(X) REP16(X) REP16(X)

__device__ __forceinline__ uint64_t stamp() {
  uint64_t t; asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory"); return t;
}

template <int OP, int ILP>
__global__ void lat(uint32_t* out, uint64_t* cyc, uint32_t a) {
  uint32_t x0 = threadIdx.x + a, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
  uint32_t y0 = a ^ 0x55, y1 = a ^ 0x66, y2 = a ^ 0x77, y3 = a ^ 0x88;
  double d0 = x0, d1 = x1, d2 = x2, d3 = x3, one = (double)(a & 1) + 1.0;
  uint64_t t0 = stamp();
#define ONE(x, y, d) \
  if (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(a)); \
  if (OP == 1) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(a)); \
  if (OP == 2) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(a)); \
  if (OP == 3) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "v"(a)); \
  if (OP == 4) { uint64_t t; asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(t) : "v"(x), "v"(a) : "vcc"); x = (uint32_t)(t >> 32) ^ (uint32_t)t; } \
  if (OP == 5) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d) : "v"(one)); \
  if (OP == 6) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d) : "v"(one)); \
  if (OP == 7) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(d) : "v"(x)); \
  if (OP == 7) asm volatile("v_cvt_u32_f64 %0, %1" : "=v"(x) : "v"(d)); \
  if (OP == 8) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(x) : "v"(y)); \
  if (OP == 9) asm volatile("v_cmp_ge_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(y) : "vcc"); \
  if (OP == 10) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x) : "v"(a)); \
  if (OP == 11) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(x) : "v"(a)); \
  if (OP == 12) { uint64_t t = ((uint64_t)y << 32) | x; asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(t)); x = (uint32_t)t; y = (uint32_t)(t >> 32); } \
  if (OP == 13) asm volatile("v_rcp_f64 %0, %0" : "+v"(d)); \
  if (OP == 14) asm volatile("v_trunc_f64 %0, %0" : "+v"(d)); \
  if (OP == 15) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(x)); \
  if (OP == 16) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d) : "v"(one)); \
  if (OP == 17) asm volatile("v_mad_i32_i24 %0, %0, %1, %1" : "+v"(x) : "v"(a)); \
  if (OP == 18) { uint64_t e_; asm volatile("v_cmp_ge_u32_e64 %1, %0, %2\n\tv_cndmask_b32_e64 %0, %0, %2, %1" : "+v"(x), "=s"(e_) : "v"(y)); } \
  if (OP == 19) asm volatile("v_or_b32 %0, 0x43300000, %0" : "+v"(x)); \
  if (OP == 20) asm volatile("v_sub_u32 %0, %1, %0" : "+v"(x) : "v"(y));
  for (int it = 0; it < 4; ++it) {
    if (ILP == 1) { REP64(ONE(x0, y0, d0)) }
    if (ILP == 4) { REP16(ONE(x0, y0, d0) ONE(x1, y1, d1) ONE(x2, y2, d2) ONE(x3, y3, d3)) }
  }
  uint64_t t1 = stamp();
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + (uint32_t)(d0 + d1 + d2 + d3) + y0;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}


__global__ void clk(uint64_t* out, uint32_t a, int iters) {
  uint32_t x = threadIdx.x;
  uint64_t t0, r0, t1, r1;
  asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0), "=s"(r0) :: "memory");
  for (int i = 0; i < iters; ++i) { REP64(asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(a));) }
  asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1), "=s"(r1) :: "memory");
  if (threadIdx.x == 0) { out[2 * blockIdx.x] = t1 - t0; out[2 * blockIdx.x + 1] = r1 - r0; }
  if (x == 12345) out[0] = 0;
}

template <int OP, int ILP>
static int run(const char* name, uint32_t* d_out, uint64_t* d_cyc) {
  hipLaunchKernelGGL((lat<OP, ILP>), dim3(1), dim3(64), 0, 0, d_out, d_cyc, 3u);
  hipLaunchKernelGGL((lat<OP, ILP>), dim3(1), dim3(64), 0, 0, d_out, d_cyc, 3u);
  CK(hipDeviceSynchronize());
  uint64_t c; CK(hipMemcpy(&c, d_cyc, 8, hipMemcpyDeviceToHost));
  printf("%-22s ILP%d: %6.2f cyc/op\n", name, ILP, (double)c / 256.0);
  return 0;
}

int main() {
  uint32_t* d_out; uint64_t* d_cyc;
  CK(hipMalloc(&d_out, 4096 * 4)); CK(hipMalloc(&d_cyc, 64 * 8));
#define BOTH(OP, NAME) run<OP, 1>(NAME, d_out, d_cyc); run<OP, 4>(NAME, d_out, d_cyc);
  BOTH(0, "v_add_u32")
  BOTH(1, "v_mul_lo_u32")
  BOTH(2, "v_mul_hi_u32")
  BOTH(3, "v_mul_u32_u24")
  BOTH(4, "v_mad_u64_u32+xor")
  BOTH(5, "v_mul_f64")
  BOTH(6, "v_fma_f64")
  BOTH(7, "cvt_f64_u32+cvt_u32")
  BOTH(8, "v_alignbit_b32")
  BOTH(9, "v_cmp+v_cndmask")
  BOTH(10, "v_mul_f32")
  BOTH(11, "v_mad_u32_u24")
  BOTH(12, "v_lshrrev_b64")
  BOTH(13, "v_rcp_f64")
  BOTH(14, "v_trunc_f64")
  BOTH(15, "v_cvt_f32_u32")
  BOTH(16, "v_add_f64")
  BOTH(17, "v_mad_i32_i24")
  BOTH(18, "v_cmp_e64+cndmask(sgpr)")
  BOTH(19, "v_or_b32 literal")
  BOTH(20, "v_sub_u32")
  uint64_t* d_clk; CK(hipMalloc(&d_clk, 2048 * 16));
  for (int nb : {1, 256, 1024}) {
    hipLaunchKernelGGL(clk, dim3(nb), dim3(64), 0, 0, d_clk, 3u, 20000);
    CK(hipDeviceSynchronize());
    uint64_t h[2]; CK(hipMemcpy(h, d_clk, 16, hipMemcpyDeviceToHost));
    printf("clock probe blocks=%d: %.0f cycles in %.1f us -> %.3f GHz ; chain %.2f cyc/op\n", nb, (double)h[0], h[1] / 100.0, h[0] / (h[1] / 100.0) / 1000.0, (double)h[0] / (20000.0 * 64));
  }
  return 0;
}
