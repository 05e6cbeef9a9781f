// Single-wave VALU issue rate on gfx950: 8 independent chains per lane, per op type;
// and the same with 2 and 4 waves resident on each SIMD (workgroup of 8 / 16 waves).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
template <int OP>
__global__ void iss(uint32_t* out, uint64_t* cyc, uint32_t a) {
  uint32_t x[8]; double d[8]; uint64_t y[8];
  for (int i = 0; i < 8; ++i) { x[i] = threadIdx.x + i + a; d[i] = x[i]; y[i] = x[i]; }
  double one = (double)(a & 1) + 1.0;
  uint64_t t0; asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0) :: "memory");
  for (int it = 0; it < 64; ++it) {
#define OPX(i) \
    if (OP == 0) asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(x[i]) : "v"(a)); \
    if (OP == 1) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d[i]) : "v"(one)); \
    if (OP == 2) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(d[i]) : "v"(x[i])); \
    if (OP == 3) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[i]) : "v"(a)); \
    if (OP == 4) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d[i]) : "v"(one)); \
    if (OP == 5) asm volatile("v_cvt_u32_f64 %0, %1" : "=v"(x[i]) : "v"(d[i])); \
    if (OP == 6) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[i]) : "v"(one)); \
    if (OP == 7) asm volatile("v_mul_u32_u24_e32 %0, %0, %1" : "+v"(x[i]) : "v"(a)); \
    if (OP == 8) asm volatile("v_alignbit_b32 %0, %0, %1, 17" : "+v"(x[i]) : "v"(a)); \
    if (OP == 9) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(x[i]) : "v"(a)); \
    if (OP == 10) asm volatile("v_cmp_ge_u32_sdwa vcc, %0, %1 src0_sel:WORD_1 src1_sel:DWORD\n\tv_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(x[i]) : "v"(a) : "vcc"); \
    if (OP == 11) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[0:1]" : "+v"(x[i]) : "v"(a)); \
    if (OP == 12) asm volatile("v_add_u32_e32 %0, %0, %0" : "+v"(x[0])); \
    if (OP == 13) { uint64_t co; asm volatile("v_mad_u64_u32 %0, %1, %2, %2, %0" : "+v"(y[i]), "=s"(co) : "v"(a)); } \
    if (OP == 14) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x[i]) : "v"(a)); \
    if (OP == 15) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(x[i]) : "v"(a)); \
    if (OP == 16) asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(y[i])); \
    if (OP == 17) asm volatile("v_cmp_gt_u64_e32 vcc, %2, %1\n\tv_cndmask_b32_e32 %0, %0, %3, vcc" : "+v"(x[i]) : "v"(y[i]), "v"(y[(i + 1) & 7]), "v"(a) : "vcc"); \
    if (OP == 18) asm volatile("v_bfe_u32 %0, %0, 1, %1" : "+v"(x[i]) : "v"(a)); \
    if (OP == 19) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(a), "s"(0x07060302u)); \
    if (OP == 20) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(x[i]) : "v"(a));
    R8(OPX)
  }
  uint64_t t1; asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1) :: "memory");
  uint32_t acc = 0; for (int i = 0; i < 8; ++i) acc += x[i] + (uint32_t)d[i] + (uint32_t)y[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
}
template <int OP>
static int run(const char* name, uint32_t* d_out, uint64_t* d_cyc) {
  for (int waves : {1, 4, 8, 16}) {
    hipLaunchKernelGGL((iss<OP>), dim3(1), dim3(64 * waves), 0, 0, d_out, d_cyc, 3u);
    hipLaunchKernelGGL((iss<OP>), dim3(1), dim3(64 * waves), 0, 0, d_out, d_cyc, 3u);
    CK(hipDeviceSynchronize());
    uint64_t c[16]; CK(hipMemcpy(c, d_cyc, 16 * 8, hipMemcpyDeviceToHost));
    uint64_t mx = 0; for (int w = 0; w < waves; ++w) mx = c[w] > mx ? c[w] : mx;
    printf("%-16s waves/WG %2d (per SIMD %d): %6.2f cyc per op per wave\n", name, waves, (waves + 3) / 4, (double)mx / 512.0);
  }
  return 0;
}
int main() {
  uint32_t* d_out; uint64_t* d_cyc;
  CK(hipMalloc(&d_out, 4096 * 4)); CK(hipMalloc(&d_cyc, 64 * 16 * 8));
  run<0>("v_add_u32", d_out, d_cyc);
  run<1>("v_mul_f64", d_out, d_cyc);
  run<2>("v_cvt_f64_u32", d_out, d_cyc);
  run<3>("v_mul_lo_u32", d_out, d_cyc);
  run<4>("v_fma_f64", d_out, d_cyc);
  run<5>("v_cvt_u32_f64", d_out, d_cyc);
  run<6>("v_add_f64", d_out, d_cyc);
  run<7>("v_mul_u32_u24", d_out, d_cyc);
  run<8>("v_alignbit", d_out, d_cyc);
  run<9>("v_add3_u32", d_out, d_cyc);
  run<10>("cmp_sdwa+cndmask", d_out, d_cyc);
  run<11>("v_cndmask_e64", d_out, d_cyc);
  run<12>("dep v_add_u32", d_out, d_cyc);
  run<13>("v_mad_u64_u32", d_out, d_cyc);
  run<14>("v_mul_hi_u32", d_out, d_cyc);
  run<15>("v_bcnt_u32", d_out, d_cyc);
  run<16>("v_lshrrev_b64", d_out, d_cyc);
  run<17>("cmp_u64+cndmask", d_out, d_cyc);
  run<18>("v_bfe_u32", d_out, d_cyc);
  run<19>("v_perm_b32", d_out, d_cyc);
  run<20>("v_mul_hi_u32_u24", d_out, d_cyc);
  return 0;
}
