// Micro-benchmark: the rANS decode step of k_drans in isolation (LDS slot table, cumulative
// table, staged payload), cycles per step per wave vs occupancy and per feature.
//   V0 full step (table + cum + 64-bit advance + refill from LDS payload)
//   V1 V0 + one scattered global u16 store per step
//   V2 V0 with the 64-bit advance replaced by 32-bit arithmetic (chain-latency probe)
//   V3 V0 without the cum read (f, c from registers: LDS round-trip probe)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int PB = 15, M = 1 << PB, STEPS = 256;

template <int V>
__global__ __launch_bounds__(256) void dstep(const uint32_t* cum_g, const uint8_t* tb_g, const uint16_t* sy_g,
                                             const uint32_t* pw_g, uint16_t* out, uint64_t* cyc, uint32_t* sink) {
  __shared__ uint32_t cum_s[258];
  __shared__ uint16_t sy_s[1024];
  __shared__ uint8_t tb[M];
  __shared__ uint32_t pw[8192];
  const int tid = threadIdx.x;
  for (int i = tid; i < 257; i += 256) cum_s[i] = cum_g[i];
  for (int i = tid; i < 1024; i += 256) sy_s[i] = sy_g[i];
  for (int i = tid; i < M / 4; i += 256) ((uint32_t*)tb)[i] = ((const uint32_t*)tb_g)[i];
  for (int i = tid; i < 8192; i += 256) pw[i] = pw_g[i];
  __syncthreads();
  uint64_t x = 0x80000000ull + (uint64_t)tid * 0x9E3779B9ull;
  uint32_t wi = tid * 16;
  uint32_t acc = 0;
  uint16_t* o = out + (size_t)(blockIdx.x * 256 + tid) * 130;
  uint64_t t0;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int i = 0; i < STEPS; i++) {
    const uint32_t nw = pw[wi & 8191];
    const uint32_t slot = (uint32_t)x & (M - 1);
    const uint32_t sym = sy_s[slot >> 5] + tb[slot];
    uint32_t cc, f;
    if (V == 3) { cc = slot & ~255u; f = 256; }
    else { cc = cum_s[sym]; f = cum_s[sym + 1] - cc; }
    acc += sym;
    if (V == 1) o[i * 65] = (uint16_t)sym;
    if (V == 2) {
      uint32_t xl = (uint32_t)x;
      xl = f * (xl >> PB) + (slot - cc);
      x = xl < (1u << 31) ? ((uint64_t)xl << 32 | nw) : xl;
      if (xl < (1u << 31)) wi++;
    } else {
      x = (uint64_t)f * (x >> PB) + (slot - cc);
      if (x < (1ull << 31)) { x = (x << 32) | nw; wi++; }
    }
  }
  uint64_t t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  sink[blockIdx.x * 256 + tid] = acc + (uint32_t)x;
  if ((tid & 63) == 0) cyc[blockIdx.x * 4 + (tid >> 6)] = t1 - t0;
}

template <int V>
static int run(const char* name, const uint32_t* cum, const uint8_t* tb, const uint16_t* sy, const uint32_t* pw,
               uint16_t* out, uint64_t* cyc, uint32_t* sink, int ncu) {
  for (int per : {1, 2, 3}) {
    const int nb = ncu * per;
    hipLaunchKernelGGL(dstep<V>, dim3(nb), dim3(256), 0, 0, cum, tb, sy, pw, out, cyc, sink);
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(dstep<V>, dim3(nb), dim3(256), 0, 0, cum, tb, sy, pw, out, cyc, sink);
    CK(hipEventRecord(b));
    CK(hipDeviceSynchronize());
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    std::vector<uint64_t> c(nb * 4);
    CK(hipMemcpy(c.data(), cyc, nb * 4 * 8, hipMemcpyDeviceToHost));
    double s = 0; for (auto v : c) s += v;
    printf("%-28s WG/CU %d: %7.1f clk/step/wave (s_memtime), kernel %.3f ms\n", name, per, s / c.size() / STEPS, ms);
  }
  return 0;
}

int main() {
  // Laplacian-ish normalized table over 256 symbols summing to 2^15
  std::vector<uint32_t> f(256), cum(258, 0);
  uint32_t tot = 0;
  for (int s = 0; s < 256; s++) { int d = s < 128 ? s : 256 - s; f[s] = 1 + (uint32_t)(6000.0 * __builtin_exp(-d / 2.5)); tot += f[s]; }
  // fix to 2^15
  int diff = (int)M - (int)tot; f[0] += diff;
  for (int s = 0; s < 256; s++) cum[s + 1] = cum[s] + f[s];
  std::vector<uint16_t> sy(1024);
  std::vector<uint8_t> tb(M);
  for (int b = 0; b < 1024; b++) { uint32_t sl = b * 32; int s = 0; while (cum[s + 1] <= sl) s++; sy[b] = s; }
  for (uint32_t sl = 0; sl < M; sl++) { int s = sy[sl >> 5]; while (cum[s + 1] <= sl) s++; tb[sl] = (uint8_t)(s - sy[sl >> 5]); }
  std::vector<uint32_t> pw(8192);
  for (int i = 0; i < 8192; i++) pw[i] = 0x12345678u * (i + 1);
  uint32_t *d_cum, *d_pw, *sink; uint8_t* d_tb; uint16_t *d_sy, *out; uint64_t* cyc;
  int ncu = 256;
  CK(hipMalloc(&d_cum, 258 * 4)); CK(hipMalloc(&d_pw, 8192 * 4)); CK(hipMalloc(&d_tb, M)); CK(hipMalloc(&d_sy, 2048));
  CK(hipMalloc(&out, (size_t)ncu * 3 * 256 * 130 * 2 + 4096 * 65 * 2)); CK(hipMalloc(&cyc, ncu * 3 * 4 * 8)); CK(hipMalloc(&sink, ncu * 3 * 256 * 4));
  CK(hipMemcpy(d_cum, cum.data(), 258 * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_pw, pw.data(), 8192 * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_tb, tb.data(), M, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_sy, sy.data(), 2048, hipMemcpyHostToDevice));
  run<0>("V0 full step", d_cum, d_tb, d_sy, d_pw, out, cyc, sink, ncu);
  run<1>("V1 + scattered store", d_cum, d_tb, d_sy, d_pw, out, cyc, sink, ncu);
  run<2>("V2 32-bit advance", d_cum, d_tb, d_sy, d_pw, out, cyc, sink, ncu);
  run<3>("V3 no cum read", d_cum, d_tb, d_sy, d_pw, out, cyc, sink, ncu);
  return 0;
}
