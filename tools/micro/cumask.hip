// Where do workgroups of a CU-masked stream land?  Prints, per mask, the (XCC, SE, CU) of 2048
// one-wave workgroups.  Measurement only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <map>

__global__ void probe(uint32_t* out) {
  uint32_t hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  if (threadIdx.x == 0) { out[2 * blockIdx.x] = hw; out[2 * blockIdx.x + 1] = xcc; }
  // keep the wave alive a little so blocks spread
  uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < 2000) {}
}

static void run(const char* name, const std::vector<uint32_t>& mask) {
  hipStream_t s;
  if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size() * 32, mask.data()) != hipSuccess) { printf("mask fail\n"); return; }
  const int nb = 2048;
  uint32_t* d;
  hipMalloc(&d, nb * 8);
  hipLaunchKernelGGL(probe, dim3(nb), dim3(64), 0, s, d);
  std::vector<uint32_t> h(nb * 2);
  hipMemcpyAsync(h.data(), d, nb * 8, hipMemcpyDeviceToHost, s);
  hipStreamSynchronize(s);
  std::map<int, int> perx;
  std::map<int, int> units;
  for (int i = 0; i < nb; i++) {
    const uint32_t hw = h[2 * i], x = h[2 * i + 1] & 15;
    const int cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
    perx[x]++;
    units[x * 1000 + se * 100 + sh * 20 + cu]++;
  }
  printf("%s: %zu distinct CUs; per XCC:", name, units.size());
  for (auto& kv : perx) printf(" %d:%d", kv.first, kv.second);
  printf("\n");
  hipFree(d);
  hipStreamDestroy(s);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int ncu = p.multiProcessorCount, nw = (ncu + 31) / 32;
  printf("CUs %d\n", ncu);
  std::vector<uint32_t> all(nw, 0xffffffffu), first32(nw, 0), every8(nw, 0), mod8lt1(nw, 0), low4(nw, 0);
  first32[0] = 0xffffffffu;
  for (int i = 0; i < ncu; i++) {
    if (i % 8 == 0) every8[i / 32] |= 1u << (i % 32);
    if ((i / 8) % 8 == 0) mod8lt1[i / 32] |= 1u << (i % 32);
    if (i < 4) low4[i / 32] |= 1u << (i % 32);
  }
  run("all", all);
  run("first32", first32);
  run("every8th", every8);
  run("blocks-of-8 every 64", mod8lt1);
  run("first4", low4);
  return 0;
}
