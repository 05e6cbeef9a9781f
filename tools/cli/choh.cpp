// choh drop-in (choh.cpp:394-527): `choh in.rgb out.hoh width height [-sN]` on the GPU.
// Writes the bytes the reference writes and prints the size it prints (header +
// tile size for untiled images, of which only the header is written).  Speeds -s0..-s4 as in the
// reference (choh.cpp:408-427): default and unknown settings mean -s1 (the reference reads
// argv[5] unchecked when it is missing; here that is the documented default).
// `--gpus N` / `--devices a,b,..` (tools/cli/gpus.h) encode over several GPUs in this one process
// (hoh_mgpu_encode_image: a band of tile rows per device, one RCCL gather); same bytes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../../include/hoh_ans.h"
#include "gpus.h"

static bool read_file(const char* path, std::vector<uint8_t>& b) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return false;
  std::fseek(f, 0, SEEK_END);
  const long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  b.resize(n > 0 ? (size_t)n : 0);
  const bool ok = b.empty() || std::fread(b.data(), 1, b.size(), f) == b.size();
  std::fclose(f);
  return ok;
}

int main(int argc, char** argv) {
  const std::vector<int> devices = take_devices(argc, argv);
  if (argc < 5) {
    std::printf("not enough arguments\nusage: choh infile.rgb outfile.hoh width height -s0\n");
    return 1;
  }
  const int W = std::atoi(argv[3]), H = std::atoi(argv[4]);
  if (W == 0 || H == 0) {
    std::printf("invalid width or height\n");
    return 2;
  }
  int speed = 1;
  if (argc > 5) {
    static const char* names[5] = {"-s0", "-s1", "-s2", "-s3", "-s4"};
    int k = 0;
    while (k < 5 && std::strcmp(argv[5], names[k]) != 0) k++;
    if (k < 5) speed = k;
    else std::printf("invalid speed setting\nusage: choh infile.rgb outfile.hoh width height -sN\n");
  }
  std::vector<uint8_t> in;
  if (!read_file(argv[1], in)) { std::printf("could not read %s\n", argv[1]); return 3; }
  const size_t raw = (size_t)W * H * 3;
  if (in.size() < raw) { std::printf("input shorter than width*height*3\n"); return 3; }
  hoh_ctx* ctx = nullptr;
  const int dev0 = devices.empty() ? 0 : devices[0];   // --devices 3 / one entry: that GPU
  hoh_mgpu* mg = nullptr;
  int r = devices.size() > 1 ? hoh_mgpu_create(&mg, (int)devices.size(), devices.data()) : hoh_ctx_create(&ctx, dev0);
  if (r != HOH_OK) { std::fprintf(stderr, "choh: %s\n", hoh_strerror(r)); return r; }
  const size_t cap = hoh_encode_bound(W, H);
  uint8_t *d_in = nullptr, *d_out = nullptr;
  (void)hipSetDevice(dev0);
  if (!mg && hipMalloc(&d_in, raw) != hipSuccess) return HOH_E_HIP;
  if (hipMalloc(&d_out, cap) != hipSuccess) return HOH_E_HIP;
  if (!mg && hipMemcpy(d_in, in.data(), raw, hipMemcpyHostToDevice) != hipSuccess) return HOH_E_HIP;
  size_t n = 0, printed = 0;
  r = mg ? hoh_mgpu_encode_image(mg, in.data(), W, H, speed, d_out, cap, &n, &printed)
         : hoh_encode_image(ctx, d_in, W, H, speed, d_out, cap, &n, &printed, nullptr);
  if (r != HOH_OK) { std::fprintf(stderr, "choh: %s\n", hoh_strerror(r)); return r; }
  std::vector<uint8_t> out(n);
  if (n && hipMemcpy(out.data(), d_out, n, hipMemcpyDeviceToHost) != hipSuccess) return HOH_E_HIP;
  std::printf("%d\n", (int)printed);
  FILE* f = std::fopen(argv[2], "wb");
  if (!f || (n && std::fwrite(out.data(), 1, n, f) != n)) { std::printf("could not write %s\n", argv[2]); return 3; }
  std::fclose(f);
  if (d_in) (void)hipFree(d_in);
  (void)hipFree(d_out);
  if (mg) hoh_mgpu_destroy(mg);
  if (ctx) hoh_ctx_destroy(ctx);
  return 0;
}
