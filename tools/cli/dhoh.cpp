// dhoh drop-in (dhoh.cpp:297-420): `dhoh in.hoh out.rgb` on the GPU.  Decodes tiled RGB .hoh
// files as written by choh -s0 (the reference crashes on them) and writes the raw
// interleaved RGB bytes.  Return codes: 3/4 not a .hoh, 5 unknown pixel format, and the
// library's status code for anything it cannot decode.  `--gpus N` / `--devices a,b,..`
// (tools/cli/gpus.h) decode over several GPUs in this process (hoh_mgpu_decode_image).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../../include/hoh_ans.h"
#include "gpus.h"

int main(int argc, char** argv) {
  const std::vector<int> devices = take_devices(argc, argv);
  if (argc == 2 && (!std::strcmp(argv[1], "--help") || !std::strcmp(argv[1], "-h"))) {
    std::printf("usage: dhoh infile.hoh outfile.rgb\n");
    return 0;
  }
  if (argc == 2 && !std::strcmp(argv[1], "--version")) { std::printf("%s\n", hoh_version()); return 0; }
  if (argc < 3) { std::printf("not enough arguments!\nusage: dhoh infile.hoh outfile.rgb\n"); return 1; }
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) { std::printf("could not read %s\n", argv[1]); return 3; }
  std::vector<uint8_t> in;
  {
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    in.resize(n > 0 ? (size_t)n : 0);
    if (!in.empty() && std::fread(in.data(), 1, in.size(), f) != in.size()) { std::fclose(f); return 3; }
    std::fclose(f);
  }
  if (in.size() < 8) { std::printf("not a valid hoh file!\n"); return 3; }
  if (in[0] != 153 || in[1] != 72 || in[2] != 79 || in[3] != 72) { std::printf("not a valid hoh file!\n"); return 4; }
  static const char* fmt[] = {"bit", "greyscale", "rgb", "greyscale + alpha", "rgb + alpha"};
  if (in[4] <= 4) std::printf("pixel format: %s\n", fmt[in[4]]);
  else if (in[4] == 255) { std::printf("invalid pixel format!\n"); return 4; }
  else { std::printf("unknown pixel format!\n"); return 5; }
  int W = 0, H = 0, xt = 0, yt = 0;
  int r = hoh_peek_header(in.data(), in.size(), &W, &H, &xt, &yt);
  if (r != HOH_OK) { std::fprintf(stderr, "dhoh: %s\n", hoh_strerror(r)); return r; }
  std::printf("width: %d\nheight: %d\n", W, H);
  hoh_ctx* ctx = nullptr;
  const int dev0 = devices.empty() ? 0 : devices[0];   // --devices 3 / one entry: that GPU
  hoh_mgpu* mg = nullptr;
  r = devices.size() > 1 ? hoh_mgpu_create(&mg, (int)devices.size(), devices.data()) : hoh_ctx_create(&ctx, dev0);
  if (r != HOH_OK) { std::fprintf(stderr, "dhoh: %s\n", hoh_strerror(r)); return r; }
  const size_t raw = (size_t)W * H * 3;
  uint8_t *d_in = nullptr, *d_rgb = nullptr;
  (void)hipSetDevice(dev0);
  if (hipMalloc(&d_in, in.size()) != hipSuccess || (!mg && hipMalloc(&d_rgb, raw) != hipSuccess)) return HOH_E_HIP;
  if (hipMemcpy(d_in, in.data(), in.size(), hipMemcpyHostToDevice) != hipSuccess) return HOH_E_HIP;
  std::vector<uint8_t> out(raw);
  if (mg) {
    r = hoh_mgpu_decode_image(mg, d_in, in.size(), out.data(), raw, &W, &H);
  } else {
    r = hoh_decode_image(ctx, d_in, in.size(), d_rgb, raw, &W, &H, nullptr);
    if (r == HOH_OK && hipMemcpy(out.data(), d_rgb, raw, hipMemcpyDeviceToHost) != hipSuccess) r = HOH_E_HIP;
  }
  if (r != HOH_OK) { std::fprintf(stderr, "dhoh: %s\n", hoh_strerror(r)); return r; }
  FILE* o = std::fopen(argv[2], "wb");
  if (!o || std::fwrite(out.data(), 1, raw, o) != raw) { std::printf("could not write %s\n", argv[2]); return 3; }
  std::fclose(o);
  (void)hipFree(d_in);
  if (d_rgb) (void)hipFree(d_rgb);
  if (mg) hoh_mgpu_destroy(mg);
  if (ctx) hoh_ctx_destroy(ctx);
  return 0;
}
