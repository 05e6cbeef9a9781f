// Shared plumbing of the drop-in headers (include/hoh/*.hpp): one process-wide library context on
// device 0 (HOH_DEVICE overrides), created on first use.  The reference's free functions have no
// error channel beyond asserts / return values, so failures are reported on stderr and surface
// as the return values documented per function.
#pragma once
#include <cstdio>
#include <cstdlib>
#include "../hoh_ans.h"

namespace hoh_gpu {

inline hoh_ctx* ctx() {
  static hoh_ctx* c = [] {
    hoh_ctx* p = nullptr;
    const char* d = std::getenv("HOH_DEVICE");
    const int r = hoh_ctx_create(&p, d ? std::atoi(d) : 0);
    if (r != HOH_OK) {
      std::fprintf(stderr, "hoh-ans: no GPU context (%s)\n", hoh_strerror(r));
      std::abort();              // the product path never falls back to a CPU implementation
    }
    return p;
  }();
  return c;
}

inline bool ok(int r, const char* what) {
  if (r == HOH_OK) return true;
  std::fprintf(stderr, "hoh-ans: %s: %s\n", what, hoh_strerror(r));
  return false;
}

}  // namespace hoh_gpu
