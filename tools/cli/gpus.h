// Device-list options shared by the choh / dhoh drop-ins: `--gpus N` (devices 0 .. N-1) or
// `--devices a,b,...` (a device may repeat: several shards on one GPU).  Both are removed from
// argv so the positional arguments keep the reference's order (choh.cpp:385-427, dhoh.cpp:298-310).
#pragma once
#include <cstdlib>
#include <cstring>
#include <vector>

static std::vector<int> take_devices(int& argc, char** argv) {
  std::vector<int> dev;
  int w = 1;
  for (int i = 1; i < argc; i++) {
    if (!std::strcmp(argv[i], "--gpus") && i + 1 < argc) {
      const int n = std::atoi(argv[++i]);
      dev.clear();
      for (int k = 0; k < n; k++) dev.push_back(k);
    } else if (!std::strcmp(argv[i], "--devices") && i + 1 < argc) {
      dev.clear();
      for (const char* p = argv[++i]; *p;) {
        dev.push_back(std::atoi(p));
        while (*p && *p != ',') p++;
        if (*p == ',') p++;
      }
    } else {
      argv[w++] = argv[i];
    }
  }
  argc = w;
  return dev;
}
