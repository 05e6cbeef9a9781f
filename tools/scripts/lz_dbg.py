#!/usr/bin/env python3
"""Measurement (HOH_LIB = a -DLZ_DBG build): per-tile k_lz timing of the natural 8192^2 image at
-s0 -- phase-1 (segment walks) ticks, total ticks (100 MHz), stitch re-walk visits, max visits
of a segment walk."""
import ctypes as C
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "hoh-ans_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import hoh_ans  # noqa: E402

W = 8192
c = hoh_ans.Context(0)
rgb = hoh_ans.natural_rgb_dev(W, W, 1, ctx=c)
for _ in range(2):
    out, n, _ = hoh_ans.encode_image(rgb, W, W, ctx=c)
torch.cuda.synchronize()
ntiles = (W // 256) ** 2
npix_cap = 65536
lz_cap = ((npix_cap // 4 + npix_cap // 255 + 16) + 7) // 8 * 8
words = ntiles * 3 * (lz_cap + 1)
buf = np.zeros(words, dtype=np.uint32)
L = hoh_ans.lib()
L.hoh_debug_read.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t]
assert L.hoh_debug_read(c.h, 0, buf.ctypes.data, buf.nbytes) == 0
m = buf.reshape(ntiles, 3 * (lz_cap + 1))[:, 3 * lz_cap:]
w0, w1, w2 = m[:, 0].astype(np.int64), m[:, 1].astype(np.int64), m[:, 2].astype(np.int64)
p1 = w0 / 100.0
vis, fix, rounds = w1 & 0xffff, w1 >> 16, w2
print("slowest wave us: max %.0f p99 %.0f median %.0f" % (p1.max(), np.percentile(p1, 99), np.median(p1)))
print("stitch visits max %d" % fix.max())
o = np.argsort(-p1)[:12]
for t in o:
    print("tile %4d (%2d,%2d): slowest wave %6.0f us, visits %5d, rounds %6d -> %.2f us/visit, %.3f us/round" %
          (t, t % 32, t // 32, p1[t], vis[t], rounds[t], p1[t] / max(vis[t], 1), p1[t] / max(rounds[t], 1)))
print("all tiles: us/visit median %.2f" % np.median(p1 / np.maximum(vis, 1)))
