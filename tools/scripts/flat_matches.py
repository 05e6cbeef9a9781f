#!/usr/bin/env python3
"""Debug (GPU box, HOH_LIB = a -DHOH_DEBUG_READ build): tile 0's LZ match list of a 256^2 test
image at -sN from the GPU against a direct restatement of lz.hpp:32-95 (fast enough for images
whose matches short-circuit)."""
import ctypes as C
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "hoh-ans_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import hoh_ans  # noqa: E402

sp = int(sys.argv[1]) if len(sys.argv) > 1 else 2
kind = sys.argv[2] if len(sys.argv) > 2 else "flat"
W = H = 256
img = np.full((H, W, 3), 77, np.uint8)
if kind == "halfflat":
    img[128:] = 9
c = hoh_ans.Context(0)
data, printed = hoh_ans.choh(img, ctx=c, speed=sp)
npix = W * H
lz_cap = ((npix // 4 + npix // 255 + 16) + 7) // 8 * 8
buf = np.zeros(3 * (lz_cap + 1), np.uint32)
L = hoh_ans.lib()
L.hoh_debug_read.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t]
assert L.hoh_debug_read(c.h, 0, buf.ctypes.data, buf.nbytes) == 0
gpu = []
for k in range(lz_cap):
    q, ln, b = buf[3 * k:3 * k + 3]
    if ln == 0:
        break
    gpu.append((int(q), int(ln), int(b)))
# restatement (pixels as tuples, tile raster order)
px = [tuple(v) for v in img.reshape(-1, 3)]
limit = 1 << {1: 10, 2: 11, 3: 12, 4: 14}[sp]
ref, i = [], 0
while i < npix:
    longest, best = 0, -1
    for back in range(1, min(limit, i) + 1):
        o = 0
        while i + o < npix and px[i + o] == px[i - back + o] and o < 259:
            o += 1
        if o > longest:
            longest, best = o, back
            if o == 259:
                break
    if longest < 259:
        back = W
        while back <= (1 << 16) and i - back >= 0:
            o = 0
            while i + o < npix and px[i + o] == px[i - back + o] and o < 259:
                o += 1
            if o > longest:
                longest, best = o, back
                if o == 259:
                    back = limit
            back += W
    if longest < 4:
        i += 1
    else:
        ref.append((i, longest, best))
        i += longest
print("-s%d %s: printed %d, gpu matches %d, ref matches %d" % (sp, kind, printed, len(gpu), len(ref)))
for k in range(max(len(gpu), len(ref))):
    a = gpu[k] if k < len(gpu) else None
    b = ref[k] if k < len(ref) else None
    if a != b:
        print("  first difference at match %d: gpu %s ref %s; around: gpu %s ref %s" % (k, a, b, gpu[max(0, k - 2):k + 3], ref[max(0, k - 2):k + 3]))
        break
else:
    print("  match lists equal")
