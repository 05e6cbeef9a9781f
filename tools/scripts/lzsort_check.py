#!/usr/bin/env python3
"""Measurement (HOH_LIB = a `make DEBUG_READ=1`-style build exporting hoh_debug_read): checks
k_lzsort's posting lists after each of REPS -s2 encodes of the natural 8192^2 image against an
exact recomputation from what k_lzfp wrote (fingerprints, pixels, runs) -- per tile the listed
positions' keys pos | hash << 16 in ascending order (hash-major, position-minor: the stable LSD
sort; a flat run's positions after its start are not listed), the sorted fingerprints and run
ends beside them, and the rank of every position (of its run's start for the unlisted ones).  Prints, per encode, the file SHA and the number of tiles
whose lists differ (any nonzero count is the race).

Usage: HOH_LIB=var/dbg.so python3 tools/scripts/lzsort_check.py [speed=2] [reps=10]"""
import ctypes as C
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "hoh-ans_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import hoh_ans  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "tests"))
from checklib import check_posting_lists  # noqa: E402

speed = int(sys.argv[1]) if len(sys.argv) > 1 else 2
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
W = 8192
ntiles, cap = (W // 256) ** 2, 65536
per = ntiles * cap
L = hoh_ans.lib()
L.hoh_debug_read.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t]
c = hoh_ans.Context(0)
rgb = hoh_ans.natural_rgb_dev(W, W, 1, ctx=c)
lzs = np.zeros(per * 5, np.uint32)               # entries, first-pass entries (key, fingerprint: u32 pairs), rank, end (u16 each)
fpb = np.zeros(per * 13 // 4, np.uint32)         # F, pixels, transposed F (u32 each), run8 (u8)
bad_total = 0
for r in range(reps):
    out, n, _ = hoh_ans.encode_image(rgb, W, W, ctx=c, speed=speed)
    torch.cuda.synchronize()
    sha = hashlib.sha256(out[:n].cpu().numpy().tobytes()).hexdigest()[:16]
    assert L.hoh_debug_read(c.h, 3, lzs.ctypes.data, lzs.nbytes) == 0
    assert L.hoh_debug_read(c.h, 4, fpb.ctypes.data, fpb.nbytes) == 0
    bad, bad_s, bad_t, bad_r = check_posting_lists(fpb, lzs, ntiles, cap)
    bad_total += int(bad.sum())
    first = np.flatnonzero(bad)[:4].tolist()
    print("rep %d: %d B sha %s  tiles with wrong lists: %d (keys %d, fingerprints %d, ranks %d) first %s" %
          (r, n, sha, bad.sum(), bad_s.sum(), bad_t.sum(), bad_r.sum(), first), flush=True)
print("TOTAL wrong tile lists over %d encodes: %d" % (reps, bad_total))
