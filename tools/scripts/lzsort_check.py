#!/usr/bin/env python3
"""Measurement (HOH_LIB = a `make DEBUG_READ=1`-style build exporting hoh_debug_read): checks
k_lzsort's posting lists after each of REPS -s2 encodes of the natural 8192^2 image against an
exact recomputation from the fingerprints k_lzfp wrote -- per tile the keys pos | hash << 16 in
ascending order (hash-major, position-minor: the stable LSD sort), the sorted fingerprints beside
them and the rank of every position.  Prints, per encode, the file SHA and the number of tiles
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

speed = int(sys.argv[1]) if len(sys.argv) > 1 else 2
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
W = 8192
ntiles, cap = (W // 256) ** 2, 65536
per = ntiles * cap
L = hoh_ans.lib()
L.hoh_debug_read.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t]
c = hoh_ans.Context(0)
rgb = hoh_ans.natural_rgb_dev(W, W, 1, ctx=c)
lzs = np.zeros(per * 5 // 2, np.uint32)          # S, T (u32 each), rank (u16)
fpb = np.zeros(per, np.uint32)
bad_total = 0
for r in range(reps):
    out, n, _ = hoh_ans.encode_image(rgb, W, W, ctx=c, speed=speed)
    torch.cuda.synchronize()
    sha = hashlib.sha256(out[:n].cpu().numpy().tobytes()).hexdigest()[:16]
    assert L.hoh_debug_read(c.h, 3, lzs.ctypes.data, lzs.nbytes) == 0
    assert L.hoh_debug_read(c.h, 4, fpb.ctypes.data, fpb.nbytes) == 0
    F = fpb.reshape(ntiles, cap)
    S = lzs[:per].reshape(ntiles, cap)
    T = lzs[per:2 * per].reshape(ntiles, cap)
    R = lzs[2 * per:].view(np.uint16)[:per].reshape(ntiles, cap)
    h = ((F.astype(np.uint64) * 0x9E3779B1) & 0xffffffff) >> 16
    want = np.sort((h << 16).astype(np.uint32) | np.arange(cap, dtype=np.uint32)[None, :], axis=1)
    pos = want & 0xffff
    bad_s = np.any(S != want, axis=1)
    bad_t = np.any(T != np.take_along_axis(F, pos.astype(np.int64), axis=1), axis=1)
    rank = np.empty_like(pos)
    np.put_along_axis(rank, pos.astype(np.int64), np.arange(cap, dtype=np.uint32)[None, :].repeat(ntiles, 0), axis=1)
    bad_r = np.any(R != rank, axis=1)
    bad = bad_s | bad_t | bad_r
    bad_total += int(bad.sum())
    first = np.flatnonzero(bad)[:4].tolist()
    print("rep %d: %d B sha %s  tiles with wrong lists: %d (keys %d, fingerprints %d, ranks %d) first %s" %
          (r, n, sha, bad.sum(), bad_s.sum(), bad_t.sum(), bad_r.sum(), first), flush=True)
print("TOTAL wrong tile lists over %d encodes: %d" % (reps, bad_total))
