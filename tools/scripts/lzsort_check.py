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
ar = np.arange(cap, dtype=np.int64)[None, :]
for r in range(reps):
    out, n, _ = hoh_ans.encode_image(rgb, W, W, ctx=c, speed=speed)
    torch.cuda.synchronize()
    sha = hashlib.sha256(out[:n].cpu().numpy().tobytes()).hexdigest()[:16]
    assert L.hoh_debug_read(c.h, 3, lzs.ctypes.data, lzs.nbytes) == 0
    assert L.hoh_debug_read(c.h, 4, fpb.ctypes.data, fpb.nbytes) == 0
    F = fpb[:per].reshape(ntiles, cap)
    TP = fpb[per:2 * per].reshape(ntiles, cap) & 0xffffff                    # rgb | run8 << 24
    R8 = fpb[3 * per:].view(np.uint8)[:per].reshape(ntiles, cap)
    S = lzs[:2 * per:2].reshape(ntiles, cap)
    T = lzs[1:2 * per:2].reshape(ntiles, cap)                                 # the sorted fingerprints
    R = lzs[4 * per:].view(np.uint16)[:per].reshape(ntiles, cap)
    E = lzs[4 * per:].view(np.uint16)[per:2 * per].reshape(ntiles, cap)
    start = np.ones_like(TP, dtype=bool)
    start[:, 1:] = TP[:, 1:] != TP[:, :-1]
    inner = (R8 >= 4) & ~start
    h = ((F.astype(np.uint64) * 0x9E3779B1) & 0xffffffff) >> 16
    key = np.where(inner, np.uint64(1 << 32) + ar.astype(np.uint64), (h << 16) | ar.astype(np.uint64))
    order = np.argsort(key, axis=1, kind="stable")
    sk = np.take_along_axis(key, order, axis=1)
    nl = (~inner).sum(axis=1)
    listed = ar < nl[:, None]
    pos = (sk & 0xffff).astype(np.int64)
    bad_s = np.any(listed & (S != (sk & 0xffffffff).astype(np.uint32)), axis=1)
    bad_t = np.any(listed & (T != np.take_along_axis(F, pos, axis=1)), axis=1)
    sidx = np.maximum.accumulate(np.where(start, ar, 0), axis=1)         # each position's run start
    nxt = np.minimum.accumulate(np.where(start, ar, cap)[:, ::-1], axis=1)[:, ::-1]
    runend = np.empty_like(nxt)
    runend[:, :-1] = nxt[:, 1:] - 1
    runend[:, -1] = cap - 1
    want_e = np.where(np.take_along_axis(R8, pos, axis=1) >= 4, np.take_along_axis(runend, pos, axis=1), pos)
    bad_e = np.any(listed & (E != want_e), axis=1)
    rank = np.zeros((ntiles, cap + 1), np.int64)                        # column cap: unlisted slots
    np.put_along_axis(rank, np.where(listed, pos, cap), np.broadcast_to(ar, pos.shape), axis=1)
    rank = rank[:, :cap]
    # an unlisted position: the last listed position before it in its group (its run's start, or
    # a hash-colliding listed position after that start)
    want_r = rank.copy()
    for tb in range(ntiles):
        lk = sk[tb, :nl[tb]]
        iq = np.flatnonzero(inner[tb])
        want_r[tb, iq] = np.searchsorted(lk, (h[tb, iq] << np.uint64(16)) | iq.astype(np.uint64)) - 1
    bad_r = np.any(R != want_r, axis=1)
    bad_s |= bad_e
    bad = bad_s | bad_t | bad_r
    bad_total += int(bad.sum())
    first = np.flatnonzero(bad)[:4].tolist()
    for tb in first[:1]:                                                # detail of the first wrong tile
        d = np.flatnonzero(R[tb] != want_r[tb])[:8]
        for p in d.tolist():
            print("  tile %d pos %d: rank %d want %d inner %d start %d R8 %d runstart %d F %08x h %04x" % (
                tb, p, R[tb, p], want_r[tb, p], inner[tb, p], start[tb, p], R8[tb, p], sidx[tb, p], F[tb, p],
                h[tb, p]), flush=True)
    print("rep %d: %d B sha %s  tiles with wrong lists: %d (keys %d, fingerprints %d, ranks %d) first %s" %
          (r, n, sha, bad.sum(), bad_s.sum(), bad_t.sum(), bad_r.sum(), first), flush=True)
print("TOTAL wrong tile lists over %d encodes: %d" % (reps, bad_total))
