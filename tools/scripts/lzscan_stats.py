#!/usr/bin/env python3
"""Measurement (HOH_LIB = a -DHOH_DEBUG_READ build): k_lzscan's per-tile counters (EncodeJob::dbg)
after encoding the natural 8192^2 image at each given speed: totals, per-measure averages and the
wave-cycle split (s_memtime).
    HOH_LIB=var/dbg.so python tools/scripts/lzscan_stats.py [speeds]"""
import ctypes as C
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "hoh-ans_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import hoh_ans  # noqa: E402

W = 8192
L = hoh_ans.lib()
L.hoh_debug_read.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t]
c = hoh_ans.Context(0)
rgb = hoh_ans.natural_rgb_dev(W, W, 1, ctx=c)
names = ["measures", "posting_batches", "hits", "ring_runs", "image_runs", "ring_trips", "image_trips", "vert_runs",
         "cyc_measure", "cyc_vertical", "cyc_posting", "cyc_wave", "matches", "stitch_measures"]
for sp in [int(a) for a in sys.argv[1:]] or [1, 4]:
    out, n, _ = hoh_ans.encode_image(rgb, W, W, ctx=c, speed=sp)
    torch.cuda.synchronize()
    d = np.zeros((1024, 64), np.uint32)
    assert L.hoh_debug_read(c.h, 5, d.ctypes.data, d.nbytes) == 0
    d = d.astype(np.float64)
    tot = {nm: d[:, i].sum() for i, nm in enumerate(names)}
    print("-s%d: file %d B" % (sp, n))
    for nm in names:
        print("  %-16s total %14.0f  per tile mean %12.1f  max %12.0f" % (nm, tot[nm], d[:, names.index(nm)].mean(),
                                                                       d[:, names.index(nm)].max()))
    m = max(tot["measures"], 1)
    print("  per measure: posting batches %.2f, hits %.2f, ring runs %.2f (trips %.2f), image runs %.2f (trips %.2f), "
          "vertical runs %.2f; cycles: measure %.0f = posting %.0f + vertical %.0f + rest" % (
              tot["posting_batches"] / m, tot["hits"] / m, tot["ring_runs"] / m, tot["ring_trips"] / m,
              tot["image_runs"] / m, tot["image_trips"] / m, tot["vert_runs"] / m, tot["cyc_measure"] / m,
              tot["cyc_posting"] / m, tot["cyc_vertical"] / m))
    print("  wave cycles: measure share %.2f of the segment walks" % (tot["cyc_measure"] / max(tot["cyc_wave"], 1)))
    kept = d[:, 40:49].sum(axis=0)
    print("  prob_bits ladder (k_prune_s): planes by trials kept 0..8: %s" % " ".join("%d" % v for v in kept))
