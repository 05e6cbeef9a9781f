#!/usr/bin/env python3
"""Measurement (HOH_LIB = a -DDEC_DBG build): per-workgroup start/end of the k_dunpred_lz "many"
launch decoding the natural 8192^2 -s0 file: chain workgroups vs wavefront workgroups."""
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
ix = hoh_ans.Index()
out, n, _ = hoh_ans.encode_image(rgb, W, W, ctx=c, index=ix)
dec = torch.empty(W * W * 3, dtype=torch.uint8, device="cuda")
for _ in range(2):
    hoh_ans.decode_image(out, n, out_dev=dec, ctx=c, index=ix)
torch.cuda.synchronize()
print("lossless", bool(torch.equal(dec, rgb)))
buf = np.zeros(1 << 14, dtype=np.uint32)
L = hoh_ans.lib()
L.hoh_debug_read.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t]
assert L.hoh_debug_read(c.h, 2, buf.ctypes.data, buf.nbytes) == 0
m = buf[8192:].reshape(-1, 2).astype(np.int64)
gc = (1024 + 9) // 10
valid = m[:, 1] > 0
t0 = m[valid, 0].min()
s, e = (m[:, 0] - t0) / 100.0, (m[:, 1] - t0) / 100.0
ch = np.arange(len(m)) < gc
wf = valid & ~ch
print("launch span %.0f us" % (e[valid].max()))
d = e - s
print("chains: %d WGs, start max %.0f us, duration max %.0f median %.0f us, end max %.0f" % (
    (valid & ch).sum(), s[valid & ch].max(), d[valid & ch].max(), np.median(d[valid & ch]), e[valid & ch].max()))
print("wavefront: %d WGs, start max %.0f us, duration max %.0f median %.0f us, end max %.0f" % (
    wf.sum(), s[wf].max(), d[wf].max(), np.median(d[wf]), e[wf].max()))
print("chain durations sorted (us):", np.sort(d[valid & ch])[::-1][:20].round())
