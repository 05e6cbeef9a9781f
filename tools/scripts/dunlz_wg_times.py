#!/usr/bin/env python3
"""Measurement (HOH_LIB = a -DDEC_DBG -DHOH_DEBUG_READ build): per-workgroup start/end
(s_memrealtime, 100 MHz) of both k_dunpred_lz launches while decoding the synthetic 8192^2 bench
image (no LZ tiles: every workgroup should leave at once)."""
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
rgb = hoh_ans.synth_rgb_dev(W, W, 1, 4, ctx=c)
ix = hoh_ans.Index()
out, n, _ = hoh_ans.encode_image(rgb, W, W, ctx=c, index=ix)
dec = torch.empty(W * W * 3, dtype=torch.uint8, device="cuda")
for _ in range(3):
    hoh_ans.decode_image(out, n, out_dev=dec, ctx=c, index=ix)
torch.cuda.synchronize()
print("lossless", bool(torch.equal(dec, rgb)))
buf = np.zeros(1 << 14, dtype=np.uint32)
L = hoh_ans.lib()
L.hoh_debug_read.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t]
assert L.hoh_debug_read(c.h, 2, buf.ctypes.data, buf.nbytes) == 0
gc = (1024 + 9) // 10
for name, part, nwg in (("few (many=0)", buf[:8192], 256 + gc), ("many=1", buf[8192:], 1024 + gc)):
    m = part.reshape(-1, 2).astype(np.int64)[:nwg]
    valid = m[:, 1] > 0
    if not valid.any():
        print(name, "no records")
        continue
    t0 = m[valid, 0].min()
    s, e = (m[:, 0] - t0) / 100.0, (m[:, 1] - t0) / 100.0
    ch = np.arange(len(m)) < gc
    print("%s: %d records, span %.1f us; chain WGs start max %.1f dur max %.1f; wavefront WGs start max %.1f "
          "dur max %.1f" % (name, valid.sum(), e[valid].max(), s[valid & ch].max() if (valid & ch).any() else -1,
                            (e - s)[valid & ch].max() if (valid & ch).any() else -1,
                            s[valid & ~ch].max() if (valid & ~ch).any() else -1,
                            (e - s)[valid & ~ch].max() if (valid & ~ch).any() else -1))
    print("  start times (us) by WG index, every 16th:", s[::16].round(1).tolist())
