#!/usr/bin/env python3
"""Measurement: 8192^2 natural-statistic image (hoh_ans.natural, BASELINE configs[4]) encoded at
-sN and decoded, a few times, one image at a time; prints ms per encode / decode and the file
size.  Run under rocprofv3 --kernel-trace --stats for the per-kernel split."""
import hashlib
import os
import sys
import time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "hoh-ans_amd"))
import torch  # noqa: E402
import hoh_ans  # noqa: E402

W = H = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
speed = int(sys.argv[2]) if len(sys.argv) > 2 else 0
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
c = hoh_ans.Context(0)
rgb = hoh_ans.natural_rgb_dev(W, H, 1, ctx=c)
ix = hoh_ans.Index()
out, n, _ = hoh_ans.encode_image(rgb, W, H, ctx=c, index=ix, speed=speed)
torch.cuda.synchronize()
te = []
for _ in range(reps):
    t = time.perf_counter()
    out, n, _ = hoh_ans.encode_image(rgb, W, H, out_dev=out, ctx=c, index=ix, speed=speed)
    torch.cuda.synchronize()
    te.append(time.perf_counter() - t)
dec = torch.empty(W * H * 3, dtype=torch.uint8, device="cuda")
td = []
for _ in range(reps if speed == 0 else 0):          # the decoder takes -s0 files
    t = time.perf_counter()
    hoh_ans.decode_image(out, n, out_dev=dec, ctx=c, index=ix if speed == 0 else None)
    torch.cuda.synchronize()
    td.append(time.perf_counter() - t)
print("natural %dx%d -s%d: %d B (sha %s), encode %.2f ms, decode %s ms, lossless %s" %
      (W, H, speed, n, hashlib.sha256(out[:n].cpu().numpy().tobytes()).hexdigest()[:12], min(te) * 1e3,
       "%.2f" % (min(td) * 1e3) if td else "-", bool(torch.equal(dec, rgb)) if td else "-"), flush=True)
