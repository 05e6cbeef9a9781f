#!/usr/bin/env python3
"""Measurement: dhoh WITHOUT the side index (a foreign .hoh: every stream one serial rANS chain)
of an 8192^2 image, one image at a time.  Prints ms per decode (best of N), the rANS stage's
device time (profiling marks) and whether the decode is lossless.

    python tools/scripts/noix_bench.py [synth|natural] [size] [reps] [adaptive|lanes|multi|wave]
The last argument pins the chain kernel (hoh_ctx_set_option HOH_OPT_NOIX_DECODER); wave is the
round-2 decoder (one wave per stream)."""
import os
import sys
import time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "hoh-ans_amd"))
import torch  # noqa: E402
import hoh_ans  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "synth"
W = H = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
mode = sys.argv[4] if len(sys.argv) > 4 else "adaptive"
c = hoh_ans.Context(0)
c.set_option(hoh_ans.OPT_NOIX_DECODER, {"adaptive": hoh_ans.NOIX_ADAPTIVE, "lanes": hoh_ans.NOIX_LANES,
                                        "multi": hoh_ans.NOIX_MULTI, "wave": hoh_ans.NOIX_WAVE}[mode])
rgb = hoh_ans.natural_rgb_dev(W, H, 1, ctx=c) if kind == "natural" else hoh_ans.synth_rgb_dev(W, H, 1, 4, ctx=c)
out, n, _ = hoh_ans.encode_image(rgb, W, H, ctx=c)
dec = torch.empty(W * H * 3, dtype=torch.uint8, device="cuda")
hoh_ans.decode_image(out, n, out_dev=dec, ctx=c, index=None)
torch.cuda.synchronize()
c.profiling(True)
c.reset_stats()
td = []
for _ in range(reps):
    dec.zero_()
    torch.cuda.synchronize()
    t = time.perf_counter()
    hoh_ans.decode_image(out, n, out_dev=dec, ctx=c, index=None)
    torch.cuda.synchronize()
    td.append(time.perf_counter() - t)
st = {k: v[0] / v[1] for k, v in c.kernel_stats().items() if v[1]}
print("no-index %s %dx%d (%s): %d B, decode %.2f ms (%.1f GB/s), stages %s, lossless %s" %
      (kind, W, H, mode, n, min(td) * 1e3,
       W * H * 3 / min(td) / 1e9, {k: round(v, 3) for k, v in st.items()}, bool(torch.equal(dec, rgb))), flush=True)
