#!/usr/bin/env python3
"""Measurement: pipelined throughput of encode only, decode only and encode+decode at D images in
flight (8192^2 synthetic, one image per slot), enqueue-only calls from one host thread.  Prints
ms per image for each mode.  Not part of the product or the bench line."""
import os
import sys
import time

D = int(sys.argv[1]) if len(sys.argv) > 1 else 20
K = int(sys.argv[2]) if len(sys.argv) > 2 else 200
MODES = sys.argv[3].split(",") if len(sys.argv) > 3 else ["enc", "dec", "both"]
os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, D))
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "hoh-ans_amd"))
import torch  # noqa: E402
import hoh_ans  # noqa: E402

W = H = 8192
L = hoh_ans.lib()
slots = []
for k in range(D):
    c = hoh_ans.Context(0)
    s = torch.cuda.Stream()
    rgb = hoh_ans.synth_rgb_dev(W, H, 1 + k, 4, ctx=c)
    out = torch.empty(L.hoh_encode_bound(W, H), dtype=torch.uint8, device="cuda")
    dec = torch.empty(W * H * 3, dtype=torch.uint8, device="cuda")
    ix = hoh_ans.Index()
    slots.append((c, s, rgb, out, dec, ix))
st = torch.zeros((K + D, 4), dtype=torch.int64, device="cuda")


def run(mode, n):
    for i in range(n):
        c, s, rgb, out, dec, ix = slots[i % D]
        with torch.cuda.stream(s):
            if mode in ("enc", "both"):
                hoh_ans.encode_image_async(rgb, W, H, out, st[i, 0:2], ctx=c, index=ix)
            if mode in ("dec", "both"):
                hoh_ans.decode_image_async(out, out.numel(), W, H, dec, st[i, 2:4], ctx=c, index=ix)


run(MODES[-1], D)
torch.cuda.synchronize()
for mode in MODES + MODES:
    run(mode, D)
    torch.cuda.synchronize()
    t = time.perf_counter()
    run(mode, K)
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    print("%-4s D=%d: %.3f ms/image (%.1f GB/s raw)" % (mode, D, el / K * 1e3, W * H * 3 * K / el / 1e9), flush=True)
if "both" in MODES:
    ok = all(bool(torch.equal(x[4], x[2])) for x in slots)
    print("lossless", ok)
