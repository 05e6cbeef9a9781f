#!/usr/bin/env python3
"""Measurement: pipelined throughput of the batched path (hoh_encode_images_async /
hoh_decode_images_async) for encode only, decode only and both: D slots (contexts + streams) of B
8192^2 synthetic images, K steps, HIP's default hardware queues.  Prints ms per image per mode.
    python tools/scripts/batch_pipe.py [D] [B] [K] [modes]"""
import os
import sys
import time

D = int(sys.argv[1]) if len(sys.argv) > 1 else 4
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
K = int(sys.argv[3]) if len(sys.argv) > 3 else 40
MODES = sys.argv[4].split(",") if len(sys.argv) > 4 else ["enc", "dec", "both"]
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "hoh-ans_amd"))
import torch  # noqa: E402
import hoh_ans  # noqa: E402

W = H = 8192
img = W * H * 3
L = hoh_ans.lib()
stride = L.hoh_encode_bound(W, H)
slots = []
for k in range(D):
    c = hoh_ans.Context(0)
    s = torch.cuda.Stream()
    rgb = torch.empty(B * img, dtype=torch.uint8, device="cuda")
    for b in range(B):
        rgb[b * img:(b + 1) * img] = hoh_ans.synth_rgb_dev(W, H, 1 + k * B + b, 4, ctx=c)
    out = torch.empty(B * stride, dtype=torch.uint8, device="cuda")
    dec = torch.empty(B * img, dtype=torch.uint8, device="cuda")
    slots.append((c, s, rgb, out, dec, hoh_ans.Index()))
st = torch.zeros((D, 4 * B), dtype=torch.int64, device="cuda")
torch.cuda.synchronize()


def run(mode, n):
    for i in range(n):
        c, s, rgb, out, dec, ix = slots[i % D]
        with torch.cuda.stream(s):
            if mode in ("enc", "both"):
                hoh_ans.encode_images_async(rgb, B, W, H, out, stride, st[i % D, :2 * B], ctx=c, index=ix)
            if mode in ("dec", "both"):
                hoh_ans.decode_images_async(out, B, stride, W, H, dec, st[i % D, 2 * B:], ctx=c, index=ix)


run(MODES[0] if MODES == ["enc"] else "both", D)
torch.cuda.synchronize()
for mode in MODES:
    run(mode, D)
    torch.cuda.synchronize()
    t = time.perf_counter()
    run(mode, K)
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    print("%-4s D=%d B=%d: %.3f ms/image (%.1f GB/s raw)" % (mode, D, B, el / K / B * 1e3, img * B * K / el / 1e9),
          flush=True)
if "both" in MODES:
    print("lossless", all(bool(torch.equal(x[4], x[2])) for x in slots))
