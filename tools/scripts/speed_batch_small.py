#!/usr/bin/env python3
"""Measurement: -s>=1 batches of small images, stacked (the library's default stacks) against one
image per stack (HOH_SPEED_STACK_TILES=1: needs a knobs build, e.g. HOH_LIB=.../libhohgpu_check.so).
    python tools/scripts/speed_batch_small.py W H N SPEED REPS
Prints ms per image of hoh_encode_images_async over N natural images (seeds 1..N)."""
import os
import sys
import time

W, H, N, SPEED, REPS = (int(a) for a in sys.argv[1:6])
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "hoh-ans_amd"))
import torch  # noqa: E402
import hoh_ans  # noqa: E402

ctx = hoh_ans.Context(0)
stride = hoh_ans.lib().hoh_encode_bound(W, H)
img = W * H * 3
rgb = torch.empty(N * img, dtype=torch.uint8, device="cuda")
for i in range(N):
    rgb[i * img:(i + 1) * img] = hoh_ans.natural_rgb_dev(W, H, 1 + i, ctx=ctx)
out = torch.empty(N * stride, dtype=torch.uint8, device="cuda")
st = torch.zeros(2 * N, dtype=torch.int64, device="cuda")
torch.cuda.synchronize()
best = 1e9
for r in range(REPS + 1):
    t = time.perf_counter()
    hoh_ans.encode_images_async(rgb, N, W, H, out, stride, st, ctx=ctx, speed=SPEED)
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    if r:
        best = min(best, el)
s = st.cpu().numpy()
for i in range(N):
    hoh_ans.check_status(s[2 * i:2 * i + 2], "image %d" % i)
print("W=%d H=%d N=%d -s%d stack=%s: %.3f ms/image (%.1f MB/s)" % (
    W, H, N, SPEED, os.environ.get("HOH_SPEED_STACK_TILES", "default"), best / N * 1e3, img * N / best / 1e6))
