#!/usr/bin/env python3
"""Measurement (GPU box): the bench's natural -s0 leg alone -- D contexts x batches of B natural
8192^2 images (seed 1), encode + decode through the batched calls, K steps; prints MB/s and
checks the decode against the input.   python3 tools/scripts/nat0_pipe.py [D] [B] [K]"""
import os
import sys
import time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "hoh-ans_amd"))
import torch  # noqa: E402
import hoh_ans  # noqa: E402

D = int(sys.argv[1]) if len(sys.argv) > 1 else 4
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
K = int(sys.argv[3]) if len(sys.argv) > 3 else 6
W = H = 8192
img = W * H * 3
L = hoh_ans.lib()
stride = L.hoh_encode_bound(W, H)
slots = []
for k in range(D):
    c = hoh_ans.Context(0)
    one = hoh_ans.natural_rgb_dev(W, H, 1, ctx=c)
    rgb = torch.empty(B * img, dtype=torch.uint8, device="cuda")
    for b in range(B):
        rgb[b * img:(b + 1) * img] = one
    slots.append(dict(ctx=c, s=torch.cuda.Stream(), rgb=rgb, out=torch.empty(B * stride, dtype=torch.uint8, device="cuda"),
                      dec=torch.empty(B * img, dtype=torch.uint8, device="cuda"), idx=hoh_ans.Index(),
                      st=torch.zeros(4 * B, dtype=torch.int64, device="cuda")))
torch.cuda.synchronize()


def step():
    for sl in slots:
        with torch.cuda.stream(sl["s"]):
            hoh_ans.encode_images_async(sl["rgb"], B, W, H, sl["out"], stride, sl["st"][:2 * B], ctx=sl["ctx"], index=sl["idx"])
            hoh_ans.decode_images_async(sl["out"], B, stride, W, H, sl["dec"], sl["st"][2 * B:], ctx=sl["ctx"], index=sl["idx"])


step()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(K):
    step()
torch.cuda.synchronize()
el = time.perf_counter() - t
ok = all(bool(torch.equal(sl["dec"], sl["rgb"])) for sl in slots)
print("natural -s0 pipeline D=%d B=%d: %.1f MB/s (%.3f ms per image), lossless %s" % (
    D, B, img * D * B * K / el / 1e6, el / (D * B * K) * 1e3, ok), flush=True)
