#!/usr/bin/env python3
"""Measurement (GPU box): pipelined -sN encodes of the natural 8192^2 image, D contexts in flight
(each on its own torch stream; an -s>=1 encode also uses its context's side stream), K encodes per
context; prints MB/s per (speed, D) and checks every file's SHA against golden_natural.json.
    python3 tools/scripts/speed_pipe.py SPEEDS DS [K]      e.g. 1,4 1,2,3,4 6"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "hoh-ans_amd"))
import torch  # noqa: E402
import hoh_ans  # noqa: E402

speeds = [int(x) for x in sys.argv[1].split(",")]
ds = [int(x) for x in sys.argv[2].split(",")]
K = int(sys.argv[3]) if len(sys.argv) > 3 else 6
W = H = 8192
img = W * H * 3
g = json.load(open(os.path.join(ROOT, "tests", "golden", "golden_natural.json")))
gold = {}
for r in g["files"]:
    sp = r["spec"]
    if sp.get("W") == W and sp.get("H") == H and sp.get("seed") == 1:
        gold[sp["speed"]] = r["out"]["sha256"]
L = hoh_ans.lib()
stride = L.hoh_encode_bound(W, H)
dmax = max(ds)
ctxs = [hoh_ans.Context(0) for _ in range(dmax)]
streams = [torch.cuda.Stream() for _ in range(dmax)]
rgb = hoh_ans.natural_rgb_dev(W, H, 1, ctx=ctxs[0])
outs = [torch.empty(stride, dtype=torch.uint8, device="cuda") for _ in range(dmax)]
st = torch.zeros((dmax, 2), dtype=torch.int64, device="cuda")
torch.cuda.synchronize()
for sp in speeds:
    for D in ds:
        def step():
            for k in range(D):
                with torch.cuda.stream(streams[k]):
                    hoh_ans.encode_image_async(rgb, W, H, outs[k], st[k], ctx=ctxs[k], speed=sp)
        step()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(K):
            step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t
        s = st.cpu().numpy()
        ok = all(hashlib.sha256(outs[k][:int(s[k][1])].cpu().numpy().tobytes()).hexdigest() == gold.get(sp)
                 for k in range(D))
        print("-s%d D=%d: %.1f MB/s (%.2f ms per image), files golden %s" % (sp, D, img * D * K / el / 1e6,
                                                                         el / (D * K) * 1e3, ok), flush=True)
