#!/usr/bin/env python3
"""Debug: batch encode (hoh_encode_images_async) vs single-image encodes, first differing byte."""
import os, sys
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "hoh-ans_amd"))
import numpy as np, torch, hoh_ans as hoh
for W, n in [(int(a.split('x')[0]), int(a.split('x')[1])) for a in (sys.argv[1:] or ['2048x4', '8192x4'])]:
    H = W
    ctx = hoh.Context(0)
    img = W * H * 3
    stride = hoh.lib().hoh_encode_bound(W, H)
    rgb = torch.empty(n * img, dtype=torch.uint8, device="cuda")
    for i in range(n):
        rgb[i * img:(i + 1) * img] = hoh.synth_rgb_dev(W, H, i + 1, 4, ctx=ctx)
    out = torch.full((n * stride,), 0xAB, dtype=torch.uint8, device="cuda")
    st = torch.zeros(2 * n, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()              # NULL stream: the library runs on the context's own stream
    hoh.encode_images_async(rgb, n, W, H, out, stride, st, ctx=ctx)
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    res = []
    for i in range(n):
        one, m, _ = hoh.encode_image(rgb[i * img:(i + 1) * img], W, H, ctx=ctx)
        a = out[i * stride:i * stride + m].cpu().numpy(); b = one[:m].cpu().numpy()
        d = np.flatnonzero(a != b)
        res.append((int(s[2 * i]), int(s[2 * i + 1]) == m, len(d), int(d[0]) if len(d) else -1))
        if len(d):
            print("  image %d: batch %s single %s" % (i, a[:16].tolist(), b[:16].tolist()))
    print(W, n, res, flush=True)
    ctx.close(); del rgb, out
