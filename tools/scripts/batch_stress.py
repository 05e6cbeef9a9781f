#!/usr/bin/env python3
"""Stress (GPU box): the bench's pipeline -- D slots of B images, encode + decode per step through
the batched calls (or the single-image calls with B = 1) -- repeated for SECONDS; every step's
files are compared with the first step's (which are SHA-checked against the reference goldens)
and every decode with its input.  A difference prints the step, slot, image, first differing
byte and the tile it falls in.

    python tools/scripts/batch_stress.py [D] [B] [SECONDS] [HWQ]"""
import hashlib
import json
import os
import sys
import time

D = int(sys.argv[1]) if len(sys.argv) > 1 else 4
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
SECS = float(sys.argv[3]) if len(sys.argv) > 3 else 60
if len(sys.argv) > 4:
    os.environ["GPU_MAX_HW_QUEUES"] = sys.argv[4]
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "hoh-ans_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import hoh_ans as hoh  # noqa: E402

W = H = 8192
img = W * H * 3
L = hoh.lib()
stride = L.hoh_encode_bound(W, H)
g = json.load(open(os.path.join(ROOT, "tests", "golden", "golden_bench.json")))
gold = {r["spec"]["seed"]: r["out"]["sha256"] for r in g["files"] if (r["spec"]["W"], r["spec"]["H"], r["spec"]["noise"]) == (8192, 8192, 4)}


class Slot:
    def __init__(self, k):
        self.seeds = [1 + k * B + b for b in range(B)]
        self.ctx = hoh.Context(0)
        self.stream = torch.cuda.Stream()
        self.rgb = torch.empty(B * img, dtype=torch.uint8, device="cuda")
        for b, sd in enumerate(self.seeds):
            self.rgb[b * img:(b + 1) * img] = hoh.synth_rgb_dev(W, H, sd, 4, ctx=self.ctx)
        self.index = hoh.Index()
        self.out = torch.zeros(B * stride, dtype=torch.uint8, device="cuda")
        self.dec = torch.zeros(B * img, dtype=torch.uint8, device="cuda")
        self.st = torch.zeros(4 * B, dtype=torch.int64, device="cuda")
        self.ref = None


slots = [Slot(k) for k in range(D)]
torch.cuda.synchronize()


def step(s):
    with torch.cuda.stream(s.stream):
        if B > 1:
            hoh.encode_images_async(s.rgb, B, W, H, s.out, stride, s.st[:2 * B], ctx=s.ctx, index=s.index)
            hoh.decode_images_async(s.out, B, stride, W, H, s.dec, s.st[2 * B:], ctx=s.ctx, index=s.index)
        else:
            hoh.encode_image_async(s.rgb, W, H, s.out, s.st[0:2], ctx=s.ctx, index=s.index)
            hoh.decode_image_async(s.out, s.out.numel(), W, H, s.dec, s.st[2:4], ctx=s.ctx, index=s.index)


def tile_of(data, off):
    """tile index of byte offset `off` of a .hoh (header 12 bytes at 8192^2, then 1023 varints)"""
    p, sizes = 12, []
    for _ in range(1023):
        b0 = data[p]; p += 1
        v = b0
        if b0 & 0x80:
            b1 = data[p]; p += 1
            v = ((b0 & 0x7f) << 7) + b1
            if b1 & 0x80:
                b2 = data[p]; p += 1
                v = ((b0 & 0x7f) << 14) + ((b1 & 0x7f) << 7) + b2
        sizes.append(v)
    if off < p:
        return "table"
    pos = p
    for t, z in enumerate(sizes):
        if off < pos + z:
            return "tile %d (+%d of %d)" % (t, off - pos, z)
        pos += z
    return "tile 1023 (+%d)" % (off - pos)


t0 = time.time()
rounds, bad = 0, 0
while time.time() - t0 < SECS:
    for s in slots:
        step(s)
    torch.cuda.synchronize()
    for k, s in enumerate(slots):
        st = s.st.cpu().numpy()
        for b in range(B):
            code, n = int(st[2 * b]), int(st[2 * b + 1])
            dcode = int(st[2 * B + 2 * b])
            o = s.out[b * stride:b * stride + n]
            if s.ref is None or len(s.ref) <= b:
                if s.ref is None:
                    s.ref = []
                sha = hashlib.sha256(o.cpu().numpy().tobytes()).hexdigest()
                print("slot %d image %d seed %d: %d B, golden %s" % (k, b, s.seeds[b], n, gold.get(s.seeds[b]) == sha),
                      flush=True)
                s.ref.append(o.clone())
                continue
            ok_file = code == 0 and n == s.ref[b].numel() and bool(torch.equal(o, s.ref[b]))
            ok_dec = dcode == 0 and bool(torch.equal(s.dec[b * img:(b + 1) * img], s.rgb[b * img:(b + 1) * img]))
            if not (ok_file and ok_dec):
                bad += 1
                msg = "ROUND %d slot %d image %d seed %d: enc code %d size %d (ref %d) dec code %d file_ok %s dec_ok %s" % (
                    rounds, k, b, s.seeds[b], code, n, s.ref[b].numel(), dcode, ok_file, ok_dec)
                if code == 0 and n == s.ref[b].numel() and not ok_file:
                    a, r = o.cpu().numpy(), s.ref[b].cpu().numpy()
                    d = np.flatnonzero(a != r)
                    msg += "; %d bytes differ, first at %d (%s), last at %d (%s)" % (
                        len(d), d[0], tile_of(r, int(d[0])), d[-1], tile_of(r, int(d[-1])))
                if not ok_dec:
                    x = s.dec[b * img:(b + 1) * img].cpu().numpy(), s.rgb[b * img:(b + 1) * img].cpu().numpy()
                    d = np.flatnonzero(x[0] != x[1])
                    if len(d):
                        px = d[0] // 3
                        msg += "; decode: %d bytes differ, first pixel (%d, %d) tile (%d, %d)" % (
                            len(d), px % W, px // W, (px % W) // 256, (px // W) // 256)
                print(msg, flush=True)
    rounds += 1
print("rounds %d (x %d images), failures %d, %.1f s" % (rounds, D * B, bad, time.time() - t0), flush=True)
