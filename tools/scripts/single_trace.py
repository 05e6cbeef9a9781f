#!/usr/bin/env python3
"""Measurement: one synthetic 8192^2 image at a time (encode with side index + decode, host-
synchronous), REPS times.  Run under `rocprofv3 --kernel-trace --output-format csv`; then
`single_trace.py --show TRACE.csv` prints the last encode+decode's kernels in issue order with
start offset, duration and the idle gap before each (what one-image latency is made of)."""
import csv
import os
import sys
import time

if len(sys.argv) > 2 and sys.argv[1] == "--show":
    rows = []
    for r in csv.DictReader(open(sys.argv[2])):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:40]))
    rows.sort()
    # the last iteration: from the last k_colours (first encode kernel after the memsets)
    starts = [i for i, r in enumerate(rows) if r[2].startswith("k_colours")]
    i0 = starts[-1] - 2 if starts else 0
    t0, prev = rows[i0][0], rows[i0][0]
    busy = 0
    for s, e, n in rows[i0:]:
        print("%8.3f ms  %8.4f ms  gap %7.4f  %s" % ((s - t0) / 1e6, (e - s) / 1e6, max(0, s - prev) / 1e6, n))
        busy += e - s
        prev = max(prev, e)
    print("span %.3f ms, kernel time %.3f ms" % ((prev - t0) / 1e6, busy / 1e6))
    sys.exit(0)
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "hoh-ans_amd"))
import torch  # noqa: E402
import hoh_ans  # noqa: E402
W = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
c = hoh_ans.Context(0)
rgb = hoh_ans.synth_rgb_dev(W, W, 1, 4, ctx=c)
ix = hoh_ans.Index()
out = torch.empty(hoh_ans.lib().hoh_encode_bound(W, W), dtype=torch.uint8, device="cuda")
dec = torch.empty(W * W * 3, dtype=torch.uint8, device="cuda")
for r in range(reps):
    torch.cuda.synchronize()
    t = time.perf_counter()
    _, n, _ = hoh_ans.encode_image(rgb, W, W, out_dev=out, ctx=c, index=ix)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    hoh_ans.decode_image(out, n, out_dev=dec, ctx=c, index=ix)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("encode %.3f ms decode %.3f ms" % ((t1 - t) * 1e3, (t2 - t1) * 1e3), flush=True)
assert torch.equal(dec, rgb)
