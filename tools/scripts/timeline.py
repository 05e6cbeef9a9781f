#!/usr/bin/env python3
"""Timeline of the last K images of a rocprofv3 kernel trace (csv): per time bucket, how many
launches of each stage are running.  python tools/scripts/timeline.py run_kernel_trace.csv [K] [bucket_ms]"""
import csv
import sys

path = sys.argv[1]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
B = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
rows = []
with open(path) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]))
rows.sort()


def cat(n):
    if "k_front" in n or "k_colours" in n or "k_palette" in n:
        return "front"
    if "k_rans_fast" in n or "k_rans_gen" in n:
        return "chain"
    if "k_drans" in n or "k_dparse" in n or "k_dtable" in n:
        return "drans"
    if "k_dunpred" in n or "k_dlz" in n or "k_dcompose" in n or "k_dbackmap" in n:
        return "dunpred"
    if n.startswith("k_"):
        return "enc_misc"
    return None


fronts = [r for r in rows if r[2].startswith("k_front")]
t0 = fronts[-K][0]
sel = [r for r in rows if r[0] >= t0 and cat(r[2])]
t1 = max(r[1] for r in sel)
print("window %.2f ms, %d launches" % ((t1 - t0) / 1e6, len(sel)))
cats = ["front", "enc_misc", "chain", "drans", "dunpred"]
print("  ms   " + " ".join("%8s" % c for c in cats))
nb = int((t1 - t0) / 1e6 / B) + 1
for b in range(nb):
    a, z = t0 + b * B * 1e6, t0 + (b + 1) * B * 1e6
    occ = {c: 0.0 for c in cats}
    for s, e, n, q in sel:
        ov = min(e, z) - max(s, a)
        if ov > 0:
            occ[cat(n)] += ov / (B * 1e6)
    print("%5.1f  " % (b * B) + " ".join("%8.2f" % occ[c] for c in cats))
# per image (queue) finish times
fin = {}
for s, e, n, q in sel:
    fin[q] = max(fin.get(q, 0), e)
print("queue finish ms:", sorted(round((v - t0) / 1e6, 1) for v in fin.values()))
ch = sorted(((s - t0) / 1e6, (e - t0) / 1e6) for s, e, n, q in sel if "k_rans_fast<0>" in n)
print("chains (start, end) ms:", [(round(a, 1), round(b, 1)) for a, b in ch])
