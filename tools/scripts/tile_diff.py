# First difference between the GPU file and the oracle's for one test image (debugging aid).
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "hoh-ans_amd"))
import numpy as np, hoh_ans, oracle as O
from hoh_ans.synth import synth_rgb
W, H, seed, noise = map(int, sys.argv[1:5])
img = synth_rgb(W, H, seed, noise)
a, pa = hoh_ans.choh(img)
b, pb = O.choh(img)
print("gpu", len(a), pa, "oracle", len(b), pb)
n = min(len(a), len(b))
d = next((i for i in range(n) if a[i] != b[i]), None)
print("first diff", d)
if d is not None:
    lo = max(0, d - 16)
    print("gpu   ", a[lo:d + 32].hex())
    print("oracle", b[lo:d + 32].hex())
diffs = [i for i in range(n) if a[i] != b[i]]
print("ndiff", len(diffs), "ranges:")
rs = []
for i in diffs:
    if rs and i - rs[-1][1] <= 8: rs[-1][1] = i
    else: rs.append([i, i])
print(rs[:40])
