#!/usr/bin/env python3
"""Debug (GPU box): choh -sN of small test images on the GPU against the oracle: sizes and the
first differing byte.  HOH_LIB selects the library (knobs builds take HOH_* knobs)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "hoh-ans_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import hoh_ans  # noqa: E402
import oracle  # noqa: E402

imgs = {"flat": np.full((256, 512, 3), 77, np.uint8),
        "flat256": np.full((256, 256, 3), 77, np.uint8),
        "halfflat": np.concatenate([np.full((128, 512, 3), 77, np.uint8), np.full((128, 512, 3), 9, np.uint8)], 0)}
for name, img in imgs.items():
    for sp in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,2,3,4").split(",")]:
        ref, rp = oracle.choh(img, sp)
        got, gp = hoh_ans.choh(img, speed=sp)
        d = next((i for i in range(min(len(ref), len(got))) if ref[i] != got[i]), None)
        print("%-9s -s%d: ref %d B (printed %d), gpu %d B (printed %d), first diff %s" % (name, sp, len(ref), rp, len(got), gp, d),
              flush=True)
