"""Determinism check: the natural 8192^2 image encoded REPS times at each speed given (default
3 4), with and without a side index; prints the distinct (size, sha256) pairs (more than one = a
race)."""
import os, sys
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "hoh-ans_amd"))
import hashlib
import torch, hoh_ans
reps = int(os.environ.get("REPS", "4"))
speeds = [int(a) for a in sys.argv[1:]] or [3, 4]
c = hoh_ans.Context(0)
rgb = hoh_ans.natural_rgb_dev(8192, 8192, 1, ctx=c)
for sp in speeds:
    for use_ix in (False, True):
        ns = []
        for r in range(reps):
            ix = hoh_ans.Index() if use_ix else None
            out, n, _ = hoh_ans.encode_image(rgb, 8192, 8192, ctx=c, index=ix, speed=sp)
            torch.cuda.synchronize()
            ns.append((n, hashlib.sha256(out[:n].cpu().numpy().tobytes()).hexdigest()[:12]))
        print("speed", sp, "index", use_ix, "distinct", sorted(set(ns)), "of", len(ns), flush=True)
