"""Golden SHA-256 of every bench slot's file: the reference's own choh -s0 (compiled in place by
oracle/ref/Makefile) on the deterministic 8192^2 synthetic image of each seed bench.py puts in
flight (seeds 1..40, noise 4: slot k holds seed 1 + k, or seeds 1 + k*B .. with --batch B).  bench.py compares every slot's file
with these after the timed region.  ~7 s per seed on one core (run in parallel here).

    python tests/golden/make_golden_bench.py [--size S] [--height H] [--seeds A B] [--jobs J]   (needs /root/reference)

--height (default S) makes the weak-scaling images of bench.py's N > 1 line (8192 x 8192 N).
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "hoh-ans_amd"))
sys.path.insert(0, os.path.join(HERE, "..", ".."))


def main():
    import oracle as O
    from hoh_ans.synth import synth_rgb
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--seeds", type=int, nargs=2, default=[1, 20])
    ap.add_argument("--height", type=int, default=0)
    ap.add_argument("--noise", type=int, default=4)
    ap.add_argument("--jobs", type=int, default=6)
    a = ap.parse_args()
    exe = O.ref_bin("choh")
    assert exe, "reference choh not built (oracle/ref/Makefile)"
    W = a.size
    H = a.height or a.size
    d = tempfile.mkdtemp(dir="/tmp")

    def one(seed):
        src = os.path.join(d, "img%d.rgb" % seed)
        dst = os.path.join(d, "out%d.hoh" % seed)
        with open(src, "wb") as f:
            f.write(synth_rgb(W, H, seed, a.noise).tobytes())
        r = subprocess.run([exe, src, dst, str(W), str(H), "-s0"], capture_output=True, check=True)
        data = open(dst, "rb").read()
        os.unlink(src)
        os.unlink(dst)
        return {"spec": {"W": W, "H": H, "seed": seed, "noise": a.noise, "speed": 0},
                "out": {"len": len(data), "sha256": hashlib.sha256(data).hexdigest()},
                "printed": int(r.stdout.split()[-1])}

    with ThreadPoolExecutor(a.jobs) as ex:
        recs = list(ex.map(one, range(a.seeds[0], a.seeds[1] + 1)))
    path = os.path.join(HERE, "golden_bench.json")
    out = json.load(open(path)) if os.path.exists(path) else {"files": []}
    key = lambda f: (f["spec"]["W"], f["spec"]["H"], f["spec"]["seed"], f["spec"]["noise"])  # noqa: E731
    keys = {key(r) for r in recs}
    out["files"] = [f for f in out["files"] if key(f) not in keys] + recs
    out["files"].sort(key=key)
    out["generator"] = "tests/golden/make_golden_bench.py (reference choh built by oracle/ref/Makefile)"
    json.dump(out, open(path, "w"), indent=1)
    for r in recs:
        print(r)


if __name__ == "__main__":
    main()
