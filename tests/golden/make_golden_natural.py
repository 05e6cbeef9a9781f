"""Golden whole-file vectors for the natural-statistic generator (hoh_ans/natural.py), made by
running the reference's own choh (compiled in place by oracle/ref/Makefile) -- BASELINE.json
configs[4] / SURVEY §8(d) config 5.  Stores size, printed size and SHA-256 only.

Default jobs (run in parallel, one process each):
    8192^2 seed 1 at -s0 .. -s4, 2048^2 seed 1 at -s4, 16384^2 seed 1 at -s0, and
    1024^2 seed 3 / 768x512 seed 4 (odd tiling) at -s0 .. -s4.
-s3 / -s4 at 8192^2 take ~15 / ~30 minutes on one core.

    python tests/golden/make_golden_natural.py [WxH:seed:speed ...]   (needs /root/reference)
"""
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

DEFAULT = (["8192x8192:1:%d" % s for s in (4, 3, 2, 1, 0)] + ["16384x16384:1:0", "2048x2048:1:4"] +
           ["1024x1024:3:%d" % s for s in range(5)] + ["768x512:4:%d" % s for s in range(5)])


def main():
    import oracle as O
    from hoh_ans.natural import natural_rgb
    exe = O.ref_bin("choh")
    assert exe, "reference choh not built (oracle/ref/Makefile)"
    jobs = []
    for a in (sys.argv[1:] or DEFAULT):
        wh, seed, sp = a.split(":")
        W, H = (int(v) for v in wh.split("x"))
        jobs.append((W, H, int(seed), int(sp)))
    d = tempfile.mkdtemp(dir="/tmp")
    srcs = {}
    for W, H, seed, _ in jobs:
        if (W, H, seed) not in srcs:
            p = os.path.join(d, "nat_%dx%d_%d.rgb" % (W, H, seed))
            with open(p, "wb") as f:
                for r0 in range(0, H, 1024):
                    f.write(natural_rgb(W, H, seed, row0=r0, rows=min(1024, H - r0)).tobytes())
            srcs[(W, H, seed)] = p
    path = os.path.join(HERE, "golden_natural.json")

    def run(job):
        W, H, seed, sp = job
        dst = os.path.join(d, "out_%dx%d_%d_s%d.hoh" % (W, H, seed, sp))
        r = subprocess.run([exe, srcs[(W, H, seed)], dst, str(W), str(H), "-s%d" % sp], capture_output=True,
                           check=True)
        data = open(dst, "rb").read()
        os.unlink(dst)
        rec = {"spec": {"W": W, "H": H, "seed": seed, "gen": "natural", "speed": sp},
               "out": {"len": len(data), "sha256": hashlib.sha256(data).hexdigest()},
               "printed": int(r.stdout.split()[-1])}
        print(rec, flush=True)
        return rec

    with ThreadPoolExecutor(max_workers=min(8, len(jobs))) as ex:
        recs = list(ex.map(run, jobs))
    out = json.load(open(path)) if os.path.exists(path) else {"files": []}
    keys = {(r["spec"]["W"], r["spec"]["H"], r["spec"]["seed"], r["spec"]["speed"]) for r in recs}
    out["files"] = [f for f in out["files"]
                    if (f["spec"]["W"], f["spec"]["H"], f["spec"]["seed"], f["spec"]["speed"]) not in keys] + recs
    out["files"].sort(key=lambda f: (f["spec"]["W"] * f["spec"]["H"], f["spec"]["seed"], f["spec"]["speed"]))
    out["generator"] = ("tests/golden/make_golden_natural.py: hoh_ans/natural.py images through the reference "
                        "choh built by oracle/ref/Makefile")
    json.dump(out, open(path, "w"), indent=1)
    for p in srcs.values():
        os.unlink(p)


if __name__ == "__main__":
    main()
