"""Golden whole-file vectors made by running the reference's own choh (compiled in place by
oracle/ref/Makefile) on the deterministic synthetic image: choh -s1..-s4 on the 8192^2 bench
image (compressed-size parity at -s>=1) and choh -s0 on 16384^2 (config 4,
the sharded size).  Stores size, printed size and SHA-256 only (the files are 86-400 MB).  Takes
~5 / 7 / 20 / 90 minutes per speed at 8192^2 and ~1 minute for 16384^2 -s0 on one core.

    python tests/golden/make_golden_speed.py [--size S --seed K] [speeds...]   (needs /root/reference)
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "hoh-ans_amd"))
sys.path.insert(0, os.path.join(HERE, "..", ".."))


def main():
    import oracle as O
    from hoh_ans.synth import synth_rgb
    exe = O.ref_bin("choh")
    assert exe, "reference choh not built (oracle/ref/Makefile)"
    args = sys.argv[1:]
    W = H = 8192
    seed, noise = 1, 4
    if "--size" in args:
        i = args.index("--size")
        W = H = int(args[i + 1])
        del args[i:i + 2]
    if "--seed" in args:
        i = args.index("--seed")
        seed = int(args[i + 1])
        del args[i:i + 2]
    speeds = [int(a) for a in args] or [1, 2, 3]
    path = os.path.join(HERE, "golden_speed.json")
    out = json.load(open(path)) if os.path.exists(path) else {"files": []}
    d = tempfile.mkdtemp()
    src = os.path.join(d, "img.rgb")
    with open(src, "wb") as f:
        f.write(synth_rgb(W, H, seed, noise).tobytes())
    for sp in speeds:
        dst = os.path.join(d, "out.hoh")
        r = subprocess.run([exe, src, dst, str(W), str(H), "-s%d" % sp], capture_output=True, check=True)
        data = open(dst, "rb").read()
        rec = {"spec": {"W": W, "H": H, "seed": seed, "noise": noise, "speed": sp},
               "out": {"len": len(data), "sha256": hashlib.sha256(data).hexdigest()},
               "printed": int(r.stdout.split()[-1])}
        out["files"] = [f for f in out["files"] if (f["spec"]["speed"], f["spec"]["W"]) != (sp, W)] + [rec]
        print(rec, flush=True)
    out["files"].sort(key=lambda f: (f["spec"]["W"], f["spec"]["speed"]))
    out["generator"] = "tests/golden/make_golden_speed.py (reference choh built by oracle/ref/Makefile)"
    json.dump(out, open(path, "w"), indent=1)


if __name__ == "__main__":
    main()
