"""Generate tests/golden/golden.json from the REFERENCE ITSELF (oracle/_ref, compiled in place
from /root/reference by oracle/ref/Makefile).  Run here, where /root/reference exists:

    python tests/golden/make_golden.py

The GPU box has no /root/reference; the committed json pins the oracle there.  Inputs are
regenerated from the specs by tests/golden/gen.py.  Also records the reference's own fixtures
(example.rgb / example.hoh, which are data) as hex.
"""
import ctypes as C
import hashlib
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "hoh-ans_amd"))
sys.path.insert(0, HERE)

import oracle  # noqa: E402
from gen import make_image, make_plane, make_symbols  # noqa: E402

REF_DIR = "/root/reference"


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def rec(out):
    out = bytes(out)
    d = {"len": len(out), "sha256": sha(out)}
    if len(out) <= 4096:
        d["hex"] = out.hex()
    return d


def main():
    oracle.build()
    R = oracle.ref()
    assert R is not None, "build oracle/_ref first (needs /root/reference)"
    u8p, u16p = oracle.u8p, oracle.u16p
    G = {"generator": "tests/golden/make_golden.py", "reference": "hohMiyazawa/hoh-ANS @ v1 (/root/reference)"}

    # 1. Rans64EncSymbolInit (rans64.hpp:167-247) for every freq at several scale_bits
    esym = {}
    for pb in (8, 10, 12, 15):
        h = hashlib.sha256()
        samples = []
        for f in range(1, (1 << pb) + 1):
            start = ((1 << pb) - f) // 3
            rcp = C.c_uint64(); bias = C.c_uint32(); cmpl = C.c_uint32(); sh = C.c_uint32()
            R.ref_esym_init(start, f, pb, C.byref(rcp), C.byref(bias), C.byref(cmpl), C.byref(sh))
            t = (start, f, rcp.value, bias.value, cmpl.value, sh.value)
            h.update(("%d,%d,%d,%d,%d,%d;" % t).encode())
            if f % 97 == 1 or f in (2, 3, (1 << pb) - 1, 1 << pb):
                samples.append(t)
        esym[str(pb)] = {"sha256": h.hexdigest(), "samples": samples}
    G["esym_init"] = esym

    # 2. normalize_freqs (stattools.hpp:13-70)
    norm = []
    cases = [
        ("ones512", [1] * 512, 1 << 15), ("ones256", [1] * 256, 1 << 10),
        ("dominant", [0] * 100 + [100000] + [1] * 50 + [0] * 105, 1 << 12),
        ("tail", [2 ** (20 - min(20, abs(i - 128) // 3)) if abs(i - 128) < 60 else (1 if i % 7 == 0 else 0) for i in range(256)], 1 << 15),
        ("zeros_many", [0 if i % 3 else 5 for i in range(512)], 1 << 10),
    ]
    rs = np.random.RandomState(1234)
    for k in range(6):
        v = (rs.geometric(0.02 + 0.05 * k, size=512) - 1)
        hist = np.bincount(np.minimum(v, 511), minlength=512).astype(np.uint32)
        cases.append(("geo%d" % k, hist.tolist(), 1 << (10 + k)))
    for name, f, tgt in cases:
        fa = np.array(f, dtype=np.uint32)
        cum = np.zeros(fa.size + 1, np.uint32)
        fo = fa.copy()
        R.ref_normalize_freqs(fo.ctypes.data_as(oracle.u32p), cum.ctypes.data_as(oracle.u32p), fa.size, tgt)
        norm.append({"name": name, "freqs": fa.tolist(), "target": tgt, "out": fo.tolist()})
    G["normalize_freqs"] = norm

    # 3. + 8. encode_entropy / decode_entropy (entropy_encoding.hpp:8, entropy_decoding.hpp:134)
    streams = []
    specs = []
    for n in (0, 1, 3, 257, 4096, 65536):
        for rng in (1, 2, 5, 256, 512):
            for pb in (8, 10, 12, 15):
                if rng > (1 << pb) or (n > 4096 and pb in (8, 12)):
                    continue
                kind = "laplace" if rng >= 5 else "uniform"
                specs.append({"kind": kind, "n": n, "range": rng, "seed": n * 7 + rng * 3 + pb, "scale_x16": 40, "pb": pb})
    specs += [
        {"kind": "laplace", "n": 1048576, "range": 512, "seed": 11, "scale_x16": 48, "pb": 15},
        {"kind": "laplace", "n": 65536, "range": 256, "seed": 12, "scale_x16": 8, "pb": 15},
        {"kind": "laplace", "n": 65536, "range": 512, "seed": 13, "scale_x16": 1600, "pb": 15},
        {"kind": "uniform", "n": 65536, "range": 512, "seed": 14, "pb": 15},          # stored (Q7)
        {"kind": "uniform", "n": 4096, "range": 256, "seed": 15, "pb": 10},
        {"kind": "const", "n": 257, "range": 256, "value": 255, "pb": 10},           # Q6 (LZ stream 0)
        {"kind": "const", "n": 65536, "range": 512, "value": 256, "pb": 15},         # Q6 plane
        {"kind": "const", "n": 100, "range": 256, "value": 0, "pb": 15},
        {"kind": "few", "n": 20000, "range": 512, "seed": 16, "k": 3, "pb": 15},
        {"kind": "few", "n": 20000, "range": 256, "seed": 17, "k": 9, "pb": 12},
        {"kind": "laplace", "n": 30000, "range": 200, "seed": 18, "scale_x16": 3000, "pb": 8},  # raw table (Q4)
        {"kind": "laplace", "n": 5000, "range": 256, "seed": 19, "scale_x16": 600, "pb": 8},
    ]
    for sp in specs:
        sym = make_symbols(sp)
        out = np.empty(oracle.lib().or_entropy_bound(sym.size, sp["range"], sp["pb"]) + 64, np.uint8)
        if sp["pb"] in (8, 12, 16) and sp["kind"] == "const":
            continue  # reference writes past a stack array (oracle: OR_E_UB)
        r = R.ref_encode_entropy(sym.ctypes.data_as(u16p), sym.size, sp["range"], sp["pb"], out.ctypes.data_as(u8p))
        enc = out[:r].tobytes()
        d = {"spec": sp, "enc": rec(enc)}
        # the reference decoder on its own stream (first stream of a buffer: Q1 does not bite)
        try:
            oracle.decode_entropy(enc)
            decodable = True
        except oracle.OracleError:
            decodable = False     # e.g. raw table with truncated frequencies
        d["decodable"] = decodable
        if sym.size and sp["kind"] != "const" and decodable:
            buf = np.frombuffer(enc + b"\0" * 16, np.uint8).copy()
            dec = np.empty(sym.size, np.uint16)
            m = R.ref_decode_entropy(buf.ctypes.data_as(u8p), buf.size, 0, dec.ctypes.data_as(u16p), dec.size)
            d["ref_decode_equal"] = bool(m == sym.size and np.array_equal(dec, sym))
        streams.append(d)
    G["entropy"] = streams

    # 4. channelpredict_fastpath (prediction.hpp:6-44) and 5. layer_encode -s0 (layer_encode.hpp:11)
    pred, layers = [], []
    for sp in ({"W": 256, "H": 256, "seed": 21, "noise": 4, "plane": "G"},
               {"W": 256, "H": 256, "seed": 22, "noise": 4, "plane": "R"},
               {"W": 256, "H": 256, "seed": 23, "noise": 12, "plane": "B"},
               {"W": 300, "H": 17, "seed": 24, "noise": 2, "plane": "R"},
               {"W": 1, "H": 9, "seed": 25, "noise": 2, "plane": "G"}):
        p = make_plane(sp)
        depth = 8 if sp["plane"] == "G" else 9
        res = np.empty_like(p)
        R.ref_channelpredict_fastpath(p.ctypes.data_as(u16p), sp["W"], sp["H"], depth, res.ctypes.data_as(u16p))
        pred.append({"spec": sp, "depth": depth, "res": rec(res.tobytes())})
        nuke = np.zeros(p.size, np.uint8)
        if sp["seed"] == 22:
            nuke[1000:1037] = 1
            nuke[5000:5300] = 1
        out = np.empty(p.size * 4 + 8192, np.uint8)
        r = R.ref_layer_encode(p.ctypes.data_as(u16p), p.size, sp["W"], sp["H"], depth, 0,
                               nuke.ctypes.data_as(u8p), out.ctypes.data_as(u8p))
        layers.append({"spec": sp, "depth": depth, "nuke_ranges": [[1000, 1037], [5000, 5300]] if sp["seed"] == 22 else [],
                       "out": rec(out[:r].tobytes())})
    G["predict_fastpath"] = pred
    G["layer_encode_s0"] = layers

    # 6. encode_tile -s0 (choh.cpp:104-383)
    tiles = []
    for sp in ({"W": 64, "H": 64, "seed": 31, "noise": 4}, {"W": 256, "H": 256, "seed": 32, "noise": 4},
               {"W": 256, "H": 256, "seed": 33, "noise": 0}, {"W": 2, "H": 2, "seed": 34, "noise": 4},
               {"W": 256, "H": 256, "seed": 35, "noise": 30}, {"W": 333, "H": 257, "seed": 36, "noise": 1}):
        img = make_image(sp)
        out = np.empty(img.size * 6 + 8192, np.uint8)
        r = R.ref_encode_tile(img.ctypes.data_as(u8p), sp["W"], sp["H"], 0, out.ctypes.data_as(u8p))
        tiles.append({"spec": sp, "out": rec(out[:r].tobytes())})
    G["encode_tile_s0"] = tiles

    # 7. whole-file choh -s0 (choh.cpp:394-527) via the reference binary itself
    files = []
    choh = oracle.ref_bin("choh")
    for sp in ({"W": 512, "H": 512, "seed": 41, "noise": 4}, {"W": 1024, "H": 1024, "seed": 42, "noise": 4},
               {"W": 768, "H": 520, "seed": 43, "noise": 2}, {"W": 2, "H": 2, "seed": 44, "noise": 4},
               {"W": 1000, "H": 600, "seed": 45, "noise": 8}, {"W": 8192, "H": 8192, "seed": 1, "noise": 4}):
        img = make_image(sp)
        img.tofile("/tmp/_golden.rgb")
        res = subprocess.run([choh, "/tmp/_golden.rgb", "/tmp/_golden.hoh", str(sp["W"]), str(sp["H"]), "-s0"],
                             capture_output=True, text=True, check=True)
        data = open("/tmp/_golden.hoh", "rb").read()
        files.append({"spec": sp, "out": rec(data), "printed": int(res.stdout.strip().splitlines()[-1])})
    G["choh_s0"] = files

    # the reference's own fixtures (data): example.rgb (2x2), example.hoh (hand-written store file)
    G["reference_fixtures"] = {
        "example.rgb": open(os.path.join(REF_DIR, "example.rgb"), "rb").read().hex(),
        "example.hoh": open(os.path.join(REF_DIR, "example.hoh"), "rb").read().hex(),
    }
    # entropy_roundtrip_test.sh encodes a reference source file; record only its digests
    src = open(os.path.join(REF_DIR, "simple_entropy_encoder.cpp"), "rb").read()
    res = subprocess.run([oracle.ref_bin("simple_entropy_encoder"), os.path.join(REF_DIR, "simple_entropy_encoder.cpp"),
                          "/tmp/_golden.ent"], capture_output=True, check=True)
    enc = open("/tmp/_golden.ent", "rb").read()
    G["entropy_roundtrip_test"] = {"input_len": len(src), "input_sha256": sha(src), "enc": {"len": len(enc), "sha256": sha(enc)},
                                   "note": "input is reference source text: not stored; test runs only where /root/reference exists"}
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(G, f, indent=1)
    print("wrote", os.path.join(HERE, "golden.json"), os.path.getsize(os.path.join(HERE, "golden.json")), "bytes")


if __name__ == "__main__":
    main()
