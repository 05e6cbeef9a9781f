"""GPU parity on the natural-statistic image (hoh_ans/natural.py; BASELINE.json configs[4], SURVEY
§8(d) config 5) and the decoder's real path: a .hoh with no side index (dhoh.cpp:297-396,
entropy_decoding.hpp:268-276 -- every stream decoded serially from the file alone) at full size.

Goldens: tests/golden/golden_natural.json, made by the reference's own choh
(tests/golden/make_golden_natural.py); the small cases are also checked against the oracle."""
import hashlib
import json
import os
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def hoh():
    import hoh_ans
    return hoh_ans


def natural_goldens():
    p = os.path.join(HERE, "golden", "golden_natural.json")
    if not os.path.exists(p):
        return []
    with open(p) as f:
        return json.load(f)["files"]


def sha(t, n):
    return hashlib.sha256(t[:n].cpu().numpy().tobytes()).hexdigest()


def test_device_generator_matches_numpy(hoh):
    """hoh_natural_rgb_rows (k_natural) writes the bytes of hoh_ans.natural.natural_rgb"""
    import torch
    from hoh_ans.natural import natural_rgb
    for W, row0, rows, seed in ((1024, 0, 64, 1), (777, 1000, 33, 5), (16384, 16000, 4, 1)):
        d = hoh.natural_rgb_dev(W, rows, seed, row0=row0)
        torch.cuda.synchronize()
        assert np.array_equal(d.cpu().numpy().reshape(rows, W, 3), natural_rgb(W, row0 + rows, seed, row0=row0))


def small_cases():
    return [f for f in natural_goldens() if f["spec"]["W"] * f["spec"]["H"] <= 1024 * 1024]


@pytest.mark.parametrize("g", small_cases(), ids=lambda g: "%dx%d-s%d" % (g["spec"]["W"], g["spec"]["H"],
                                                                          g["spec"]["speed"]))
def test_natural_small_vs_reference_and_oracle(hoh, orc, g):
    import torch
    sp = g["spec"]
    W, H = sp["W"], sp["H"]
    d = hoh.natural_rgb_dev(W, H, sp["seed"])
    ix = hoh.Index() if sp["speed"] == 0 else None
    out, n, printed = hoh.encode_image(d, W, H, speed=sp["speed"], index=ix)
    torch.cuda.synchronize()
    assert (n, printed) == (g["out"]["len"], g["printed"])
    assert sha(out, n) == g["out"]["sha256"]
    if W * H <= 768 * 512:
        img = d.cpu().numpy().reshape(H, W, 3)
        assert out[:n].cpu().numpy().tobytes() == orc.choh(img, sp["speed"])[0]
    if sp["speed"] == 0:                                   # -s>=1 layers are undecodable (Q14)
        for index in (ix, None):
            rgb, _, _ = hoh.decode_image(out, n, index=index)
            torch.cuda.synchronize()
            assert torch.equal(rgb, d)


@pytest.mark.parametrize("speed", [0, 1, 2, 3, 4])
def test_natural_8192_vs_reference(hoh, speed):
    """config 5: 8192^2 natural image at -s0..-s4, whole file against the reference choh's SHA"""
    import torch
    gs = [f for f in natural_goldens() if f["spec"]["W"] == 8192 and f["spec"]["speed"] == speed]
    if not gs:
        pytest.skip("no golden for -s%d" % speed)
    g = gs[0]
    d = hoh.natural_rgb_dev(8192, 8192, g["spec"]["seed"])
    torch.cuda.synchronize()
    t = time.perf_counter()
    out, n, printed = hoh.encode_image(d, 8192, 8192, speed=speed)
    torch.cuda.synchronize()
    print("natural 8192^2 -s%d: %d B (%.4f of raw) in %.1f ms" % (speed, n, n / (8192 * 8192 * 3),
                                                                 (time.perf_counter() - t) * 1e3))
    assert (n, printed) == (g["out"]["len"], g["printed"])
    assert sha(out, n) == g["out"]["sha256"]
    if speed == 0:
        rgb, _, _ = hoh.decode_image(out, n, index=None)   # the file alone: serial streams
        torch.cuda.synchronize()
        assert torch.equal(rgb, d)


def test_natural_2048_s4_vs_reference(hoh):
    import torch
    g = [f for f in natural_goldens() if f["spec"]["W"] == 2048 and f["spec"]["speed"] == 4][0]
    d = hoh.natural_rgb_dev(2048, 2048, g["spec"]["seed"])
    out, n, printed = hoh.encode_image(d, 2048, 2048, speed=4)
    torch.cuda.synchronize()
    assert (n, printed) == (g["out"]["len"], g["printed"])
    assert sha(out, n) == g["out"]["sha256"]


def serial_decode(hoh, d, W, H, golden_len, golden_sha):
    """encode (checked against the reference's SHA), then decode the bytes alone -- a copy of the
    file with no side index, as dhoh reads it from disk -- and compare with the input"""
    import torch
    out, n, _ = hoh.encode_image(d, W, H)
    torch.cuda.synchronize()
    assert n == golden_len and sha(out, n) == golden_sha
    f = out[:n].clone()                                    # only the file's bytes
    del out
    t = time.perf_counter()
    rgb, w, h = hoh.decode_image(f, n, index=None)
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    print("%dx%d serial (no index) decode: %.1f ms, %.1f MB/s" % (W, H, el * 1e3, W * H * 3 / el / 1e6))
    assert (w, h) == (W, H)
    assert torch.equal(rgb, d)


def test_serial_decode_8192_gradient(hoh, golden):
    f = [c for c in golden["choh_s0"] if c["spec"]["W"] == 8192][0]
    sp = f["spec"]
    serial_decode(hoh, hoh.synth_rgb_dev(8192, 8192, sp["seed"], sp["noise"]), 8192, 8192, f["out"]["len"],
                  f["out"]["sha256"])


def test_serial_decode_16384_gradient(hoh):
    g = json.load(open(os.path.join(HERE, "golden", "golden_speed.json")))
    f = [c for c in g["files"] if c["spec"]["W"] == 16384 and c["spec"]["speed"] == 0][0]
    sp = f["spec"]
    serial_decode(hoh, hoh.synth_rgb_dev(16384, 16384, sp["seed"], sp["noise"]), 16384, 16384, f["out"]["len"],
                  f["out"]["sha256"])


def test_serial_decode_16384_natural(hoh):
    gs = [f for f in natural_goldens() if f["spec"]["W"] == 16384 and f["spec"]["speed"] == 0]
    if not gs:
        pytest.skip("no 16384^2 natural golden")
    g = gs[0]
    serial_decode(hoh, hoh.natural_rgb_dev(16384, 16384, g["spec"]["seed"]), 16384, 16384, g["out"]["len"],
                  g["out"]["sha256"])


@pytest.mark.parametrize("speed", [1, 2, 3, 4])
def test_natural_8192_repeatable(hoh, speed):
    """The same image encoded again on the same context gives the same file (a race in the search
    or LZ kernels shows up as run-to-run differences; tools/scripts/rep_speed.py).  Round 4's
    differences came from k_lzsort's count reset racing the next chunk's count store (DESIGN.md
    section 2); tools/scripts/lzsort_check.py checks the posting lists directly."""
    import torch
    d = hoh.natural_rgb_dev(8192, 8192, 1)
    shas = set()
    for _ in range(6):
        out, n, _ = hoh.encode_image(d, 8192, 8192, speed=speed)
        torch.cuda.synchronize()
        shas.add((n, sha(out, n)))
    assert len(shas) == 1, shas


@pytest.mark.parametrize("mode", ["lanes", "multi", "wave", "adaptive"])
def test_no_index_decoders(hoh, golden, mode):
    """Every no-index chain kernel (hoh_ctx_set_option HOH_OPT_NOIX_DECODER; dhoh.cpp:297-396 reads
    the file alone, entropy_decoding.hpp:268-276 per stream) decodes losslessly, pinned per
    context rather than left to the adaptive choice: the synthetic 8192^2 bench file (reference
    SHA), the natural 1024^2 -s0 file (LZ streams, reference SHA), and a high-noise 2048^2 image
    (triangular noise k = 40) whose wide residual tables put more than three symbol starts into
    many 64-slot buckets (k_drans_lanes' walk past its three-entry window)."""
    import torch
    ctx = hoh.Context(0)
    ctx.set_option(hoh.OPT_NOIX_DECODER, {"lanes": hoh.NOIX_LANES, "multi": hoh.NOIX_MULTI,
                                          "wave": hoh.NOIX_WAVE, "adaptive": hoh.NOIX_ADAPTIVE}[mode])
    f = [c for c in golden["choh_s0"] if c["spec"]["W"] == 8192][0]
    g = [x for x in natural_goldens() if (x["spec"]["W"], x["spec"]["speed"]) == (1024, 0)][0]
    cases = [(hoh.synth_rgb_dev(8192, 8192, f["spec"]["seed"], f["spec"]["noise"], ctx=ctx), 8192, f["out"]),
             (hoh.natural_rgb_dev(1024, 1024, g["spec"]["seed"], ctx=ctx), 1024, g["out"]),
             (hoh.synth_rgb_dev(2048, 2048, 7, 40, ctx=ctx), 2048, None)]
    for d, W, want in cases:
        out, n, _ = hoh.encode_image(d, W, W, ctx=ctx)
        torch.cuda.synchronize()
        if want is not None:
            assert n == want["len"] and sha(out, n) == want["sha256"]
        f2 = out[:n].clone()
        rgb, w, h = hoh.decode_image(f2, n, ctx=ctx, index=None)
        torch.cuda.synchronize()
        assert (w, h) == (W, W) and torch.equal(rgb, d), (mode, W)
    with pytest.raises(hoh.HohError):
        ctx.set_option(hoh.OPT_NOIX_DECODER, 3)
    ctx.close()
