"""GPU -s1..-s4 (choh cruncher_mode >= 1: LZ seek distance 10-14 + vertical search, 40-px grid
predictor search, prob_bits ladder with the Q14 prefix, palette and RGB colour modes) against the
oracle, which is pinned to the reference's own choh (tests/test_oracle_vs_reference.py).  The
files are byte-identical, so their sizes are too (SURVEY §8(d) config 5 asks for size parity)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hoh():
    import hoh_ans
    return hoh_ans


def cases():
    from hoh_ans.synth import synth_rgb
    rs = np.random.RandomState(21)
    out = []
    for sp in (1, 2, 3, 4):
        out.append(("synth512x256-s%d" % sp, sp, synth_rgb(512, 256, sp, 3)))
    out.append(("synth600x520-s1", 1, synth_rgb(600, 520, 7, 4)))      # edge tiles 300x260
    out.append(("synth768x512-s3", 3, synth_rgb(768, 512, 8, 2)))
    img = synth_rgb(512, 512, 9, 4)
    img[300:, :] = img[:212, :]                                           # vertical repeats
    for _ in range(200):
        y, x, L, b = rs.randint(0, 512), rs.randint(300, 480), rs.randint(4, 30), rs.randint(1, 900)
        if x - b >= 0:
            img[y, x:x + L] = img[y, x - b:x - b + L]
    out.append(("repeats-s1", 1, img.copy()))
    out.append(("repeats-s2", 2, img.copy()))
    pal = np.stack([rs.randint(0, 256, 40), np.full(40, 9), rs.randint(0, 256, 40)], 1).astype(np.uint8)
    img = synth_rgb(512, 256, 10, 3)
    img[:, 256:] = pal[rs.randint(0, 40, (256, 256))]
    out.append(("palette-s1", 1, img.copy()))
    out.append(("palette-s3", 3, img.copy()))
    out.append(("flat-s1", 1, np.full((256, 512, 3), 77, np.uint8)))
    for sp in (2, 4):
        out.append(("flat-s%d" % sp, sp, np.full((256, 512, 3), 77, np.uint8)))
    # long runs of a few colours (runs of 1..700 pixels, many starting at tile row starts, colour
    # repeats): the run-length shortcut, the flat-run posting walk and k_lzfp's run lengths at
    # chunk boundaries
    cols = rs.randint(0, 256, (6, 3)).astype(np.uint8)
    flat = rs.randint(0, 256, (256 * 512, 3)).astype(np.uint8)            # > 256 colours: RGB tiles
    p = 0
    while p < flat.shape[0]:
        n = int(rs.choice([1, 3, 5, 40, 254, 255, 256, 300, 700]))
        if rs.randint(0, 3):
            flat[p:p + n] = cols[rs.randint(0, 6)]
        p += n
    runs = flat.reshape(256, 512, 3)
    runs[100:110] = 9                                                     # two flat tile-row bands
    for sp in (1, 2, 3, 4):
        out.append(("runs-s%d" % sp, sp, runs.copy()))
    half = np.full((256, 512, 3), 77, np.uint8)
    half[128:] = 9
    out.append(("halfflat-s3", 3, half))
    out.append(("untiled200x100-s2", 2, synth_rgb(200, 100, 11, 3)))
    # one tile of fewer than 65,536 positions at -s3/-s4 (k_lzsort's 512-thread shape: partial
    # chunks, ranks built in parts of 16,384 with a partial last part)
    out.append(("untiled200x100-s4", 4, synth_rgb(200, 100, 13, 3)))
    out.append(("untiled250x250-s3", 3, synth_rgb(250, 250, 14, 3)))
    out.append(("tiny30x20-s1", 1, synth_rgb(30, 20, 12, 3)))
    return out


@pytest.mark.parametrize("name,sp,img", cases(), ids=[c[0] for c in cases()])
def test_choh_speed_parity(hoh, orc, name, sp, img):
    try:
        ref, ref_printed = orc.choh(img, sp)
    except orc.OracleError as e:
        assert e.code == -4, e
        with pytest.raises(hoh.HohError) as g:
            hoh.choh(img, speed=sp)
        assert g.value.code == 5
        return
    data, printed = hoh.choh(img, speed=sp)
    assert printed == ref_printed
    assert len(data) == len(ref)
    assert data == ref


def test_choh_8192_speed_golden(hoh):
    """config 5: 8192^2 at -s1/-s2/-s3 against the reference choh's own output (size + SHA-256)"""
    import hashlib
    import json
    import os
    import time
    import torch
    g = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_speed.json")))
    for f in g["files"]:
        sp = f["spec"]
        if sp["W"] != 8192:
            continue
        d = hoh.synth_rgb_dev(sp["W"], sp["H"], sp["seed"], sp["noise"])
        torch.cuda.synchronize()
        t = time.perf_counter()
        out, n, printed = hoh.encode_image(d, sp["W"], sp["H"], speed=sp["speed"])
        torch.cuda.synchronize()
        el = time.perf_counter() - t
        print("-s%d 8192^2: %d B in %.1f ms" % (sp["speed"], n, el * 1e3))
        assert n == f["out"]["len"]
        assert printed == f["printed"]
        assert hashlib.sha256(out[:n].cpu().numpy().tobytes()).hexdigest() == f["out"]["sha256"]
