"""GPU encode parity: libhohgpu's choh -s0 bytes against the oracle (and, for 8192^2, the golden
sha256 of the compiled reference's own output)."""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hoh():
    import hoh_ans
    return hoh_ans


def cases():
    from hoh_ans.synth import synth_rgb
    rs = np.random.RandomState(5)
    out = [("synth512", synth_rgb(512, 512, 1, 4)), ("synth1024", synth_rgb(1024, 1024, 2, 4)),
           ("synth768x520", synth_rgb(768, 520, 3, 2)), ("synth600x1000", synth_rgb(600, 1000, 4, 8)),
           ("gradient-lz", synth_rgb(256, 512, 5, 0)), ("synth1000x600", synth_rgb(1000, 600, 45, 8)),
           ("noisy40", synth_rgb(512, 512, 9, 40))]
    img = synth_rgb(512, 512, 7, 4)
    img[100:300, 50:400] = [10, 20, 30]
    out.append(("flat-block", img))
    img = synth_rgb(512, 512, 8, 4)
    for _ in range(300):                                   # repeats at random back distances
        y, x, L, b = rs.randint(0, 512), rs.randint(70, 400), rs.randint(4, 80), rs.randint(1, 65)
        img[y, x:x + L] = img[y, x - b:x - b + L]
    out.append(("repeats", img))
    out.append(("uniform", rs.randint(0, 256, (512, 768, 3)).astype(np.uint8)))   # stored planes
    out.append(("tiny2x2", np.array([[[255, 0, 0], [0, 255, 0]], [[255, 255, 0], [0, 0, 255]]], np.uint8)))
    out.append(("untiled300x200", synth_rgb(300, 200, 10, 4)))
    # untiled and wider than k_front's pixel ring (neighbours read from memory); 1100 just fits it
    out.append(("untiled2000x100", synth_rgb(2000, 100, 13, 4)))
    out.append(("untiled1100x150", synth_rgb(1100, 150, 14, 3)))
    img = synth_rgb(1500, 120, 15, 2)
    for _ in range(100):
        y, x, L, b = rs.randint(0, 120), rs.randint(70, 1400), rs.randint(4, 60), rs.randint(1, 65)
        img[y, x:x + L] = img[y, x - b:x - b + L]
    out.append(("untiled1500x120-repeats", img))
    # flat gradients (dense LZ candidates) at the widest tile each k_front pixel ring takes
    out.append(("untiled271x200-lz", synth_rgb(271, 200, 19, 0)))
    out.append(("untiled511x200-lz", synth_rgb(511, 200, 16, 0)))
    out.append(("untiled1200x120-lz", synth_rgb(1200, 120, 17, 0)))
    out.append(("untiled512x100-lz", synth_rgb(512, 100, 18, 0)))
    out += palette_cases()
    return out


def palette_cases():
    """Tiles with <= 256 colours (choh.cpp:298-308 palette_encode competes with sub-green)."""
    from hoh_ans.synth import synth_rgb
    rs = np.random.RandomState(11)
    out = []
    # constant G, random R/B from a 64-colour palette: the indexed layer wins and is longer than
    # the G layer, so the Q15 prefix is reproducible
    pal = np.stack([rs.randint(0, 256, 64), np.full(64, 100), rs.randint(0, 256, 64)], 1).astype(np.uint8)
    out.append(("palette-g-const", pal[rs.randint(0, 64, (512, 512))]))
    # palette tiles next to sub-green tiles, with LZ runs inside the palette tiles
    img = synth_rgb(768, 512, 12, 4)
    pal2 = np.stack([rs.randint(0, 256, 200), np.full(200, 7), rs.randint(0, 256, 200)], 1).astype(np.uint8)
    blk = pal2[rs.randint(0, 200, (256, 256))]
    blk[10:20, :] = blk[9:10, :]
    img[256:512, 256:512] = blk
    img[0:256, 512:768] = (img[0:256, 512:768] // 64) * 64        # posterised: <= 64 colours
    out.append(("palette-mixed", img))
    # few colours: LZ break-even bonus (choh.cpp:139-154) together with the palette
    four = np.array([[0, 0, 0], [255, 0, 0], [0, 255, 0], [0, 0, 255]], np.uint8)
    out.append(("palette-4col", four[(np.arange(512)[:, None] // 3 + np.arange(512)[None, :] // 5) % 4]))
    # 256 / 257 colours in one tile
    p256 = np.stack([np.arange(256), np.full(256, 50), 255 - np.arange(256)], 1).astype(np.uint8)
    out.append(("palette-256", p256[rs.randint(0, 256, (512, 512))]))
    img = p256[rs.randint(0, 256, (512, 512))]
    img[5, 5] = [1, 2, 3]
    out.append(("palette-257", img))
    # random palettes: the prefix is reproducible or not, the GPU must agree with the oracle
    for k in range(3):
        pk = rs.randint(0, 256, (32 + 50 * k, 3)).astype(np.uint8)
        out.append(("palette-rand%d" % k, pk[rs.randint(0, len(pk), (512, 512))]))
    return out


@pytest.mark.parametrize("name,img", cases(), ids=[c[0] for c in cases()])
def test_choh_parity(hoh, orc, name, img):
    try:
        ref, ref_printed = orc.choh(img)
    except orc.OracleError as e:
        # the reference would copy uninitialised bytes (grey tiles, Q15 prefix past the layer)
        assert e.code == -4, e
        with pytest.raises(hoh.HohError) as g:
            hoh.choh(img)
        assert g.value.code == 5
        return
    data, printed = hoh.choh(img)
    assert len(data) == len(ref)
    assert data == ref
    assert printed == ref_printed


def test_synth_device_matches_numpy(hoh):
    import torch
    from hoh_ans.synth import synth_rgb
    for W, H, seed, noise in ((512, 300, 3, 4), (1000, 77, 9, 0), (64, 64, 123456789, 40)):
        d = hoh.synth_rgb_dev(W, H, seed, noise)
        torch.cuda.synchronize()
        assert np.array_equal(d.cpu().numpy().reshape(H, W, 3), synth_rgb(W, H, seed, noise))


def test_choh_8192_golden(hoh, golden):
    import torch
    f = [f for f in golden["choh_s0"] if f["spec"]["W"] == 8192][0]
    sp = f["spec"]
    d = hoh.synth_rgb_dev(sp["W"], sp["H"], sp["seed"], sp["noise"])
    out, n, printed = hoh.encode_image(d, sp["W"], sp["H"])
    torch.cuda.synchronize()
    data = out[:n].cpu().numpy().tobytes()
    assert n == f["out"]["len"]
    assert hashlib.sha256(data).hexdigest() == f["out"]["sha256"]
    assert printed == f["printed"]


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("pb", [9, 10, 12, 15])
def test_normalize_steals_many_levels(seed, pb):
    """normalize_freqs (stattools.hpp:13-70) with many symbols scaled to zero width, so the steals
    drain several width levels (k_tables places them all at once): stream bytes equal the
    oracle's for skewed histograms with long tails of rare symbols."""
    import oracle
    import hoh_ans
    rng = np.random.default_rng(1000 + seed * 7 + pb)
    rng_sz = 512
    n = int(rng.integers(3000, 60000))
    body = np.minimum(rng.geometric(rng.uniform(0.05, 0.5), n), 40).astype(np.int64)
    tail = rng.choice(np.arange(41, rng_sz), size=int(rng.integers(50, 400)), replace=True)
    mids = rng.choice(np.arange(41, rng_sz), size=int(rng.integers(0, 300)))
    sym = np.concatenate([body, tail, np.repeat(mids, rng.integers(1, 6, mids.size))])
    rng.shuffle(sym)
    sym = sym.astype(np.uint16)
    want = oracle.encode_entropy(sym, rng_sz, pb)
    got = hoh_ans.encode_entropy(sym, rng_sz, pb)
    assert bytes(got) == bytes(want)


@pytest.mark.parametrize("pb", [7, 8, 9, 10, 11, 12, 13, 14, 16, 17, 18, 19])
def test_fast_chain_all_prob_bits(pb):
    """The f64-quotient chain (k_rans_fast KIND 1) at every prob_bits of the -s>=1 ladder
    (layer_encode.hpp:326-391) against the oracle (rans64.hpp:262-278): geometric, uniform and
    peaked histograms, one-symbol streams and ranges 2..512.  Every stream at prob_bits 7..19
    takes the chain: its f64 floors are exact for every f <= 2^19 (k_rans_enc.hip, step15's
    bound), so the peaked pb-19 cases (frequencies up to 2^19) check that bound."""
    import oracle
    import hoh_ans
    rng = np.random.default_rng(77 + pb)
    cases = []
    for rg in (2, 16, 100, 256, 512):
        if rg > (1 << pb):
            continue
        for kind in ("geo", "uni", "peak", "one"):
            n = int(rng.integers(1, 70000))
            if kind == "geo":
                s = np.minimum(rng.geometric(rng.uniform(0.05, 0.6), n) - 1, rg - 1)
            elif kind == "uni":
                s = rng.integers(0, rg, n)
            elif kind == "peak":
                s = np.where(rng.random(n) < 0.9, 0, rng.integers(0, rg, n))
            else:
                s = np.full(n, rg - 1)
            cases.append((s.astype(np.uint16), rg))
    for s, rg in cases:
        want = oracle.encode_entropy(s, rg, pb)
        got = hoh_ans.encode_entropy(s, rg, pb)
        assert bytes(got) == bytes(want), (pb, rg, s.size)
