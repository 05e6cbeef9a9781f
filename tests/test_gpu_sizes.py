"""Odd image sizes with dense LZ (flat gradients, copied runs): GPU .hoh bytes equal the oracle's
(choh.cpp:394-527 tiling incl. partial edge tiles and Q13 untiled images), and tiled files decode
losslessly.  Sizes straddle the tile width (256), the tiling threshold (512) and k_front's pixel
ring widths (271 / 1279)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SIZES = [(257, 512, 0), (300, 513, 2), (513, 257, 0), (777, 300, 1), (1023, 260, 0), (1025, 512, 2),
         (272, 200, 0), (1279, 100, 0), (1280, 90, 0), (640, 640, 0)]


def _img(W, H, noise, seed):
    from hoh_ans.synth import synth_rgb
    img = synth_rgb(W, H, seed, noise)
    rs = np.random.RandomState(seed)
    for _ in range(60):                                      # copies at back distances 1..64
        y, L, b = rs.randint(0, H), rs.randint(4, 40), rs.randint(1, 65)
        if W > b + L + 1:
            x = rs.randint(b, W - L)
            img[y, x:x + L] = img[y, x - b:x - b + L]
    return img


@pytest.fixture(scope="module")
def hoh():
    import hoh_ans
    return hoh_ans


@pytest.mark.parametrize("W,H,noise", SIZES, ids=["%dx%d-n%d" % s for s in SIZES])
def test_sizes_parity_and_roundtrip(hoh, orc, W, H, noise):
    img = _img(W, H, noise, W * 7 + H)
    try:
        ref, ref_printed = orc.choh(img)
    except orc.OracleError as e:                             # reference would copy garbage
        assert e.code == -4, e
        with pytest.raises(hoh.HohError):
            hoh.choh(img)
        return
    data, printed = hoh.choh(img)
    assert printed == ref_printed
    assert data == ref
    tiled = hoh.tiling(W, H)[0]
    if tiled:
        try:
            out = hoh.dhoh(data)
        except hoh.HohError as e:                            # palette tiles (Q15) are undecodable
            assert e.code == 6, e
            return
        assert np.array_equal(out.reshape(H, W, 3), img)


LARGE_UNTILED = [(5000, 250, 0), (12000, 200, 0), (1000, 200, 1)]


@pytest.mark.parametrize("W,H,speed", LARGE_UNTILED, ids=["%dx%d-s%d" % s for s in LARGE_UNTILED])
def test_large_untiled_parity(hoh, orc, W, H, speed):
    """Untiled images (H < 256) are one tile of W*H pixels: k_nuke's bitmap + count histograms
    no longer fit the 160 KB LDS above ~1.1 M px and take the global-memory walk
    (k_lz.hip nuke_tile).  Natural statistics, so most of the tile is LZ copies.  The file is
    header-only (Q13); the printed size carries the whole encode."""
    from hoh_ans.natural import natural_rgb
    img = natural_rgb(W, H, 5)
    ref, ref_printed = orc.choh(img, speed)
    data, printed = hoh.choh(img, speed=speed)
    assert printed == ref_printed
    assert data == ref


def test_untiled_search_grid_limit(hoh):
    """-s>=1 on an untiled image whose 40-px predictor grid exceeds the search kernel's LDS map
    (HOH_MAPCAP cells): refused with HOH_E_UNSUPPORTED, never a corrupt map."""
    from hoh_ans.natural import natural_rgb
    with pytest.raises(hoh.HohError) as e:
        hoh.choh(natural_rgb(1500, 200, 5), speed=1)
    assert e.value.code == 6
