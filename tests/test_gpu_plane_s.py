"""GPU plane-level -s>=1 entry points (prediction.hpp:46-229, unprediction.hpp:6-91,
layer_encode.hpp:11-412 at cruncher 1..4, layer_decode.hpp:128-278) against the oracle, which
tests/test_oracle_vs_reference.py pins to the reference's own functions."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MASKS = [1, 2, 0x20, 0x10, 0xffbf, 3, 0xfffd, 0xfffb, 0xfff7, 0xffef, 0xffdf, 0xff7f, 0xfdff, 0xffff]


@pytest.fixture(scope="module")
def hoh():
    import hoh_ans
    return hoh_ans


def _smooth(rs, h, w, depth, noise):
    y, x = np.mgrid[0:h, 0:w]
    v = (x * rs.randint(1, 5) + y * rs.randint(1, 5)) // 3 + rs.randint(-noise, noise + 1, (h, w))
    return (v % (1 << depth)).astype(np.uint16)


def test_predict_section_and_all(hoh, orc):
    rs = np.random.RandomState(31)
    n = 0
    while n < 40:
        w, h, depth = int(rs.randint(1, 300)), int(rs.randint(1, 300)), int(rs.choice([8, 9]))
        d = _smooth(rs, h, w, depth, int(rs.choice([0, 2, 30]))) if n % 2 else \
            rs.randint(0, 1 << depth, (h, w)).astype(np.uint16)
        xt, yt = int(rs.randint(1, 9)), int(rs.randint(1, 9))
        cx, cy = int(rs.randint(0, xt)), int(rs.randint(0, yt))
        if cx * ((w + xt - 1) // xt) >= w or cy * ((h + yt - 1) // yt) >= h:
            continue
        mask = int(rs.choice(MASKS + [int(rs.randint(1, 65536))]))
        assert np.array_equal(hoh.predict_section(d, depth, xt, yt, cx, cy, mask),
                              orc.predict_section(d, depth, xt, yt, cx, cy, mask)), (w, h, xt, yt, cx, cy, mask)
        tm = rs.choice(MASKS, xt * yt).astype(np.uint16)
        assert np.array_equal(hoh.predict_all(d, depth, xt, yt, tm), orc.predict_all(d, depth, xt, yt, tm))
        n += 1


def test_unpredict_all_maps(hoh, orc):
    rs = np.random.RandomState(32)
    for it in range(20):
        w, h, depth = int(rs.randint(2, 260)), int(rs.randint(2, 260)), int(rs.choice([8, 9]))
        xt, yt = int(rs.randint(1, 8)), int(rs.randint(1, 8))
        tm = rs.choice(MASKS, xt * yt).astype(np.uint16)
        if xt == 1 and yt == 1 and tm[0] == 0x10:
            tm[0] = 0xffff
        d = _smooth(rs, h, w, depth, int(rs.choice([0, 3, 20])))
        res = orc.predict_all(d, depth, xt, yt, tm)
        assert np.array_equal(hoh.unpredict_all(res, w, h, depth, xt, yt, tm), d), it
        br = np.zeros(w * h, np.uint16)
        for _ in range(8):
            i, L, b = int(rs.randint(0, w * h)), int(rs.randint(1, 30)), int(rs.randint(1, 200))
            for k in range(i, min(w * h, i + L)):
                if k >= b:
                    br[k] = b
        r2 = rs.randint(0, 1 << depth, int((br == 0).sum())).astype(np.uint16)
        assert np.array_equal(hoh.unpredict_all(r2, w, h, depth, xt, yt, tm, br),
                              orc.unpredict_all(r2, w, h, depth, xt, yt, tm, br)), it


@pytest.mark.parametrize("speed", [1, 2, 3, 4])
def test_layer_encode_speeds(hoh, orc, speed):
    rs = np.random.RandomState(40 + speed)
    for it in range(4):
        w, h = int(rs.choice([30, 64, 100, 256])), int(rs.choice([20, 41, 128, 256]))
        depth = int(rs.choice([8, 9]))
        d = _smooth(rs, h, w, depth, int(rs.choice([1, 3, 8])))
        nuke = (rs.rand(h, w) < 0.05).astype(np.uint8) if it % 2 else None
        want = orc.layer_encode(d, depth, speed, nuke)
        assert hoh.layer_encode(d, depth, nuke, speed=speed) == want, (it, w, h, depth)


def test_layer_decode_predictor_map(hoh, orc):
    """a layer with a predictor map (layer_decode.hpp:196-256), built from its parts"""
    rs = np.random.RandomState(33)
    for it in range(6):
        w, h, depth = int(rs.choice([64, 100, 256])), int(rs.choice([48, 256])), int(rs.choice([8, 9]))
        xt, yt = (w + 39) // 40, (h + 39) // 40
        used = sorted(set(int(m) for m in rs.choice(len(MASKS), 3)))
        pidx = rs.choice(len(used), xt * yt).astype(np.uint16)
        tm = np.array([MASKS[used[k]] for k in pidx], np.uint16)
        d = _smooth(rs, h, w, depth, 4)
        res = orc.predict_all(d, depth, xt, yt, tm)
        hdr = bytes([0x10, xt - 1, yt - 1, len(used)]) + b"".join(bytes([MASKS[m] >> 8, MASKS[m] & 255]) for m in used)
        layer = hdr + orc.encode_entropy(pidx, len(used), 8) + orc.encode_entropy(res, 1 << depth, 15)
        assert np.array_equal(hoh.layer_decode(layer, w, h, depth), d), it
