"""Direct oracle-vs-reference comparisons on fresh random inputs (runs only where the reference
was built in place: oracle/_ref/libref.so)."""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.skipif(O.ref() is None, reason="oracle/_ref not built (no /root/reference)")


def ref_encode(sym, rng, pb):
    R = O.ref()
    out = np.empty(O.lib().or_entropy_bound(sym.size, rng, pb) + 64, np.uint8)
    r = R.ref_encode_entropy(sym.ctypes.data_as(O.u16p), sym.size, rng, pb, out.ctypes.data_as(O.u8p))
    return out[:r].tobytes()


def test_random_streams():
    rs = np.random.RandomState(7)
    for it in range(300):
        rng = int(rs.choice([2, 3, 17, 64, 255, 256, 300, 511, 512]))
        pb = int(rs.choice([p for p in (9, 10, 11, 12, 13, 14, 15) if (1 << p) >= rng]))
        n = int(rs.choice([1, 2, 10, 100, 1000, 5000]))
        scale = rs.uniform(0.3, 60)
        v = np.floor(rs.exponential(scale, n)).astype(np.int64) * rs.choice([-1, 1], n)
        sym = ((rng // 2 + v) % rng).astype(np.uint16)
        assert O.encode_entropy(sym, rng, pb) == ref_encode(sym, rng, pb), (rng, pb, n)


def test_lz_and_tiles_random_patterns():
    """tiles with repeats (LZ matches), few colours and flat areas"""
    rs = np.random.RandomState(11)
    R = O.ref()
    for it in range(12):
        w, h = int(rs.choice([64, 100, 256])), int(rs.choice([48, 256]))
        base = rs.randint(0, 256, size=(h, w, 3)).astype(np.uint8)
        pal = rs.randint(0, 256, size=(int(rs.choice([3, 20, 300])), 3)).astype(np.uint8)
        img = pal[rs.randint(0, len(pal), size=(h, w))]
        # repeat runs
        for _ in range(20):
            y, x, L = rs.randint(0, h), rs.randint(8, w), rs.randint(4, 40)
            img[y, x:x + L] = img[y, x - 8:x - 8 + L][: max(0, min(L, w - x))]
        if it % 3 == 0:
            img = np.where(rs.rand(h, w, 1) < 0.7, img, base)
        img = np.ascontiguousarray(img)
        out = np.empty(img.size * 6 + 8192, np.uint8)
        r = R.ref_encode_tile(img.ctypes.data_as(O.u8p), w, h, 0, out.ctypes.data_as(O.u8p))
        try:
            mine = O.encode_tile(img)
        except O.OracleError as e:
            assert e.code == -4  # unreproducible in the reference (uninitialised bytes)
            continue
        assert mine == out[:r].tobytes(), it


def test_single_symbol_overrun():
    """single-symbol streams at prob_bits 8/12/16 make the reference write one element past its
    clamp array (entropy_encoding.hpp:72,103); the oracle drops that write -- same bytes."""
    for n, rng, pb, v in [(65536, 256, 12, 7), (65536, 256, 8, 200), (5000, 512, 12, 3), (70000, 2, 8, 1),
                          (100000, 256, 16, 9), (65536, 1024, 12, 5), (1, 256, 8, 3), (3, 5, 12, 4)]:
        sym = np.full(n, v, np.uint16)
        assert O.encode_entropy(sym, rng, pb) == ref_encode(sym, rng, pb), (n, rng, pb)


def test_palette_files_vs_reference_choh(tmp_path):
    """whole files with palette tiles (choh.cpp:298-308, Q15) through the reference's own choh"""
    import importlib.util
    import os
    import subprocess
    exe = O.ref_bin("choh")
    if exe is None:
        pytest.skip("reference choh not built")
    here = os.path.dirname(os.path.abspath(__file__))
    spec = importlib.util.spec_from_file_location("tge", os.path.join(here, "test_gpu_encode.py"))
    tge = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(tge)
    n_ok = 0
    for name, img in tge.palette_cases():
        try:
            mine, printed = O.choh(img)
        except O.OracleError as e:
            assert e.code == -4, name
            continue
        H, W, _ = img.shape
        src, dst = tmp_path / (name + ".rgb"), tmp_path / (name + ".hoh")
        src.write_bytes(np.ascontiguousarray(img).tobytes())
        r = subprocess.run([exe, str(src), str(dst), str(W), str(H), "-s0"], capture_output=True, timeout=120)
        assert r.returncode == 0, name
        assert int(r.stdout.split()[-1]) == printed, name
        assert dst.read_bytes() == mine, name
        n_ok += 1
    assert n_ok >= 4


def _smooth(rs, h, w, depth, noise):
    y, x = np.mgrid[0:h, 0:w]
    v = (x * rs.randint(1, 5) + y * rs.randint(1, 5)) // 3 + rs.randint(-noise, noise + 1, (h, w))
    return (v % (1 << depth)).astype(np.uint16)


def test_predict_section_and_all_vs_reference():
    """channelpredict_section / channelpredict_all (prediction.hpp:46-229), the -s>=1 predictors"""
    rs = np.random.RandomState(3)
    R = O.ref()
    masks = [1, 2, 0x20, 0x10, 0xffbf, 3, 0xfffd, 0xfffb, 0xfff7, 0xffef, 0xffdf, 0xff7f, 0xfdff, 0xffff]
    n = 0
    while n < 120:
        w, h, depth = int(rs.randint(1, 100)), int(rs.randint(1, 100)), int(rs.choice([8, 9]))
        d = _smooth(rs, h, w, depth, int(rs.choice([0, 2, 30]))) if n % 2 else \
            rs.randint(0, 1 << depth, (h, w)).astype(np.uint16)
        xt, yt = int(rs.randint(1, 5)), int(rs.randint(1, 5))
        cx, cy = int(rs.randint(0, xt)), int(rs.randint(0, yt))
        if cx * ((w + xt - 1) // xt) >= w or cy * ((h + yt - 1) // yt) >= h:
            continue
        mask = int(rs.choice(masks + [int(rs.randint(1, 65536))]))
        mine = O.predict_section(d, depth, xt, yt, cx, cy, mask)
        out = np.empty(w * h + 64, np.uint16)
        k = R.ref_channelpredict_section(d.ctypes.data_as(O.u16p), w, h, depth, xt, yt, cx, cy, mask,
                                         out.ctypes.data_as(O.u16p))
        assert k == mine.size and np.array_equal(out[:k], mine), (w, h, xt, yt, cx, cy, mask)
        tm = rs.choice(masks, xt * yt).astype(np.uint16)
        out = np.empty(w * h, np.uint16)
        R.ref_channelpredict_all(d.ctypes.data_as(O.u16p), w, h, depth, xt, yt, tm.ctypes.data_as(O.u16p),
                                 out.ctypes.data_as(O.u16p))
        assert np.array_equal(out, O.predict_all(d, depth, xt, yt, tm)), (w, h, xt, yt)
        n += 1


def test_layer_encode_all_speeds_vs_reference():
    """layer_encode at cruncher 1..4 (layer_encode.hpp:122-392): search, map stream, prob_bits
    ladder and the Q14 stale-prefix output"""
    rs = np.random.RandomState(4)
    R = O.ref()
    for it in range(12):
        w, h = int(rs.choice([30, 64, 100, 256])), int(rs.choice([20, 41, 128]))
        depth, cr = int(rs.choice([8, 9])), 1 + it % 4
        d = _smooth(rs, h, w, depth, int(rs.choice([1, 3, 8])))
        nuke = (rs.rand(h, w) < 0.05).astype(np.uint8) if it % 3 == 0 else np.zeros((h, w), np.uint8)
        mine = O.layer_encode(d, depth, cr, nuke)
        out = np.empty(len(mine) + (1 << 20), np.uint8)
        r = R.ref_layer_encode(d.ctypes.data_as(O.u16p), w * h, w, h, depth, cr, nuke.ctypes.data_as(O.u8p),
                               out.ctypes.data_as(O.u8p))
        assert out[:r].tobytes() == mine, (it, w, h, depth, cr)


def test_tiles_all_speeds_vs_reference():
    """encode_tile at -s1..-s4: LZ seek distance 10-14 + vertical search with 4 streams, palette
    and RGB colour modes"""
    from hoh_ans.synth import synth_rgb
    rs = np.random.RandomState(5)
    R = O.ref()
    seen = 0
    for it in range(16):
        w, h = int(rs.choice([48, 64, 100])), int(rs.choice([40, 64, 100]))
        cr = 1 + it % 4
        img = synth_rgb(w, h, it, int(rs.choice([0, 2, 4, 16])))
        if it % 4 == 1:     # palette with constant G: the indexed layer wins, prefix reproducible
            pal = np.stack([rs.randint(0, 256, 40), np.full(40, 9), rs.randint(0, 256, 40)], 1).astype(np.uint8)
            img = pal[rs.randint(0, 40, (h, w))]
        if it % 5 == 2:
            img[h // 2:, :] = img[:h - h // 2, :]
        img = np.ascontiguousarray(img)
        out = np.empty(img.size * 8 + 65536, np.uint8)
        r = R.ref_encode_tile(img.ctypes.data_as(O.u8p), w, h, cr, out.ctypes.data_as(O.u8p))
        try:
            mine = O.encode_tile(img, cr)
        except O.OracleError as e:
            assert e.code == -4
            continue
        assert out[:r].tobytes() == mine, (it, w, h, cr)
        seen += 1
    assert seen >= 12


def test_choh_speeds_vs_reference_binary(tmp_path):
    import subprocess
    from hoh_ans.synth import synth_rgb
    exe = O.ref_bin("choh")
    if exe is None:
        pytest.skip("reference choh not built")
    for W, H, sp, seed, noise in [(512, 256, 1, 1, 3), (256, 512, 2, 2, 2), (512, 256, 3, 3, 4)]:
        img = synth_rgb(W, H, seed, noise)
        (tmp_path / "a.rgb").write_bytes(img.tobytes())
        r = subprocess.run([exe, str(tmp_path / "a.rgb"), str(tmp_path / "a.hoh"), str(W), str(H), "-s%d" % sp],
                           capture_output=True, timeout=300)
        mine, printed = O.choh(img, sp)
        assert (tmp_path / "a.hoh").read_bytes() == mine, (W, H, sp)
        assert int(r.stdout.split()[-1]) == printed


def test_unpredict_all_maps_vs_reference():
    """unpredict_all (unprediction.hpp:6-91) with predictor maps and LZ back references; and the
    round trip channelpredict_all -> unpredict_all"""
    rs = np.random.RandomState(8)
    R = O.ref()
    masks = [1, 2, 0x20, 0x10, 0xffbf, 3, 0xfffd, 0xffff]
    for it in range(60):
        w, h, depth = int(rs.randint(1, 90)), int(rs.randint(1, 90)), int(rs.choice([8, 9]))
        xt, yt = int(rs.randint(1, 4)), int(rs.randint(1, 4))
        tm = rs.choice(masks, xt * yt).astype(np.uint16)
        d = _smooth(rs, h, w, depth, int(rs.choice([0, 3, 20])))
        res = O.predict_all(d, depth, xt, yt, tm)
        assert np.array_equal(O.unpredict_all(res, w, h, depth, xt, yt, tm), d), it
        br = np.zeros(w * h, np.uint16)
        if it % 2:
            for _ in range(5):
                i, L, b = int(rs.randint(0, w * h)), int(rs.randint(1, 20)), int(rs.randint(1, 60))
                for k in range(i, min(w * h, i + L)):
                    if k >= b:
                        br[k] = b
        r2 = rs.randint(0, 1 << depth, w * h).astype(np.uint16)
        nres = int((br == 0).sum())
        out = np.empty(w * h, np.uint16)
        R.ref_unpredict_map(r2.ctypes.data_as(O.u16p), w, h, depth, xt, yt, tm.ctypes.data_as(O.u16p),
                            br.ctypes.data_as(O.u16p), out.ctypes.data_as(O.u16p))
        mine = O.unpredict_all(r2[:nres], w, h, depth, xt, yt, tm, br)
        assert np.array_equal(mine.reshape(-1), out), it
