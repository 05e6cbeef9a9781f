"""GPU decode: lossless round trip of choh -s0 files (with and without the side index), decode
of files made by the reference itself, and the stream / plane level drop-in entry points."""
import os

import numpy as np
import pytest

import hoh_ans
from gen import make_plane, make_symbols

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hoh():
    import hoh_ans
    return hoh_ans


def images():
    from hoh_ans.synth import synth_rgb
    rs = np.random.RandomState(7)
    out = [("synth512", synth_rgb(512, 512, 1, 4)), ("synth768x520", synth_rgb(768, 520, 3, 2)),
           ("gradient-lz", synth_rgb(256, 512, 5, 0)), ("synth1000x600", synth_rgb(1000, 600, 45, 8)),
           ("wide511", synth_rgb(511, 600, 12, 4))]
    img = synth_rgb(512, 512, 8, 4)
    for _ in range(300):
        y, x, L, b = rs.randint(0, 512), rs.randint(70, 400), rs.randint(4, 80), rs.randint(1, 65)
        img[y, x:x + L] = img[y, x - b:x - b + L]
    out.append(("repeats", img))
    out.append(("uniform", rs.randint(0, 256, (512, 768, 3)).astype(np.uint8)))
    return out


@pytest.mark.parametrize("name,img", images(), ids=[c[0] for c in images()])
def test_roundtrip(hoh, orc, name, img):
    import torch
    H, W, _ = img.shape
    d = torch.from_numpy(img.reshape(-1).copy()).cuda()
    ix = hoh.Index()
    out, n, _ = hoh.encode_image(d, W, H, index=ix)
    data = out[:n].cpu().numpy().tobytes()
    assert data == orc.choh(img)[0]                        # encoder parity
    for index in (ix, None):                               # segmented and serial rANS decode
        rgb, w, h = hoh.decode_image(out, n, index=index)
        torch.cuda.synchronize()
        assert (w, h) == (W, H)
        assert np.array_equal(rgb.cpu().numpy().reshape(H, W, 3), img), ("index" if index else "serial")


def test_decode_reference_made_file(hoh, golden):
    """bytes written by the compiled reference choh (golden sha) decode losslessly"""
    import hashlib
    from hoh_ans.synth import synth_rgb
    from oracle import choh as ochoh
    sp = [f for f in golden["choh_s0"] if f["spec"]["W"] == 1024][0]["spec"]
    img = synth_rgb(sp["W"], sp["H"], sp["seed"], sp["noise"])
    data, _ = ochoh(img)
    f = [f for f in golden["choh_s0"] if f["spec"]["W"] == 1024][0]
    assert hashlib.sha256(data).hexdigest() == f["out"]["sha256"]
    assert np.array_equal(hoh.dhoh(data), img)


def test_roundtrip_8192(hoh):
    import torch
    W = H = 8192
    d = hoh.synth_rgb_dev(W, H, 1, 4)
    ix = hoh.Index()
    out, n, _ = hoh.encode_image(d, W, H, index=ix)
    rgb, w, h = hoh.decode_image(out, n, index=ix)
    torch.cuda.synchronize()
    assert torch.equal(rgb, d)


def test_entropy_streams_vs_golden(hoh, golden, orc):
    import hashlib
    done = 0
    for e in golden["entropy"]:
        sp = e["spec"]
        if sp["n"] > 70000:
            continue
        sym = make_symbols(sp)
        enc = hoh.encode_entropy(sym, sp["range"], sp["pb"])
        assert len(enc) == e["enc"]["len"] and hashlib.sha256(enc).hexdigest() == e["enc"]["sha256"], sp
        if e.get("decodable", True) and sym.size:
            dec, bp = hoh.decode_entropy(enc + b"\0" * 8)
            assert np.array_equal(dec, sym), sp
            assert bp == len(enc)
        done += 1
    assert done > 50


def test_entropy_1m_single_stream(hoh, orc):
    """config 2: one stream of 1,048,576 symbols"""
    sp = {"kind": "laplace", "n": 1048576, "range": 512, "seed": 11, "scale_x16": 48, "pb": 15}
    sym = make_symbols(sp)
    enc = hoh.encode_entropy(sym, 512, 15)
    assert enc == orc.encode_entropy(sym, 512, 15)
    dec, bp = hoh.decode_entropy(enc)
    assert np.array_equal(dec, sym) and bp == len(enc)


def test_stream_sequence_q1(hoh, orc):
    """three streams back to back: the decoder must land on each next stream"""
    parts = [make_symbols({"kind": "laplace", "n": n, "range": r, "seed": n, "scale_x16": 30}) for n, r in
             ((257, 256), (5000, 512), (3, 256))]
    blob = b"".join(orc.encode_entropy(p, 256 if p.max() < 256 else 512, 10 if i != 1 else 15) for i, p in enumerate(parts))
    bp = 0
    for p in parts:
        dec, bp = hoh.decode_entropy(blob + b"\0" * 8, bp)
        assert np.array_equal(dec, p)
    assert bp == len(blob)


def test_layer_and_predictor(hoh, orc, golden):
    import hashlib
    for g in golden["layer_encode_s0"]:
        sp = g["spec"]
        plane = np.ascontiguousarray(make_plane(sp))
        nuke = np.zeros(plane.size, np.uint8)
        for a, b in g["nuke_ranges"]:
            nuke[a:b] = 1
        out = hoh.layer_encode(plane, g["depth"], nuke=nuke if g["nuke_ranges"] else None)
        assert hashlib.sha256(out).hexdigest() == g["out"]["sha256"], sp
    for p in golden["predict_fastpath"]:
        plane = make_plane(p["spec"])
        res = hoh.channelpredict_fastpath(plane, p["depth"])
        assert hashlib.sha256(res.tobytes()).hexdigest() == p["res"]["sha256"]
        back = hoh.unpredict_fastpath(res.reshape(-1), plane.shape[1], plane.shape[0], p["depth"])
        assert np.array_equal(back, plane)


def test_subtract_green(hoh, orc):
    from hoh_ans.synth import synth_rgb
    img = synth_rgb(300, 200, 3, 30)
    a = hoh.subtract_green(img)
    b = orc.subtract_green(img)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


def test_entropy_roundtrip_text_pb12():
    """entropy_roundtrip_test.sh's shape on the GPU: a text file's bytes as one stream (range 256,
    prob_bits 12: the generic chain), bytes equal to the oracle's and a lossless round trip.  The
    reference's own input (its source text) is not shipped; this repository's bench.py stands in."""
    import oracle
    data = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py"), "rb").read()
    sym = np.frombuffer(data, np.uint8).astype(np.uint16)
    got = hoh_ans.encode_entropy(sym, 256, 12)
    assert bytes(got) == bytes(oracle.encode_entropy(sym, 256, 12))
    dec, bp = hoh_ans.decode_entropy(got)
    assert bytes(np.asarray(dec, np.uint8)) == data and bp == len(got)
