"""The reference's own test flow, run through the GPU drop-ins.

oracle/ref/Makefile `dropin` compiles the reference's callers UNCHANGED -- simple_entropy_encoder.cpp
(:26-33, encode_entropy(bytes, n, 256, out, 12, 1)), simple_entropy_decoder.cpp (:28-34,
decode_entropy_8bit), layer_roundtrip_test.cpp (:7-59, layer_encode cruncher 2 -> decode_layer) and
the encoder itself, choh.cpp (:394-527, encode_tile -> layer_encode / encode_entropy per tile) --
against include/hoh/*.hpp, linked to libhohgpu.so, into oracle/_ref/dropin/.  These tests run
the flow of entropy_roundtrip_test.sh:1-11 and the layer round trip with those binaries:
  * the drop-in encoder's stream must equal the reference encoder's (oracle/_ref, the reference
    binary built from the same source without the drop-ins) byte for byte;
  * the drop-in decoder must restore the input (cmp), from its own stream and the reference's;
  * the reference decoder must read the drop-in's stream back too (one stream: Q1 does not bite),
    except the single-symbol table it cannot read (Q6);
  * layer_roundtrip_test must print "Layer roundtrip: OK" and exit 0 through the GPU;
  * choh's files and printed sizes must equal the reference binary's, tiled at -s0..-s4 (with the
    RGB and palette colour modes) and header-only.
The inputs are repository files (the reference encodes its own source text; that file is not
kept here), plus byte patterns that reach the stored fallback and a single-symbol table (Q6)."""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref")
DROP = os.path.join(REF, "dropin")


def _bin(d, name):
    p = os.path.join(d, name)
    assert os.path.exists(p), "%s not built (make -C oracle/ref all dropin, in the container)" % p
    return p


def _run(args, **kw):
    return subprocess.run(args, capture_output=True, text=True, timeout=120, **kw)


def _inputs(tmp_path):
    files = [os.path.join(ROOT, "tools", "cli", "choh.cpp"), os.path.join(ROOT, "bench.py"),
             os.path.join(ROOT, "include", "hoh_ans.h")]
    rng = np.random.default_rng(5)
    extra = {
        "wide.bin": rng.integers(0, 256, 20000, dtype=np.uint8).tobytes(),          # stored fallback (Q7)
        "one.bin": bytes([200]) * 4097,                                             # one symbol (Q6)
        "geo.bin": np.minimum(rng.geometric(0.08, 70000) - 1, 255).astype(np.uint8).tobytes(),
    }
    for k, v in extra.items():
        p = tmp_path / k
        p.write_bytes(v)
        files.append(str(p))
    return files


def test_entropy_roundtrip_flow(tmp_path):
    """entropy_roundtrip_test.sh:1-11 with the drop-in binaries, plus byte equality with the
    reference encoder and cross-decoding in both directions."""
    enc_d, dec_d = _bin(DROP, "simple_entropy_encoder"), _bin(DROP, "simple_entropy_decoder")
    enc_r, dec_r = _bin(REF, "simple_entropy_encoder"), _bin(REF, "simple_entropy_decoder")
    for i, f in enumerate(_inputs(tmp_path)):
        src = open(f, "rb").read()
        cg, cr = tmp_path / ("c_gpu%d" % i), tmp_path / ("c_ref%d" % i)
        r = _run([enc_d, f, str(cg)])
        assert r.returncode == 0, r.stdout + r.stderr
        assert "wrote %d bytes" % cg.stat().st_size in r.stdout
        r = _run([enc_r, f, str(cr)])
        assert r.returncode == 0, r.stdout + r.stderr
        assert cg.read_bytes() == cr.read_bytes(), f
        # the reference decoder cannot read a single-symbol table (its frequency overflows the
        # field): only the drop-in decoder reads that one back
        pairs = ((dec_d, cg), (dec_d, cr)) + (((dec_r, cg),) if not f.endswith("one.bin") else ())
        for dec, c in pairs:
            out = tmp_path / ("d%d" % i)
            r = _run([dec, str(c), str(out)])
            assert r.returncode == 0, r.stdout + r.stderr
            assert out.read_bytes() == src, (dec, f)           # cmp -s
            out.unlink()


def test_layer_roundtrip_flow():
    """layer_roundtrip_test.cpp:7-59 (5x4 plane, depth 8, cruncher 2, no LZ) through the GPU
    drop-ins, beside the reference binary of the same source."""
    r = _run([_bin(DROP, "layer_roundtrip_test")])
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Layer roundtrip: OK" in r.stdout
    r = _run([_bin(REF, "layer_roundtrip_test")])
    assert r.returncode == 0 and "Layer roundtrip: OK" in r.stdout


def _choh_cases():
    # (name, W, H, speed): tiled images (768x512: 3x2 tiles of 256; 1024^2: 4x4) at -s0..-s4, plus
    # an untiled one (header only).  -s3/-s4 take choh.cpp:265-325's RGB colour-mode
    # branch (layer_encode per R, G, B plane with cruncher 3/4) and seek distances 12/14
    # (choh.cpp:132-137); "palette" tiles hold <= 256 colours (palette_encode, choh.cpp:48-102, Q15)
    return [("synth", 768, 512, 0), ("synth", 768, 512, 1), ("natural", 1024, 1024, 0),
            ("natural", 1024, 1024, 1), ("synth", 768, 512, 2), ("synth", 320, 200, 0),
            ("synth", 768, 512, 3), ("natural", 768, 512, 3), ("natural", 768, 512, 4),
            ("palette", 512, 256, 3), ("palette", 512, 256, 4), ("natural", 768, 512, 2)]


def _image(kind, W, H):
    import hoh_ans.natural as nat
    from hoh_ans import synth
    if kind == "synth":
        return synth.synth_rgb(W, H, seed=3, noise=4)
    if kind == "natural":
        return nat.natural_rgb(W, H, 1)
    rs = np.random.RandomState(21)                 # test_gpu_search.py's palette image
    pal = np.stack([rs.randint(0, 256, 40), np.full(40, 9), rs.randint(0, 256, 40)], 1).astype(np.uint8)
    img = synth.synth_rgb(W, H, 10, 3)
    img[:, W // 2:] = pal[rs.randint(0, 40, (H, W - W // 2))]
    return img


@pytest.mark.parametrize("case", _choh_cases(), ids=lambda c: "%s-%dx%d-s%d" % c)
def test_choh_through_dropins(tmp_path, case):
    """The reference's own encoder main (choh.cpp:394-527: header, tiling, encode_tile per tile,
    which calls layer_encode (layer_encode.hpp:11-20) per plane and encode_entropy for the LZ and
    palette streams) compiled unchanged against the drop-ins and run on the GPU: its file and
    printed size must equal the reference binary's (oracle/_ref/choh, same source, no drop-ins)."""
    kind, W, H, speed = case
    img = _image(kind, W, H)
    src = tmp_path / "in.rgb"
    src.write_bytes(np.ascontiguousarray(img, dtype=np.uint8).tobytes())
    outs = {}
    for tag, exe in (("dropin", _bin(DROP, "choh")), ("ref", _bin(REF, "choh"))):
        o = tmp_path / ("%s.hoh" % tag)
        r = subprocess.run([exe, str(src), str(o), str(W), str(H), "-s%d" % speed], capture_output=True,
                           text=True, timeout=600)
        assert r.returncode == 0, (tag, r.stdout + r.stderr)
        outs[tag] = (o.read_bytes(), r.stdout.strip().splitlines()[-1])
    assert outs["dropin"][1] == outs["ref"][1], "printed sizes differ"
    assert outs["dropin"][0] == outs["ref"][0], "files differ (%d vs %d bytes)" % (len(outs["dropin"][0]),
                                                                                   len(outs["ref"][0]))
