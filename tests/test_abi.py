"""CPU-side checks of the C ABI boundary: the in-tree library loads and exports every function
include/hoh_ans.h declares (no GPU needed: nothing is called)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "hoh-ans_amd", "lib", "libhohgpu.so")


def declared():
    src = open(os.path.join(ROOT, "include", "hoh_ans.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hoh_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = declared()
    for n in ("hoh_encode_image", "hoh_decode_image", "hoh_encode_entropy", "hoh_decode_entropy",
              "hoh_layer_encode", "hoh_layer_decode", "hoh_predict_fastpath", "hoh_unpredict_fastpath",
              "hoh_subtract_green", "hoh_encode_tiles", "hoh_file_prefix"):
        assert n in names


@pytest.mark.skipif(not os.path.exists(LIB), reason="libhohgpu.so not built")
def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(LIB)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing


@pytest.mark.skipif(not os.path.exists(LIB), reason="libhohgpu.so not built")
def test_host_only_helpers():
    """pure-host helpers of the ABI work without a GPU: tiling, prefix, header peek, bounds"""
    import numpy as np
    import hoh_ans
    assert hoh_ans.tiling(8192, 8192) == (True, 32, 32, 256, 256)
    assert hoh_ans.tiling(2, 2)[0] is False
    assert hoh_ans.tiling(1000, 600) == (True, 3, 2, 334, 300)
    pre = hoh_ans.file_prefix(1000, 600, [100, 200000, 3, 4, 5, 6])
    assert pre[:8] == bytes([153, 72, 79, 72, 2, 8]) + bytes([0x87, 0x67])
    W, H, xt, yt = hoh_ans.peek_header(pre)
    assert (W, H, xt, yt) == (1000, 600, 3, 2)
    assert hoh_ans.lib().hoh_encode_bound(8192, 8192) > 8192 * 8192 * 3


@pytest.mark.skipif(not os.path.exists(LIB), reason="libhohgpu.so not built")
def test_entropy_parse_framing():
    """hoh_entropy_parse (decode_entropy_simple's walk, host only) ends every stream exactly
    where the oracle's decoder does, over rANS streams with clamped / raw tables and stored
    streams, and back to back."""
    import numpy as np
    import hoh_ans
    import oracle
    rng = np.random.default_rng(11)
    seen = set()
    cat = b""
    ends = []
    for trial in range(60):
        rg = int(rng.choice([2, 3, 16, 256, 511, 512, 1024, 4096]))
        pb = int(rng.integers(12, 16))    # the metadata byte holds 4 bits of prob_bits (entropy_encoding.hpp)
        n = int(rng.choice([0, 1, 3, 40, 500, 5000]))
        kind = trial % 3
        if kind == 0:
            sym = np.minimum(rng.geometric(0.2, n) - 1, rg - 1)
        elif kind == 1:
            sym = rng.integers(0, rg, n)
        else:
            sym = np.full(n, rg - 1)
        s = oracle.encode_entropy(sym.astype(np.uint16), rg, pb)
        try:
            _, bp = oracle.decode_entropy(s + b"\x00" * 8)
        except oracle.OracleError:
            continue               # tables the reference writes but cannot read back
        h = hoh_ans.entropy_parse(s)
        assert h["stream_end"] == bp == len(s), (rg, pb, n, kind, h)
        assert h["count"] == n and h["range"] == rg
        seen.add((h["entropy_mode"], h["table_mode"]))
        cat += s
        ends.append(len(cat))
    assert (0, 0) in seen and (1, 2) in seen, seen
    p = 0
    for e in ends:
        p = hoh_ans.entropy_parse(cat, p)["stream_end"]
        assert p == e


@pytest.mark.skipif(not os.path.exists(LIB), reason="libhohgpu.so not built")
def test_no_device_fails_loudly():
    """without a GPU the product path must refuse, never fall back to the CPU"""
    import hoh_ans
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is present")
    except ImportError:
        pass
    with pytest.raises(hoh_ans.HohError) as e:
        hoh_ans.Context(0)
    assert e.value.code == 8


def test_dropin_headers_compile(tmp_path):
    """include/hoh/*.hpp re-expose the reference's call surface; they must compile as C++17
    with nothing but the C ABI header (no HIP, no torch)."""
    import subprocess
    src = tmp_path / "t.cpp"
    inc = os.path.join(ROOT, "include", "hoh")
    src.write_text("".join('#include "%s"\n' % os.path.join(inc, h) for h in sorted(os.listdir(inc))) +
                   "int main() { return 0; }\n")
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


REF = "/root/reference"
DROPINS_ENTROPY = ("entropy_encoding.hpp", "entropy_decoding.hpp")
DROPINS_ALL = DROPINS_ENTROPY + ("layer_encode.hpp", "layer_decode.hpp", "prediction.hpp", "unprediction.hpp")
CALLERS = ("simple_entropy_encoder.cpp", "simple_entropy_decoder.cpp", "layer_roundtrip_test.cpp", "dhoh.cpp",
           "choh.cpp")


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree absent (GPU box)")
@pytest.mark.parametrize("swap", ["entropy", "all"])
def test_reference_callers_compile_against_dropins(tmp_path, swap):
    """The reference's own translation units compile, unchanged, with its headers replaced by the
    drop-ins: the callers of decode_entropy_8bit (layer_decode.hpp:223, un_lz.hpp:103-139,
    simple_entropy_decoder.cpp:28), of decode_entropy_simple (layer_decode.hpp:97-117,
    un_lz.hpp:30-57) and of every other replaced function.  The reference tree is mirrored by
    symlinks in a temporary directory (quoted includes resolve next to the including file), the
    replaced headers point at include/hoh/; compile only (-fsyntax-only), nothing is kept."""
    import subprocess
    stage = tmp_path / "ref"
    stage.mkdir()
    os.symlink(os.path.join(ROOT, "include", "hoh_ans.h"), tmp_path / "hoh_ans.h")
    inc = os.path.join(ROOT, "include", "hoh")
    swapped = DROPINS_ENTROPY if swap == "entropy" else DROPINS_ALL
    for f in os.listdir(REF):
        if os.path.isfile(os.path.join(REF, f)) and f not in swapped:
            os.symlink(os.path.join(REF, f), stage / f)
    for f in swapped + ("hoh_gpu.hpp",):
        os.symlink(os.path.join(inc, f), stage / f)
    errs = []
    for cpp in CALLERS:
        r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-w", str(stage / cpp)], capture_output=True,
                           text=True, cwd=str(stage))
        if r.returncode:
            errs.append("%s:\n%s" % (cpp, r.stderr[-3000:]))
    assert not errs, "\n".join(errs)
