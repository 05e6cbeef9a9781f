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
