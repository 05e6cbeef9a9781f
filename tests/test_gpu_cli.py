"""The choh / dhoh drop-in CLIs and the drop-in C++ headers (include/hoh) on the GPU.

choh must write the bytes the reference choh -s0 writes and print the size it prints
(choh.cpp:394-527); dhoh must restore the RGB bytes (the reference dhoh crashes on tiled files,
SURVEY Q1, so the oracle's corrected decoder is the check)."""
import os
import subprocess

import numpy as np
import pytest

import oracle
from hoh_ans import synth

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "hoh-ans_amd", "bin")


def _run(args):
    return subprocess.run(args, capture_output=True, text=True, timeout=120)


@pytest.mark.parametrize("W,H", [(768, 512), (1000, 600), (300, 200)])
def test_choh_dhoh_cli(tmp_path, W, H):
    img = synth.synth_rgb(W, H, seed=21, noise=4)
    src = tmp_path / "in.rgb"
    src.write_bytes(img.tobytes())
    r = _run([os.path.join(BIN, "choh"), str(src), str(tmp_path / "o.hoh"), str(W), str(H), "-s0"])
    assert r.returncode == 0, r.stderr
    want, printed = oracle.choh(img)
    got = (tmp_path / "o.hoh").read_bytes()
    assert got == want
    assert int(r.stdout.strip().splitlines()[-1]) == printed
    tiled = (W >= 512 or H >= 512) and W >= 256 and H >= 256
    if tiled:
        r = _run([os.path.join(BIN, "dhoh"), str(tmp_path / "o.hoh"), str(tmp_path / "back.rgb")])
        assert r.returncode == 0, r.stdout + r.stderr
        assert (tmp_path / "back.rgb").read_bytes() == img.tobytes()


@pytest.mark.parametrize("speed", [1, 3])
def test_choh_speeds(tmp_path, speed):
    from hoh_ans.synth import synth_rgb
    img = synth_rgb(512, 256, 30 + speed, 3)
    src = tmp_path / "in.rgb"
    src.write_bytes(img.tobytes())
    r = _run([os.path.join(BIN, "choh"), str(src), str(tmp_path / "o.hoh"), "512", "256", "-s%d" % speed])
    assert r.returncode == 0, r.stderr
    want, printed = oracle.choh(img, speed)
    assert (tmp_path / "o.hoh").read_bytes() == want
    assert int(r.stdout.strip().splitlines()[-1]) == printed


def test_dropin_headers_roundtrip():
    r = _run([os.path.join(BIN, "dropin_test")])
    assert r.returncode == 0, r.stdout + r.stderr
    assert "drop-in headers ok" in r.stdout
