"""choh / dhoh over several devices in ONE process (hoh_mgpu_*, tools/cli --gpus/--devices):
bands of tile rows (choh.cpp:464-500), one gather into the file on the first device.  On a
one-GPU machine the devices repeat (several shards on GPU 0: the gather moves by device copies)
and a one-device list builds a real RCCL communicator (ncclCommInitAll) and encodes through it.
Files must equal the single-GPU / reference bytes (golden sha256 of the reference choh at 8192^2),
and decodes must be lossless."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest
import torch

import hoh_ans
from hoh_ans import synth

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "hoh-ans_amd", "bin")


def _golden(W, H, seed, noise):
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))
    for c in g["choh_s0"]:
        sp = c["spec"]
        if (sp.get("W"), sp.get("H"), sp.get("seed"), sp.get("noise")) == (W, H, seed, noise):
            return c["out"]["sha256"] if isinstance(c["out"], dict) else hashlib.sha256(bytes.fromhex(c["out"])).hexdigest()
    return None


def test_rccl_single_device_communicator():
    m = hoh_ans.MultiGPU([0])
    assert m.transport() == 1                   # librccl loaded, ncclCommInitAll built the communicator
    img = synth.synth_rgb(1024, 768, seed=4, noise=4)
    got, printed = m.encode_image(img)
    want, wp = hoh_ans.choh(img)
    assert got == want and printed == wp
    assert np.array_equal(m.decode_image(got), img)
    m.close()


@pytest.mark.parametrize("nshard", [2, 3, 4])
def test_shards_on_one_gpu_8192_golden(nshard):
    m = hoh_ans.MultiGPU([0] * nshard)
    assert m.transport() == 0
    img = synth.synth_rgb(8192, 8192, seed=1, noise=4)
    got, printed = m.encode_image(img)
    assert hashlib.sha256(got).hexdigest() == _golden(8192, 8192, 1, 4)
    assert printed == len(got)
    assert np.array_equal(m.decode_image(got), img)
    m.close()


@pytest.mark.parametrize("W,H,nshard", [(1000, 600, 2), (777, 1300, 3), (300, 200, 2), (2304, 1536, 4)])
def test_shards_odd_sizes(W, H, nshard):
    img = synth.synth_rgb(W, H, seed=9, noise=3)
    want, wp = hoh_ans.choh(img)
    m = hoh_ans.MultiGPU([0] * nshard)
    got, printed = m.encode_image(img)
    assert got == want and printed == wp
    tiled = (W >= 512 or H >= 512) and W >= 256 and H >= 256
    if tiled:
        assert np.array_equal(m.decode_image(got), img)
    m.close()


def test_cli_devices(tmp_path):
    W, H = 1536, 1024
    img = synth.synth_rgb(W, H, seed=12, noise=4)
    src = tmp_path / "in.rgb"
    src.write_bytes(img.tobytes())
    r = subprocess.run([os.path.join(BIN, "choh"), "--devices", "0,0,0", str(src), str(tmp_path / "o.hoh"), str(W),
                        str(H), "-s0"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    want, printed = hoh_ans.choh(img)
    assert (tmp_path / "o.hoh").read_bytes() == want
    assert int(r.stdout.strip().splitlines()[-1]) == printed
    r = subprocess.run([os.path.join(BIN, "dhoh"), "--devices", "0,0", str(tmp_path / "o.hoh"),
                        str(tmp_path / "back.rgb")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert (tmp_path / "back.rgb").read_bytes() == img.tobytes()
