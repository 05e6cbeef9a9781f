"""GPU: batches at the search speeds (-s1..-s4, choh.cpp:125-137): hoh_encode_images_async and
hoh_encode_tiles_images_async stack the n images' (or shards') tiles into one tile grid exactly as
at -s0, so every -s>=1 kernel (predictor search, LZ screen / scan, prob_bits ladder, chains) covers
the whole batch per launch; k_layout_s lays out one file per image.

Every batched file must be the single-image call's bytes, and so the reference choh's where
tests/golden/golden_natural.json holds its SHA.  -s>=1 files are undecodable by construction
(SURVEY Q14), so there is no round trip here.  The 8-image 8192^2 case pushes the job's
stream tables past 4 GB: the -s>=1 chains address them through 64-bit per-lane addresses."""
import hashlib
import json
import os

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def hoh():
    import hoh_ans
    return hoh_ans


def _golden(W, H, seed, speed):
    g = json.load(open(os.path.join(HERE, "golden", "golden_natural.json")))
    for r in g["files"]:
        s = r["spec"]
        if (s["W"], s["H"], s["seed"], s["speed"], s["gen"]) == (W, H, seed, speed, "natural"):
            return r["out"]["len"], r["out"]["sha256"]
    return None


def _sha(t):
    return hashlib.sha256(t.cpu().numpy().tobytes()).hexdigest()


def _images(hoh, ctx, W, H, specs):
    """specs: ("natural", seed) or ("synth", seed, noise)"""
    import torch
    img = W * H * 3
    rgb = torch.empty(len(specs) * img, dtype=torch.uint8, device="cuda")
    for i, sp in enumerate(specs):
        if sp[0] == "natural":
            rgb[i * img:(i + 1) * img] = hoh.natural_rgb_dev(W, H, sp[1], ctx=ctx)
        else:
            rgb[i * img:(i + 1) * img] = hoh.synth_rgb_dev(W, H, sp[1], sp[2], ctx=ctx)
    torch.cuda.synchronize()
    return rgb


def _batch_vs_single(hoh, W, H, speed, specs):
    import torch
    ctx = hoh.Context(0)
    L = hoh.lib()
    stride = L.hoh_encode_bound(W, H)
    img = W * H * 3
    n = len(specs)
    rgb = _images(hoh, ctx, W, H, specs)
    out = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    st = torch.zeros(2 * n, dtype=torch.int64, device="cuda")
    ix = hoh.Index()
    hoh.encode_images_async(rgb, n, W, H, out, stride, st, ctx=ctx, index=ix, speed=speed)
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    sizes = [hoh.check_status(s[2 * i:2 * i + 2], "batch -s%d image %d" % (speed, i)) for i in range(n)]
    for i, sp in enumerate(specs):
        one, m, _ = hoh.encode_image(rgb[i * img:(i + 1) * img], W, H, ctx=ctx, speed=speed)
        torch.cuda.synchronize()
        assert sizes[i] == m and torch.equal(out[i * stride:i * stride + m], one[:m]), (W, H, speed, i, sp)
        if sp[0] == "natural":
            g = _golden(W, H, sp[1], speed)
            if g:
                assert (m, _sha(out[i * stride:i * stride + m])) == g, (W, H, speed, sp)
    ctx.close()
    return sizes


@pytest.mark.parametrize("speed", [1, 2, 3, 4])
def test_batch_speed_natural_768x512(hoh, speed):
    """three images of one batch: the golden natural image between two others"""
    _batch_vs_single(hoh, 768, 512, speed, [("natural", 5), ("natural", 4), ("synth", 7, 4)])


@pytest.mark.parametrize("speed", [2, 4])
def test_batch_speed_1024(hoh, speed):
    _batch_vs_single(hoh, 1024, 1024, speed, [("natural", 3), ("synth", 2, 1)])


_EIGHT_CHILD = r"""
import hashlib, json, sys
import torch
sys.path.insert(0, sys.argv[1])
import hoh_ans as hoh
W = H = 8192
n = 8
ctx = hoh.Context(0)
stride = hoh.lib().hoh_encode_bound(W, H)
one = hoh.natural_rgb_dev(W, H, 1, ctx=ctx)
rgb = one.repeat(n)
del one
out = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
st = torch.zeros(2 * n, dtype=torch.int64, device="cuda")
torch.cuda.synchronize()
hoh.encode_images_async(rgb, n, W, H, out, stride, st, ctx=ctx, speed=1)
torch.cuda.synchronize()
s = st.cpu().numpy()
res = []
for i in range(n):
    m = hoh.check_status(s[2 * i:2 * i + 2], "image %d" % i)
    res.append([m, hashlib.sha256(out[i * stride:i * stride + m].cpu().numpy().tobytes()).hexdigest()])
ctx.close()
print("RESULT " + json.dumps(res))
"""


@pytest.mark.parametrize("stack", [0, 8192])
def test_batch_speed_8192_eight_images(stack):
    """8 x the golden natural 8192^2 image at -s1 in a fresh process.  stack 0: the product library
    (stacks of up to 1024 tiles: one image each, one after another); 8192: the checking build
    with SPEED_STACK_TILES=8192, one stack of all eight -- 8192 tiles x 70 streams of 8 KB tables
    (4.7 GB), so the chains' 64-bit table addresses are what makes the files right"""
    import subprocess
    import sys
    pkg = os.path.join(os.path.dirname(HERE), "hoh-ans_amd")
    env = dict(os.environ, HOH_QUIET="1")
    if stack:
        env.update(HOH_LIB=os.path.join(pkg, "lib", "libhohgpu_check.so"), HOH_SPEED_STACK_TILES=str(stack))
    p = subprocess.run([sys.executable, "-c", _EIGHT_CHILD, pkg], env=env, capture_output=True, text=True, timeout=200)
    assert p.returncode == 0, p.stderr[-3000:]
    res = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")][-1][7:])
    want = list(_golden(8192, 8192, 1, 1))
    assert all(r == want for r in res), res


def test_batch_speed_shards(hoh):
    """hoh_encode_tiles_images_async at -s3: 2 shards x a batch of 2, each blob the single-shard
    call's, the assembled file the reference's (golden natural 1024^2 seed 3 as image 1)"""
    import numpy as np
    import torch
    from hoh_ans import dist as hd
    W = H = 1024
    speed = 3
    ctx = hoh.Context(0)
    L = hoh.lib()
    specs = [("synth", 9, 2), ("natural", 3)]
    n = len(specs)
    full = _images(hoh, ctx, W, H, specs)
    img = W * H * 3
    blobs = [[] for _ in specs]
    sizes = [[] for _ in specs]
    for r in range(2):
        t0, nt, y0, y1 = hd.shard(W, H, r, 2)
        band = W * (y1 - y0) * 3
        rgb = torch.cat([full[i * img + y0 * W * 3:i * img + y1 * W * 3] for i in range(n)])
        stride = L.hoh_encode_bound(W, y1 - y0)
        out = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
        ts = torch.zeros(n * nt, dtype=torch.int32, device="cuda")
        st = torch.zeros(2 * n, dtype=torch.int64, device="cuda")
        hoh.encode_tiles_images_async(rgb, n, W, H, t0, nt, out, stride, ts, st, ctx=ctx, speed=speed)
        torch.cuda.synchronize()
        s = st.cpu().numpy()
        tsh = ts.cpu().numpy().astype(np.uint32).reshape(n, nt)
        for i in range(n):
            size = hoh.check_status(s[2 * i:2 * i + 2], "shard %d image %d" % (r, i))
            o1 = torch.zeros(stride, dtype=torch.uint8, device="cuda")
            t1 = torch.zeros(nt, dtype=torch.int32, device="cuda")
            s1 = torch.zeros(2, dtype=torch.int64, device="cuda")
            hoh.encode_tiles_async(rgb[i * band:(i + 1) * band], W, H, t0, nt, o1, t1, s1, ctx=ctx, row0=y0,
                                   speed=speed)
            torch.cuda.synchronize()
            assert hoh.check_status(s1.cpu().numpy(), "single shard") == size
            assert torch.equal(o1[:size], out[i * stride:i * stride + size]), (r, i)
            assert torch.equal(t1, ts[i * nt:(i + 1) * nt]), (r, i)
            blobs[i].append(out[i * stride:i * stride + size].cpu().numpy().tobytes())
            sizes[i].append(tsh[i])
    f = hoh.file_prefix(W, H, np.concatenate(sizes[1])) + b"".join(blobs[1])
    assert (len(f), hashlib.sha256(f).hexdigest()) == _golden(W, H, 3, speed)
    ctx.close()
