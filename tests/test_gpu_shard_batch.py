"""GPU: batched shards (hoh_encode_tiles_images_async / hoh_decode_tiles_images_async) -- the
calls bench.py's N > 1 path runs on every rank: the same band of tile rows (choh.cpp:454-506's
tiling and tile table) of n images per call.

Every blob must equal the single-shard call's (hoh_encode_tiles_async) byte for byte, with the same
tile sizes; the ranks' blobs behind hoh_file_prefix must be the reference choh's file (8192^2 bench
seeds: tests/golden/golden_bench.json); every band must decode losslessly with the batch's side
index and without; shapes whose bands do not stack (H not a multiple of 256) run shard after
shard with the same bytes.  Also pins the Python mirror's stream fences on torch's default stream
(include/hoh_ans.h: a NULL stream is the context's own)."""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
from hoh_ans import synth

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def hoh():
    import hoh_ans
    return hoh_ans


def _bands(hoh, ctx, W, H, y0, y1, seeds, noise=4):
    import torch
    band = W * (y1 - y0) * 3
    rgb = torch.empty(len(seeds) * band, dtype=torch.uint8, device="cuda")
    for i, sd in enumerate(seeds):
        rgb[i * band:(i + 1) * band] = hoh.synth_rgb_dev(W, y1 - y0, sd, noise, ctx=ctx, row0=y0)
    return rgb


def _run(hoh, W, H, world, seeds, use_index):
    """every rank's batched blobs -> (files per seed, every band lossless)"""
    import torch
    from hoh_ans import dist as hd
    ctx = hoh.Context(0)
    L = hoh.lib()
    n = len(seeds)
    blobs = [[] for _ in seeds]
    sizes = [[] for _ in seeds]
    for r in range(world):
        t0, nt, y0, y1 = hd.shard(W, H, r, world)
        band = W * (y1 - y0) * 3
        stride = L.hoh_encode_bound(W, y1 - y0)
        rgb = _bands(hoh, ctx, W, H, y0, y1, seeds)
        out = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
        ts = torch.zeros(n * nt, dtype=torch.int32, device="cuda")
        st = torch.zeros(2 * n, dtype=torch.int64, device="cuda")
        ix = hoh.Index() if use_index else None
        hoh.encode_tiles_images_async(rgb, n, W, H, t0, nt, out, stride, ts, st, ctx=ctx, index=ix)
        s = st.cpu().numpy()
        tsh = ts.cpu().numpy().astype(np.uint32).reshape(n, nt)
        for i in range(n):
            size = hoh.check_status(s[2 * i:2 * i + 2], "shard %d image %d" % (r, i))
            assert int(tsh[i].sum()) == size
            # the single-shard call on the same band: same blob, same tile sizes
            o1 = torch.zeros(stride, dtype=torch.uint8, device="cuda")
            t1 = torch.zeros(nt, dtype=torch.int32, device="cuda")
            s1 = torch.zeros(2, dtype=torch.int64, device="cuda")
            hoh.encode_tiles_async(rgb[i * band:(i + 1) * band], W, H, t0, nt, o1, t1, s1, ctx=ctx, row0=y0)
            assert hoh.check_status(s1.cpu().numpy(), "single shard") == size
            assert torch.equal(o1[:size], out[i * stride:i * stride + size]), (r, i)
            assert torch.equal(t1, ts[i * nt:(i + 1) * nt]), (r, i)
            blobs[i].append(out[i * stride:i * stride + size].cpu().numpy().tobytes())
            sizes[i].append(tsh[i])
        for index in ((ix, None) if ix is not None else (None,)):
            dec = torch.zeros_like(rgb)
            ds = torch.zeros(2 * n, dtype=torch.int64, device="cuda")
            hoh.decode_tiles_images_async(out, n, stride, W, H, t0, nt, ts, dec, ds, ctx=ctx, index=index)
            d = ds.cpu().numpy()
            for i in range(n):
                assert hoh.check_status(d[2 * i:2 * i + 2], "decode shard %d image %d" % (r, i)) == band
            assert torch.equal(dec, rgb), (r, "index" if index is not None else "no index")
    ctx.close()
    files = [hoh.file_prefix(W, H, np.concatenate(sizes[i])) + b"".join(blobs[i]) for i in range(n)]
    return files


def test_batched_shards_8192_vs_reference_goldens(hoh):
    """4 ranks x a batch of 3 bench seeds at 8192^2: assembled files == the reference choh's"""
    g = json.load(open(os.path.join(HERE, "golden", "golden_bench.json")))
    want = {r["spec"]["seed"]: (r["out"]["len"], r["out"]["sha256"]) for r in g["files"]
            if (r["spec"]["W"], r["spec"]["H"], r["spec"]["noise"], r["spec"]["speed"]) == (8192, 8192, 4, 0)}
    seeds = [5, 6, 7]
    files = _run(hoh, 8192, 8192, 4, seeds, True)
    for sd, f in zip(seeds, files):
        assert (len(f), hashlib.sha256(f).hexdigest()) == want[sd], sd


@pytest.mark.parametrize("W,H,world,n,use_index", [(768, 1024, 2, 3, True), (1024, 768, 3, 2, False),
                                                   (1000, 1300, 3, 2, False), (512, 512, 1, 4, True)])
def test_batched_shards_small_vs_oracle(hoh, W, H, world, n, use_index):
    """(1000, 1300): tile rows of 325 -- the bands do not stack and run one after another"""
    seeds = list(range(31, 31 + n))
    if H % 256 and use_index:
        use_index = False
    files = _run(hoh, W, H, world, seeds, use_index)
    for sd, f in zip(seeds, files):
        assert f == oracle.choh(synth.synth_rgb(W, H, sd, 4))[0], sd


def test_batched_shards_arguments(hoh):
    import torch
    W, H = 768, 1024
    L = hoh.lib()
    ctx = hoh.Context(0)
    out = torch.zeros(2 * L.hoh_encode_bound(W, H), dtype=torch.uint8, device="cuda")
    ts = torch.zeros(64, dtype=torch.int32, device="cuda")
    st = torch.zeros(4, dtype=torch.int64, device="cuda")
    rgb = torch.zeros(2 * W * H * 3, dtype=torch.uint8, device="cuda")
    with pytest.raises(hoh.HohError):          # not whole tile rows (x_tiles = 3)
        hoh.encode_tiles_images_async(rgb, 2, W, H, 1, 3, out, L.hoh_encode_bound(W, H), ts, st, ctx=ctx)
    with pytest.raises(hoh.HohError) as e:     # untiled image: no tiles to shard (Q13)
        hoh.encode_tiles_images_async(rgb, 2, 320, 200, 0, 1, out, 4096, ts, st, ctx=ctx)
    assert e.value.code == 6
    # an index recorded for a batch of 2 does not serve a batch of 1
    stride = L.hoh_encode_bound(W, 512)
    ix = hoh.Index()
    rgb2 = _bands(hoh, ctx, W, H, 0, 512, [1, 2])
    hoh.encode_tiles_images_async(rgb2, 2, W, H, 0, 6, out, stride, ts, st, ctx=ctx, index=ix)
    hoh.check_status(st.cpu().numpy()[:2], "enc")
    dec = torch.zeros_like(rgb2)
    with pytest.raises(hoh.HohError):
        hoh.decode_tiles_images_async(out, 1, stride, W, H, 0, 6, ts, dec, st, ctx=ctx, index=ix)
    ctx.close()


def test_default_stream_fences(hoh):
    """Library calls on torch's default stream (handle 0: the context's own stream) are ordered
    against torch's work on it without host waits: a buffer torch zero-fills just before the call
    is filled by the call, and a torch op issued right after the call sees its output."""
    import torch
    W = H = 8192
    g = json.load(open(os.path.join(HERE, "golden", "golden_bench.json")))
    want = {r["spec"]["seed"]: r["out"]["sha256"] for r in g["files"]
            if (r["spec"]["W"], r["spec"]["H"], r["spec"]["noise"], r["spec"]["speed"]) == (8192, 8192, 4, 0)}
    ctx = hoh.Context(0)
    stride = hoh.lib().hoh_encode_bound(W, H)
    img = W * H * 3
    rgb = torch.empty(2 * img, dtype=torch.uint8, device="cuda")
    for i, sd in enumerate((1, 2)):
        rgb[i * img:(i + 1) * img] = hoh.synth_rgb_dev(W, H, sd, 4, ctx=ctx)
    assert torch.cuda.current_stream().cuda_stream == 0
    for rep in range(3):
        out = torch.full((2 * stride,), 0xAB, dtype=torch.uint8, device="cuda")   # queued on the default stream
        st = torch.full((4,), -1, dtype=torch.int64, device="cuda")
        hoh.encode_images_async(rgb, 2, W, H, out, stride, st, ctx=ctx)
        got = out.clone()                                                        # torch op right behind the call
        sizes = st.clone()
        dec = torch.zeros_like(rgb)
        ds = torch.full((4,), -1, dtype=torch.int64, device="cuda")
        hoh.decode_images_async(got, 2, stride, W, H, dec, ds, ctx=ctx)
        same = torch.equal(dec, rgb)                                             # reads the decode's output
        s = sizes.cpu().numpy()
        for i, sd in enumerate((1, 2)):
            n = hoh.check_status(s[2 * i:2 * i + 2], "encode %d" % i)
            assert hashlib.sha256(got[i * stride:i * stride + n].cpu().numpy().tobytes()).hexdigest() == want[sd]
        assert all(int(x) == 0 for x in ds.cpu().numpy()[0::2]) and same, rep
    ctx.close()


def test_weak_scaling_image_golden(hoh):
    """bench.py's N = 2 weak-scaling image (8192 x 16384, seed 1) as 2 batched shards of 2 images
    (seeds 1, 2): the assembled files equal the reference choh's (golden_bench.json, made by
    make_golden_bench.py --height 16384)"""
    g = json.load(open(os.path.join(HERE, "golden", "golden_bench.json")))
    want = {r["spec"]["seed"]: (r["out"]["len"], r["out"]["sha256"]) for r in g["files"]
            if (r["spec"]["W"], r["spec"]["H"], r["spec"]["noise"], r["spec"]["speed"]) == (8192, 16384, 4, 0)}
    files = _run(hoh, 8192, 16384, 2, [1, 2], False)
    for sd, f in zip((1, 2), files):
        assert (len(f), hashlib.sha256(f).hexdigest()) == want[sd], sd
