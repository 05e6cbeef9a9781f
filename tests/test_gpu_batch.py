"""GPU: the batched enqueue-only image path (hoh_encode_images_async / hoh_decode_images_async).

A batch runs choh.cpp:464-500's tile loop over n images in each launch.  (The calls below pass
torch's default stream, i.e. NULL: the library then runs on the context's own stream, so every
buffer torch fills is synchronised before a call.)  Its files must be the
bytes of the single-image calls (and so of the reference choh: tests/golden/golden_bench.json
holds the reference's SHA of every bench seed at 8192^2), every image must decode losslessly with
and without the batch's side index, and per-image statuses must isolate per-image failures."""
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


def _batch(hoh, ctx, W, H, seeds, noise=4):
    import torch
    img = W * H * 3
    rgb = torch.empty(len(seeds) * img, dtype=torch.uint8, device="cuda")
    for i, sd in enumerate(seeds):
        rgb[i * img:(i + 1) * img] = hoh.synth_rgb_dev(W, H, sd, noise, ctx=ctx)
    torch.cuda.synchronize()
    return rgb


def _sha(t):
    return hashlib.sha256(t.cpu().numpy().tobytes()).hexdigest()


@pytest.mark.parametrize("W,H,n", [(1024, 1024, 3), (768, 512, 5), (1280, 768, 2), (1000, 600, 3), (1024, 1024, 1)])
def test_batch_equals_single_and_roundtrips(hoh, W, H, n):
    """(1000, 600) does not stack (tile rows of 300): the call runs the images one by one"""
    import torch
    ctx = hoh.Context(0)
    L = hoh.lib()
    stride = L.hoh_encode_bound(W, H)
    img = W * H * 3
    rgb = _batch(hoh, ctx, W, H, list(range(11, 11 + n)))
    out = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    st = torch.zeros(2 * n, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    stack = W >= 256 and H % 256 == 0
    idx = hoh.Index() if (stack or n == 1) else None
    hoh.encode_images_async(rgb, n, W, H, out, stride, st, ctx=ctx, index=idx)
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    for i in range(n):
        size = hoh.check_status(s[2 * i:2 * i + 2], "batch encode %d" % i)
        one, m, _ = hoh.encode_image(rgb[i * img:(i + 1) * img], W, H, ctx=ctx)
        torch.cuda.synchronize()
        assert size == m and torch.equal(out[i * stride:i * stride + m], one[:m]), (W, H, i)
    for index in ((idx, None) if idx is not None else (None,)):
        dec = torch.zeros(n * img, dtype=torch.uint8, device="cuda")
        ds = torch.zeros(2 * n, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        hoh.decode_images_async(out, n, stride, W, H, dec, ds, ctx=ctx, index=index)
        torch.cuda.synchronize()
        d = ds.cpu().numpy()
        for i in range(n):
            assert hoh.check_status(d[2 * i:2 * i + 2], "batch decode %d" % i) == img
        assert torch.equal(dec, rgb), ("index" if index is not None else "no index")
    ctx.close()


def test_batch_8192_vs_reference_goldens(hoh):
    """four bench seeds at 8192^2 in one batch: every file's SHA equals the reference choh's, and
    the batch decodes losslessly with and without the side index"""
    import torch
    g = json.load(open(os.path.join(HERE, "golden", "golden_bench.json")))
    want = {r["spec"]["seed"]: (r["out"]["len"], r["out"]["sha256"]) for r in g["files"]
            if (r["spec"]["W"], r["spec"]["H"], r["spec"]["noise"], r["spec"]["speed"]) == (8192, 8192, 4, 0)}
    seeds = [1, 2, 3, 4]
    ctx = hoh.Context(0)
    W = H = 8192
    stride = hoh.lib().hoh_encode_bound(W, H)
    rgb = _batch(hoh, ctx, W, H, seeds)
    out = torch.zeros(len(seeds) * stride, dtype=torch.uint8, device="cuda")
    st = torch.zeros(2 * len(seeds), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    idx = hoh.Index()
    hoh.encode_images_async(rgb, len(seeds), W, H, out, stride, st, ctx=ctx, index=idx)
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    for i, sd in enumerate(seeds):
        size = hoh.check_status(s[2 * i:2 * i + 2], "encode seed %d" % sd)
        assert (size, _sha(out[i * stride:i * stride + size])) == want[sd], sd
    dec = torch.zeros_like(rgb)
    ds = torch.zeros_like(st)
    torch.cuda.synchronize()
    hoh.decode_images_async(out, len(seeds), stride, W, H, dec, ds, ctx=ctx, index=idx)
    torch.cuda.synchronize()
    assert all(int(x) == 0 for x in ds.cpu().numpy()[0::2])
    assert torch.equal(dec, rgb)
    # the files alone (no side index): 12,288 plane chains, more than one round of k_drans_multi,
    # so the adaptive choice takes k_drans_lanes (k_decode.hip, the one-round rule)
    dec.zero_()
    ds.zero_()
    torch.cuda.synchronize()
    hoh.decode_images_async(out, len(seeds), stride, W, H, dec, ds, ctx=ctx, index=None)
    torch.cuda.synchronize()
    assert all(int(x) == 0 for x in ds.cpu().numpy()[0::2])
    assert torch.equal(dec, rgb)
    ctx.close()


def test_batch_index_layout_checked(hoh):
    """a batch's side index only serves the same batch layout; per-image HOH_E_CAP isolation"""
    import torch
    ctx = hoh.Context(0)
    W, H, n = 1024, 512, 3
    stride = hoh.lib().hoh_encode_bound(W, H)
    rgb = _batch(hoh, ctx, W, H, [3, 4, 5])
    out = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    st = torch.zeros(2 * n, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    idx = hoh.Index()
    hoh.encode_images_async(rgb, n, W, H, out, stride, st, ctx=ctx, index=idx)
    torch.cuda.synchronize()
    dec = torch.zeros(n * W * H * 3, dtype=torch.uint8, device="cuda")
    ds = torch.zeros(2 * n, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    with pytest.raises(hoh.HohError):           # index of 3 files at `stride`, decoded as 2
        hoh.decode_images_async(out, 2, stride, W, H, dec, ds, ctx=ctx, index=idx)
    with pytest.raises(hoh.HohError):           # single-image decode with a batch index
        hoh.decode_image(out, stride, ctx=ctx, index=idx)
    # image 1 made incompressible noise that cannot fit a stride sized for image 0's file: only
    # its slot reports HOH_E_CAP, the others' files are exact
    sizes = [hoh.check_status(x, "enc") for x in st.cpu().numpy().reshape(-1, 2)]
    small = max(sizes[0], sizes[2]) + 64
    rgb2 = rgb.clone()
    img = W * H * 3
    rgb2[img:2 * img] = hoh.synth_rgb_dev(W, H, 9, 60, ctx=ctx)
    out2 = torch.zeros(n * small, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    hoh.encode_images_async(rgb2, n, W, H, out2, small, st, ctx=ctx)
    torch.cuda.synchronize()
    codes = st.cpu().numpy().reshape(-1, 2)
    assert codes[1][0] == 2 and codes[0][0] == 0 and codes[2][0] == 0, codes
    assert torch.equal(out2[:sizes[0]], out[:sizes[0]])
    assert torch.equal(out2[2 * small:2 * small + sizes[2]], out[2 * stride:2 * stride + sizes[2]])
    ctx.close()


@pytest.mark.parametrize("n", [1, 2])
def test_batch_untiled_shape_unsupported(hoh, n):
    """untiled shapes (header-only files) are refused by the batched calls for any n,
    as by the single-image async calls (include/hoh_ans.h); the synchronous call encodes them"""
    import torch
    W, H = 320, 200
    ctx = hoh.Context(0)
    rgb = torch.zeros(n * W * H * 3, dtype=torch.uint8, device="cuda")
    stride = hoh.lib().hoh_encode_bound(W, H)
    out = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
    st = torch.zeros(2 * n, dtype=torch.int64, device="cuda")
    with pytest.raises(hoh.HohError) as e:
        hoh.encode_images_async(rgb, n, W, H, out, stride, st, ctx=ctx)
    assert e.value.code == 6
    with pytest.raises(hoh.HohError) as e:
        hoh.decode_images_async(out, n, stride, W, H, rgb, st, ctx=ctx)
    assert e.value.code == 6
    f, m, _ = hoh.encode_image(rgb[:W * H * 3], W, H, ctx=ctx)
    assert m == 10                                 # the header only (choh.cpp:508-520): 6 + 2 varints
    ctx.close()


def test_batch_truncated_file_reads_corrupt(hoh):
    """A file cut short by the batch stride must read as corrupt: the decoder bounds file i's parse
    by [i*stride, (i+1)*stride) and never runs on into file i+1's bytes."""
    import torch
    W, H = 1024, 512
    ctx = hoh.Context(0)
    img = W * H * 3
    rgb = torch.empty(2 * img, dtype=torch.uint8, device="cuda")
    rgb[:img] = hoh.synth_rgb_dev(W, H, 3, 8, ctx=ctx)      # the larger file
    rgb[img:] = hoh.synth_rgb_dev(W, H, 4, 2, ctx=ctx)
    stride = hoh.lib().hoh_encode_bound(W, H)
    out = torch.zeros(2 * stride, dtype=torch.uint8, device="cuda")
    st = torch.zeros(4, dtype=torch.int64, device="cuda")
    hoh.encode_images_async(rgb, 2, W, H, out, stride, st, ctx=ctx)
    s0, s1 = [hoh.check_status(x, "enc") for x in st.cpu().numpy().reshape(2, 2)]
    assert s0 > s1 + 64
    for cut in (s0 - 1, s0 - 40, (s0 + s1) // 2):
        tight = max(cut, s1)
        buf = torch.zeros(2 * tight, dtype=torch.uint8, device="cuda")
        buf[:tight] = out[:tight]                          # file 0 truncated to `tight` bytes
        buf[tight:tight + s1] = out[stride:stride + s1]    # file 1 right behind it
        dec = torch.zeros(2 * img, dtype=torch.uint8, device="cuda")
        ds = torch.full((4,), -1, dtype=torch.int64, device="cuda")
        hoh.decode_images_async(buf, 2, tight, W, H, dec, ds, ctx=ctx)
        codes = ds.cpu().numpy().reshape(2, 2)[:, 0]
        assert codes[0] == 7, (cut, codes)
    # the same files at a stride that holds both decode
    dec = torch.zeros(2 * img, dtype=torch.uint8, device="cuda")
    ds = torch.full((4,), -1, dtype=torch.int64, device="cuda")
    hoh.decode_images_async(out, 2, stride, W, H, dec, ds, ctx=ctx)
    assert all(int(c) == 0 for c in ds.cpu().numpy()[0::2]) and torch.equal(dec, rgb)
    ctx.close()
