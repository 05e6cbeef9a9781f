"""Enqueue-only image path (hoh_encode_image_async / hoh_decode_image_async): the same bytes as
the synchronous calls and the oracle, lossless decode, several images in flight on several
streams with no host wait in between, and errors reported through the status words."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hoh():
    import hoh_ans
    return hoh_ans


def _status(torch):
    return torch.zeros(4, dtype=torch.int64, device="cuda")


@pytest.mark.parametrize("W,H,seed,noise", [(512, 512, 1, 4), (768, 520, 3, 2), (1000, 600, 45, 8), (256, 512, 5, 0)])
def test_async_matches_oracle(hoh, orc, W, H, seed, noise):
    import torch
    from hoh_ans.synth import synth_rgb
    img = synth_rgb(W, H, seed, noise)
    d = torch.from_numpy(img.reshape(-1).copy()).cuda()
    ctx = hoh.Context(0)
    ix = hoh.Index()
    out = torch.empty(hoh.lib().hoh_encode_bound(W, H), dtype=torch.uint8, device="cuda")
    dec = torch.empty(W * H * 3, dtype=torch.uint8, device="cuda")
    st = _status(torch)
    hoh.encode_image_async(d, W, H, out, st[0:2], ctx=ctx, index=ix)
    hoh.decode_image_async(out, out.numel(), W, H, dec, st[2:4], ctx=ctx, index=ix)
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    n = hoh.check_status(s[0:2], "encode")
    assert hoh.check_status(s[2:4], "decode") == W * H * 3
    assert out[:n].cpu().numpy().tobytes() == orc.choh(img)[0]
    assert np.array_equal(dec.cpu().numpy(), img.reshape(-1))
    ctx.close()


def test_async_many_in_flight(hoh):
    """4 lanes x 3 images each, all enqueued before any wait; different images per lane"""
    import torch
    W, H = 1024, 768
    imgs = [hoh.synth_rgb_dev(W, H, seed=10 + k, noise=2 + k % 3) for k in range(4)]
    ref = []
    for k in range(4):
        o, n, _ = hoh.encode_image(imgs[k], W, H)
        ref.append(o[:n].cpu().numpy().tobytes())
    lanes = []
    for k in range(4):
        lanes.append(dict(ctx=hoh.Context(0), s=torch.cuda.Stream(), ix=hoh.Index(),
                          out=torch.empty(hoh.lib().hoh_encode_bound(W, H), dtype=torch.uint8, device="cuda"),
                          dec=torch.empty(W * H * 3, dtype=torch.uint8, device="cuda")))
    st = torch.zeros((12, 4), dtype=torch.int64, device="cuda")
    for i in range(12):
        k = i % 4
        ln = lanes[k]
        with torch.cuda.stream(ln["s"]):
            hoh.encode_image_async(imgs[(k + i // 4) % 4], W, H, ln["out"], st[i, 0:2], ctx=ln["ctx"], index=ln["ix"])
            hoh.decode_image_async(ln["out"], ln["out"].numel(), W, H, ln["dec"], st[i, 2:4], ctx=ln["ctx"],
                                   index=ln["ix"])
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    for i in range(12):
        n = hoh.check_status(s[i, 0:2], "encode %d" % i)
        hoh.check_status(s[i, 2:4], "decode %d" % i)
        assert n == len(ref[(i % 4 + i // 4) % 4])
    for k, ln in enumerate(lanes):
        last = (k + 2) % 4                     # image of the lane's third step
        n = int(s[8 + k, 1])
        assert ln["out"][:n].cpu().numpy().tobytes() == ref[last]
        assert torch.equal(ln["dec"], imgs[last])
        ln["ctx"].close()


def test_async_errors_in_status(hoh):
    """wrong dimensions / a corrupt header come back as HOH_E_CORRUPT in the status word, and the
    stream stays usable"""
    import torch
    W, H = 512, 512
    rgb = hoh.synth_rgb_dev(W, H, seed=2, noise=4)
    ctx = hoh.Context(0)
    out = torch.empty(hoh.lib().hoh_encode_bound(W, H), dtype=torch.uint8, device="cuda")
    dec = torch.empty(1024 * 512 * 3, dtype=torch.uint8, device="cuda")
    st = torch.zeros((4, 4), dtype=torch.int64, device="cuda")
    hoh.encode_image_async(rgb, W, H, out, st[0, 0:2], ctx=ctx)
    hoh.decode_image_async(out, out.numel(), 1024, 512, dec, st[0, 2:4], ctx=ctx)      # wrong W
    bad = out.clone()
    bad[0] = 0
    hoh.decode_image_async(bad, bad.numel(), W, H, dec, st[1, 2:4], ctx=ctx)           # bad magic
    hoh.decode_image_async(out, out.numel(), W, H, dec, st[2, 2:4], ctx=ctx)           # fine again
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    hoh.check_status(s[0, 0:2], "encode")
    assert s[0, 2] == 7
    assert s[1, 2] == 7
    assert s[2, 2] == 0
    assert torch.equal(dec[:W * H * 3], rgb)
    # untiled images are rejected up front (the sync call writes their header-only file)
    small = hoh.synth_rgb_dev(64, 64, seed=1, noise=2)
    with pytest.raises(hoh.HohError):
        hoh.encode_image_async(small, 64, 64, out, st[3, 0:2], ctx=ctx)
    ctx.close()


@pytest.mark.parametrize("speed", [1, 3])
def test_async_speed_matches_sync(hoh, speed):
    """-s1 / -s3 encodes enqueued without host waits give the synchronous call's bytes"""
    import torch
    from hoh_ans.synth import synth_rgb
    W, H = 768, 520
    img = synth_rgb(W, H, 21, 3)
    d = torch.from_numpy(img.reshape(-1).copy()).cuda()
    want, n, _ = hoh.encode_image(d, W, H, speed=speed)
    want = want[:n].cpu().numpy().tobytes()
    ctx = hoh.Context(0)
    out = torch.empty(hoh.lib().hoh_encode_bound(W, H), dtype=torch.uint8, device="cuda")
    st = _status(torch)
    hoh.encode_image_async(d, W, H, out, st[0:2], ctx=ctx, speed=speed)
    torch.cuda.synchronize()
    m = hoh.check_status(st.cpu().numpy()[0:2], "encode")
    assert out[:m].cpu().numpy().tobytes() == want
    ctx.close()


def test_async_unsupported_in_status(hoh):
    """a file with an indexed (palette, mode 127) tile decodes to HOH_E_UNSUPPORTED through the
    status word, like the synchronous call's return code"""
    import torch
    rs = np.random.RandomState(11)
    pal = np.stack([rs.randint(0, 256, 64), np.full(64, 100), rs.randint(0, 256, 64)], 1).astype(np.uint8)
    img = pal[rs.randint(0, 64, (512, 512))]
    H, W, _ = img.shape
    d = torch.from_numpy(img.reshape(-1).copy()).cuda()
    ctx = hoh.Context(0)
    out = torch.empty(hoh.lib().hoh_encode_bound(W, H), dtype=torch.uint8, device="cuda")
    dec = torch.empty(W * H * 3, dtype=torch.uint8, device="cuda")
    st = _status(torch)
    hoh.encode_image_async(d, W, H, out, st[0:2], ctx=ctx)
    hoh.decode_image_async(out, out.numel(), W, H, dec, st[2:4], ctx=ctx)
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    hoh.check_status(s[0:2], "encode")
    assert s[2] == 6
    ctx.close()
