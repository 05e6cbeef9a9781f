"""Sharded (multi-GPU) entry points on one GPU: encode_tiles / decode_tiles per band of tile
rows, prefix + concatenation == the single-call choh -s0 file (choh.cpp:464-527), and each
shard decodes losslessly from its own blob, with and without the side index."""
import numpy as np
import pytest

import oracle
from hoh_ans import synth

pytestmark = pytest.mark.gpu


def _shards(W, H, world, seed, use_index, check_oracle):
    import torch
    import hoh_ans
    from hoh_ans import dist as hd
    ctx = hoh_ans.default_ctx()
    L = hoh_ans.lib()
    blobs, sizes = [], []
    for r in range(world):
        t0, nt, y0, y1 = hd.shard(W, H, r, world)
        rows = y1 - y0
        rgb = hoh_ans.synth_rgb_dev(W, rows, seed, 4, ctx=ctx, row0=y0)
        want_rows = synth.synth_rgb(W, H, seed, 4)[y0:y1] if check_oracle else None
        if want_rows is not None:
            assert np.array_equal(rgb.cpu().numpy().reshape(rows, W, 3), want_rows)
        out = torch.empty(L.hoh_encode_bound(W, rows), dtype=torch.uint8, device="cuda")
        sz = torch.empty(nt, dtype=torch.int32, device="cuda")
        ix = hoh_ans.Index() if use_index else None
        n = hoh_ans.encode_tiles(rgb, W, H, t0, nt, out, sz, ctx=ctx, index=ix, row0=y0)
        ts = sz.cpu().numpy().astype(np.uint32)
        assert int(ts.sum()) == n
        dec = torch.zeros(W * rows * 3, dtype=torch.uint8, device="cuda")
        hoh_ans.decode_tiles(out, n, W, H, t0, ts, dec, ctx=ctx, index=ix, row0=y0)
        torch.cuda.synchronize()
        assert torch.equal(dec, rgb), "shard %d not lossless" % r
        blobs.append(out[:n].cpu().numpy().tobytes())
        sizes.append(ts)
    return hoh_ans.file_prefix(W, H, np.concatenate(sizes)) + b"".join(blobs)


@pytest.mark.parametrize("W,H,world,use_index", [(768, 1024, 2, True), (768, 1024, 4, False),
                                                 (1000, 1300, 3, True)])
def test_shards_small_vs_oracle(W, H, world, use_index):
    f = _shards(W, H, world, 11, use_index, True)
    want, _ = oracle.choh(synth.synth_rgb(W, H, 11, 4))
    assert f == want


def test_shards_8192_golden(golden):
    import hashlib
    f = _shards(8192, 8192, 4, 1, True, False)
    g = [c for c in golden["choh_s0"] if c["spec"]["W"] == 8192][0]["out"]
    assert len(f) == g["len"] and hashlib.sha256(f).hexdigest() == g["sha256"]


def test_synth_rows_match_numpy():
    import hoh_ans
    W, H = 640, 300
    full = synth.synth_rgb(W, H, 9, 3)
    for y0, y1 in [(0, 300), (17, 200), (299, 300)]:
        d = hoh_ans.synth_rgb_dev(W, y1 - y0, 9, 3, row0=y0).cpu().numpy().reshape(y1 - y0, W, 3)
        assert np.array_equal(d, full[y0:y1])


@pytest.mark.parametrize("speed", [1, 3])
def test_shards_speed_assemble_to_file(speed):
    """config 5 on N GPUs: -s>=1 tiles sharded by bands of tile rows, prefix + concatenation is
    the single-call file (and the oracle's)"""
    import torch
    import hoh_ans
    from hoh_ans import dist as hd
    W, H, world, seed = 1024, 768, 3, 5
    img = synth.synth_rgb(W, H, seed, 4)
    L = hoh_ans.lib()
    blobs, sizes = [], []
    for r in range(world):
        t0, nt, y0, y1 = hd.shard(W, H, r, world)
        rgb = torch.from_numpy(img[y0:y1].reshape(-1).copy()).cuda()
        out = torch.empty(L.hoh_encode_bound(W, y1 - y0), dtype=torch.uint8, device="cuda")
        sz = torch.empty(nt, dtype=torch.int32, device="cuda")
        n = hoh_ans.encode_tiles(rgb, W, H, t0, nt, out, sz, row0=y0, speed=speed)
        ts = sz.cpu().numpy().astype(np.uint32)
        assert int(ts.sum()) == n
        blobs.append(out[:n].cpu().numpy().tobytes())
        sizes.append(ts)
    f = hoh_ans.file_prefix(W, H, np.concatenate(sizes)) + b"".join(blobs)
    assert f == hoh_ans.choh(img, speed=speed)[0]
    assert f == oracle.choh(img, speed)[0]


def test_16384_golden_single_and_sharded():
    """config 4: 16384^2 -s0, one call and as 4 shards (bands of tile rows) + prefix, against the
    reference choh's own file (tests/golden/golden_speed.json)"""
    import hashlib
    import json
    import os
    import torch
    import hoh_ans
    from hoh_ans import dist as hd
    g = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_speed.json")))
    recs = [f for f in g["files"] if f["spec"]["W"] == 16384 and f["spec"]["speed"] == 0]
    if not recs:
        pytest.skip("no 16384^2 golden")
    sp = recs[0]["spec"]
    W = H = 16384
    rgb = hoh_ans.synth_rgb_dev(W, H, sp["seed"], sp["noise"])
    out, n, printed = hoh_ans.encode_image(rgb, W, H)
    torch.cuda.synchronize()
    assert n == recs[0]["out"]["len"] and printed == recs[0]["printed"]
    assert hashlib.sha256(out[:n].cpu().numpy().tobytes()).hexdigest() == recs[0]["out"]["sha256"]
    del out
    L = hoh_ans.lib()
    h = hashlib.sha256()
    blobs, sizes = [], []
    for r in range(4):
        t0, nt, y0, y1 = hd.shard(W, H, r, 4)
        o = torch.empty(L.hoh_encode_bound(W, y1 - y0), dtype=torch.uint8, device="cuda")
        sz = torch.empty(nt, dtype=torch.int32, device="cuda")
        nb = hoh_ans.encode_tiles(rgb[y0 * W * 3:y1 * W * 3], W, H, t0, nt, o, sz, row0=y0)
        blobs.append(o[:nb].cpu().numpy().tobytes())
        sizes.append(sz.cpu().numpy().astype(np.uint32))
        del o
    h.update(hoh_ans.file_prefix(W, H, np.concatenate(sizes)))
    for b in blobs:
        h.update(b)
    assert h.hexdigest() == recs[0]["out"]["sha256"]
