"""The host-buffer drop-ins (encode_entropy, decode_entropy, layer_encode/decode, the predictor and
unpredictor, subtract_green; entropy_encoding.hpp:8-15, entropy_decoding.hpp:134-140,
layer_encode.hpp:11-20, layer_decode.hpp:128-136, prediction.hpp:6-13, unprediction.hpp:6-16,
channel.hpp:73) reuse the context's grow-only device workspaces: after one call of a given shape,
repeating the calls makes no device allocation (the reference's TUs call them per plane)."""
import numpy as np
import pytest

import hoh_ans

pytestmark = pytest.mark.gpu


def _calls(ctx, rng):
    sym = np.minimum(rng.geometric(0.05, 70000) - 1, 255).astype(np.uint16)
    s = hoh_ans.encode_entropy(sym, 256, 15, ctx=ctx)
    d, _ = hoh_ans.decode_entropy(s, ctx=ctx)
    assert np.array_equal(np.asarray(d, np.uint16), sym)
    plane = (rng.integers(0, 40, (200, 256)) + np.arange(256)[None, :] // 4).astype(np.uint16) & 511
    res = hoh_ans.channelpredict_fastpath(plane, 9, ctx=ctx)
    back = hoh_ans.unpredict_fastpath(res, 256, 200, 9, ctx=ctx)
    assert np.array_equal(back, plane)
    for speed in (0, 1):
        lay = hoh_ans.layer_encode(plane, 9, ctx=ctx, speed=speed)
        if speed == 0:
            assert np.array_equal(hoh_ans.layer_decode(lay, 256, 200, 9, ctx=ctx), plane)
    tm = np.array([0x0010, 0x0001, 0x0002, 0x0020], np.uint16)
    pa = hoh_ans.predict_all(plane, 9, 2, 2, tm, ctx=ctx)
    assert np.array_equal(hoh_ans.unpredict_all(pa, 256, 200, 9, 2, 2, tm, ctx=ctx), plane)
    hoh_ans.predict_section(plane, 9, 2, 2, 1, 1, 0x0003, ctx=ctx)
    rgb = rng.integers(0, 256, (64, 64, 3)).astype(np.uint8)
    hoh_ans.subtract_green(rgb, ctx=ctx)
    small = (rng.integers(0, 8, (100, 120, 3)) + 60).astype(np.uint8)
    hoh_ans.choh(small, ctx=ctx)                       # untiled image: header only (Q13), scratch encode


def test_dropins_allocate_nothing_after_first_call():
    ctx = hoh_ans.Context(0)
    _calls(ctx, np.random.default_rng(1))
    before = hoh_ans.device_alloc_count()
    for k in range(3):
        _calls(ctx, np.random.default_rng(1))
    after = hoh_ans.device_alloc_count()
    ctx.close()
    assert after == before, "%d device allocations in repeated drop-in calls" % (after - before)
