"""GPU encode parity: libhohgpu's choh -s0 bytes against the oracle (and, for 8192^2, the golden
sha256 of the compiled reference's own output)."""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hoh():
    import hoh_ans
    return hoh_ans


def cases():
    from hoh_ans.synth import synth_rgb
    rs = np.random.RandomState(5)
    out = [("synth512", synth_rgb(512, 512, 1, 4)), ("synth1024", synth_rgb(1024, 1024, 2, 4)),
           ("synth768x520", synth_rgb(768, 520, 3, 2)), ("synth600x1000", synth_rgb(600, 1000, 4, 8)),
           ("gradient-lz", synth_rgb(256, 512, 5, 0)), ("synth1000x600", synth_rgb(1000, 600, 45, 8)),
           ("noisy40", synth_rgb(512, 512, 9, 40))]
    img = synth_rgb(512, 512, 7, 4)
    img[100:300, 50:400] = [10, 20, 30]
    out.append(("flat-block", img))
    img = synth_rgb(512, 512, 8, 4)
    for _ in range(300):                                   # repeats at random back distances
        y, x, L, b = rs.randint(0, 512), rs.randint(70, 400), rs.randint(4, 80), rs.randint(1, 65)
        img[y, x:x + L] = img[y, x - b:x - b + L]
    out.append(("repeats", img))
    out.append(("uniform", rs.randint(0, 256, (512, 768, 3)).astype(np.uint8)))   # stored planes
    out.append(("tiny2x2", np.array([[[255, 0, 0], [0, 255, 0]], [[255, 255, 0], [0, 0, 255]]], np.uint8)))
    out.append(("untiled300x200", synth_rgb(300, 200, 10, 4)))
    return out


@pytest.mark.parametrize("name,img", cases(), ids=[c[0] for c in cases()])
def test_choh_parity(hoh, orc, name, img):
    if name == "tiny2x2":
        # 4 colours: palette_encode competes (choh.cpp:298-308) -- not on the GPU path yet
        with pytest.raises(hoh.HohError) as e:
            hoh.choh(img)
        assert e.value.code == 6
        return
    data, printed = hoh.choh(img)
    ref, ref_printed = orc.choh(img)
    assert len(data) == len(ref)
    assert data == ref
    assert printed == ref_printed


def test_synth_device_matches_numpy(hoh):
    import torch
    from hoh_ans.synth import synth_rgb
    for W, H, seed, noise in ((512, 300, 3, 4), (1000, 77, 9, 0), (64, 64, 123456789, 40)):
        d = hoh.synth_rgb_dev(W, H, seed, noise)
        torch.cuda.synchronize()
        assert np.array_equal(d.cpu().numpy().reshape(H, W, 3), synth_rgb(W, H, seed, noise))


def test_choh_8192_golden(hoh, golden):
    import torch
    f = [f for f in golden["choh_s0"] if f["spec"]["W"] == 8192][0]
    sp = f["spec"]
    d = hoh.synth_rgb_dev(sp["W"], sp["H"], sp["seed"], sp["noise"])
    out, n, printed = hoh.encode_image(d, sp["W"], sp["H"])
    torch.cuda.synchronize()
    data = out[:n].cpu().numpy().tobytes()
    assert n == f["out"]["len"]
    assert hashlib.sha256(data).hexdigest() == f["out"]["sha256"]
    assert printed == f["printed"]
