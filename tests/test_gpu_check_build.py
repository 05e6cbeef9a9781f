"""GPU, through the checking build (tests/checklib.py: the product sources with workspace read-back
and measurement knobs; k_lzsort, k_lzfp and the ladder kernels compile identically):

* Posting-list exactness in ONE run.  The round-4 -s2..-s4 race (k_lzsort's per-wave count reset,
  DESIGN.md section 2) lost a posting-list entry in a few encodes of a hundred, so repeating encodes
  only catches a recurrence by chance.  Here every tile's lists, fingerprints, run ends and ranks
  after an -s2 and an -s4 encode of the natural 8192^2 image are compared with an exact
  recomputation from k_lzfp's fingerprints and pixels (lz.hpp:35-53's candidate order: longest
  match, smallest back), and the file with the reference choh's SHA.
* The prob_bits ladder's pruning (k_prune_s) without pruning: with LADDER_PRUNE=0 every trial is
  encoded, every size-only trial's rANS word count must lie in the analytic bounds [wlo, whi] that
  the pruning trusts (k_tables), and the file must still equal the reference's (so the pruned
  product run, which the other tests pin to the same SHA, makes the same choices)."""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def golden_natural(W, H, seed, speed):
    with open(os.path.join(HERE, "golden", "golden_natural.json")) as f:
        for r in json.load(f)["files"]:
            sp = r["spec"]
            if (sp["W"], sp["H"], sp["seed"], sp["speed"]) == (W, H, seed, speed):
                return r["out"]["sha256"]
    return None


@pytest.mark.parametrize("speed", [2, 4])
def test_posting_lists_exact_natural_8192(speed):
    import torch
    from checklib import CheckLib, check_posting_lists
    W, cap = 8192, 65536
    ntiles = (W // 256) ** 2
    per = ntiles * cap
    c = CheckLib()
    try:
        rgb = c.natural(W, W, 1, torch)
        f = c.encode(rgb, W, W, speed, torch)
        want = golden_natural(W, W, 1, speed)
        assert want and hashlib.sha256(f).hexdigest() == want
        lzs = c.read(3, np.zeros(per * 5, np.uint32))
        fpb = c.read(4, np.zeros(per * 13 // 4, np.uint32))
    finally:
        c.close()
    bad, bad_s, bad_t, bad_r = check_posting_lists(fpb, lzs, ntiles, cap)
    assert not bad.any(), ("tiles with wrong lists: %d (keys %d, fingerprints %d, ranks %d), first %s"
                           % (bad.sum(), bad_s.sum(), bad_t.sum(), bad_r.sum(), np.flatnonzero(bad)[:8].tolist()))


_LADDER_CHILD = r"""
import hashlib, json, sys
import numpy as np
import torch
sys.path.insert(0, sys.argv[1])
from checklib import CheckLib, SM_RANS
W = int(sys.argv[2]); speeds = [int(s) for s in sys.argv[3].split(",")]
c = CheckLib()
rgb = c.natural(W, W, 1, torch)
ntiles = (W // 256) ** 2
res = {}
for sp in speeds:
    f = c.encode(rgb, W, W, sp, torch)
    st = c.streams(ntiles * 70)                    # SPT_S stream records per tile
    # k_finalize may turn a counted trial into a stored stream afterwards; its words stay counted
    trial = (st["sizeonly"] == 1) & (st["fast"] == 1) & (st["mode"] >= SM_RANS) & (st["err"] == 0) & (st["words"] > 0)
    bounded = trial & (st["whi"] >= st["wlo"]) & (st["wlo"] >= 2)
    out = bounded & ((st["words"] < st["wlo"]) | (st["words"] > st["whi"]))
    res[sp] = {"sha": hashlib.sha256(f).hexdigest(), "trials": int(trial.sum()), "bounded": int(bounded.sum()),
               "outside": int(out.sum()), "pruned": int((st["sizeonly"] == 2).sum()),
               "first_outside": np.flatnonzero(out)[:5].tolist()}
c.close()
print("RESULT " + json.dumps(res))
"""


def test_ladder_bounds_hold_unpruned():
    """natural 8192^2 at -s1..-s4 with LADDER_PRUNE=0 (a fresh process: knobs are read once)"""
    env = dict(os.environ, HOH_LADDER_PRUNE="0", HOH_QUIET="1")
    p = subprocess.run([sys.executable, "-c", _LADDER_CHILD, HERE, "8192", "1,2,3,4"], env=env,
                       capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    res = json.loads(line[7:])
    for sp, r in res.items():
        assert r["pruned"] == 0, (sp, r)                       # the knob really encoded every trial
        assert r["bounded"] > 1000, (sp, r)                    # the bounds were exercised
        assert r["outside"] == 0, (sp, r)
        assert r["sha"] == golden_natural(8192, 8192, 1, int(sp)), (sp, r)
