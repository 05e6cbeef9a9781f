# Decode kernel timing on the bench image (measurement only; HOH_DEC_DBG knobs break output).
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "hoh-ans_amd"))
import torch, hoh_ans
W = H = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
ctx = hoh_ans.default_ctx()
d = hoh_ans.synth_rgb_dev(W, H, 1, 4)
out = torch.empty(hoh_ans.lib().hoh_encode_bound(W, H), dtype=torch.uint8, device="cuda")
ix = hoh_ans.Index()
_, n, _ = hoh_ans.encode_image(d, W, H, out_dev=out, index=ix)
dec = torch.empty_like(d)
for dbg in [0] + [int(a) for a in sys.argv[2:]]:
    os.environ["HOH_DEC_DBG"] = str(dbg)
    ctx.profiling(True)
    ctx.reset_stats()
    for it in range(5):
        try:
            hoh_ans.decode_image(out, n, out_dev=dec, index=ix)
        except hoh_ans.HohError as e:
            pass
    st = ctx.kernel_stats()
    print("dbg=%d " % dbg + " ".join("%s=%.3f" % (k, v[0] / v[1]) for k, v in st.items()), flush=True)
