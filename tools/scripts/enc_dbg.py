# Encoder kernel timing under HOH_ENC_DBG knobs (measurement only; knobs change the output).
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "hoh-ans_amd"))
import torch, hoh_ans
W = H = int(sys.argv[1])
ctx = hoh_ans.default_ctx()
d = hoh_ans.synth_rgb_dev(W, H, 1, 4)
out = torch.empty(hoh_ans.lib().hoh_encode_bound(W, H), dtype=torch.uint8, device="cuda")
for dbg in [0] + [int(a) for a in sys.argv[2:]]:
    os.environ["HOH_ENC_DBG"] = str(dbg)
    ctx.profiling(True)
    ctx.reset_stats()
    for it in range(4):
        try:
            hoh_ans.encode_image(d, W, H, out_dev=out)
        except hoh_ans.HohError:
            pass
    st = ctx.kernel_stats()
    print("dbg=%d " % dbg + " ".join("%s=%.3f" % (k, v[0] / v[1]) for k, v in st.items() if v[0] / v[1] > 0.05), flush=True)
