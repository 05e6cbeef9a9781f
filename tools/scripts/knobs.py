# Per-kernel time (one image in flight) under HOH_ENC_DBG measurement knobs; errors ignored
# (the knobs may break the output).  usage: python knobs.py KERNEL DBG [DBG ...]
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "hoh-ans_amd"))
import torch, hoh_ans
kern = sys.argv[1]
W = H = 8192
rgb = hoh_ans.synth_rgb_dev(W, H, 1, 4)
ctx = hoh_ans.Context(0)
out = torch.empty(hoh_ans.lib().hoh_encode_bound(W, H), dtype=torch.uint8, device="cuda")
for dbg in sys.argv[2:]:
    os.environ["HOH_ENC_DBG"] = dbg
    ctx.profiling(True)
    for it in range(6):
        if it == 2:
            ctx.reset_stats()
        try:
            hoh_ans.encode_image(rgb, W, H, out_dev=out, ctx=ctx)
        except hoh_ans.HohError:
            pass
    st = ctx.kernel_stats()
    tot, cnt = st.get(kern, (0, 1))
    print("dbg=%s %s %.4f ms" % (dbg, kern, tot / max(cnt, 1)), flush=True)
