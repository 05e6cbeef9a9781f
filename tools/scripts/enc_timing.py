import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "hoh-ans_amd"))
import torch, hoh_ans
W = H = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
ctx = hoh_ans.default_ctx()
d = hoh_ans.synth_rgb_dev(W, H, 1, 4)
out = torch.empty(hoh_ans.lib().hoh_encode_bound(W, H), dtype=torch.uint8, device="cuda")
for it in range(3):
    torch.cuda.synchronize(); t = time.time()
    _, n, _ = hoh_ans.encode_image(d, W, H, out_dev=out)
    torch.cuda.synchronize(); dt = time.time() - t
    print("encode %dx%d: %.3f ms  %d bytes  %.1f MB/s" % (W, H, dt * 1e3, n, W * H * 3 / dt / 1e6))
ctx.profiling(True)
hoh_ans.encode_image(d, W, H, out_dev=out)
for name, ms in ctx.kernel_ms():
    print("  %-16s %8.3f ms" % (name, ms))
