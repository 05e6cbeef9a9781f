# Pipelined throughput of encode-only / decode-only / both with D images in flight (measurement
# only: HOH_ENC_DBG / HOH_DEC_DBG knobs may change or break the output, errors are ignored).
# usage: python pipe.py MODE D K [size]   MODE in enc, dec, both
import sys, os, time, threading
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "hoh-ans_amd"))
mode, D, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
W = H = int(sys.argv[4]) if len(sys.argv) > 4 else 8192
# one hardware queue per image in flight, as bench.py does (the GPU box exports 4); an explicit
# PIPE_QUEUES overrides for queue-count experiments
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("PIPE_QUEUES", str(min(32, max(4, D))))
import torch, hoh_ans
rgb = hoh_ans.synth_rgb_dev(W, H, 1, 4)
L = hoh_ans.lib()
encdbg = os.environ.pop("HOH_ENC_DBG", "0")
decdbg = os.environ.pop("HOH_DEC_DBG", "0")


class Lane:
    def __init__(self):
        self.ctx = hoh_ans.Context(0)
        self.s = torch.cuda.Stream()
        self.ix = hoh_ans.Index()
        self.out = torch.empty(L.hoh_encode_bound(W, H), dtype=torch.uint8, device="cuda")
        self.dec = torch.empty_like(rgb)
        with torch.cuda.stream(self.s):
            _, self.n, _ = hoh_ans.encode_image(rgb, W, H, out_dev=self.out, ctx=self.ctx, index=self.ix)
            self.s.synchronize()

    def run(self, c):
        with torch.cuda.stream(self.s):
            for _ in range(c):
                try:
                    if mode in ("enc", "both"):
                        _, self.n, _ = hoh_ans.encode_image(rgb, W, H, out_dev=self.out, ctx=self.ctx, index=self.ix)
                    if mode in ("dec", "both"):
                        hoh_ans.decode_image(self.out, self.n, out_dev=self.dec, ctx=self.ctx, index=self.ix)
                except hoh_ans.HohError:
                    pass
                self.s.synchronize()


lanes = [Lane() for _ in range(D)]
ASYNC = os.environ.get("PIPE_ASYNC", "1") == "1"
status = torch.zeros(4, dtype=torch.int64, device="cuda")


def go_async(total):
    # enqueue-only from one thread (statuses ignored: the knobs may break the output)
    for i in range(total):
        ln = lanes[i % D]
        with torch.cuda.stream(ln.s):
            if mode in ("enc", "both"):
                hoh_ans.encode_image_async(rgb, W, H, ln.out, status[0:2], ctx=ln.ctx, index=ln.ix)
            if mode in ("dec", "both"):
                hoh_ans.decode_image_async(ln.out, ln.out.numel(), W, H, ln.dec, status[2:4], ctx=ln.ctx, index=ln.ix)
os.environ["HOH_ENC_DBG"] = encdbg
os.environ["HOH_DEC_DBG"] = decdbg


def go(total):
    if ASYNC:
        return go_async(total)
    th = [threading.Thread(target=ln.run, args=(total // D,)) for ln in lanes]
    [x.start() for x in th]
    [x.join() for x in th]


go(2 * D)
torch.cuda.synchronize()
t = time.perf_counter()
go(K)
torch.cuda.synchronize()
el = time.perf_counter() - t
print("mode=%s D=%d enc=%s dec=%s ms/image=%.3f GB/s=%.1f" % (mode, D, encdbg, decdbg, el * 1e3 / (K // D * D),
      W * H * 3 * (K // D * D) / el / 1e9), flush=True)
