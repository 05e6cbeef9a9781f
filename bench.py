#!/usr/bin/env python3
"""hoh-ANS MI355X bench: MB/s encode+decode (bit-exact) of synthetic 8-bit RGB.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One step = one pass of the hot path over the workload, inputs resident in HBM:
  N = 1: choh -s0 of the 8192x8192 image (BASELINE.json configs[2]: 1024 tiles of 256x256,
         3072 tile-plane rANS streams) into HBM (hoh_encode_image_ix, which also records the
         decode side index), then dhoh of that file back into HBM (hoh_decode_image_ix).
  N > 1: weak scaling -- the image is 8192 x (8192*N) and rank r owns tile rows
         [32r, 32r+32) (8192^2 pixels per GPU, configs[3]'s sharding).  A step is: encode the
         shard's tiles (hoh_encode_tiles_ix), gather every shard to rank 0 over RCCL, where the
         .hoh is assembled (prefix + concatenation; byte-identical to a 1-GPU encode), and
         decode the shard (hoh_decode_tiles).
value = raw RGB bytes of all ranks x K / max-over-ranks(time of the K steps) / 1e6.
Images in flight (--inflight; default 20 at N = 1, 12 at N > 1): each GPU keeps D images in
flight, one library context,
HIP stream and hardware queue per slot (GPU_MAX_HW_QUEUES raised to D), steps dealt round-robin
to the slots.  At N = 1 one host thread enqueues every step through the enqueue-only calls
(hoh_encode_image_async / hoh_decode_image_async): no host round trip inside the timed region,
the per-step status words are checked afterwards (--threads: one host thread per slot with the
synchronous calls instead, which is what N > 1 does because the gather needs the tile sizes on
the host).  The serial rANS chain of one image (65,536 dependent steps per tile-plane) leaves
most CUs idle; the other images' kernels fill them.  detail.latency_ms_* is the per-image latency
under that load (HIP events on each slot's stream at N = 1); --inflight 1 measures one image at a
time.

Outside the timed region: the decoded image is compared with the input (lossless), and at
N = 1 the encoded file's sha256 with the golden of the compiled reference (tests/golden).

roofline: rans_enc_fast (the dominant kernel), average launch duration from HIP events
recorded on the encoder's stream around that launch during the timed steps; algorithmic bytes
per launch = 2 B read per symbol (its u16 residual) + the stream payload bytes written (DESIGN.md
"Measurement").  `traffic` is filled from profiles/r01_pmc.json when that PMC summary (made by
tools/scripts/pmc.sh for this same workload) is present.

cpu_baseline: rank 0, N = 1 only -- oracle/_ref/ref_bench, the reference's own encode_tile(-s0)
+ decode_entropy/unpredict_all compiled from its sources, one thread, on the first
--cpu-tiles tiles of the same image.  Falls back to the C restatement (oracle, kind "port") if
the reference harness was not built.
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "hoh-ans_amd"))

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md


def metric_name():
    try:
        with open(os.path.join(ROOT, "BASELINE.json")) as f:
            return json.load(f)["metric"]
    except Exception:
        return "MB/s encode+decode (bit-exact) on 8-bit RGB"


def golden_sha(W, H, seed, noise):
    try:
        with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
            g = json.load(f)
        for c in g.get("choh_s0", []):
            sp, out = c.get("spec", {}), c.get("out")
            if (sp.get("W"), sp.get("H"), sp.get("seed"), sp.get("noise")) == (W, H, seed, noise) \
                    and isinstance(out, dict):
                return out.get("sha256")
    except Exception:
        pass
    return None


def cpu_baseline(rgb_host, W, H, tiles):
    """Reference CPU hot path on a bounded sample (first `tiles` tiles); returns the JSON object."""
    import numpy as np
    xt = W // 256
    rows = min(H, -(-tiles // xt) * 256)
    tiles = min(tiles, xt * (rows // 256))
    sample = "first %d of %d tiles (%dx%d rows 0-%d) of the bench image" % (tiles, xt * (H // 256), W, rows, rows - 1)
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_bench")
    if os.path.exists(exe):
        with tempfile.NamedTemporaryFile(suffix=".rgb", dir="/tmp", delete=False) as f:
            f.write(rgb_host[:W * rows * 3].tobytes())
            path = f.name
        try:
            r = subprocess.run([exe, path, str(W), str(rows), str(tiles)], capture_output=True, text=True,
                               timeout=300, check=True)
            d = json.loads(r.stdout.strip().splitlines()[-1])
        finally:
            os.unlink(path)
        return {"value": round(d["raw_bytes"] / (d["t_enc"] + d["t_dec"]) / 1e6, 3), "unit": "MB/s",
                "cores": 1, "kind": "reference",
                "sample": sample + "; encode_tile -s0 + decode_entropy/unpredict_all, 1 thread",
                "enc_MBps": d["enc_MBps"], "dec_MBps": d["dec_MBps"]}
    import oracle
    img = rgb_host[:W * rows * 3].reshape(rows, W, 3)
    t = time.perf_counter()
    data, _ = oracle.choh(img)
    te = time.perf_counter() - t
    t = time.perf_counter()
    back = oracle.dhoh(data)
    td = time.perf_counter() - t
    assert np.array_equal(back, img)
    raw = img.size
    return {"value": round(raw / (te + td) / 1e6, 3), "unit": "MB/s", "cores": 1, "kind": "port",
            "sample": "%dx%d rows of the bench image; oracle choh + dhoh, 1 thread" % (W, rows),
            "enc_MBps": round(raw / te / 1e6, 3), "dec_MBps": round(raw / td / 1e6, 3)}


def pmc_traffic(kernel, W, H):
    p = os.path.join(ROOT, "profiles", "r01_pmc.json")
    try:
        with open(p) as f:
            d = json.load(f)
        if d.get("W") == W and d.get("H") == H:
            return d["kernels"][kernel]["hbm_bytes_per_launch"]
    except Exception:
        pass
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=12)
    ap.add_argument("--size", type=int, default=8192, help="image width; height per GPU")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--noise", type=int, default=4)
    ap.add_argument("--cpu-tiles", type=int, default=512)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-index", action="store_true", help="decode without the side index (serial rANS)")
    ap.add_argument("--threads", action="store_true",
                    help="N=1: one host thread per lane with synchronous calls (the N>1 mode) instead of "
                         "enqueue-only calls from one thread")
    ap.add_argument("--inflight", type=int, default=0,
                    help="images in flight per GPU (each with its own context/stream); 1 = one at a time; "
                         "default 20 at N = 1 (enqueue-only lanes), 12 at N > 1 (a process group per lane)")
    args = ap.parse_args()
    if args.inflight <= 0:
        args.inflight = 20 if int(os.environ.get("WORLD_SIZE", "1")) == 1 else 12
    # one hardware queue per in-flight image (HIP reads this at runtime init; <= 32 allowed here)
    try:
        q = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    except ValueError:
        q = 4
    if q < args.inflight:
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, args.inflight))

    import numpy as np
    import torch
    import torch.distributed as dist
    import hoh_ans
    from hoh_ans import dist as hd

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE %d" % (args.gpus, world))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        dist.init_process_group("nccl", device_id=dev)

    L = hoh_ans.lib()
    W = args.size
    H = args.size * world
    if world == 1:
        t0, nt, y0, y1 = 0, 0, 0, H
    else:
        t0, nt, y0, y1 = hd.shard(W, H, rank, world)
    rows = y1 - y0
    D = max(1, args.inflight)
    rgb = hoh_ans.synth_rgb_dev(W, rows, args.seed, args.noise, row0=y0)
    torch.cuda.synchronize()

    class Lane:
        """One in-flight image slot: its own library context (HIP stream + workspaces), torch
        stream, buffers, side index and (N > 1) process group for the gather."""

        def __init__(self, k):
            self.ctx = hoh_ans.Context(local)
            self.stream = torch.cuda.Stream(device=dev)
            self.index = None if args.no_index else hoh_ans.Index()
            self.out = torch.empty(L.hoh_encode_bound(W, rows), dtype=torch.uint8, device=dev)
            self.dec = torch.empty(W * rows * 3, dtype=torch.uint8, device=dev)
            self.sizes = torch.empty(max(nt, 1), dtype=torch.int32, device=dev)
            self.group = dist.new_group(list(range(world))) if world > 1 else None
            self.gather = hd.FileGather(W, H, dev, group=self.group) if world > 1 else None
            self.t_enc = self.t_dec = 0.0
            self.n = 0

        def step(self):
            with torch.cuda.stream(self.stream):
                ta = time.perf_counter()
                if world == 1:
                    _, n, _ = hoh_ans.encode_image(rgb, W, H, out_dev=self.out, ctx=self.ctx, index=self.index)
                    tb = time.perf_counter()
                    hoh_ans.decode_image(self.out, n, out_dev=self.dec, ctx=self.ctx, index=self.index)
                else:
                    n = hoh_ans.encode_tiles(rgb, W, H, t0, nt, self.out, self.sizes, ctx=self.ctx,
                                             index=self.index, row0=y0)
                    ts = self.sizes[:nt].cpu().numpy().astype(np.uint32)
                    self.gather(self.out, n, ts)
                    tb = time.perf_counter()
                    hoh_ans.decode_tiles(self.out, n, W, H, t0, ts, self.dec, ctx=self.ctx, index=self.index,
                                         row0=y0)
                self.stream.synchronize()
                tc = time.perf_counter()
            self.n = n
            self.t_enc += tb - ta
            self.t_dec += tc - tb

        def run(self, count):
            for _ in range(count):
                self.step()

        def enqueue(self, status):
            """One step without any host wait: encode and decode enqueued on the lane's stream;
            their status words land in `status` (4 x int64, device); events bracket the two
            halves for the per-image latency."""
            with torch.cuda.stream(self.stream):
                e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                e0.record()
                hoh_ans.encode_image_async(rgb, W, H, self.out, status[0:2], ctx=self.ctx, index=self.index)
                e1.record()
                hoh_ans.decode_image_async(self.out, self.out.numel(), W, H, self.dec, status[2:4], ctx=self.ctx,
                                           index=self.index)
                e2.record()
            self.events.append((e0, e1, e2))

    lanes = [Lane(k) for k in range(D)]
    for ln in lanes:
        ln.events = []
    # N = 1: enqueue-only -- one host thread deals the steps round-robin to the lanes and never
    # waits inside the timed region (statuses are checked afterwards).  N > 1 needs the tile sizes
    # on the host for the gather, so each lane is a host thread running synchronous steps.
    use_async = world == 1 and not args.threads
    status = torch.zeros((max(args.steps, args.warmup, D), 4), dtype=torch.int64, device=dev)

    def run_all(total):
        if use_async:
            for i in range(total):
                lanes[i % D].enqueue(status[i])
            return
        # steps are dealt round-robin to the lanes; each lane runs its share back to back
        shares = [total // D + (1 if k < total % D else 0) for k in range(D)]
        if D == 1:
            lanes[0].run(shares[0])
            return
        th = [threading.Thread(target=ln.run, args=(c,)) for ln, c in zip(lanes, shares)]
        for x in th:
            x.start()
        for x in th:
            x.join()

    def check_status(total):
        st = status[:total].cpu().numpy()
        for i in range(total):
            hoh_ans.check_status(st[i, 0:2], "encode (step %d)" % i)
            hoh_ans.check_status(st[i, 2:4], "decode (step %d)" % i)
        return int(st[total - 1, 1])

    for ln in lanes:
        ln.ctx.profiling(True)
    run_all(max(args.warmup, D))
    torch.cuda.synchronize()
    if use_async:
        check_status(max(args.warmup, D))
    for ln in lanes:
        ln.ctx.reset_stats()
        ln.t_enc = ln.t_dec = 0.0
        ln.events = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t = time.perf_counter()
    run_all(args.steps)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    stats = {}
    for ln in lanes:
        for k, (tot, cnt) in ln.ctx.kernel_stats().items():
            a0, c0 = stats.get(k, (0.0, 0))
            stats[k] = (a0 + tot, c0 + cnt)
        ln.ctx.profiling(False)
    if use_async:
        n_async = check_status(args.steps)
        for ln in lanes:
            ln.n = n_async
            for e0, e1, e2 in ln.events:
                ln.t_enc += e0.elapsed_time(e1) * 1e-3
                ln.t_dec += e1.elapsed_time(e2) * 1e-3
    t_enc = sum(ln.t_enc for ln in lanes)
    t_dec = sum(ln.t_dec for ln in lanes)
    # per-kernel durations of one image alone (no other image in flight), for the record
    iso = {}
    if D > 1:
        ln = lanes[0]
        ln.ctx.profiling(True)
        ln.ctx.reset_stats()
        ln.run(3)
        iso = {k: v[0] / v[1] for k, v in ln.ctx.kernel_stats().items() if v[1]}
        ln.ctx.profiling(False)

    # checks outside the timed region
    lossless = all(bool(torch.equal(ln.dec, rgb)) for ln in lanes)
    n = lanes[0].n
    out = lanes[0].out
    index = lanes[0].index
    sha = None
    if world == 1:
        sha = hashlib.sha256(out[:n].cpu().numpy().tobytes()).hexdigest()
    if world > 1:
        tt = torch.tensor([el, 0.0 if lossless else 1.0, t_enc, t_dec], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el, bad, t_enc, t_dec = tt.tolist()
        lossless = bad == 0.0
        nn = torch.tensor([n], dtype=torch.int64, device=dev)
        dist.all_reduce(nn)
        comp_total = int(nn.item())
    else:
        comp_total = n
    raw_total = W * H * 3
    value = raw_total * args.steps / el / 1e6

    if rank == 0:
        K = args.steps
        kavg = {k: v[0] / v[1] for k, v in stats.items() if v[1]}
        dom = "rans_enc_fast"
        rows_raw = W * rows * 3
        n_rank = n
        alg = 2 * rows_raw + n_rank          # u16 residual in + payload out, one launch = one shard
        kms = kavg.get(dom)
        achieved = alg / (kms * 1e-3) / 1e9 if kms else None
        ratio = comp_total / raw_total
        roof = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2) if achieved else None,
                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5) if achieved else None,
                "traffic": pmc_traffic(dom, W, rows), "algorithmic_bytes": alg,
                "avg_launch_ms": round(kms, 4) if kms else None}
        pipeline_bytes = 2 * (1 + ratio) * raw_total
        golden = golden_sha(W, H, args.seed, args.noise) if world == 1 else None
        res = {
            "metric": metric_name(),
            "value": round(value, 2),
            "unit": "MB/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(el / K * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {
                "workload": ("%dx%d synthetic RGB (gradient + triangular noise k=%d, seed %d), 256x256 tiles, "
                             "choh -s0 encode + dhoh decode, %s, %d image(s) in flight"
                             % (W, H, args.noise, args.seed, "side index" if index else "serial decode", D)),
                "W": W, "H": H, "tiles": (W // 256) * (H // 256), "per_gpu": "%dx%d" % (W, rows),
                "parallelism": "tile rows sharded over %d GPU(s), RCCL gather to rank 0" % world
                               if world > 1 else "1 GPU",
            },
            "roofline": roof,
            "detail": {
                "inflight": D,
                "latency_ms_enc": round(t_enc / K * 1e3, 3),
                "latency_ms_dec": round(t_dec / K * 1e3, 3),
                "compressed_bytes": comp_total,
                "ratio": round(ratio, 5),
                "lossless": lossless,
                "file_sha256": sha,
                "bit_exact_vs_reference": (sha == golden) if golden else None,
                "pipeline_hbm_frac": round(pipeline_bytes * K / el / 1e9 / HBM_PEAK_GBS, 5),
                "kernel_avg_ms": {k: round(v, 4) for k, v in kavg.items()},
                "kernel_avg_ms_one_in_flight": {k: round(v, 4) for k, v in iso.items()},
            },
        }
        if world == 1 and not args.no_cpu_baseline:
            try:
                res["cpu_baseline"] = cpu_baseline(rgb.cpu().numpy(), W, H, args.cpu_tiles)
            except Exception as e:      # reported, never silently replaced
                res["cpu_baseline"] = {"value": None, "error": repr(e)[:200]}
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not lossless:
        sys.exit(3)


if __name__ == "__main__":
    main()
