#!/usr/bin/env python3
"""hoh-ANS MI355X bench: MB/s encode+decode (bit-exact) of synthetic 8-bit RGB.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--strong]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One step = one pass of the hot path over one batch of the workload, inputs resident in HBM:
  N = 1: choh -s0 of a batch of B = --batch (default 8) 8192x8192 images (BASELINE.json
         configs[2]: 1024 tiles of 256x256 each, 3072 tile-plane rANS streams) into HBM
         (hoh_encode_images_async: every kernel covers the B images' tiles; it also records the
         decode side index), then dhoh of the B files back into HBM (hoh_decode_images_async).
         --batch 1: one image per step through hoh_encode_image_async / hoh_decode_image_async.
  N > 1: weak scaling (default) -- the images are 8192 x (8192*N) and rank r owns a band of tile
         rows (8192^2 pixels per GPU per image).  --strong: configs[3], 16384x16384 images sharded
         over the N GPUs.  A step is: encode the shard of B images (hoh_encode_tiles_images_async:
         every kernel covers the B bands' tiles), gather each image's shards over RCCL to its root
         rank b % N (one all-gather of the B images' tile sizes, point-to-point blobs straight
         into the root's file behind its header + tile table: byte-identical to a 1-GPU encode;
         the roots spread the blobs over every xGMI link), and decode the
         B bands (hoh_decode_tiles_images_async, tile sizes read on the device).
value = raw RGB bytes of the step's images x K / max-over-ranks(time of the K steps) / 1e6.

Slots in flight (--inflight): at N = 1 D = 4 slots of B = 8 images (32 images in flight), each
slot with its own library context (HIP stream, workspaces) and its OWN input images (seeds 1..32,
so no image is a cache hit of another's), at HIP's default of 4 hardware queues (nothing set); the
N > 1 path runs the same 4 slots x 8 images per GPU; --batch 1 keeps 20 single-image slots on up to
20 queues.  One host thread per rank
deals the steps round-robin to the slots through enqueue-only calls; at N > 1 the gathers are
issued in step order on one process group (hoh_ans.dist.run_pipeline).  A set-up pass of one
step per slot (workspaces sized outside the timed region), then W warmup steps, then K timed.

Outside the timed region: every slot's decoded image is compared with its input (lossless), and
at N = 1 slot 0's file (seed 1) with the sha256 golden of the compiled reference (tests/golden).
Also at N = 1: detail.single_image_MBps (one image at a time, host-synchronous calls) and
detail.no_index_decode_MBps (dhoh of slot 0's file WITHOUT the side index: the serial rANS decode
any foreign .hoh gets, checked lossless).

roofline: the dominant kernel k_rans_fast01 (one launch = all 3 plane streams of every tile of one
image, and its LZ streams in otherwise idle blocks).  avg_launch_ms is its average duration with one image in flight (HIP events on the
encoder's stream, 5 launches; rocprofv3 agrees: profiles/), algorithmic bytes per launch = 2 B
read per symbol + the payload written.  The kernel is bounded by the latency of
its serial coder chain, not by HBM ("limiter"); roofline.pipeline_* is the whole pipeline's
algorithmic traffic 2(1+r)*raw per image against HBM peak.  traffic = HBM bytes per launch
measured in this run by rocprofv3 --pmc (FETCH_SIZE x2 per the gfx950 correction, + WRITE_SIZE;
two passes of `bench.py --pmc-probe`, started before this process touches the GPU), or null
when rocprofv3 is unavailable or the bench itself runs under a profiler.

cpu_baseline (rank 0, N = 1): the reference compiled from its own sources (oracle/_ref):
ref_bench = encode_tile(-s0) + decode_entropy/unpredict_all per tile on the same image, one
process per CPU of the box's quota (cgroup / worker-pool share, not nproc) over disjoint tile
ranges (value; cores and their source stated, nproc beside) and one thread on 512
tiles (single_thread), plus the reference's own choh binary (-s0, one thread, whole image;
its file's sha256 is compared with the golden).
"""
import argparse
import csv
import glob
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "hoh-ans_amd"))

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
DOM = "rans_enc_fast"   # stage name of the dominant kernel (k_rans_fast)
PMC_KERNELS = {"k_rans_fast": "rans_enc_fast", "k_rans_fast01": "rans_enc_fast", "k_front": "front", "k_front256": "front", "k_drans": "drans",
               "k_dunpred_fast": "dunpred_fast", "k_tables": "tables", "k_streambytes": "streambytes",
               "k_dunpred_lz": "dunpred_lz", "k_nuke": "nuke"}


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


def host_cores():
    """every CPU of this process's affinity mask"""
    try:
        n = len(os.sched_getaffinity(0))
    except Exception:
        n = os.cpu_count() or 1
    return max(1, n)


def cpu_quota():
    """(CPUs this process may actually use, where that number came from): the cgroup CPU quota
    (v2 cpu.max, v1 cfs_quota_us / cfs_period_us) when one is set, else the box's worker-pool
    setting (OMP_NUM_THREADS), else the affinity mask -- whichever is smallest.  A GPU box shows
    hundreds of CPUs in its affinity mask but grants a share of ~16-20."""
    aff = host_cores()
    cands = [(aff, "affinity mask")]
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            cands.append((max(1, int(int(q) / int(per))), "cgroup v2 cpu.max %s/%s" % (q, per)))
    except Exception:
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                cands.append((max(1, q // per), "cgroup v1 cfs_quota_us %d/%d" % (q, per)))
        except Exception:
            pass
    try:
        omp = int(os.environ.get("OMP_NUM_THREADS", "0"))
        if omp > 0:
            cands.append((omp, "OMP_NUM_THREADS=%d (the box's worker-pool share)" % omp))
    except ValueError:
        pass
    return min(cands)


# ------------------------------------------------------------------------------ PMC traffic

def under_profiler():
    return any(k.startswith(("ROCPROF", "ROCP_")) for k in os.environ) or "rocprof" in os.environ.get("LD_PRELOAD", "")


def pmc_probe(args):
    """Child of rocprofv3 --pmc: two encode+decode passes of slot 0's image (seed 1), then exit."""
    import torch
    import hoh_ans
    W, H = args.size, args.size
    ctx = hoh_ans.Context(0)
    rgb = hoh_ans.synth_rgb_dev(W, H, args.seed, args.noise, ctx=ctx)
    idx = hoh_ans.Index()
    out = torch.empty(hoh_ans.lib().hoh_encode_bound(W, H), dtype=torch.uint8, device="cuda")
    dec = torch.empty(W * H * 3, dtype=torch.uint8, device="cuda")
    for _ in range(2):
        _, n, _ = hoh_ans.encode_image(rgb, W, H, out_dev=out, ctx=ctx, index=idx)
        hoh_ans.decode_image(out, n, out_dev=dec, ctx=ctx, index=idx)
    torch.cuda.synchronize()
    assert torch.equal(dec, rgb)
    print(json.dumps({"probe": "ok", "n": n}))


def pmc_passes(passes, probe_argv, keep_last=None):
    """Run `bench.py <probe_argv>` under one rocprofv3 --pmc pass per entry of `passes` (each a
    tuple of counters that fits one pass), each under timeout -s KILL.  Returns ({kernel base name:
    {"launches": n, "ns": summed dispatch durations, counter: summed value}}, error or None).
    keep_last: keep only each kernel's last `keep_last` fraction of dispatches (the probe's final
    encode, past first-call set-up)."""
    exe = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(exe):
        return None, "rocprofv3 not found"
    res = {}
    tmp = tempfile.mkdtemp(prefix="hohpmc", dir="/tmp")
    try:
        for i, ctrs in enumerate(passes):
            d = os.path.join(tmp, "p%d" % i)
            cmd = ["timeout", "-s", "KILL", "150", exe, "--pmc", *ctrs, "--output-format", "csv", "-d", d, "-o", "p",
                   "--", sys.executable, os.path.abspath(__file__), *probe_argv]
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=180)
            files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
            if r.returncode != 0 or not files:
                return None, "rocprofv3 --pmc %s failed (rc %d): %s" % (" ".join(ctrs), r.returncode, (r.stderr or "")[-200:])
            per = {}     # kernel -> {dispatch: [ns, {ctr: value}]}
            for row in csv.DictReader(open(files[0])):
                if row.get("Counter_Name") not in ctrs:
                    continue
                k = row["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].strip()
                dd = per.setdefault(k, {}).setdefault(int(row["Dispatch_Id"]),
                                                       [int(row["End_Timestamp"]) - int(row["Start_Timestamp"]), {}])
                dd[1][row["Counter_Name"]] = dd[1].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
            for k, disp in per.items():
                ids = sorted(disp)
                if keep_last:
                    ids = ids[len(ids) - max(1, int(round(len(ids) * keep_last))):]
                e = res.setdefault(k, {})
                if "launches" not in e:
                    e["launches"] = len(ids)
                    e["ns"] = sum(disp[j][0] for j in ids)
                for c in ctrs:
                    e[c] = sum(disp[j][1].get(c, 0.0) for j in ids)
                e.setdefault("n_" + str(i), len(ids))
    except Exception as e:      # reported, never invented
        return None, "pmc: %r" % (e,)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return res, None


def pmc_traffic_live(args):
    """HBM bytes per launch of each main kernel, from two rocprofv3 --pmc passes (FETCH_SIZE and
    WRITE_SIZE do not fit one pass) over `bench.py --pmc-probe`.  Returns (per-kernel dict, note)."""
    res, err = pmc_passes([("FETCH_SIZE",), ("WRITE_SIZE",)],
                          ["--pmc-probe", "--size", str(args.size), "--seed", str(args.seed), "--noise", str(args.noise)])
    if err:
        return None, err
    vals = {}
    for k, e in res.items():
        name = PMC_KERNELS.get(k)
        if name is None or "FETCH_SIZE" not in e or "WRITE_SIZE" not in e:
            continue
        v = vals.setdefault(name, {"FETCH_SIZE": 0.0, "WRITE_SIZE": 0.0, "n0": 0, "n1": 0})
        v["FETCH_SIZE"] += e["FETCH_SIZE"] * 1024.0    # KB
        v["WRITE_SIZE"] += e["WRITE_SIZE"] * 1024.0
        v["n0"] += e.get("n_0", 0)
        v["n1"] += e.get("n_1", 0)
    out = {}
    for name, v in vals.items():
        if v["n0"] and v["n1"]:
            f, w = v["FETCH_SIZE"] / v["n0"], v["WRITE_SIZE"] / v["n1"]
            out[name] = {"fetch_raw": round(f), "write": round(w), "hbm_bytes": round(2 * f + w)}
    return out, "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE (separate passes), bench.py --pmc-probe, " \
                "per launch; hbm_bytes = 2 x FETCH_SIZE (gfx950 correction) + WRITE_SIZE"


def pmc_probe_speed(args):
    """Child of rocprofv3 --pmc: configs[4]'s natural image encoded twice at choh -s<speed>."""
    import torch
    import hoh_ans
    W, H = args.size, args.size
    ctx = hoh_ans.Context(0)
    rgb = hoh_ans.natural_rgb_dev(W, H, args.seed, ctx=ctx)
    out = torch.empty(hoh_ans.lib().hoh_encode_bound(W, H), dtype=torch.uint8, device="cuda")
    for _ in range(2):
        _, n, _ = hoh_ans.encode_image(rgb, W, H, out_dev=out, ctx=ctx, speed=args.pmc_probe_speed)
    torch.cuda.synchronize()
    print(json.dumps({"probe": "ok", "n": n}))


PMC_SETUP_KERNELS = ("k_natural", "k_synth")   # the probe's input generation, not the encode
SPEED_PMC_TOP = 8        # kernels reported per speed, by summed duration
VALU_SIMDS = 1024        # 256 CUs x 4 SIMDs
VALU_CYCLES = 2          # measured: one wave64 VALU instruction issues per 2 cycles per SIMD
CLOCK_HZ = 2.4e9         # MI355X max engine clock (MI355X_MICROARCH.md)


def speed_roofline_live(args, speed):
    """Roofline fractions of the -s<speed> encode's kernels (k_lzscan,
    k_search_walk_multi, k_search ...), from three rocprofv3 --pmc passes over `bench.py
    --pmc-probe-speed`: FETCH_SIZE | WRITE_SIZE | SQ_INSTS_VALU + SQ_INSTS_LDS, the second encode's
    dispatches only.  Per kernel, per launch: HBM bytes (2 x FETCH_SIZE + WRITE_SIZE), duration
    (dispatch timestamps of the FETCH pass: the profiler serialises dispatches, so this is the
    kernel alone, not beside the other stream), hbm GB/s and its fraction of 8 TB/s, and the VALU
    issue fraction = VALU wave-instructions x 2 cycles / (duration x 1024 SIMDs x 2.4 GHz)."""
    res, err = pmc_passes([("FETCH_SIZE",), ("WRITE_SIZE",), ("SQ_INSTS_VALU", "SQ_INSTS_LDS")],
                          ["--pmc-probe-speed", str(speed), "--size", str(args.size), "--seed", str(args.seed)],
                          keep_last=0.5)
    if err:
        return {"error": err}
    rows = []
    for k, e in res.items():
        if not e.get("launches") or "FETCH_SIZE" not in e or "WRITE_SIZE" not in e or k in PMC_SETUP_KERNELS:
            continue
        n = e["launches"]
        ns = e["ns"] / n
        hb = (2 * e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024.0 / n
        valu = e.get("SQ_INSTS_VALU", 0.0) / n
        r = {"launches_per_encode": n, "ms": round(ns / 1e6, 4), "hbm_bytes": round(hb),
             "hbm_GBps": round(hb / ns, 1) if ns else None,
             "hbm_frac": round(hb / ns / HBM_PEAK_GBS, 4) if ns else None,
             "valu_insts": round(valu), "lds_insts": round(e.get("SQ_INSTS_LDS", 0.0) / n),
             "valu_frac": round(valu * VALU_CYCLES / (ns * 1e-9 * VALU_SIMDS * CLOCK_HZ), 4) if ns else None}
        rows.append((e["ns"], k, r))
    rows.sort(reverse=True)
    out = {k: r for _, k, r in rows[:SPEED_PMC_TOP]}
    out["source"] = ("rocprofv3 --pmc, 3 passes over bench.py --pmc-probe-speed %d (natural %dx%d, second "
                     "encode); durations are each kernel alone (the profiler serialises dispatches); "
                     "valu_frac = VALU x %d cycles / (ms x %d SIMDs x %.1f GHz)"
                     % (speed, args.size, args.size, VALU_CYCLES, VALU_SIMDS, CLOCK_HZ / 1e9))
    return out


def cpu_baseline(rgb_host, W, H, args):
    """The reference's CPU hot path (oracle/_ref, compiled from its own sources) on the bench
    image: all host cores (one ref_bench process per core over disjoint tile ranges), one thread
    (first --cpu-tiles tiles), and the reference choh binary itself (one thread, whole image)."""
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_bench")
    if not os.path.exists(exe):
        return {"value": None, "error": "oracle/_ref/ref_bench not built (make -C oracle/ref)"}
    affinity = host_cores()
    quota, quota_src = cpu_quota()
    if args.cpu_procs > 0:
        quota, quota_src = args.cpu_procs, "--cpu-procs"
    xt, yt = W // 256, H // 256
    ntiles = xt * yt
    P = min(quota, ntiles)
    res = {}
    with tempfile.NamedTemporaryFile(suffix=".rgb", dir="/tmp", delete=False) as f:
        f.write(rgb_host.tobytes())
        path = f.name
    try:
        # all cores: one process per CPU of the quota, disjoint contiguous tile ranges covering
        # the whole image; each process clocks only encode_tile and the decode calls
        # (ref_bench.cpp), and the image's time is the slowest process's
        per = -(-ntiles // P)
        t = time.perf_counter()
        procs = [subprocess.Popen([exe, path, str(W), str(H), str(per), str(k * per)], stdout=subprocess.PIPE,
                                  text=True) for k in range(P) if k * per < ntiles]
        outs = [p.communicate(timeout=600)[0] for p in procs]
        wall = time.perf_counter() - t
        ds = [json.loads(o.strip().splitlines()[-1]) for o in outs]
        raw = sum(d["raw_bytes"] for d in ds)
        bad = sum(d["mismatch_excl_last_row"] for d in ds)
        work = max(d["t_enc"] + d["t_dec"] for d in ds)
        res.update({"value": round(raw / work / 1e6, 3), "unit": "MB/s", "cores": len(procs), "kind": "reference",
                    "cores_source": quota_src, "nproc": os.cpu_count(), "affinity_cpus": affinity,
                    "sample": "whole bench image (%d tiles), one ref_bench process per CPU of the quota (%d) on "
                              "disjoint tile ranges (%d tiles each); value = raw bytes of the tiles whose encode and "
                              "decode were both timed / the slowest process's encode_tile -s0 + "
                              "decode_entropy/unpredict_all time" % (ntiles, len(procs), per),
                    "tiles_skipped": sum(d.get("tiles_skipped", 0) for d in ds),
                    "wall_clock_MBps": round(raw / wall / 1e6, 3),
                    "wall_clock_note": "process start, band read and the LZ locate of ref_bench included",
                    "ref_decode_mismatch_excl_last_row": bad,
                    "ref_decode_note": "each tile decoded by the reference's decode_entropy + unpredict_all with its real "
                                       "LZ back-reference map (oracle/ref/ref_bench.cpp lz_backref, outside the clock); "
                                       "mismatch = decoded bytes that differ from the input, the last row excluded "
                                       "(the reference decodes it with its non-MED edge rule, SURVEY Q9)"})
        # one thread on a bounded sample
        nt1 = min(args.cpu_tiles, ntiles)
        r = subprocess.run([exe, path, str(W), str(H), str(nt1), "0"], capture_output=True, text=True, timeout=600,
                           check=True)
        d = json.loads(r.stdout.strip().splitlines()[-1])
        st = d["raw_bytes"] / (d["t_enc"] + d["t_dec"]) / 1e6
        res["single_thread"] = {"value": round(st, 3), "cores": 1,
                                "sample": "first %d of %d tiles" % (nt1, ntiles),
                                "enc_MBps": d["enc_MBps"], "dec_MBps": d["dec_MBps"]}
        res["all_cores_vs_single_x_cores"] = round(res["value"] / (st * len(procs)), 3)
        res["effective_cores"] = round(res["value"] / st, 1)
        # the reference's own choh binary, -s0, one thread, whole image (dhoh cannot run: SURVEY Q1)
        choh = os.path.join(ROOT, "oracle", "_ref", "choh")
        if os.path.exists(choh) and not args.no_choh_binary:
            outp = path + ".hoh"
            t = time.perf_counter()
            subprocess.run([choh, path, outp, str(W), str(H), "-s0"], capture_output=True, timeout=900, check=True)
            te = time.perf_counter() - t
            sha = hashlib.sha256(open(outp, "rb").read()).hexdigest()
            os.unlink(outp)
            g = golden_sha(W, H, args.seed, args.noise)
            res["choh_binary"] = {"encode_MBps": round(W * H * 3 / te / 1e6, 3), "cores": 1,
                                  "seconds": round(te, 3), "sha256": sha,
                                  "sha_matches_golden": (sha == g) if g else None}
    finally:
        os.unlink(path)
    return res


# ------------------------------------------------------------------------------ config 2

def config2_leg(args):
    """BASELINE configs[1]: one 1024x1024 plane (the G residuals of the synthetic image, MED
    fast path) as ONE rans64 stream of 1,048,576 symbols (range 256, prob_bits 15) -- a serial
    chain, so a latency config: GPU encode_entropy / decode_entropy ns per symbol (host buffers,
    one stream; the 2 MB of PCIe copies are included) beside the C restatement of the reference
    (oracle, one thread) on the same symbols; the GPU stream must equal the oracle's byte for byte
    and round-trip."""
    import numpy as np
    import hoh_ans
    from hoh_ans import synth
    import oracle
    img = synth.synth_rgb(1024, 1024, seed=args.seed, noise=args.noise)
    sym = hoh_ans.channelpredict_fastpath(img[:, :, 1].astype(np.uint16), 8).reshape(-1)
    n = sym.size

    def best(f, k=3):
        ts = []
        for _ in range(k):
            t = time.perf_counter()
            r = f()
            ts.append(time.perf_counter() - t)
        return r, min(ts)

    g_enc, t_ge = best(lambda: hoh_ans.encode_entropy(sym, 256, 15))
    (g_dec, _), t_gd = best(lambda: hoh_ans.decode_entropy(g_enc))
    c_enc, t_ce = best(lambda: oracle.encode_entropy(sym, 256, 15))
    (c_dec, _), t_cd = best(lambda: oracle.decode_entropy(c_enc))
    return {"symbols": n, "stream_bytes": len(g_enc),
            "gpu_encode_ns_per_symbol": round(t_ge / n * 1e9, 2), "gpu_decode_ns_per_symbol": round(t_gd / n * 1e9, 2),
            "cpu_port_encode_ns_per_symbol": round(t_ce / n * 1e9, 2),
            "cpu_port_decode_ns_per_symbol": round(t_cd / n * 1e9, 2),
            "bytes_equal_cpu": bytes(g_enc) == bytes(c_enc),
            "roundtrip": bool(np.array_equal(np.asarray(g_dec, np.uint16), sym)),
            "note": "one serial coder chain: ~140 GPU cycles per dependent step against ~11 on a CPU core; "
                    "the GPU's rate comes from thousands of streams (configs[2])"}


# ------------------------------------------------------------------------------ detail legs

def golden_natural_sha(W, H, seed, speed=0):
    try:
        with open(os.path.join(ROOT, "tests", "golden", "golden_natural.json")) as f:
            for r in json.load(f)["files"]:
                sp = r["spec"]
                if (sp["W"], sp["H"], sp["seed"], sp["speed"]) == (W, H, seed, speed):
                    return r["out"]["sha256"]
    except Exception:
        pass
    return None


class SlotIO:
    """The detail legs' calls on a slot: its B images per step through the batched calls
    (hoh_*_images_async) when B > 1, else the single-image calls; status row i holds {code, size}
    of every image's encode, then of every image's decode."""

    def __init__(self, hoh_ans, W, H, B, stride):
        self.h, self.W, self.H, self.B, self.stride = hoh_ans, W, H, B, stride

    def encode(self, s, inp, row, index=None, speed=0):
        if self.B > 1:
            self.h.encode_images_async(inp, self.B, self.W, self.H, s.out, self.stride, row[:2 * self.B], ctx=s.ctx,
                                       index=index, speed=speed)
        else:
            self.h.encode_image_async(inp, self.W, self.H, s.out, row[0:2], ctx=s.ctx, index=index, speed=speed)

    def decode(self, s, row, index=None):
        if self.B > 1:
            self.h.decode_images_async(s.out, self.B, self.stride, self.W, self.H, s.dec, row[2 * self.B:4 * self.B],
                                       ctx=s.ctx, index=index)
        else:
            self.h.decode_image_async(s.out, s.out.numel(), self.W, self.H, s.dec, row[2:4], ctx=s.ctx, index=index)

    def check(self, st, total, what, decode=True):
        for i in range(total):
            for b in range(self.B):
                self.h.check_status(st[i, 2 * b:2 * b + 2], "%s encode (step %d image %d)" % (what, i, b))
                if decode:
                    self.h.check_status(st[i, 2 * self.B + 2 * b:2 * self.B + 2 * b + 2],
                                        "%s decode (step %d image %d)" % (what, i, b))


def extra_legs(args, slots, W, H, D, B, stride, status, torch, hoh_ans, hd):
    """N = 1 detail legs on the bench's own slots (contexts, streams, buffers), D slots of B images
    in flight (the headline's calls), one set-up pass per slot, then --leg-steps timed steps,
    lossless-checked afterwards:
      no_index_pipeline: the same synthetic images, encoded without recording a side index and
        decoded from the file alone (what a foreign .hoh gets: every stream one serial chain);
      natural_s0_pipeline: configs[4]'s natural-statistic image (seed --seed, generated into every
        slot's own buffer: other seeds hold palette tiles, which the format cannot decode, SURVEY
        Q15), choh -s0 + dhoh with the side index; slot 0's file is compared with the reference
        choh's SHA."""
    out = {}
    K = max(1, args.leg_steps)
    io = SlotIO(hoh_ans, W, H, B, stride)
    img = W * H * 3

    def leg(inputs, use_index):
        idx = [hoh_ans.Index() if use_index else None for _ in range(D)]

        def enq(k, i):
            s = slots[k]
            with torch.cuda.stream(s.stream):
                io.encode(s, inputs[k], status[i], index=idx[k])
                io.decode(s, status[i], index=idx[k])

        def chk(total):
            io.check(status[:total].cpu().numpy(), total, "leg")

        hd.run_pipeline(D, D, enq, lambda k, i: None)
        torch.cuda.synchronize()
        chk(D)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for c in range(0, K, status.shape[0]):      # status rows are reused per chunk of steps
            hd.run_pipeline(D, min(status.shape[0], K - c), enq, lambda k, i: None)
            torch.cuda.synchronize()
            chk(min(status.shape[0], K - c))
        el = time.perf_counter() - t
        ok = all(bool(torch.equal(slots[k].dec, inputs[k])) for k in range(D))
        n0 = int(status[min(status.shape[0], K) - 1 - ((min(status.shape[0], K) - 1) % D), 1].item())
        return img * B * K / el / 1e6, ok, el / K * 1e3, n0

    try:
        v, ok, ms, _ = leg([s.rgb for s in slots], False)
        out["no_index_pipeline_MBps"] = round(v, 1)
        out["no_index_pipeline_ms_per_step"] = round(ms, 4)
        out["no_index_pipeline_lossless"] = ok
    except Exception as e:      # reported, never silently replaced
        out["no_index_pipeline_error"] = repr(e)[:300]
    nat = None
    try:
        one = hoh_ans.natural_rgb_dev(W, H, args.seed, ctx=slots[0].ctx)
        nat = [one.repeat(B) for _ in range(D)]
        del one
        torch.cuda.synchronize()
        v, ok, ms, n0 = leg(nat, True)
        sha = hashlib.sha256(slots[0].out[:n0].cpu().numpy().tobytes()).hexdigest()
        g = golden_natural_sha(W, H, args.seed)
        out["natural_s0_MBps"] = round(v, 1)
        out["natural_s0_ms_per_step"] = round(ms, 4)
        out["natural_s0_lossless"] = ok
        out["natural_s0_file_bytes"] = n0
        out["natural_s0_bit_exact_vs_reference"] = (sha == g) if g else None
        # one image at a time (latency): best of 3 synchronous encodes and decodes on slot 0
        s0, ix = slots[0], hoh_ans.Index()
        te, tdl = [], []
        for r in range(4):
            torch.cuda.synchronize()
            t = time.perf_counter()
            _, n1, _ = hoh_ans.encode_image(nat[0][:img], W, H, out_dev=s0.out0, ctx=s0.ctx, index=ix)
            torch.cuda.synchronize()
            te.append(time.perf_counter() - t)
            t = time.perf_counter()
            hoh_ans.decode_image(s0.out0, n1, out_dev=s0.dec0, ctx=s0.ctx, index=ix)
            torch.cuda.synchronize()
            tdl.append(time.perf_counter() - t)
        ms_e, ms_d = min(te[1:]) * 1e3, min(tdl[1:]) * 1e3
        out["natural_s0_single_enc_ms"] = round(ms_e, 3)
        out["natural_s0_single_dec_ms"] = round(ms_d, 3)
        out["natural_s0_single_MBps"] = round(W * H * 3 / (ms_e + ms_d) / 1e3, 1)
        out["natural_s0_single_lossless"] = bool(torch.equal(s0.dec0, nat[0][:img]))
    except Exception as e:
        out["natural_s0_error"] = repr(e)[:300]
        nat = None
    if nat is not None and args.speed_legs:
        out.update(speed_legs(args, slots, nat, W, H, D, B, stride, status, torch, hoh_ans, hd))
    del nat
    out["legs_note"] = ("%d slots x %d image(s) in flight, one set-up pass per slot, then %d timed steps each; inputs "
                        "resident in HBM" % (D, B, K))
    return out


def speed_legs(args, slots, nat, W, H, D, B, stride, status, torch, hoh_ans, hd):
    """BASELINE configs[4] at the search speeds: the natural-statistic image (seed --seed in every
    slot) encoded at choh -s1..-s4 (full predictor search, layer_encode.hpp:122-319, and the
    seek-distance LZ, lz.hpp:32-95 at 10..14), D slots of B images in flight (at -s>=1
    hoh_encode_images_async stacks up to 1024 tiles per job: one 8192^2 image, which fills the
    device alone -- stacks of two measured 3-6 % slower here), encode only (-s>=1
    layers are undecodable by construction), one set-up pass per slot, then
    --speed-leg-steps timed steps.  EVERY image's last file is SHA-compared with the reference
    choh's (golden_natural.json); one image at a time: the best of 3 synchronous encodes on slot 0."""
    out = {}
    K = max(1, args.speed_leg_steps)
    io = SlotIO(hoh_ans, W, H, B, stride)
    img = W * H * 3
    for speed in [int(x) for x in args.speed_legs.split(",") if x.strip()]:
        key = "natural_s%d" % speed
        try:
            def enq(k, i):
                s = slots[k]
                with torch.cuda.stream(s.stream):
                    io.encode(s, nat[k], status[i], speed=speed)

            def chk(total):
                st = status[:total].cpu().numpy()
                io.check(st, total, key, decode=False)
                return st

            hd.run_pipeline(D, D, enq, lambda k, i: None)
            torch.cuda.synchronize()
            chk(D)
            steps, el = 0, 0.0
            for c in range(0, K, status.shape[0]):
                n = min(status.shape[0], K - c)
                torch.cuda.synchronize()
                t = time.perf_counter()
                hd.run_pipeline(D, n, enq, lambda k, i: None)
                torch.cuda.synchronize()
                el += time.perf_counter() - t
                st = chk(n)
                steps = n
            g = golden_natural_sha(W, H, args.seed, speed)
            match, checked = 0, 0
            for k in range(min(D, steps)):
                row = k + ((steps - 1 - k) // D) * D
                for b in range(B):
                    n_k = int(st[row, 2 * b + 1])
                    checked += 1
                    o = slots[k].out[b * stride:b * stride + n_k]
                    match += g is not None and hashlib.sha256(o.cpu().numpy().tobytes()).hexdigest() == g
            te = []
            for r in range(4):
                torch.cuda.synchronize()
                t = time.perf_counter()
                _, n1, _ = hoh_ans.encode_image(nat[0][:img], W, H, out_dev=slots[0].out0, ctx=slots[0].ctx, speed=speed)
                torch.cuda.synchronize()
                te.append(time.perf_counter() - t)
            single_ok = g is not None and hashlib.sha256(slots[0].out0[:n1].cpu().numpy().tobytes()).hexdigest() == g
            out[key + "_MBps"] = round(img * B * K / el / 1e6, 1)
            out[key + "_ms_per_step"] = round(el / K * 1e3, 3)
            out[key + "_file_bytes"] = n1
            out[key + "_slot_files_bit_exact"] = "%d of %d" % (match + single_ok, checked + 1)
            out[key + "_bit_exact_vs_reference"] = (match == checked and single_ok) if g else None
            out[key + "_single_enc_ms"] = round(min(te[1:]) * 1e3, 3)
        except Exception as e:      # reported, never silently replaced
            out[key + "_error"] = repr(e)[:300]
    out["speed_legs_note"] = ("configs[4] natural 8192^2 image, choh -sN encode only (Q14: -s>=1 layers are "
                              "undecodable), %d slots x %d image(s) in flight, %d timed steps per speed; every "
                              "image's file SHA-checked against the reference choh's (golden_natural.json)"
                              % (D, B, K))
    return out


# ------------------------------------------------------------------------------ bench

class GpuShardOps:
    """Device side of hoh_ans.dist.run_sharded_leg for bench.py's N > 1 path: rank `rank` owns the
    tile-row band [t0, t0+nt) of every W x H image.  A slot holds the bands of B images; a step
    encodes them in one batched call (hoh_encode_tiles_images_async: every kernel covers the B
    bands' tiles, tile sizes and statuses stay on the device), copies the tile sizes to pinned host
    memory behind an event and, when the step finishes, all-gathers the B images' sizes once, sends
    the B blobs to their files' root ranks (image b's file on rank b % N, each blob straight into
    its place behind hoh_file_prefix: hoh_ans.dist.BatchGather) and
    decodes the B bands (hoh_decode_tiles_images_async, tile sizes read on the device) on the slot's
    stream.  The same D slots x B images schedule as the N = 1 line, at HIP's default queues."""

    def __init__(self, args, W, H, seed0, rank, world, dev, torch, hoh_ans, hd, nrows, B):
        self.args, self.W, self.H, self.seed0, self.B = args, W, H, seed0, B
        self.torch, self.hoh_ans, self.hd, self.dev = torch, hoh_ans, hd, dev
        self.device = dev
        self.t0, self.nt, self.y0, y1 = hd.shard(W, H, rank, world)
        self.rows = y1 - self.y0
        self.band = W * self.rows * 3
        self.L = hoh_ans.lib()
        self.stride = self.L.hoh_encode_bound(W, self.rows)
        self.status = torch.zeros((nrows, 4 * B), dtype=torch.int64, device=dev)

    def new_slot(self, k):
        torch, hoh_ans, B = self.torch, self.hoh_ans, self.B

        class Slot:
            pass
        s = Slot()
        s.seeds = [self.seed0 + k * B + b for b in range(B)]
        s.seed = s.seeds[0]
        s.ctx = hoh_ans.Context(self.dev.index)
        s.stream = torch.cuda.Stream(device=self.dev)
        s.rgb = torch.empty(B * self.band, dtype=torch.uint8, device=self.dev)
        for b, sd in enumerate(s.seeds):
            s.rgb[b * self.band:(b + 1) * self.band] = hoh_ans.synth_rgb_dev(self.W, self.rows, sd, self.args.noise,
                                                                           ctx=s.ctx, row0=self.y0)
        s.index = None if self.args.no_index else hoh_ans.Index()
        s.out = torch.empty(B * self.stride, dtype=torch.uint8, device=self.dev)
        s.dec = torch.empty(B * self.band, dtype=torch.uint8, device=self.dev)
        s.events = []
        s.sizes = torch.empty(B * self.nt, dtype=torch.int32, device=self.dev)
        s.sizes_host = torch.empty(B * self.nt, dtype=torch.int32).pin_memory()
        s.enc_done = torch.cuda.Event()
        s.gather = self.hd.BatchGather(self.W, self.H, B, self.dev)
        s.ctx.profiling(True)
        return s

    def enqueue(self, s, i):
        torch, B = self.torch, self.B
        with torch.cuda.stream(s.stream):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            self.hoh_ans.encode_tiles_images_async(s.rgb, B, self.W, self.H, self.t0, self.nt, s.out, self.stride,
                                                   s.sizes, self.status[i, 0:2 * B], ctx=s.ctx, index=s.index)
            e1.record()
            s.sizes_host.copy_(s.sizes, non_blocking=True)
            s.enc_done.record()
            s.events.append((e0, e1))

    def finish(self, s, i):
        import numpy as np
        torch, B = self.torch, self.B
        s.enc_done.synchronize()
        ts = s.sizes_host.numpy().astype(np.uint32).reshape(B, self.nt)
        with torch.cuda.stream(s.stream):
            res = s.gather(s.out, self.stride, ts, wait=False)
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            self.hoh_ans.decode_tiles_images_async(s.out, B, self.stride, self.W, self.H, self.t0, self.nt, s.sizes,
                                                   s.dec, self.status[i, 2 * B:4 * B], ctx=s.ctx, index=s.index)
            e2 = torch.cuda.Event(enable_timing=True)
            e2.record()
            s.events[-1] = s.events[-1] + (e1, e2)
            for q in res[2]:
                q.wait()              # RCCL: the slot's stream (not the host) waits before reusing the blobs

    def drain(self):
        self.torch.cuda.synchronize()

    def check(self, total):
        st = self.status[:total].cpu().numpy()
        B = self.B
        for i in range(total):
            for b in range(B):
                self.hoh_ans.check_status(st[i, 2 * b:2 * b + 2], "encode (step %d image %d)" % (i, b))
                self.hoh_ans.check_status(st[i, 2 * B + 2 * b:2 * B + 2 * b + 2], "decode (step %d image %d)" % (i, b))

    def reset(self, slots):
        for s in slots:
            s.ctx.reset_stats()
            s.events = []

    def lossless(self, s):
        return bool(self.torch.equal(s.dec, s.rgb))


def shard_one_in_flight(ops, s, torch, hoh_ans, n=5):
    """The dominant kernel's launch duration with ONE shard in flight on this rank (the N = 1
    line's one-in-flight measurement, on the N > 1 path): n host-synchronous shard encodes of
    slot s's first band (hoh_encode_tiles_async, B = 1) with the library's HIP-event stage timing
    on the call's stream; the bytes are checked against the batched blob of that band."""
    out = torch.empty(ops.stride, dtype=torch.uint8, device=ops.dev)
    sizes = torch.empty(ops.nt, dtype=torch.int32, device=ops.dev)
    st = torch.zeros(2, dtype=torch.int64, device=ops.dev)
    rgb0 = s.rgb[:ops.band]
    with torch.cuda.stream(s.stream):
        s.ctx.profiling(True)
        s.ctx.reset_stats()
        for _ in range(n):
            hoh_ans.encode_tiles_async(rgb0, ops.W, ops.H, ops.t0, ops.nt, out, sizes, st, ctx=s.ctx,
                                       row0=ops.y0)
            s.stream.synchronize()
        iso = {k: v[0] / v[1] for k, v in s.ctx.kernel_stats().items() if v[1]}
        s.ctx.profiling(False)
    size = hoh_ans.check_status(st.cpu().numpy(), "one-in-flight shard encode")
    same = bool(torch.equal(out[:size], s.out[:size])) and bool(torch.equal(sizes, s.sizes[:ops.nt]))
    return iso, same


def sharded_leg(args, W, H, D, B, K, warm, seed0, rank, world, dev, torch, hoh_ans, hd, one_in_flight=False):
    """One N > 1 leg (or its one-rank rehearsal, --sharded): returns a dict of its numbers; on
    rank 0 the SHA of slot 0's first image's gathered file (seed seed0) is reported, and every slot's
    images' files of their last step against the reference choh's SHAs where known (each file is
    assembled on its root rank, hoh_ans.dist.BatchGather, and hashed there)."""
    import numpy as np
    import torch.distributed as dist
    ops = GpuShardOps(args, W, H, seed0, rank, world, dev, torch, hoh_ans, hd, max(K, warm, D), B)
    slots, el, lossless = hd.run_sharded_leg(ops, D, K, warm)
    t_enc = sum(ev[0].elapsed_time(ev[1]) for s in slots for ev in s.events) * 1e-3
    t_dec = sum(ev[-2].elapsed_time(ev[-1]) for s in slots for ev in s.events) * 1e-3
    stats = {}
    for s in slots:
        for k, (tot, cnt) in s.ctx.kernel_stats().items():
            a0, c0 = stats.get(k, (0.0, 0))
            stats[k] = (a0 + tot, c0 + cnt)
        s.ctx.profiling(False)
    iso, iso_same = (None, None)
    if one_in_flight:
        iso, iso_same = shard_one_in_flight(ops, slots[0], torch, hoh_ans)
    tt = torch.tensor([t_enc, t_dec, iso.get(DOM, 0.0) if iso else 0.0], dtype=torch.float64, device=dev)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    t_enc, t_dec, iso_dom = tt.tolist()
    n_rank = int(slots[0].sizes_host.numpy().astype(np.int64)[:ops.nt].sum())
    nn = torch.tensor([n_rank], dtype=torch.int64, device=dev)
    dist.all_reduce(nn)
    # every slot's files of its last step (header + tile table + every rank's blob), hashed on the
    # rank that assembled each (image b of a slot on rank b % world), collected on every rank
    mine = {}
    for s in slots:
        g = s.gather
        for b in g.own:
            mine[s.seeds[b]] = hashlib.sha256(g.files[g.row(b), :g.totals[b]].cpu().numpy().tobytes()).hexdigest()
    allh = [None] * world
    dist.all_gather_object(allh, mine)
    shas = {k: v for d in allh for k, v in d.items()}
    sha = shas.get(seed0)
    res = {"el": el, "K": K, "D": D, "B": B, "lossless": lossless, "t_enc": t_enc, "t_dec": t_dec,
           "comp_total": int(nn.item()), "sha": sha, "shas": shas, "stats": stats, "rows": ops.rows,
           "iso": iso, "iso_dom_ms_max": iso_dom if iso else None, "iso_same_bytes": iso_same,
           "value": W * H * 3 * K * B / el / 1e6}
    del slots, ops
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return res


def golden_speed_sha(W, H, seed, noise, speed=0):
    try:
        with open(os.path.join(ROOT, "tests", "golden", "golden_speed.json")) as f:
            for r in json.load(f)["files"]:
                sp = r["spec"]
                if (sp["W"], sp["H"], sp["seed"], sp["noise"], sp["speed"]) == (W, H, seed, noise, speed):
                    return r["out"]["sha256"]
    except Exception:
        pass
    return None


def golden_bench_shas(W, H, noise):
    """{seed: sha256} of the reference choh -s0 file of every bench seed (golden_bench.json)"""
    try:
        with open(os.path.join(ROOT, "tests", "golden", "golden_bench.json")) as f:
            return {r["spec"]["seed"]: r["out"]["sha256"] for r in json.load(f)["files"]
                    if (r["spec"]["W"], r["spec"]["H"], r["spec"]["noise"], r["spec"]["speed"]) == (W, H, noise, 0)}
    except Exception:
        return {}


STRONG_SIDE, STRONG_SEED = 16384, 2     # configs[3]; seed 2 is the reference choh's golden file


HW_QUEUE_CAP = 20
DEFAULT_SLOTS, DEFAULT_BATCH = 4, 8       # N = 1: 4 streams x 8 images (r05 sweep)


def hw_queue_note():
    q = os.environ.get("GPU_MAX_HW_QUEUES")
    return q if q else "4 (HIP default, GPU_MAX_HW_QUEUES unset)"


def hw_queues_for(d):
    """Hardware queues for d images in flight: d up to HW_QUEUE_CAP, else the fewest images per
    queue that fit the cap, spread evenly (24 -> 12 queues of 2, 32 -> 16 of 2, 40 -> 20 of 2)."""
    if d <= HW_QUEUE_CAP:
        return max(1, d)
    per = -(-d // HW_QUEUE_CAP)
    return -(-d // per)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=12)
    ap.add_argument("--size", type=int, default=0,
                    help="weak: image width and rows per GPU (default 8192); --strong: the whole image side "
                         "(default 16384)")
    ap.add_argument("--strong", action="store_true", help="configs[3]: one size x size image sharded over N GPUs")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--noise", type=int, default=4)
    ap.add_argument("--inflight", type=int, default=0,
                    help="slots in flight per GPU (default: 4 at N = 1, each a batch of --batch images; 20 "
                         "single images per GPU on the N > 1 path)")
    ap.add_argument("--hw-queues", type=int, default=0,
                    help="GPU_MAX_HW_QUEUES for this process (default: hw_queues_for(--inflight), at most 20)")
    ap.add_argument("--strong-inflight", type=int, default=8, help="images in flight per GPU in the 16384^2 leg")
    ap.add_argument("--batch", type=int, default=0,
                    help="N = 1: images per slot and step (default %d) through the batched calls "
                         "(hoh_*_images_async); 1: the single-image calls" % DEFAULT_BATCH)
    ap.add_argument("--no-index", action="store_true", help="decode without the side index (serial rANS)")
    ap.add_argument("--cpu-tiles", type=int, default=512)
    ap.add_argument("--cpu-procs", type=int, default=0,
                    help="reference processes of the all-cores CPU baseline (default: the cgroup CPU quota)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-choh-binary", action="store_true")
    ap.add_argument("--no-config2", action="store_true", help="skip the 1M-symbol single-stream leg")
    ap.add_argument("--no-pmc", action="store_true", help="skip the live rocprofv3 --pmc traffic passes")
    ap.add_argument("--sharded", action="store_true",
                    help="N = 1: run the N > 1 code path (tile encode, RCCL gather on a 1-rank group, tile decode)")
    ap.add_argument("--no-strong-leg", action="store_true",
                    help="N > 1 / --sharded: skip the configs[3] leg (16384^2 sharded over the ranks)")
    ap.add_argument("--no-legs", action="store_true",
                    help="skip the detail legs (no-index pipeline, natural-statistic pipeline)")
    ap.add_argument("--leg-steps", type=int, default=40, help="timed steps of each detail leg")
    ap.add_argument("--speed-legs", default="1,2,3,4",
                    help="choh -sN speeds of the natural-image encode legs (configs[4]); empty: none")
    ap.add_argument("--speed-leg-steps", type=int, default=40, help="timed steps of each -sN leg")
    ap.add_argument("--batch-only", action="store_true",
                    help="N = 1: the timed batched leg alone (no one-in-flight / no-index / roofline detail)")
    ap.add_argument("--pmc-probe", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--pmc-probe-speed", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--pmc-speed", type=int, default=4,
                    help="the -sN encode whose kernels get live PMC roofline fractions (0: none)")
    args = ap.parse_args()
    if args.size <= 0:
        args.size = STRONG_SIDE if args.strong else 8192
    if args.pmc_probe:
        pmc_probe(args)
        return
    if args.pmc_probe_speed >= 0:
        pmc_probe_speed(args)
        return
    if args.batch <= 0:
        args.batch = DEFAULT_BATCH
    if args.inflight <= 0:
        args.inflight = 20 if args.batch == 1 else DEFAULT_SLOTS
    D = max(1, args.inflight)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE %d" % (args.gpus, world))
    sharded = world > 1 or args.sharded

    # live PMC traffic first, before this process initialises the GPU
    pmc, pmc_note, pmc_speed = None, "skipped", None
    if world == 1 and not args.no_pmc and not sharded:
        if under_profiler():
            pmc_note = "skipped: the bench itself runs under a profiler"
        else:
            pmc, pmc_note = pmc_traffic_live(args)
            if args.pmc_speed > 0 and not args.no_legs and not args.batch_only:
                try:
                    pmc_speed = speed_roofline_live(args, args.pmc_speed)
                except Exception as e:      # reported, never invented
                    pmc_speed = {"error": repr(e)[:300]}

    # hardware queues (HIP reads GPU_MAX_HW_QUEUES at runtime init).  The batched paths (N = 1 and
    # N > 1 alike) run at HIP's default (4 queues: nothing is set); the single-image path (--batch
    # 1) keeps one queue per in-flight image up to HW_QUEUE_CAP, past that shared evenly
    # (docs/EXPERIMENTS.md, "in-flight sweep": more than ~20 queues per process cost 15-30%)
    if args.hw_queues > 0:
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, args.hw_queues))
    elif args.batch == 1:
        os.environ["GPU_MAX_HW_QUEUES"] = str(hw_queues_for(D))

    import torch
    import hoh_ans
    from hoh_ans import dist as hd

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if sharded:
        sharded_main(args, D, args.batch, world, rank, dev, torch, hoh_ans, hd)
    elif args.batch > 1 and args.batch_only:
        batch_main(args, D, args.batch, dev, torch, hoh_ans, hd)
    else:
        single_main(args, D, dev, torch, hoh_ans, hd, pmc, pmc_note, pmc_speed)


def roofline_obj(kms, kavg, ratio, rows_raw, raw_total, K, el, pmc, B=1):
    """SURVEY 8(d)'s encode-side algorithmic bytes charged to one launch of the dominant kernel
    (one launch = one image's or shard's encode, as measured one image in flight): 3 B/px read +
    3r B/px written = (1 + r) raw; the design's own bytes (u16 residuals in + payload out) beside
    it as design_bytes.  The pipeline figure counts the B images of every step."""
    alg = int(round((1 + ratio) * rows_raw))
    design = 2 * rows_raw + int(round(ratio * rows_raw))
    achieved = alg / (kms * 1e-3) / 1e9 if kms else None
    pipeline_gbs = 2 * (1 + ratio) * raw_total * B * K / el / 1e9
    traffic = pmc.get(DOM, {}).get("hbm_bytes") if pmc else None
    # "bound" names what limits the kernel (its serial coder chain's latency, per "limiter"); the
    # roofline it is priced against is HBM ("peak_resource"): there is no contraction for MFMA
    return {"bound": "latency", "peak_resource": "hbm", "kernel": "k_rans_fast01 (" + DOM + ")",
            "achieved": round(achieved, 2) if achieved else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5) if achieved else None,
            "traffic": traffic, "algorithmic_bytes": alg,
            "algorithmic_bytes_note": "(1 + r) x raw bytes per launch (SURVEY 8(d) encode side)",
            "design_bytes": design,
            "design_achieved": round(design / (kms * 1e-3) / 1e9, 2) if kms else None,
            "limiter": "latency of the serial rans64 coder chain (65,536 dependent steps per tile plane), "
                       "not HBM: traffic ~ design bytes (u16 residuals in + payload out)",
            "avg_launch_ms": round(kms, 4) if kms else None,
            "avg_launch_ms_source": "HIP events on the encoder's stream, one image in flight, 5 launches",
            "avg_launch_ms_under_load": round(kavg[DOM], 4) if DOM in kavg else None,
            "images_per_launch_under_load": B,
            "pipeline_achieved": round(pipeline_gbs, 2), "pipeline_frac": round(pipeline_gbs / HBM_PEAK_GBS, 5),
            "pipeline_bytes_per_image": round(2 * (1 + ratio) * raw_total)}


def strong_batch(W, H, world, B):
    """Images per slot of the configs[3] leg: about as many pixels per GPU per step as the weak
    line's B 8192^2 bands (16384^2 over N ranks: 2 images per slot at N = 1, 16 at N = 8)."""
    rows = H // max(1, world)
    return max(1, min(16, (B * 8192 * 8192) // (W * max(rows, 1))))


def sharded_main(args, D, B, world, rank, dev, torch, hoh_ans, hd):
    """N > 1 (one process per GPU, RCCL), or --sharded at N = 1 (the same code on a one-rank
    group).  The line's value is the primary leg: weak scaling 8192 x (8192 N) by default (each
    GPU always holds an 8192^2 band of every image), or configs[3] with --strong.  Each rank runs
    the N = 1 line's schedule -- D slots, each a batch of B images' bands per step through the
    batched shard calls, at HIP's default hardware queues.  Unless --strong or --no-strong-leg, the
    same launch also runs configs[3] -- 16384^2 images sharded over the N ranks, slot 0's first
    image seed 2 (the reference choh's golden file) -- into detail.strong_16384_*, with rank 0's
    gathered file hashed against tests/golden/golden_speed.json."""
    import torch.distributed as dist
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if world == 1:
        import socket
        so = socket.socket()
        so.bind(("127.0.0.1", 0))
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(so.getsockname()[1]))
        so.close()
        os.environ.setdefault("RANK", "0")
    dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)
    W = args.size
    H = args.size if args.strong else args.size * world
    K, warm = args.steps, args.warmup
    seed0 = STRONG_SEED if (args.strong and W == STRONG_SIDE) else args.seed
    Bp = strong_batch(W, H, world, B) if args.strong else B
    p = sharded_leg(args, W, H, D, Bp, K, warm, seed0, rank, world, dev, torch, hoh_ans, hd, one_in_flight=True)
    strong = None
    if not args.strong and not args.no_strong_leg and STRONG_SIDE // 256 >= world:
        Ds = max(1, min(args.strong_inflight, D))
        Bs = strong_batch(STRONG_SIDE, STRONG_SIDE, world, B)
        strong = sharded_leg(args, STRONG_SIDE, STRONG_SIDE, Ds, Bs, max(1, args.leg_steps), Ds, STRONG_SEED, rank,
                             world, dev, torch, hoh_ans, hd)
    bad = False
    if rank == 0:
        raw_total = W * H * 3
        kavg = {k: v[0] / v[1] for k, v in p["stats"].items() if v[1]}
        rows_raw = W * p["rows"] * 3
        # the one-in-flight launch is the slowest rank's
        ratio = p["comp_total"] / raw_total
        roof = roofline_obj(p["iso_dom_ms_max"] or None, kavg, ratio, rows_raw, raw_total, K, p["el"], None, Bp)
        roof["avg_launch_ms_source"] = ("HIP events on the encoder's stream, one shard (%dx%d band) in flight per "
                                        "rank, 5 launches, max over ranks" % (W, p["rows"]))
        roof["algorithmic_bytes_note"] = "(1 + r) x the band's raw bytes per launch (SURVEY 8(d) encode side)"
        gw = golden_speed_sha(W, H, seed0, args.noise) if args.strong else None
        if gw is None:
            gw = golden_sha(W, H, seed0, args.noise)
        gb = dict(golden_bench_shas(W, H, args.noise))  # 8192^2 seeds 1..40; 8192 x 8192N seeds 1..4
        if gw is not None:
            gb[seed0] = gw
        gw = gb.get(seed0)
        checked = {sd: (h == gb[sd]) for sd, h in p["shas"].items() if sd in gb}
        detail = {
            "slots": D,
            "batch": Bp,
            "inflight": D * Bp,
            "hw_queues": hw_queue_note(),
            "warmup_requested": args.warmup,
            "latency_ms_enc": round(p["t_enc"] / K * 1e3, 3),
            "latency_ms_dec": round(p["t_dec"] / K * 1e3, 3),
            "compressed_bytes": p["comp_total"],
            "ratio": round(ratio, 5),
            "lossless": p["lossless"],
            "file_sha256": p["sha"],
            "bit_exact_vs_reference": (p["sha"] == gw) if gw else None,
            "slot_files_bit_exact": "%d of %d" % (sum(checked.values()), len(checked)),
            "slot_files_checked_seeds": sorted(checked),
            "one_in_flight_shard_bytes_equal_batched": p["iso_same_bytes"],
            "setup_steps": D,
            "kernel_avg_ms_under_load": {k: round(v, 4) for k, v in kavg.items()},
            "kernel_avg_ms_one_in_flight_rank0": {k: round(v, 4) for k, v in (p["iso"] or {}).items()},
        }
        if strong is not None:
            g = golden_speed_sha(STRONG_SIDE, STRONG_SIDE, STRONG_SEED, args.noise)
            detail.update({
                "strong_16384_MBps": round(strong["value"], 1),
                "strong_16384_ms_per_step": round(strong["el"] / strong["K"] * 1e3, 4),
                "strong_16384_steps": strong["K"],
                "strong_16384_slots": strong["D"],
                "strong_16384_batch": strong["B"],
                "strong_16384_lossless": strong["lossless"],
                "strong_16384_file_sha256": strong["sha"],
                "strong_16384_bit_exact_vs_reference": (strong["sha"] == g) if g else None,
                "strong_16384_note": "BASELINE configs[3]: 16384x16384 images (slot 0's first: seed %d) sharded over "
                                     "the %d rank(s) (strong scaling), %d slots x %d images per step, RCCL gather of "
                                     "the sub-bitstreams to each image's root rank; sha256 of the gathered file against the "
                                     "reference choh's (golden_speed.json)"
                                     % (STRONG_SEED, world, strong["D"], strong["B"]),
            })
        res = {
            "metric": metric_name(),
            "value": round(p["value"], 2),
            "unit": "MB/s",
            "n_gpus": world,
            "steps": K,
            "warmup": warm,
            "ms_per_step": round(p["el"] / K * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {
                "workload": ("%dx%d synthetic RGB (gradient + triangular noise k=%d, seeds %d..%d), 256x256 tiles, "
                             "choh -s0 encode + dhoh decode, %s, %d slot(s) x a batch of %d images' bands per step "
                             "(hoh_encode_tiles_images_async / hoh_decode_tiles_images_async) per GPU, %s hardware "
                             "queues"
                             % (W, H, args.noise, seed0, seed0 + D * Bp - 1,
                                "side index" if not args.no_index else "serial decode", D, Bp, hw_queue_note())),
                "W": W, "H": H, "tiles": (W // 256) * (H // 256), "per_gpu": "%dx%d" % (W, p["rows"]), "batch": Bp,
                "parallelism": "tile rows sharded over %d GPU(s), RCCL gather of each image's shards to its "
                               "root rank (image b of a step on rank b %% N)" % world,
            },
            "roofline": roof,
            "detail": detail,
        }
        print(json.dumps(res), flush=True)
        bad = (not all(checked.values())) or detail.get("strong_16384_bit_exact_vs_reference") is False
    ok = p["lossless"] and (strong is None or strong["lossless"])
    dist.destroy_process_group()
    if not ok or bad:
        sys.exit(3)


def batch_main(args, D, B, dev, torch, hoh_ans, hd):
    """N = 1 with --batch B > 1: D slots, each step one batch of B images (seeds args.seed + k*B ..,
    contiguous in HBM) through hoh_encode_images_async + hoh_decode_images_async, whose kernels
    cover the B images' tiles per launch (choh.cpp:464-500's tile loop over the batch): fewer,
    larger launches on fewer streams, so the device fills without many hardware queues.  Every
    image's file of each slot's last step is SHA-checked against the reference's
    (golden_bench.json) and every image's decode against its input."""
    L = hoh_ans.lib()
    W = H = args.size
    img = W * H * 3
    stride = L.hoh_encode_bound(W, H)
    K, warm = args.steps, args.warmup
    status = torch.zeros((max(K, warm, D), 4 * B), dtype=torch.int64, device=dev)

    class Slot:
        def __init__(self, k):
            self.seeds = [args.seed + k * B + b for b in range(B)]
            self.ctx = hoh_ans.Context(dev.index)
            self.stream = torch.cuda.Stream(device=dev)
            self.rgb = torch.empty(B * img, dtype=torch.uint8, device=dev)
            for b, sd in enumerate(self.seeds):
                self.rgb[b * img:(b + 1) * img] = hoh_ans.synth_rgb_dev(W, H, sd, args.noise, ctx=self.ctx)
            self.index = None if args.no_index else hoh_ans.Index()
            self.out = torch.empty(B * stride, dtype=torch.uint8, device=dev)
            self.dec = torch.empty(B * img, dtype=torch.uint8, device=dev)

    slots = [Slot(k) for k in range(D)]
    torch.cuda.synchronize()

    def enqueue(k, i):
        s = slots[k]
        with torch.cuda.stream(s.stream):
            hoh_ans.encode_images_async(s.rgb, B, W, H, s.out, stride, status[i, :2 * B], ctx=s.ctx, index=s.index)
            hoh_ans.decode_images_async(s.out, B, stride, W, H, s.dec, status[i, 2 * B:], ctx=s.ctx, index=s.index)

    def run(total):
        hd.run_pipeline(D, total, enqueue, lambda k, i: None)

    def check_status(total):
        st = status[:total].cpu().numpy()
        for i in range(total):
            for b in range(B):
                hoh_ans.check_status(st[i, 2 * b:2 * b + 2], "encode (step %d image %d)" % (i, b))
                hoh_ans.check_status(st[i, 2 * B + 2 * b:2 * B + 2 * b + 2], "decode (step %d image %d)" % (i, b))
        return st

    run(D)
    torch.cuda.synchronize()
    check_status(D)
    if warm:
        run(warm)
        torch.cuda.synchronize()
        check_status(warm)
    torch.cuda.synchronize()
    t = time.perf_counter()
    run(K)
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    st = check_status(K)
    bad_dec = [(k, b) for k, s in enumerate(slots) for b in range(B)
               if not bool(torch.equal(s.dec[b * img:(b + 1) * img], s.rgb[b * img:(b + 1) * img]))]
    lossless = not bad_dec
    gb = golden_bench_shas(W, H, args.noise)
    match, checked, nogold, comp, bad_sha = 0, 0, [], None, []
    for k, s in enumerate(slots):
        if k >= K:
            continue
        row = k + ((K - 1 - k) // D) * D
        for b, sd in enumerate(s.seeds):
            n_b = int(st[row, 2 * b + 1])
            if comp is None:
                comp = n_b
            want = gb.get(sd)
            if want is None:
                nogold.append(sd)
                continue
            checked += 1
            ok = hashlib.sha256(s.out[b * stride:b * stride + n_b].cpu().numpy().tobytes()).hexdigest() == want
            match += ok
            if not ok:
                bad_sha.append((k, b, sd, n_b))
    if bad_dec or bad_sha:
        print("batch_main: lossless failures (slot, image) %s; SHA mismatches (slot, image, seed, size) %s"
              % (bad_dec, bad_sha), file=sys.stderr)
    value = B * img * K / el / 1e6
    res = {
        "metric": metric_name(), "value": round(value, 2), "unit": "MB/s", "n_gpus": 1, "steps": K, "warmup": warm,
        "ms_per_step": round(el / K * 1e3, 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic",
        "config": {"workload": ("%dx%d synthetic RGB (gradient + triangular noise k=%d, seeds %d..%d), 256x256 tiles, "
                                "choh -s0 encode + dhoh decode, %s, %d slot(s) x a batch of %d images per step "
                                "(hoh_encode_images_async / hoh_decode_images_async)"
                                % (W, H, args.noise, args.seed, args.seed + D * B - 1,
                                   "side index" if not args.no_index else "serial decode", D, B)),
                   "W": W, "H": H, "tiles": (W // 256) * (H // 256), "batch": B, "parallelism": "1 GPU"},
        "detail": {"inflight_slots": D, "batch": B, "images_in_flight": D * B,
                   "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0),
                   "lossless": lossless, "compressed_bytes": comp,
                   "slot_files_bit_exact": "%d of %d" % (match, checked),
                   "slot_files_bit_exact_all": (match == checked and not nogold) if checked else None,
                   "slot_files_no_golden_seeds": nogold},
    }
    print(json.dumps(res), flush=True)
    if not lossless or match != checked:
        sys.exit(3)


def single_main(args, D, dev, torch, hoh_ans, hd, pmc, pmc_note, pmc_speed):
    """N = 1: D slots of B = --batch images each (B * D images in flight), enqueue-only encode +
    decode, no host round trip per step.  B > 1: one step encodes and decodes the slot's B images
    through the batched calls (hoh_encode_images_async / hoh_decode_images_async: every kernel
    covers the B images' tiles); B = 1: the single-image calls."""
    L = hoh_ans.lib()
    W = H = args.size
    rows = H
    K = args.steps
    warm = args.warmup
    B = max(1, args.batch)
    img = W * rows * 3
    stride = L.hoh_encode_bound(W, rows)
    status = torch.zeros((max(K, warm, D), 4 * B), dtype=torch.int64, device=dev)

    class Slot:
        """B in-flight images (seeds args.seed + k*B .. + B-1, contiguous in HBM), one library
        context (HIP stream + workspaces), side index and output buffers; rgb0 / out0 / dec0 are
        the first image's views (one-in-flight measurements and the detail legs)."""

        def __init__(self, k):
            self.seeds = [args.seed + k * B + b for b in range(B)]
            self.seed = self.seeds[0]
            self.ctx = hoh_ans.Context(dev.index)
            self.stream = torch.cuda.Stream(device=dev)
            self.rgb = torch.empty(B * img, dtype=torch.uint8, device=dev)
            for b, sd in enumerate(self.seeds):
                self.rgb[b * img:(b + 1) * img] = hoh_ans.synth_rgb_dev(W, rows, sd, args.noise, ctx=self.ctx)
            self.index = None if args.no_index else hoh_ans.Index()
            self.out = torch.empty(B * stride, dtype=torch.uint8, device=dev)
            self.dec = torch.empty(B * img, dtype=torch.uint8, device=dev)
            self.rgb0, self.out0, self.dec0 = self.rgb[:img], self.out[:stride], self.dec[:img]
            self.events = []

    slots = [Slot(k) for k in range(D)]
    torch.cuda.synchronize()

    def enqueue(k, i):
        s = slots[k]
        with torch.cuda.stream(s.stream):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if B > 1:
                hoh_ans.encode_images_async(s.rgb, B, W, H, s.out, stride, status[i, :2 * B], ctx=s.ctx, index=s.index)
            else:
                hoh_ans.encode_image_async(s.rgb, W, H, s.out, status[i, 0:2], ctx=s.ctx, index=s.index)
            e1.record()
            if B > 1:
                hoh_ans.decode_images_async(s.out, B, stride, W, H, s.dec, status[i, 2 * B:], ctx=s.ctx, index=s.index)
            else:
                hoh_ans.decode_image_async(s.out, s.out.numel(), W, H, s.dec, status[i, 2:4], ctx=s.ctx, index=s.index)
            e2 = torch.cuda.Event(enable_timing=True)
            e2.record()
            s.events.append((e0, e1, e2))

    def run(total):
        hd.run_pipeline(D, total, enqueue, lambda k, i: None)

    def check_status(total):
        st = status[:total].cpu().numpy()
        for i in range(total):
            for b in range(B):
                hoh_ans.check_status(st[i, 2 * b:2 * b + 2], "encode (step %d image %d)" % (i, b))
                hoh_ans.check_status(st[i, 2 * B + 2 * b:2 * B + 2 * b + 2], "decode (step %d image %d)" % (i, b))
        return int(st[total - 1, 1])

    for s in slots:
        s.ctx.profiling(True)
    # set-up pass (not warmup): one step per slot sizes its context's workspaces, so no slot
    # allocates device memory inside the timed region; then exactly the requested warmup steps
    run(D)
    torch.cuda.synchronize()
    check_status(D)
    if warm:
        run(warm)
        torch.cuda.synchronize()
        check_status(warm)
    for s in slots:
        s.ctx.reset_stats()
        s.events = []
    torch.cuda.synchronize()
    t = time.perf_counter()
    run(K)
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    check_status(K)
    stats = {}
    for s in slots:
        for k, (tot, cnt) in s.ctx.kernel_stats().items():
            a0, c0 = stats.get(k, (0.0, 0))
            stats[k] = (a0 + tot, c0 + cnt)
        s.ctx.profiling(False)
    t_enc = t_dec = 0.0
    for s in slots:
        for ev in s.events:
            t_enc += ev[0].elapsed_time(ev[1]) * 1e-3
            t_dec += ev[-2].elapsed_time(ev[-1]) * 1e-3

    # per-kernel durations and the per-image rate with ONE image in flight (host-synchronous
    # calls), and the no-index (serial rANS) decode of slot 0's file
    s0 = slots[0]
    noix_ms, noix_ok = None, None
    with torch.cuda.stream(s0.stream):
        s0.ctx.profiling(True)
        s0.ctx.reset_stats()
        times = []
        for _ in range(5):
            torch.cuda.synchronize()
            ta = time.perf_counter()
            _, n0, _ = hoh_ans.encode_image(s0.rgb0, W, H, out_dev=s0.out0, ctx=s0.ctx, index=s0.index)
            hoh_ans.decode_image(s0.out0, n0, out_dev=s0.dec0, ctx=s0.ctx, index=s0.index)
            s0.stream.synchronize()
            times.append(time.perf_counter() - ta)
        iso = {k: v[0] / v[1] for k, v in s0.ctx.kernel_stats().items() if v[1]}
        s0.ctx.profiling(False)
        single_ms = sorted(times)[len(times) // 2] * 1e3
        if not args.no_index:
            noix = torch.empty_like(s0.dec0)
            times = []
            for _ in range(3):
                s0.stream.synchronize()
                ta = time.perf_counter()
                hoh_ans.decode_image(s0.out0, n0, out_dev=noix, ctx=s0.ctx, index=None)
                s0.stream.synchronize()
                times.append(time.perf_counter() - ta)
            noix_ms = min(times) * 1e3
            noix_ok = bool(torch.equal(noix, s0.rgb0))
            del noix

    # checks outside the timed region: every slot lossless, and EVERY slot's file (its last
    # timed step's) against the reference choh's sha256 for that slot's seed
    # (tests/golden/golden_bench.json, made by tests/golden/make_golden_bench.py)
    lossless = all(bool(torch.equal(s.dec, s.rgb)) for s in slots)
    sha = hashlib.sha256(s0.out0[:n0].cpu().numpy().tobytes()).hexdigest()
    gb = golden_bench_shas(W, H, args.noise)
    st = status[:K].cpu().numpy()
    slot_match, slot_checked, slot_nogolden = 0, 0, []
    for k, s in enumerate(slots):
        if k >= K:
            continue
        row = k + ((K - 1 - k) // D) * D          # the slot's last timed step
        for b, sd in enumerate(s.seeds):
            # image 0 of slot 0 was re-encoded by the one-in-flight leg (same image)
            n_k = n0 if (k == 0 and b == 0) else int(st[row, 2 * b + 1])
            want = gb.get(sd)
            if want is None:
                slot_nogolden.append(sd)
                continue
            slot_checked += 1
            slot_match += hashlib.sha256(s.out[b * stride:b * stride + n_k].cpu().numpy().tobytes()).hexdigest() == want
    comp_total = n0
    raw_total = W * H * 3
    value = raw_total * B * K / el / 1e6
    legs = {}
    if not args.no_legs:      # after the checks: the legs reuse the slots' buffers
        legs = extra_legs(args, slots, W, H, D, B, stride, status, torch, hoh_ans, hd)

    kavg = {k: v[0] / v[1] for k, v in stats.items() if v[1]}
    ratio = comp_total / raw_total
    roof = roofline_obj(iso.get(DOM) or None, kavg, ratio, W * rows * 3, raw_total, K, el, pmc, B)
    golden = golden_sha(W, H, args.seed, args.noise)
    res = {
        "metric": metric_name(),
        "value": round(value, 2),
        "unit": "MB/s",
        "n_gpus": 1,
        "steps": K,
        "warmup": warm,
        "ms_per_step": round(el / K * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {
            "workload": ("%dx%d synthetic RGB (gradient + triangular noise k=%d, seeds %d..%d: one image each), "
                         "256x256 tiles, choh -s0 encode + dhoh decode, %s, %d slot(s) x %d image(s) per step "
                         "(%s) = %d images in flight per GPU, %s hardware queues"
                         % (W, H, args.noise, args.seed, args.seed + D * B - 1,
                            "side index" if not args.no_index else "serial decode", D, B,
                            "batched calls hoh_encode_images_async / hoh_decode_images_async" if B > 1 else
                            "hoh_encode_image_async / hoh_decode_image_async", D * B, hw_queue_note())),
            "W": W, "H": H, "tiles": (W // 256) * (H // 256), "per_gpu": "%dx%d" % (W, rows), "batch": B,
            "parallelism": "1 GPU",
        },
        "roofline": roof,
        "detail": {
            "inflight": D * B,
            "slots": D,
            "batch": B,
            "hw_queues": hw_queue_note(),
            "warmup_requested": args.warmup,
            "latency_ms_enc": round(t_enc / K * 1e3, 3),
            "latency_ms_dec": round(t_dec / K * 1e3, 3),
            "compressed_bytes": comp_total,
            "ratio": round(ratio, 5),
            "lossless": lossless,
            "file_sha256": sha,
            "bit_exact_vs_reference": (sha == golden) if golden else None,
            "slot_files_bit_exact": "%d of %d" % (slot_match, slot_checked),
            "slot_files_bit_exact_all": (slot_match == slot_checked and not slot_nogolden) if slot_checked else None,
            "slot_files_no_golden_seeds": slot_nogolden,
            "single_image_MBps": round(raw_total / single_ms / 1e3, 1) if single_ms else None,
            "single_image_ms": round(single_ms, 3) if single_ms else None,
            "no_index_decode_MBps": round(raw_total / noix_ms / 1e3, 1) if noix_ms else None,
            "no_index_decode_lossless": noix_ok,
            "setup_steps": D,
            **legs,
            "kernel_avg_ms_under_load": {k: round(v, 4) for k, v in kavg.items()},
            "kernel_avg_ms_one_in_flight": {k: round(v, 4) for k, v in iso.items()},
            "pmc_hbm_bytes_per_launch": pmc,
            "pmc_source": pmc_note,
            "speed_roofline_s%d" % args.pmc_speed: pmc_speed,
        },
    }
    if not args.no_config2:
        try:
            res["detail"]["config2_single_stream"] = config2_leg(args)
        except Exception as e:      # reported, never silently replaced
            res["detail"]["config2_single_stream"] = {"error": repr(e)[:300]}
    if not args.no_cpu_baseline:
        try:
            res["cpu_baseline"] = cpu_baseline(s0.rgb0.cpu().numpy(), W, H, args)
        except Exception as e:      # reported, never silently replaced
            res["cpu_baseline"] = {"value": None, "error": repr(e)[:300]}
    print(json.dumps(res), flush=True)
    if not lossless or noix_ok is False or slot_match != slot_checked:
        sys.exit(3)


if __name__ == "__main__":
    main()
