"""World-size-2 gloo run of the multi-GPU host logic (hoh_ans.dist) on the CPU.

Each rank produces the tile blob of its shard (the oracle's encode_tile stands in for the GPU
encoder here: this tests sharding, the size exchange, the gather and the file assembly), rank 0
assembles the .hoh and it must equal the single-process choh -s0 file byte for byte
(choh.cpp:464-527 tile order / table)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle
from hoh_ans import synth

W, H = 768, 1024   # 3 x 4 tiles: ranks own 2 tile rows each


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    import torch
    import torch.distributed as dist
    import hoh_ans
    from hoh_ans import dist as hd
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        img = synth.synth_rgb(W, H, seed=5, noise=4)
        t0, nt, y0, y1 = hd.shard(W, H, rank, world)
        _, xt, yt, tw, th = hoh_ans.tiling(W, H)
        tiles = []
        for t in range(t0, t0 + nt):
            x, y = (t % xt) * tw, (t // xt) * th
            tiles.append(oracle.encode_tile(img[y:y + th, x:x + tw]))
        sizes = np.array([len(b) for b in tiles], np.uint32)
        blob = torch.zeros(4 << 20, dtype=torch.uint8)
        cat = b"".join(tiles)
        blob[:len(cat)] = torch.frombuffer(bytearray(cat), dtype=torch.uint8)
        g = hd.FileGather(W, H, "cpu")
        f, n = g(blob, len(cat), sizes)
        if rank == 0:
            with open(os.path.join(outdir, "gathered.hoh"), "wb") as fh:
                fh.write(f[:n].numpy().tobytes())
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_shard_covers_all_tiles():
    import hoh_ans
    from hoh_ans import dist as hd
    for (w, h) in [(768, 1024), (8192, 8192), (8192, 16384), (1000, 600)]:
        _, xt, yt, tw, th = hoh_ans.tiling(w, h)
        for world in (1, 2, 3, 4, 8):
            if world > yt:
                continue
            nxt = 0
            rows = 0
            for r in range(world):
                t0, nt, y0, y1 = hd.shard(w, h, r, world)
                assert t0 == nxt and nt % xt == 0 and y0 == rows
                nxt += nt
                rows = y1
            assert nxt == xt * yt and rows == h


def test_gloo_gather_matches_single_file(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = (tmp_path / "gathered.hoh").read_bytes()
    img = synth.synth_rgb(W, H, seed=5, noise=4)
    want, printed = oracle.choh(img)
    assert got == want


NSTEP, NSLOT = 5, 3


def _pipeline_worker(rank, world, port, outdir):
    """bench.py's N > 1 schedule on gloo: several images in flight per rank, one process group,
    one host thread; every step's gather must still assemble that step's file exactly."""
    import torch
    import torch.distributed as dist
    import hoh_ans
    from hoh_ans import dist as hd
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t0, nt, y0, y1 = hd.shard(W, H, rank, world)
        _, xt, yt, tw, th = hoh_ans.tiling(W, H)
        slots = [{"blob": torch.zeros(4 << 20, dtype=torch.uint8), "g": hd.FileGather(W, H, "cpu")}
                 for _ in range(NSLOT)]

        def enqueue(k, i):
            img = synth.synth_rgb(W, H, seed=10 + i, noise=4)
            tiles = []
            for t in range(t0, t0 + nt):
                x, y = (t % xt) * tw, (t // xt) * th
                tiles.append(oracle.encode_tile(img[y:y + th, x:x + tw]))
            cat = b"".join(tiles)
            slots[k]["blob"][:len(cat)] = torch.frombuffer(bytearray(cat), dtype=torch.uint8)
            slots[k]["n"] = len(cat)
            slots[k]["sizes"] = np.array([len(b) for b in tiles], np.uint32)

        def finish(k, i):
            sl = slots[k]
            res = sl["g"](sl["blob"], sl["n"], sl["sizes"], wait=False)
            for q in res[2]:
                q.wait()
            if rank == 0:
                with open(os.path.join(outdir, "step%d.hoh" % i), "wb") as fh:
                    fh.write(res[0][:res[1]].numpy().tobytes())

        order = hd.run_pipeline(NSLOT, NSTEP, enqueue, finish)
        assert order == list(range(NSTEP))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_gloo_pipeline_in_step_order(tmp_path):
    world = 2
    mp.spawn(_pipeline_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for i in range(NSTEP):
        img = synth.synth_rgb(W, H, seed=10 + i, noise=4)
        want, _ = oracle.choh(img)
        assert (tmp_path / ("step%d.hoh" % i)).read_bytes() == want, "step %d" % i


class _CpuShardOps:
    """CPU stand-in for bench.py's GpuShardOps (same interface, oracle encode_tile instead of
    hoh_encode_tiles_async, oracle dhoh of the gathered file instead of hoh_decode_tiles_async)."""

    def __init__(self, W, H, rank, world, seed0):
        import hoh_ans
        from hoh_ans import dist as hd
        self.W, self.H, self.rank, self.seed0 = W, H, rank, seed0
        self.t0, self.nt, self.y0, self.y1 = hd.shard(W, H, rank, world)
        _, self.xt, _, self.tw, self.th = hoh_ans.tiling(W, H)
        self.device = "cpu"
        self.hd = hd
        self.log = []

    def new_slot(self, k):
        import torch
        return {"seed": self.seed0 + k, "img": synth.synth_rgb(self.W, self.H, seed=self.seed0 + k, noise=4),
                "blob": torch.zeros(4 << 20, dtype=torch.uint8), "g": self.hd.FileGather(self.W, self.H, "cpu"),
                "ok": True}

    def enqueue(self, s, i):
        import torch
        tiles = []
        for t in range(self.t0, self.t0 + self.nt):
            x, y = (t % self.xt) * self.tw, (t // self.xt) * self.th
            tiles.append(oracle.encode_tile(s["img"][y:y + self.th, x:x + self.tw]))
        cat = b"".join(tiles)
        s["blob"][:len(cat)] = torch.frombuffer(bytearray(cat), dtype=torch.uint8)
        s["n"], s["sizes"] = len(cat), np.array([len(b) for b in tiles], np.uint32)

    def finish(self, s, i):
        res = s["g"](s["blob"], s["n"], s["sizes"], wait=False)
        for q in res[2]:
            q.wait()
        self.log.append(i)
        if self.rank == 0:
            f = res[0][:res[1]].numpy().tobytes()
            s["file"] = f
            s["ok"] = s["ok"] and np.array_equal(oracle.dhoh(f), s["img"])

    def drain(self):
        pass

    def check(self, total):
        pass

    def reset(self, slots):
        self.log = []

    def lossless(self, s):
        return s["ok"]


def _leg_worker(rank, world, port, outdir):
    import torch.distributed as dist
    from hoh_ans import dist as hd
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ops = _CpuShardOps(W, H, rank, world, 20)
        slots, el, ok = hd.run_sharded_leg(ops, 2, 3, 1)
        assert ok and el > 0
        assert ops.log == [0, 1, 2]            # the timed steps finished in step order
        if rank == 0:
            for s in slots:
                with open(os.path.join(outdir, "leg_seed%d.hoh" % s["seed"]), "wb") as fh:
                    fh.write(s["file"])
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_gloo_sharded_leg(tmp_path):
    """hoh_ans.dist.run_sharded_leg -- the timed leg bench.py runs at N > 1 (the weak line and the
    configs[3] strong leg) -- on two gloo ranks: set-up pass, warmup, timed steps, max-over-ranks;
    each slot's gathered file equals the single-process choh -s0 file and decodes losslessly."""
    world = 2
    mp.spawn(_leg_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for seed in (20, 21):
        want, _ = oracle.choh(synth.synth_rgb(W, H, seed=seed, noise=4))
        assert (tmp_path / ("leg_seed%d.hoh" % seed)).read_bytes() == want


class _BatchCpuShardOps(_CpuShardOps):
    """CPU stand-in for bench.py's batched GpuShardOps: a slot holds B images, a step encodes the
    rank's band of all B (the oracle's encode_tile per tile, blob i at i * STRIDE) and
    hd.BatchGather moves all of them to rank 0 with one size exchange and one batch of
    point-to-point operations."""
    B, STRIDE = 2, 2 << 20

    def new_slot(self, k):
        import torch
        seeds = [self.seed0 + k * self.B + b for b in range(self.B)]
        return {"seeds": seeds, "imgs": [synth.synth_rgb(self.W, self.H, seed=sd, noise=4) for sd in seeds],
                "blob": torch.zeros(self.B * self.STRIDE, dtype=torch.uint8),
                "g": self.hd.BatchGather(self.W, self.H, self.B, "cpu"), "ok": True}

    def enqueue(self, s, i):
        import torch
        sizes = []
        for b, img in enumerate(s["imgs"]):
            tiles = []
            for t in range(self.t0, self.t0 + self.nt):
                x, y = (t % self.xt) * self.tw, (t // self.xt) * self.th
                tiles.append(oracle.encode_tile(img[y:y + self.th, x:x + self.tw]))
            cat = b"".join(tiles)
            assert len(cat) <= self.STRIDE
            s["blob"][b * self.STRIDE:b * self.STRIDE + len(cat)] = torch.frombuffer(bytearray(cat), dtype=torch.uint8)
            sizes.append([len(t) for t in tiles])
        s["sizes"] = np.array(sizes, np.uint32)

    def finish(self, s, i):
        res = s["g"](s["blob"], self.STRIDE, s["sizes"], wait=False)
        for q in res[2]:
            q.wait()
        self.log.append(i)
        g = s["g"]                                  # image b's file is assembled on rank b % world
        s["files"] = {b: res[0][g.row(b), :res[1][b]].numpy().tobytes() for b in g.own}
        s["ok"] = s["ok"] and all(np.array_equal(oracle.dhoh(f), s["imgs"][b]) for b, f in s["files"].items())


def _batch_leg_worker(rank, world, port, outdir):
    import torch.distributed as dist
    from hoh_ans import dist as hd
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ops = _BatchCpuShardOps(W, H, rank, world, 40)
        slots, el, ok = hd.run_sharded_leg(ops, 2, 3, 1)
        assert ok and el > 0
        assert ops.log == [0, 1, 2]
        for s in slots:                             # every rank writes the files it roots
            for b, f in s["files"].items():
                with open(os.path.join(outdir, "batch_seed%d.hoh" % s["seeds"][b]), "wb") as fh:
                    fh.write(f)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_gloo_batched_sharded_leg(tmp_path):
    """bench.py's batched N > 1 schedule on two gloo ranks: 2 slots x 2 images, BatchGather (image
    b of a slot assembled on rank b % 2); every image's gathered file equals the single-process
    choh -s0 file and decodes losslessly"""
    world = 2
    mp.spawn(_batch_leg_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for seed in (40, 41, 42, 43):
        want, _ = oracle.choh(synth.synth_rgb(W, H, seed=seed, noise=4))
        assert (tmp_path / ("batch_seed%d.hoh" % seed)).read_bytes() == want, seed
