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
