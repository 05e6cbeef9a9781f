"""Multi-GPU tile sharding (one process per GPU) and the gather that assembles a .hoh.

choh walks tiles in row-major order and writes them back to back after the tile table
(choh.cpp:464-527).  Tiles are independent, so rank r encodes a contiguous band of tile rows
(encode_tiles), and one gather over RCCL/xGMI brings every rank's blob to rank 0, which writes
the header + tile table (hoh_file_prefix) and concatenates: the result is byte-identical to the
single-GPU file.  Decode runs per rank on its own blob (decode_tiles); no other exchange.

Works with any torch.distributed backend ("nccl" = RCCL on ROCm for device tensors, "gloo" for
the CPU tests); the collectives see only uint8/int64 tensors.

Several images in flight per GPU share ONE process group: a single host thread per rank deals the
steps round-robin to the in-flight slots (run_pipeline), and every rank issues the gathers in
step order, so the collectives of different slots never interleave differently across ranks.
"""
import numpy as np

from . import tiling, file_prefix


def shard(W, H, rank, world):
    """Band of tile rows owned by `rank`: (t0, ntiles, y0, y1) with rows [y0, y1) of the image."""
    tiled, xt, yt, tw, th = tiling(W, H)
    if not tiled:
        raise ValueError("untiled image (choh.cpp:454-461): nothing to shard")
    if world > yt:
        raise ValueError("more ranks (%d) than tile rows (%d)" % (world, yt))
    r0 = rank * yt // world
    r1 = (rank + 1) * yt // world
    return r0 * xt, (r1 - r0) * xt, r0 * th, min(H, r1 * th)


def shard_counts(W, H, world):
    """Tile count of every rank's shard (known to all ranks without an exchange)."""
    return [shard(W, H, r, world)[1] for r in range(world)]


def gather_sizes(tile_sizes, device, group=None, counts=None):
    """All-gather every rank's per-tile sizes -> list of np.uint32 arrays.  With `counts` (each
    rank's tile count, e.g. shard_counts) one all_gather suffices; otherwise the counts are
    exchanged first."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    ts = np.asarray(tile_sizes, dtype=np.int64)
    if counts is None:
        n = torch.tensor([ts.size], dtype=torch.int64, device=device)
        ns = [torch.zeros_like(n) for _ in range(world)]
        dist.all_gather(ns, n, group=group)
        counts = [int(x.item()) for x in ns]
    m = max(counts)
    buf = torch.zeros(m, dtype=torch.int64, device=device)
    buf[:ts.size] = torch.from_numpy(ts).to(device)
    bufs = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(bufs, buf, group=group)
    return [b[:k].cpu().numpy().astype(np.uint32) for b, k in zip(bufs, counts)]


class FileGather:
    """Brings the ranks' tile blobs to rank 0 and assembles the .hoh there.

    One all_gather of the per-tile sizes (every rank's tile count follows from the sharding),
    then each rank r > 0 sends exactly its blob to rank 0, which receives it straight into its
    place in the file buffer (after the header + tile table, hoh_file_prefix, and the blobs of
    ranks < r): no padding to the largest shard and no assembly copy.  blob: uint8 tensor on
    this rank's device, size: bytes used.  Workspaces are kept across calls (the bench calls it
    every step).  Returns (file tensor, total bytes) on rank 0, (None, 0) elsewhere."""

    def __init__(self, W, H, device, group=None):
        self.W, self.H, self.device, self.group = W, H, device, group
        self.file = None
        self.total = 0            # rank 0: bytes of the last assembled file

    def __call__(self, blob, size, tile_sizes, wait=True):
        """wait=False: return the pending point-to-point requests instead of waiting on them (the
        caller waits -- for RCCL that makes its current stream wait, not the host -- before it
        reuses `blob` or the file buffer)."""
        import torch
        import torch.distributed as dist
        rank = dist.get_rank(self.group)
        world = dist.get_world_size(self.group)
        counts = shard_counts(self.W, self.H, world)
        if len(tile_sizes) != counts[rank]:
            raise RuntimeError("rank %d holds %d tile sizes, its shard has %d tiles" % (rank, len(tile_sizes), counts[rank]))
        sizes = gather_sizes(tile_sizes, self.device, self.group, counts)
        blob_sizes = [int(s.sum(dtype=np.int64)) for s in sizes]
        if blob_sizes[rank] != size:
            raise RuntimeError("tile sizes do not add up to the blob size")
        ranks = dist.get_process_group_ranks(self.group) if self.group is not None else list(range(world))
        if rank != 0:
            reqs = dist.batch_isend_irecv([dist.P2POp(dist.isend, blob[:size], ranks[0], self.group)]) if size else []
            if wait:
                for q in reqs:
                    q.wait()
                return None, 0
            return None, 0, reqs
        prefix = file_prefix(self.W, self.H, np.concatenate(sizes))
        total = len(prefix) + sum(blob_sizes)
        self.total = total
        if self.file is None or self.file.numel() < total:
            self.file = torch.empty(total, dtype=torch.uint8, device=self.device)
        self.file[:len(prefix)] = torch.frombuffer(bytearray(prefix), dtype=torch.uint8).to(self.device)
        offs = np.cumsum([len(prefix)] + blob_sizes)
        ops = [dist.P2POp(dist.irecv, self.file[offs[r]:offs[r] + blob_sizes[r]], ranks[r], self.group)
               for r in range(1, world) if blob_sizes[r]]
        reqs = dist.batch_isend_irecv(ops) if ops else []
        self.file[offs[0]:offs[0] + blob_sizes[0]] = blob[:blob_sizes[0]]
        if not wait:
            return self.file, total, reqs
        for q in reqs:
            q.wait()
        return self.file, total


class BatchGather:
    """FileGather for B images at once (bench.py's batched N > 1 schedule: every rank encodes the
    same band of B images per step, hoh_encode_tiles_images_async).  Blob i of this rank lies at
    blob[i*stride:]; tile_sizes is a (B, ntiles) array of this rank's tile sizes.  ONE all_gather
    carries all B images' tile sizes, then ONE batch of point-to-point operations moves every
    (rank, image) blob straight into its place in image i's file behind hoh_file_prefix.

    Image i's file is assembled on its root rank root(i) = i % world (every image is still one
    gather of its sub-bitstreams): with B >= world each rank roots B / world files, so the blobs of
    a step spread over all the xGMI links instead of converging on rank 0's (at N = 8 that is an
    eighth of the bytes per link).  After a call: `own` lists the images this rank roots, `files`
    holds their files (row k = image own[k]) and `totals[i]` the size of every file (all ranks
    know them).  Returns (files, totals, requests) -- files None on a rank that roots nothing --
    or, with wait=True, (files, totals) after waiting."""

    def __init__(self, W, H, B, device, group=None):
        self.W, self.H, self.B, self.device, self.group = W, H, B, device, group
        self.files = None
        self.totals = [0] * B
        self.own = []

    @staticmethod
    def root(i, world):
        return i % world

    def row(self, i):
        """row of image i in `files` (this rank must root it)"""
        return self.own.index(i)

    def __call__(self, blob, stride, tile_sizes, wait=True):
        import torch
        import torch.distributed as dist
        B = self.B
        rank = dist.get_rank(self.group)
        world = dist.get_world_size(self.group)
        counts = shard_counts(self.W, self.H, world)
        ts = np.asarray(tile_sizes, dtype=np.int64).reshape(B, -1)
        if ts.shape[1] != counts[rank]:
            raise RuntimeError("rank %d holds %d tile sizes per image, its shard has %d tiles"
                               % (rank, ts.shape[1], counts[rank]))
        per = [s.reshape(B, c) for s, c in zip(gather_sizes(ts.reshape(-1), self.device, self.group,
                                                               [c * B for c in counts]), counts)]
        bsz = [[int(per[r][i].sum(dtype=np.int64)) for i in range(B)] for r in range(world)]
        if max(bsz[rank]) > stride:
            raise RuntimeError("a blob is larger than the stride")
        ranks = dist.get_process_group_ranks(self.group) if self.group is not None else list(range(world))
        self.own = [i for i in range(B) if self.root(i, world) == rank]
        prefixes = {i: file_prefix(self.W, self.H, np.concatenate([per[r][i] for r in range(world)]))
                    for i in range(B)}
        totals = [len(prefixes[i]) + sum(bsz[r][i] for r in range(world)) for i in range(B)]
        files = None
        if self.own:
            need = max(totals[i] for i in self.own)
            if self.files is None or self.files.shape[0] < len(self.own) or self.files.shape[1] < need:
                self.files = torch.empty((len(self.own), need + need // 16), dtype=torch.uint8, device=self.device)
            files = self.files
        ops = []
        for i in range(B):
            rt = self.root(i, world)
            if rt != rank:
                if bsz[rank][i]:
                    ops.append(dist.P2POp(dist.isend, blob[i * stride:i * stride + bsz[rank][i]], ranks[rt],
                                          self.group))
                continue
            k = self.own.index(i)
            pl = len(prefixes[i])
            files[k, :pl] = torch.frombuffer(bytearray(prefixes[i]), dtype=torch.uint8).to(self.device)
            off = pl
            for r in range(world):
                if r != rank and bsz[r][i]:
                    ops.append(dist.P2POp(dist.irecv, files[k, off:off + bsz[r][i]], ranks[r], self.group))
                off += bsz[r][i]
        reqs = dist.batch_isend_irecv(ops) if ops else []
        for i in self.own:                      # this rank's own blob of the images it roots
            k = self.own.index(i)
            off = len(prefixes[i]) + sum(bsz[r][i] for r in range(rank))
            files[k, off:off + bsz[rank][i]] = blob[i * stride:i * stride + bsz[rank][i]]
        self.totals = totals
        if not wait:
            return files, totals, reqs
        for q in reqs:
            q.wait()
        return files, totals


def run_pipeline(nslots, total, enqueue, finish):
    """Single-thread pipeline over `nslots` in-flight slots: step i goes to slot i % nslots.
    enqueue(slot, i) enqueues step i's device work without waiting on the host; finish(slot, i)
    completes its host-side part (e.g. the gather, which needs the tile sizes on the host).  Step
    i's finish runs just before its slot takes step i + nslots, and the last nslots steps finish
    at the end, so finish is called for steps 0, 1, 2, ... in order on every rank: collectives
    issued from it match across ranks with one process group."""
    pending = [None] * nslots
    order = []
    for i in range(total):
        k = i % nslots
        if pending[k] is not None:
            finish(k, pending[k])
            order.append(pending[k])
        enqueue(k, i)
        pending[k] = i
    for i in range(max(0, total - nslots), total):
        finish(i % nslots, i)
        order.append(i)
    return order


def run_sharded_leg(ops, nslots, steps, warmup):
    """One timed leg of bench.py's N > 1 path, independent of the device: `nslots` images in
    flight per rank, a set-up pass (one step per slot: workspaces are sized outside the timed
    region), `warmup` steps, then exactly `steps` steps bracketed by a barrier and a device drain
    on both sides; the leg's time is the maximum over ranks.  `ops` supplies the device side:
      new_slot(k) -> slot;  enqueue(slot, i) (encode of the shard, sizes copied to the host);
      finish(slot, i) (FileGather of the blobs to rank 0 + decode of the shard);  drain() (wait
      for the device);  check(total) (statuses of steps 0..total-1);  reset(slots) (clear timing
      state after the warmup);  lossless(slot) -> bool;  device (for the reductions).
    bench.py passes its GPU ops (hoh_encode_tiles_async / hoh_decode_tiles_async over RCCL);
    tests/test_dist_gloo.py passes CPU ops (the oracle) over gloo.
    Returns (slots, max-over-ranks seconds, lossless on every rank)."""
    import time
    import torch
    import torch.distributed as dist
    slots = [ops.new_slot(k) for k in range(nslots)]
    ops.drain()

    def run(total):
        run_pipeline(nslots, total, lambda k, i: ops.enqueue(slots[k], i), lambda k, i: ops.finish(slots[k], i))
        ops.drain()
        ops.check(total)

    run(nslots)
    if warmup:
        run(warmup)
    ops.reset(slots)
    dist.barrier()
    ops.drain()
    t = time.perf_counter()
    run_pipeline(nslots, steps, lambda k, i: ops.enqueue(slots[k], i), lambda k, i: ops.finish(slots[k], i))
    ops.drain()
    dist.barrier()
    el = time.perf_counter() - t
    ops.check(steps)
    ok = all(ops.lossless(s) for s in slots)
    tt = torch.tensor([el, 0.0 if ok else 1.0], dtype=torch.float64, device=ops.device)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    el, bad = tt.tolist()
    return slots, el, bad == 0.0
