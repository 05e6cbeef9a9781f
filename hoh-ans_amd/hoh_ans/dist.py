"""Multi-GPU tile sharding (one process per GPU) and the gather that assembles a .hoh.

choh walks tiles in row-major order and writes them back to back after the tile table
(choh.cpp:464-527).  Tiles are independent, so rank r encodes a contiguous band of tile rows
(encode_tiles), and one gather over RCCL/xGMI brings every rank's blob to rank 0, which writes
the header + tile table (hoh_file_prefix) and concatenates: the result is byte-identical to the
single-GPU file.  Decode runs per rank on its own blob (decode_tiles); no other exchange.

Works with any torch.distributed backend ("nccl" = RCCL on ROCm for device tensors, "gloo" for
the CPU tests); the collectives see only uint8/int64 tensors.
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


def gather_sizes(tile_sizes, device, group=None):
    """All-gather every rank's per-tile sizes (variable count) -> list of np.uint32 arrays."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    ts = np.asarray(tile_sizes, dtype=np.int64)
    n = torch.tensor([ts.size], dtype=torch.int64, device=device)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    ns = [int(x.item()) for x in ns]
    m = max(ns)
    buf = torch.zeros(m, dtype=torch.int64, device=device)
    buf[:ts.size] = torch.from_numpy(ts).to(device)
    bufs = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(bufs, buf, group=group)
    return [b[:k].cpu().numpy().astype(np.uint32) for b, k in zip(bufs, ns)]


class FileGather:
    """Gathers the ranks' tile blobs to rank 0 and assembles the .hoh there.

    blob: uint8 tensor on this rank's device (capacity >= the largest rank's blob), size: bytes
    used.  Workspaces are kept across calls (the bench calls it every step)."""

    def __init__(self, W, H, device, group=None):
        self.W, self.H, self.device, self.group = W, H, device, group
        self.slots = None
        self.file = None

    def __call__(self, blob, size, tile_sizes):
        import torch
        import torch.distributed as dist
        rank = dist.get_rank(self.group)
        world = dist.get_world_size(self.group)
        sizes = gather_sizes(tile_sizes, self.device, self.group)
        blob_sizes = [int(s.sum(dtype=np.int64)) for s in sizes]
        if blob_sizes[rank] != size:
            raise RuntimeError("tile sizes do not add up to the blob size")
        m = max(blob_sizes)
        if blob.numel() < m:
            raise RuntimeError("blob capacity %d < largest shard %d" % (blob.numel(), m))
        if rank == 0:
            if self.slots is None or self.slots[0].numel() < m:
                self.slots = [torch.empty(m, dtype=torch.uint8, device=self.device) for _ in range(world)]
            dist.gather(blob[:m], [s[:m] for s in self.slots], dst=0, group=self.group)
        else:
            dist.gather(blob[:m], None, dst=0, group=self.group)
            return None, 0
        all_sizes = np.concatenate(sizes)
        prefix = file_prefix(self.W, self.H, all_sizes)
        total = len(prefix) + sum(blob_sizes)
        if self.file is None or self.file.numel() < total:
            self.file = torch.empty(total, dtype=torch.uint8, device=self.device)
        self.file[:len(prefix)] = torch.frombuffer(bytearray(prefix), dtype=torch.uint8).to(self.device)
        off = len(prefix)
        for r in range(world):
            self.file[off:off + blob_sizes[r]] = self.slots[r][:blob_sizes[r]]
            off += blob_sizes[r]
        return self.file, total
