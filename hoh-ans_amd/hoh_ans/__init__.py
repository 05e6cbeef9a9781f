"""hoh_ans -- Python mirror of the hoh-ANS hot-path API on the MI355X library (libhohgpu.so).

The reference's interface is a set of C++ free functions (entropy_encoding.hpp:8,
entropy_decoding.hpp:134, layer_encode.hpp:11, layer_decode.hpp:128, prediction.hpp:6,
unprediction.hpp:6, channel.hpp:73) driven by the choh / dhoh CLIs.  This module exposes the
same operations, same names and argument meaning, over the C ABI in include/hoh_ans.h:

    encode_entropy(symbols, range, prob_bits)   -> bytes             (entropy_encoding.hpp:8)
    decode_entropy(data, byte_pointer=0)        -> (symbols, bp)     (entropy_decoding.hpp:134)
    layer_encode(plane, depth, nuke=None)       -> bytes             (layer_encode.hpp:11, -s0)
    channelpredict_fastpath(plane, depth)       -> residuals         (prediction.hpp:6)
    unpredict_fastpath(res, w, h, depth, backref=None) -> plane      (unprediction.hpp:6)
    subtract_green(rgb)                         -> (G, R-G+256, B-G+256)   (channel.hpp:73)
    choh(rgb)                                   -> (bytes, printed)  (choh.cpp:394, -s0)
    dhoh(data)                                  -> rgb               (dhoh.cpp:297, fixed)

Device-resident variants (encode_image / decode_image) take torch tensors already in HBM; they
are what bench.py times.  Errors raise HohError carrying the C status code.  There is no CPU
fallback: a missing library or GPU raises.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIBPATH = os.environ.get("HOH_LIB") or os.path.join(os.path.dirname(HERE), "lib", "libhohgpu.so")  # HOH_LIB: A/B builds

HOH_OK = 0
ERRNAMES = {1: "E_ARG", 2: "E_CAP", 3: "E_HIP", 4: "E_RANGE", 5: "E_UNREPRODUCIBLE", 6: "E_UNSUPPORTED",
            7: "E_CORRUPT", 8: "E_NODEV"}

_L = None
vp = C.c_void_p
sz = C.c_size_t
szp = C.POINTER(C.c_size_t)
ip = C.POINTER(C.c_int)


class HohError(RuntimeError):
    def __init__(self, code, what=""):
        self.code = code
        super().__init__("%s: %s (%d)" % (what, ERRNAMES.get(code, "?"), code))


def lib():
    """Load libhohgpu.so (built in-tree by `make` / __graft_entry__.build())."""
    global _L
    if _L is None:
        if not os.path.exists(LIBPATH):
            raise RuntimeError("libhohgpu.so not built: run `make` (or __graft_entry__.build())")
        L = C.CDLL(LIBPATH)
        L.hoh_ctx_create.argtypes = [C.POINTER(vp), C.c_int]
        L.hoh_ctx_destroy.argtypes = [vp]
        L.hoh_strerror.restype = C.c_char_p
        L.hoh_version.restype = C.c_char_p
        L.hoh_device_alloc_count.restype = C.c_uint64
        L.hoh_set_profiling.argtypes = [vp, C.c_int]
        L.hoh_get_kernel_ms.argtypes = [vp, C.POINTER(C.c_char_p), C.POINTER(C.c_float), C.c_int]
        L.hoh_get_kernel_stats.argtypes = [vp, C.POINTER(C.c_char_p), C.POINTER(C.c_double),
                                           C.POINTER(C.c_uint64), C.c_int]
        L.hoh_reset_kernel_stats.argtypes = [vp]
        L.hoh_reset_kernel_stats.restype = None
        L.hoh_ctx_set_option.argtypes = [vp, C.c_int, C.c_int64]
        L.hoh_ctx_stream.restype = vp
        L.hoh_ctx_stream.argtypes = [vp]
        L.hoh_encode_bound.restype = sz
        L.hoh_encode_bound.argtypes = [C.c_int, C.c_int]
        L.hoh_encode_image.argtypes = [vp, vp, C.c_int, C.c_int, C.c_int, vp, sz, szp, szp, vp]
        L.hoh_encode_image_ix.argtypes = [vp, vp, C.c_int, C.c_int, C.c_int, vp, sz, szp, szp, vp, vp]
        L.hoh_index_create.argtypes = [C.POINTER(vp)]
        L.hoh_index_destroy.argtypes = [vp]
        L.hoh_index_bytes.restype = sz
        L.hoh_index_bytes.argtypes = [vp]
        L.hoh_encode_tiles.argtypes = [vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, vp, sz, vp, szp, vp]
        L.hoh_file_prefix.restype = sz
        L.hoh_file_prefix.argtypes = [C.c_int, C.c_int, vp, C.c_int, vp, sz]
        L.hoh_tiling.argtypes = [C.c_int, C.c_int, ip, ip, ip, ip]
        L.hoh_peek_header.argtypes = [vp, sz, ip, ip, ip, ip]
        L.hoh_synth_rgb.argtypes = [vp, vp, C.c_int, C.c_int, C.c_uint64, C.c_int, vp]
        L.hoh_synth_rgb_rows.argtypes = [vp, vp, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_int, vp]
        L.hoh_natural_rgb_rows.argtypes = [vp, vp, C.c_int, C.c_int, C.c_int, C.c_uint64, vp]
        L.hoh_encode_tiles_ix.argtypes = [vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, vp, sz, vp, szp, vp, vp]
        L.hoh_encode_tiles_speed.argtypes = [vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp, sz, vp, szp,
                                             vp, vp]
        L.hoh_decode_tiles.argtypes = [vp, vp, sz, C.c_int, C.c_int, C.c_int, C.c_int, vp, vp, vp, vp]
        for name, args in (
            ("hoh_decode_image", [vp, vp, sz, vp, sz, ip, ip, vp]),
            ("hoh_decode_image_ix", [vp, vp, sz, vp, sz, ip, ip, vp, vp]),
            ("hoh_encode_image_async", [vp, vp, C.c_int, C.c_int, C.c_int, vp, sz, vp, vp, vp]),
            ("hoh_decode_image_async", [vp, vp, sz, C.c_int, C.c_int, vp, sz, vp, vp, vp]),
            ("hoh_encode_images_async", [vp, C.c_int, vp, C.c_int, C.c_int, C.c_int, vp, sz, vp, vp, vp]),
            ("hoh_decode_images_async", [vp, C.c_int, vp, sz, C.c_int, C.c_int, vp, vp, vp, vp]),
            ("hoh_encode_tiles_async", [vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp, sz, vp, vp, vp,
                                        vp]),
            ("hoh_decode_tiles_async", [vp, vp, sz, C.c_int, C.c_int, C.c_int, C.c_int, vp, vp, vp, vp, vp]),
            ("hoh_encode_tiles_images_async", [vp, C.c_int, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp, sz,
                                               vp, vp, vp, vp]),
            ("hoh_decode_tiles_images_async", [vp, C.c_int, vp, sz, C.c_int, C.c_int, C.c_int, C.c_int, vp, vp, vp,
                                               vp, vp]),
            ("hoh_mgpu_create", [C.POINTER(vp), C.c_int, ip]),
            ("hoh_mgpu_destroy", [vp]),
            ("hoh_mgpu_transport", [vp]),
            ("hoh_mgpu_encode_image", [vp, vp, C.c_int, C.c_int, C.c_int, vp, sz, szp, szp]),
            ("hoh_mgpu_decode_image", [vp, vp, sz, vp, sz, ip, ip]),
            ("hoh_encode_entropy", [vp, vp, sz, sz, C.c_uint32, vp, sz, szp]),
            ("hoh_decode_entropy", [vp, vp, sz, szp, vp, sz, szp]),
            ("hoh_entropy_count", [vp, sz, sz, szp]),
            ("hoh_entropy_parse", [vp, sz, sz, vp]),
            ("hoh_layer_encode", [vp, vp, sz, C.c_int, C.c_int, C.c_int, sz, vp, vp, sz, szp]),
            ("hoh_layer_decode", [vp, vp, sz, sz, C.c_int, C.c_int, C.c_int, vp, vp]),
            ("hoh_predict_fastpath", [vp, vp, C.c_int, C.c_int, C.c_int, vp]),
            ("hoh_unpredict_fastpath", [vp, vp, sz, vp, C.c_int, C.c_int, C.c_int, vp]),
            ("hoh_predict_section", [vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                     C.c_uint16, vp, szp]),
            ("hoh_predict_all", [vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp, vp]),
            ("hoh_unpredict_all", [vp, vp, sz, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp, vp]),
            ("hoh_subtract_green", [vp, vp, sz, vp, vp, vp]),
            ("hoh_add_green", [vp, vp, vp, vp, sz, vp]),
        ):
            if hasattr(L, name):
                getattr(L, name).argtypes = args
        if hasattr(L, "hoh_entropy_bound"):
            L.hoh_entropy_bound.restype = sz
            L.hoh_entropy_bound.argtypes = [sz, sz, C.c_uint32]
        _L = L
    return _L


def device_alloc_count():
    """hipMalloc calls the library has made so far (process-wide)."""
    return int(lib().hoh_device_alloc_count())


def check(code, what):
    if code != HOH_OK:
        raise HohError(code, what)


def _p(a):
    return a.ctypes.data_as(vp)


class Context:
    """One HIP device context (workspaces + stream).  Use one per thread per GPU."""

    def __init__(self, device=0):
        self.h = vp()
        check(lib().hoh_ctx_create(C.byref(self.h), device), "hoh_ctx_create")
        self.device = device

    def close(self):
        if self.h:
            lib().hoh_ctx_destroy(self.h)
            self.h = vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def profiling(self, on=True):
        lib().hoh_set_profiling(self.h, 1 if on else 0)

    def kernel_ms(self):
        names = (C.c_char_p * 64)()
        ms = (C.c_float * 64)()
        n = lib().hoh_get_kernel_ms(self.h, names, ms, 64)
        return [(names[i].decode(), ms[i]) for i in range(n)]

    def kernel_stats(self):
        """{stage: (total_ms, launches)} accumulated over profiled calls since reset_stats()."""
        names = (C.c_char_p * 64)()
        tot = (C.c_double * 64)()
        cnt = (C.c_uint64 * 64)()
        n = lib().hoh_get_kernel_stats(self.h, names, tot, cnt, 64)
        return {names[i].decode(): (tot[i], cnt[i]) for i in range(n)}

    def reset_stats(self):
        lib().hoh_reset_kernel_stats(self.h)

    def own_stream(self, torch):
        """The context's own HIP stream (hoh_ctx_stream) as a torch stream, for event fences."""
        if getattr(self, "_own", None) is None:
            self._own = torch.cuda.ExternalStream(int(lib().hoh_ctx_stream(self.h) or 0),
                                                  device=torch.device("cuda", self.device))
        return self._own

    def set_option(self, option, value):
        """hoh_ctx_set_option: e.g. set_option(OPT_NOIX_DECODER, NOIX_LANES)."""
        check(lib().hoh_ctx_set_option(self.h, option, value), "hoh_ctx_set_option")


# hoh_ctx_set_option (include/hoh_ans.h)
OPT_NOIX_DECODER = 1
NOIX_ADAPTIVE, NOIX_LANES, NOIX_MULTI, NOIX_WAVE = -1, 0, 1, 2


_CTX = None


def default_ctx():
    global _CTX
    if _CTX is None:
        _CTX = Context(0)
    return _CTX


def tiling(W, H):
    xt, yt, tw, th = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    tiled = lib().hoh_tiling(W, H, C.byref(xt), C.byref(yt), C.byref(tw), C.byref(th))
    return bool(tiled), xt.value, yt.value, tw.value, th.value


# ------------------------------------------------------------------ device-resident (torch) API

def _stream_ptr(torch, ctx):
    """torch's current stream as the call's stream.  torch's default stream is handle 0, which the
    C ABI reads as "the context's own stream" (include/hoh_ans.h), a stream torch does not order
    against; on it the call is fenced by events instead: the context's stream waits for the work
    torch has queued on the default stream (the call then sees the buffers torch filled), and
    _after_call makes the default stream wait for the call (torch then sees what it wrote).
    Neither side blocks the host or any other stream."""
    cur = torch.cuda.current_stream()
    if not cur.cuda_stream:
        ctx.own_stream(torch).wait_stream(cur)
    return vp(cur.cuda_stream)


def _after_call(torch, ctx):
    cur = torch.cuda.current_stream()
    if not cur.cuda_stream:
        cur.wait_stream(ctx.own_stream(torch))


class Index:
    """Decode side index (encoder checkpoints), kept beside the .hoh bytes."""

    def __init__(self):
        self.h = vp()
        check(lib().hoh_index_create(C.byref(self.h)), "hoh_index_create")

    def nbytes(self):
        return lib().hoh_index_bytes(self.h)

    def __del__(self):
        try:
            if self.h:
                lib().hoh_index_destroy(self.h)
        except Exception:
            pass


def encode_image(rgb_dev, W, H, out_dev=None, ctx=None, index=None, speed=0):
    """rgb_dev: uint8 torch tensor (W*H*3) in HBM; speed = choh's -sN.  Returns (out tensor, size,
    printed).  -s1..-s4 files carry no side index (they are undecodable by construction, Q14)."""
    import torch
    ctx = ctx or default_ctx()
    if out_dev is None:
        out_dev = torch.empty(lib().hoh_encode_bound(W, H), dtype=torch.uint8, device=rgb_dev.device)
    n, printed = C.c_size_t(0), C.c_size_t(0)
    r = lib().hoh_encode_image_ix(ctx.h, vp(rgb_dev.data_ptr()), W, H, speed, vp(out_dev.data_ptr()),
                                  out_dev.numel(), C.byref(n), C.byref(printed),
                                  index.h if index is not None else None, _stream_ptr(torch, ctx))
    check(r, "hoh_encode_image")
    _after_call(torch, ctx)
    return out_dev, n.value, printed.value


def decode_image(hoh_dev, size, out_dev=None, ctx=None, index=None):
    """hoh_dev: uint8 torch tensor holding `size` bytes of a .hoh.  Returns (rgb tensor, W, H)."""
    import torch
    ctx = ctx or default_ctx()
    head = hoh_dev[:min(size, 16)].cpu().numpy()
    W, H = peek_header(head.tobytes())[:2]
    if out_dev is None:
        out_dev = torch.empty(W * H * 3, dtype=torch.uint8, device=hoh_dev.device)
    w, h = C.c_int(), C.c_int()
    r = lib().hoh_decode_image_ix(ctx.h, vp(hoh_dev.data_ptr()), size, vp(out_dev.data_ptr()),
                                  out_dev.numel(), C.byref(w), C.byref(h),
                                  index.h if index is not None else None, _stream_ptr(torch, ctx))
    check(r, "hoh_decode_image")
    _after_call(torch, ctx)
    return out_dev, w.value, h.value


def encode_image_async(rgb_dev, W, H, out_dev, status_dev, ctx=None, index=None, speed=0):
    """Enqueue-only encode on the current stream (no host wait).  status_dev: int64 tensor of 2
    (device) receiving {HOH status code, .hoh size}; read it after synchronising the stream and
    pass it to check_status."""
    import torch
    ctx = ctx or default_ctx()
    r = lib().hoh_encode_image_async(ctx.h, vp(rgb_dev.data_ptr()), W, H, speed, vp(out_dev.data_ptr()),
                                     out_dev.numel(), index.h if index is not None else None,
                                     vp(status_dev.data_ptr()), _stream_ptr(torch, ctx))
    check(r, "hoh_encode_image_async")
    _after_call(torch, ctx)


def decode_image_async(hoh_dev, size, W, H, out_dev, status_dev, ctx=None, index=None):
    """Enqueue-only decode of a W x H .hoh (at most `size` bytes are read; a bound suffices) on
    the current stream.  status_dev receives {HOH status code, W*H*3}."""
    import torch
    ctx = ctx or default_ctx()
    r = lib().hoh_decode_image_async(ctx.h, vp(hoh_dev.data_ptr()), size, W, H, vp(out_dev.data_ptr()),
                                     out_dev.numel(), index.h if index is not None else None,
                                     vp(status_dev.data_ptr()), _stream_ptr(torch, ctx))
    check(r, "hoh_decode_image_async")
    _after_call(torch, ctx)


def encode_images_async(rgb_dev, n, W, H, out_dev, stride, status_dev, ctx=None, index=None, speed=0):
    """Enqueue-only encode of a batch: n contiguous W x H images (rgb_dev, n*W*H*3 bytes) into n
    files at out_dev + i*stride; status_dev: int64 tensor of 2n ({code, size} per image).  The
    kernels cover the whole batch per launch (hoh_encode_images_async)."""
    import torch
    ctx = ctx or default_ctx()
    assert out_dev.numel() >= n * stride and rgb_dev.numel() >= n * W * H * 3 and status_dev.numel() >= 2 * n
    r = lib().hoh_encode_images_async(ctx.h, n, vp(rgb_dev.data_ptr()), W, H, speed, vp(out_dev.data_ptr()), stride,
                                      index.h if index is not None else None, vp(status_dev.data_ptr()),
                                      _stream_ptr(torch, ctx))
    check(r, "hoh_encode_images_async")
    _after_call(torch, ctx)


def decode_images_async(hoh_dev, n, stride, W, H, out_dev, status_dev, ctx=None, index=None):
    """Enqueue-only decode of n files at hoh_dev + i*stride into n contiguous images (out_dev)."""
    import torch
    ctx = ctx or default_ctx()
    assert hoh_dev.numel() >= n * stride and out_dev.numel() >= n * W * H * 3 and status_dev.numel() >= 2 * n
    r = lib().hoh_decode_images_async(ctx.h, n, vp(hoh_dev.data_ptr()), stride, W, H, vp(out_dev.data_ptr()),
                                      index.h if index is not None else None, vp(status_dev.data_ptr()),
                                      _stream_ptr(torch, ctx))
    check(r, "hoh_decode_images_async")
    _after_call(torch, ctx)


def check_status(status, what):
    """status: the two u64 an async call wrote (any sequence); raises HohError on failure and
    returns the size word."""
    code, size = int(status[0]), int(status[1])
    check(code, what)
    return size


def encode_tiles(rgb_dev, W, H, t0, ntiles, out_dev, sizes_dev, ctx=None, index=None, row0=0, speed=0):
    """Encode tiles [t0, t0+ntiles) of a W x H image into a blob (concatenated tile byte strings).
    rgb_dev holds image rows from row0 on (a shard); only the named tiles' pixels are read.
    Returns the blob size; sizes_dev (uint32, device) receives each tile's size."""
    import torch
    ctx = ctx or default_ctx()
    n = C.c_size_t(0)
    base = rgb_dev.data_ptr() - row0 * W * 3
    r = lib().hoh_encode_tiles_speed(ctx.h, vp(base), W, H, speed, t0, ntiles, vp(out_dev.data_ptr()),
                                     out_dev.numel(), vp(sizes_dev.data_ptr()), C.byref(n),
                                     index.h if index is not None else None, _stream_ptr(torch, ctx))
    check(r, "hoh_encode_tiles")
    _after_call(torch, ctx)
    return n.value


def decode_tiles(blob_dev, size, W, H, t0, tile_sizes, out_dev, ctx=None, index=None, row0=0):
    """Inverse of encode_tiles: decodes the blob's tiles into out_dev (image rows from row0 on)."""
    import torch
    ctx = ctx or default_ctx()
    ts = np.ascontiguousarray(tile_sizes, dtype=np.uint32)
    base = out_dev.data_ptr() - row0 * W * 3
    r = lib().hoh_decode_tiles(ctx.h, vp(blob_dev.data_ptr()), size, W, H, t0, ts.size, _p(ts), vp(base),
                               index.h if index is not None else None, _stream_ptr(torch, ctx))
    check(r, "hoh_decode_tiles")
    _after_call(torch, ctx)


def encode_tiles_async(rgb_dev, W, H, t0, ntiles, out_dev, sizes_dev, status_dev, ctx=None, index=None, row0=0,
                       speed=0):
    """Enqueue-only encode_tiles on the current stream: the tile sizes land in sizes_dev (device)
    and {status, blob size} in status_dev (2 x int64, device); nothing waits on the host."""
    import torch
    ctx = ctx or default_ctx()
    base = rgb_dev.data_ptr() - row0 * W * 3
    r = lib().hoh_encode_tiles_async(ctx.h, vp(base), W, H, speed, t0, ntiles, vp(out_dev.data_ptr()),
                                     out_dev.numel(), vp(sizes_dev.data_ptr()), index.h if index is not None else None,
                                     vp(status_dev.data_ptr()), _stream_ptr(torch, ctx))
    check(r, "hoh_encode_tiles_async")
    _after_call(torch, ctx)


def decode_tiles_async(blob_dev, size, W, H, t0, ntiles, sizes_dev, out_dev, status_dev, ctx=None, index=None, row0=0):
    """Enqueue-only decode_tiles with the tile sizes in DEVICE memory (sizes_dev, as encode_tiles
    wrote them); {status, shard RGB bytes} land in status_dev."""
    import torch
    ctx = ctx or default_ctx()
    base = out_dev.data_ptr() - row0 * W * 3
    r = lib().hoh_decode_tiles_async(ctx.h, vp(blob_dev.data_ptr()), size, W, H, t0, ntiles, vp(sizes_dev.data_ptr()),
                                     vp(base), index.h if index is not None else None, vp(status_dev.data_ptr()),
                                     _stream_ptr(torch, ctx))
    check(r, "hoh_decode_tiles_async")
    _after_call(torch, ctx)


def encode_tiles_images_async(rgb_dev, n, W, H, t0, ntiles, out_dev, stride, sizes_dev, status_dev, ctx=None,
                              index=None, speed=0):
    """Enqueue-only encode of the same shard (tiles [t0, t0+ntiles), whole tile rows) of n images
    (hoh_encode_tiles_images_async): rgb_dev holds the n bands back to back, blob i goes to
    out_dev + i*stride, its tile sizes to sizes_dev[i*ntiles:(i+1)*ntiles] (int32/uint32, device),
    {status, blob size} per shard to status_dev (2n int64)."""
    import torch
    ctx = ctx or default_ctx()
    assert out_dev.numel() >= n * stride and sizes_dev.numel() >= n * ntiles and status_dev.numel() >= 2 * n
    r = lib().hoh_encode_tiles_images_async(ctx.h, n, vp(rgb_dev.data_ptr()), W, H, speed, t0, ntiles,
                                            vp(out_dev.data_ptr()), stride, vp(sizes_dev.data_ptr()),
                                            index.h if index is not None else None, vp(status_dev.data_ptr()),
                                            _stream_ptr(torch, ctx))
    check(r, "hoh_encode_tiles_images_async")
    _after_call(torch, ctx)


def decode_tiles_images_async(blob_dev, n, stride, W, H, t0, ntiles, sizes_dev, out_dev, status_dev, ctx=None,
                              index=None):
    """Inverse of encode_tiles_images_async: n blobs (tile sizes on the device) -> n bands back to
    back in out_dev; {status, band RGB bytes} per shard in status_dev."""
    import torch
    ctx = ctx or default_ctx()
    assert blob_dev.numel() >= n * stride and sizes_dev.numel() >= n * ntiles and status_dev.numel() >= 2 * n
    r = lib().hoh_decode_tiles_images_async(ctx.h, n, vp(blob_dev.data_ptr()), stride, W, H, t0, ntiles,
                                            vp(sizes_dev.data_ptr()), vp(out_dev.data_ptr()),
                                            index.h if index is not None else None, vp(status_dev.data_ptr()),
                                            _stream_ptr(torch, ctx))
    check(r, "hoh_decode_tiles_images_async")
    _after_call(torch, ctx)


def file_prefix(W, H, tile_sizes):
    ts = np.ascontiguousarray(tile_sizes, dtype=np.uint32)
    buf = np.empty(64 + 3 * ts.size, np.uint8)
    n = lib().hoh_file_prefix(W, H, _p(ts), ts.size, _p(buf), buf.size)
    if n == 0:
        raise HohError(1, "hoh_file_prefix")
    return buf[:n].tobytes()


def peek_header(data):
    b = np.frombuffer(bytes(data[:64]), np.uint8).copy()
    W, H, xt, yt = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    check(lib().hoh_peek_header(_p(b), b.size, C.byref(W), C.byref(H), C.byref(xt), C.byref(yt)), "hoh_peek_header")
    return W.value, H.value, xt.value, yt.value


def synth_rgb_dev(W, H, seed=1, noise=4, ctx=None, device="cuda", row0=0):
    """Synthetic image generated in HBM (same bytes as hoh_ans.synth.synth_rgb); with row0, rows
    [row0, row0+H) of the width-W global image (a shard)."""
    import torch
    ctx = ctx or default_ctx()
    t = torch.empty(W * H * 3, dtype=torch.uint8, device=device)
    check(lib().hoh_synth_rgb_rows(ctx.h, vp(t.data_ptr()), W, row0, H, seed, noise, _stream_ptr(torch, ctx)),
          "hoh_synth_rgb_rows")
    _after_call(torch, ctx)
    return t


def natural_rgb_dev(W, H, seed=1, ctx=None, device="cuda", row0=0):
    """Natural-statistic image generated in HBM (same bytes as hoh_ans.natural.natural_rgb);
    with row0, rows [row0, row0+H) of the width-W global image."""
    import torch
    ctx = ctx or default_ctx()
    t = torch.empty(W * H * 3, dtype=torch.uint8, device=device)
    check(lib().hoh_natural_rgb_rows(ctx.h, vp(t.data_ptr()), W, row0, H, seed, _stream_ptr(torch, ctx)),
          "hoh_natural_rgb_rows")
    _after_call(torch, ctx)
    return t


class MultiGPU:
    """choh / dhoh over several GPUs in one process (hoh_mgpu_*): a band of tile rows per device,
    one RCCL gather over xGMI into the file on the first device.  A device may repeat (the blobs
    then move by device copies: transport 0); distinct devices use RCCL (transport 1)."""

    def __init__(self, devices):
        self.h = vp()
        dv = (C.c_int * len(devices))(*devices)
        check(lib().hoh_mgpu_create(C.byref(self.h), len(devices), dv), "hoh_mgpu_create")
        self.devices = list(devices)

    def transport(self):
        return lib().hoh_mgpu_transport(self.h)

    def encode_image(self, rgb, speed=0):
        """(H, W, 3) uint8 host array -> (file bytes, printed size)."""
        import torch
        a = np.ascontiguousarray(rgb, dtype=np.uint8)
        H, W, _ = a.shape
        out = torch.empty(lib().hoh_encode_bound(W, H), dtype=torch.uint8, device="cuda:%d" % self.devices[0])
        n, printed = C.c_size_t(0), C.c_size_t(0)
        check(lib().hoh_mgpu_encode_image(self.h, _p(a), W, H, speed, vp(out.data_ptr()), out.numel(), C.byref(n),
                                          C.byref(printed)), "hoh_mgpu_encode_image")
        return out[:n.value].cpu().numpy().tobytes(), printed.value

    def decode_image(self, data):
        import torch
        b = torch.from_numpy(np.frombuffer(bytes(data), np.uint8).copy()).to("cuda:%d" % self.devices[0])
        W, H = peek_header(bytes(data[:64]))[:2]
        out = np.empty((H, W, 3), np.uint8)
        w, h = C.c_int(), C.c_int()
        check(lib().hoh_mgpu_decode_image(self.h, vp(b.data_ptr()), len(data), _p(out), out.size, C.byref(w),
                                          C.byref(h)), "hoh_mgpu_decode_image")
        return out

    def close(self):
        if self.h:
            lib().hoh_mgpu_destroy(self.h)
            self.h = vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------------------ host-buffer API (reference names)

def choh(rgb, ctx=None, speed=0):
    """`choh in out W H -sN` on an (H, W, 3) uint8 array -> (file bytes, printed size)."""
    import torch
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    H, W, _ = rgb.shape
    d = torch.from_numpy(rgb.reshape(-1)).cuda()
    out, n, printed = encode_image(d, W, H, ctx=ctx, speed=speed)
    torch.cuda.synchronize()
    return out[:n].cpu().numpy().tobytes(), printed


def dhoh(data, ctx=None, index=None):
    import torch
    b = torch.from_numpy(np.frombuffer(bytes(data), np.uint8).copy()).cuda()
    rgb, W, H = decode_image(b, len(data), ctx=ctx, index=index)
    torch.cuda.synchronize()
    return rgb.cpu().numpy().reshape(H, W, 3)


def encode_entropy(symbols, range_, prob_bits, ctx=None):
    ctx = ctx or default_ctx()
    s = np.ascontiguousarray(symbols, dtype=np.uint16)
    cap = lib().hoh_entropy_bound(s.size, range_, prob_bits)
    out = np.empty(cap, np.uint8)
    n = C.c_size_t(0)
    check(lib().hoh_encode_entropy(ctx.h, _p(s), s.size, range_, prob_bits, _p(out), cap, C.byref(n)),
          "hoh_encode_entropy")
    return out[:n.value].tobytes()


def decode_entropy(data, byte_pointer=0, ctx=None):
    ctx = ctx or default_ctx()
    b = np.frombuffer(bytes(data), np.uint8).copy()
    cnt = C.c_size_t(0)
    check(lib().hoh_entropy_count(_p(b), b.size, byte_pointer, C.byref(cnt)), "hoh_entropy_count")
    out = np.empty(max(cnt.value, 1), np.uint16)
    bp, n = C.c_size_t(byte_pointer), C.c_size_t(0)
    check(lib().hoh_decode_entropy(ctx.h, _p(b), b.size, C.byref(bp), _p(out), out.size, C.byref(n)),
          "hoh_decode_entropy")
    return out[:n.value], bp.value


class EntropyHeader(C.Structure):
    """hoh_entropy_header (include/hoh_ans.h)"""
    _fields_ = [("range", C.c_uint64), ("count", C.c_uint64), ("entropy_mode", C.c_uint32),
                ("prob_bits", C.c_uint32), ("table_mode", C.c_uint32), ("symbol_bits", C.c_uint32),
                ("table_end", C.c_uint64), ("payload_bytes", C.c_uint64), ("stream_end", C.c_uint64)]


def entropy_parse(data, byte_pointer=0):
    """Framing of one stream without decoding it (host only; decode_entropy_simple,
    entropy_decoding.hpp:8-132) -> dict of the hoh_entropy_header fields."""
    b = np.frombuffer(bytes(data), np.uint8).copy()
    h = EntropyHeader()
    check(lib().hoh_entropy_parse(_p(b), b.size, byte_pointer, C.byref(h)), "hoh_entropy_parse")
    return {f: int(getattr(h, f)) for f, _ in EntropyHeader._fields_}


def layer_encode(plane, depth, nuke=None, ctx=None, speed=0):
    """layer_encode (layer_encode.hpp:11-412) at cruncher_mode `speed` -> layer bytes."""
    ctx = ctx or default_ctx()
    p = np.ascontiguousarray(plane, dtype=np.uint16)
    h, w = p.shape
    nk = None if nuke is None else np.ascontiguousarray(nuke, dtype=np.uint8)
    cap = lib().hoh_entropy_bound(p.size, 1 << depth, 31) + 4096
    out = np.empty(cap, np.uint8)
    n = C.c_size_t(0)
    check(lib().hoh_layer_encode(ctx.h, _p(p), p.size, w, h, depth, speed, None if nk is None else _p(nk),
                                 _p(out), cap, C.byref(n)), "hoh_layer_encode")
    return out[:n.value].tobytes()


def layer_decode(data, w, h, depth, backref=None, pos=0, ctx=None):
    """decode_layer (layer_decode.hpp:128-278) -> (h, w) u16 plane (full depth)."""
    ctx = ctx or default_ctx()
    b = np.frombuffer(bytes(data), dtype=np.uint8).copy()
    br = None if backref is None else np.ascontiguousarray(backref, dtype=np.uint16)
    out = np.empty((h, w), np.uint16)
    check(lib().hoh_layer_decode(ctx.h, _p(b), b.size, pos, w, h, depth, None if br is None else _p(br), _p(out)),
          "hoh_layer_decode")
    return out


def predict_section(plane, depth, xt, yt, cx, cy, mask, ctx=None):
    """channelpredict_section (prediction.hpp:46-151) -> residuals of one cell."""
    ctx = ctx or default_ctx()
    p = np.ascontiguousarray(plane, dtype=np.uint16)
    h, w = p.shape
    out = np.empty(p.size + 64, np.uint16)
    k = C.c_size_t(0)
    check(lib().hoh_predict_section(ctx.h, _p(p), w, h, depth, xt, yt, cx, cy, mask, _p(out), C.byref(k)),
          "hoh_predict_section")
    return out[:k.value].copy()


def predict_all(plane, depth, xt, yt, tile_map, ctx=None):
    """channelpredict_all (prediction.hpp:153-229) -> residual plane (flat)."""
    ctx = ctx or default_ctx()
    p = np.ascontiguousarray(plane, dtype=np.uint16)
    tm = np.ascontiguousarray(tile_map, dtype=np.uint16)
    h, w = p.shape
    out = np.empty(p.size, np.uint16)
    check(lib().hoh_predict_all(ctx.h, _p(p), w, h, depth, xt, yt, _p(tm), _p(out)), "hoh_predict_all")
    return out


def unpredict_all(res, w, h, depth, xt, yt, tile_map, backref=None, ctx=None):
    """unpredict_all (unprediction.hpp:6-91) for any predictor map -> (h, w) plane."""
    ctx = ctx or default_ctx()
    r = np.ascontiguousarray(res, dtype=np.uint16)
    tm = np.ascontiguousarray(tile_map, dtype=np.uint16)
    br = None if backref is None else np.ascontiguousarray(backref, dtype=np.uint16)
    out = np.empty((h, w), np.uint16)
    check(lib().hoh_unpredict_all(ctx.h, _p(r), r.size, None if br is None else _p(br), w, h, depth, xt, yt, _p(tm),
                                  _p(out)), "hoh_unpredict_all")
    return out


def channelpredict_fastpath(plane, depth, ctx=None):
    ctx = ctx or default_ctx()
    p = np.ascontiguousarray(plane, dtype=np.uint16)
    h, w = p.shape
    out = np.empty_like(p)
    check(lib().hoh_predict_fastpath(ctx.h, _p(p), w, h, depth, _p(out)), "hoh_predict_fastpath")
    return out


def unpredict_fastpath(res, w, h, depth, backref=None, ctx=None):
    ctx = ctx or default_ctx()
    r = np.ascontiguousarray(res, dtype=np.uint16)
    br = None if backref is None else np.ascontiguousarray(backref, dtype=np.uint16)
    out = np.empty((h, w), np.uint16)
    check(lib().hoh_unpredict_fastpath(ctx.h, _p(r), r.size, None if br is None else _p(br), w, h, depth, _p(out)),
          "hoh_unpredict_fastpath")
    return out


def subtract_green(rgb, ctx=None):
    ctx = ctx or default_ctx()
    a = np.ascontiguousarray(rgb, dtype=np.uint8)
    n = a.size // 3
    G, R, B = (np.empty(n, np.uint16) for _ in range(3))
    check(lib().hoh_subtract_green(ctx.h, _p(a), n, _p(G), _p(R), _p(B)), "hoh_subtract_green")
    return G, R, B
