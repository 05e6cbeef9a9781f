"""Test infrastructure: the checking build of the library (hoh-ans_amd/lib/libhohgpu_check.so, the
product sources compiled with -DHOH_DEBUG_READ -DHOH_KNOBS by `make`) and the exact recomputation
of k_lzsort's posting lists from what k_lzfp wrote.  Used by tests/test_gpu_check_build.py and
tools/scripts/lzsort_check.py; never by the product.

The posting lists (lz.hpp:35-53's candidate set at seek 10-14): per tile the
listed positions' keys pos | hash << 16 in ascending order (hash-major, position-minor: a stable
LSD sort by the 16-bit fingerprint hash), the sorted fingerprints and run ends beside them, and
the rank of every position (an unlisted flat-run position: the last listed entry of its group
before it)."""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHECK_LIB = os.path.join(ROOT, "hoh-ans_amd", "lib", "libhohgpu_check.so")

# StreamInfo (hoh-ans_amd/csrc/hoh_internal.h), 112 bytes
STREAM_DTYPE = np.dtype([("sym_off", "<u8"), ("slab_off", "<u8"), ("out_off", "<u8"), ("n", "<u4"), ("range", "<u4"),
                         ("pb", "<u4"), ("slab_cap", "<u4"), ("hdr_len", "<u4"), ("vlen", "<u4"), ("maxbits", "<u4"),
                         ("words", "<u4"), ("widx_end", "<u4"), ("mode", "<u4"), ("size", "<u4"), ("err", "<u4"),
                         ("expected_stored", "<u8"), ("fast", "<u4"), ("ckpt_off", "<u4"), ("drop", "<u4"),
                         ("clip", "<u4"), ("sizeonly", "<u4"), ("hist_src", "<u4"), ("wlo", "<u4"), ("whi", "<u4")])
assert STREAM_DTYPE.itemsize == 112
SM_RANS = 1


class CheckLib:
    """ctypes over the checking build: its own context, so it can sit beside hoh_ans's product
    library in one process (each library has its own HIP streams and workspaces)."""

    def __init__(self, path=CHECK_LIB):
        if not os.path.exists(path):
            raise RuntimeError("checking build missing: run `make` (%s)" % path)
        L = C.CDLL(path)
        vp = C.c_void_p
        L.hoh_ctx_create.argtypes = [C.POINTER(vp), C.c_int]
        L.hoh_ctx_destroy.argtypes = [vp]
        L.hoh_natural_rgb_rows.argtypes = [vp, vp, C.c_int, C.c_int, C.c_int, C.c_uint64, vp]
        L.hoh_encode_image.argtypes = [vp, vp, C.c_int, C.c_int, C.c_int, vp, C.c_size_t, C.POINTER(C.c_size_t),
                                       C.POINTER(C.c_size_t), vp]
        L.hoh_encode_bound.restype = C.c_size_t
        L.hoh_encode_bound.argtypes = [C.c_int, C.c_int]
        L.hoh_debug_read.argtypes = [vp, C.c_int, vp, C.c_size_t]
        self.L = L
        self.h = vp()
        r = L.hoh_ctx_create(C.byref(self.h), 0)
        if r:
            raise RuntimeError("hoh_ctx_create: %d" % r)

    def close(self):
        if self.h:
            self.L.hoh_ctx_destroy(self.h)
            self.h = C.c_void_p()

    def natural(self, W, H, seed, torch):
        t = torch.empty(W * H * 3, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        r = self.L.hoh_natural_rgb_rows(self.h, C.c_void_p(t.data_ptr()), W, 0, H, seed, None)
        assert r == 0, r
        return t

    def encode(self, rgb, W, H, speed, torch):
        """synchronous encode on the context's own stream -> (file bytes)"""
        out = torch.empty(self.L.hoh_encode_bound(W, H), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        n, printed = C.c_size_t(0), C.c_size_t(0)
        r = self.L.hoh_encode_image(self.h, C.c_void_p(rgb.data_ptr()), W, H, speed, C.c_void_p(out.data_ptr()),
                                    out.numel(), C.byref(n), C.byref(printed), None)
        assert r == 0, r
        return out[:n.value].cpu().numpy().tobytes()

    def read(self, which, arr):
        r = self.L.hoh_debug_read(self.h, which, arr.ctypes.data, arr.nbytes)
        assert r == 0, "hoh_debug_read(%d): %d" % (which, r)
        return arr

    def streams(self, count):
        return self.read(6, np.zeros(count, STREAM_DTYPE))


def check_posting_lists(fpb, lzs, ntiles, cap):
    """fpb: k_lzfp's workspace (u32: fingerprints F, tile pixel words | run8 << 24, transposed F,
    then run8 as u8); lzs: k_lzsort's (8-byte entries key | fingerprint << 32, first-pass entries,
    u16 ranks, u16 run ends).  Returns (bad tile mask, keys bad, fingerprints bad, ranks bad)."""
    per = ntiles * cap
    ar = np.arange(cap, dtype=np.int64)[None, :]
    F = fpb[:per].reshape(ntiles, cap)
    TP = fpb[per:2 * per].reshape(ntiles, cap) & 0xffffff                    # rgb | run8 << 24
    R8 = fpb[3 * per:].view(np.uint8)[:per].reshape(ntiles, cap)
    S = lzs[:2 * per:2].reshape(ntiles, cap)
    T = lzs[1:2 * per:2].reshape(ntiles, cap)                                 # the sorted fingerprints
    R = lzs[4 * per:].view(np.uint16)[:per].reshape(ntiles, cap)
    E = lzs[4 * per:].view(np.uint16)[per:2 * per].reshape(ntiles, cap)
    start = np.ones_like(TP, dtype=bool)
    start[:, 1:] = TP[:, 1:] != TP[:, :-1]
    inner = (R8 >= 4) & ~start
    h = ((F.astype(np.uint64) * 0x9E3779B1) & 0xffffffff) >> 16
    key = np.where(inner, np.uint64(1 << 32) + ar.astype(np.uint64), (h << 16) | ar.astype(np.uint64))
    order = np.argsort(key, axis=1, kind="stable")
    sk = np.take_along_axis(key, order, axis=1)
    del order
    nl = (~inner).sum(axis=1)
    listed = ar < nl[:, None]
    pos = (sk & 0xffff).astype(np.int64)
    bad_s = np.any(listed & (S != (sk & 0xffffffff).astype(np.uint32)), axis=1)
    bad_t = np.any(listed & (T != np.take_along_axis(F, pos, axis=1)), axis=1)
    nxt = np.minimum.accumulate(np.where(start, ar, cap)[:, ::-1], axis=1)[:, ::-1]
    runend = np.empty_like(nxt)
    runend[:, :-1] = nxt[:, 1:] - 1
    runend[:, -1] = cap - 1
    want_e = np.where(np.take_along_axis(R8, pos, axis=1) >= 4, np.take_along_axis(runend, pos, axis=1), pos)
    bad_e = np.any(listed & (E != want_e), axis=1)
    rank = np.zeros((ntiles, cap + 1), np.int64)                        # column cap: unlisted slots
    np.put_along_axis(rank, np.where(listed, pos, cap), np.broadcast_to(ar, pos.shape), axis=1)
    want_r = rank[:, :cap].copy()
    for tb in range(ntiles):
        lk = sk[tb, :nl[tb]]
        iq = np.flatnonzero(inner[tb])
        want_r[tb, iq] = np.searchsorted(lk, (h[tb, iq] << np.uint64(16)) | iq.astype(np.uint64)) - 1
    bad_r = np.any(R != want_r, axis=1)
    bad_s |= bad_e
    return bad_s | bad_t | bad_r, bad_s, bad_t, bad_r
