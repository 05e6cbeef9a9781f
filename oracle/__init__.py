"""TEST INFRASTRUCTURE ONLY -- ctypes access to the CPU oracle and to the reference.

* ``lib()``  -> oracle/liboracle.so, the plain-C restatement (oracle/hoh_oracle.c).
* ``ref()``  -> oracle/_ref/libref.so, the reference's own headers compiled in place
  (oracle/ref/Makefile); None when it has not been built (e.g. a fresh clone on the GPU box).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
The product library never does.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_REF = None

u8p = C.POINTER(C.c_uint8)
u16p = C.POINTER(C.c_uint16)
u32p = C.POINTER(C.c_uint32)
szp = C.POINTER(C.c_size_t)


def build():
    """Compile the oracle (always) and the reference harness (when /root/reference exists)."""
    so = os.path.join(HERE, "liboracle.so")
    src = os.path.join(HERE, "hoh_oracle.c")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", "-o", so, src, "-lm"])
    if os.path.isdir("/root/reference"):
        subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "ref"), "all"])
        # the reference's own callers against the drop-in headers + libhohgpu (needs the library)
        if os.path.exists(os.path.join(os.path.dirname(HERE), "hoh-ans_amd", "lib", "libhohgpu.so")):
            subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "ref"), "dropin"])


def _p(a, t):
    return a.ctypes.data_as(t)


def lib():
    global _LIB
    if _LIB is None:
        so = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(so):
            build()
        L = C.CDLL(so)
        L.or_encode_entropy.restype = C.c_long
        L.or_encode_entropy.argtypes = [u16p, C.c_size_t, C.c_size_t, C.c_uint32, u8p]
        L.or_entropy_bound.restype = C.c_size_t
        L.or_entropy_bound.argtypes = [C.c_size_t, C.c_size_t, C.c_uint32]
        L.or_decode_entropy.restype = C.c_long
        L.or_decode_entropy.argtypes = [u8p, C.c_size_t, szp, u16p, C.c_size_t]
        L.or_peek_count.restype = C.c_long
        L.or_peek_count.argtypes = [u8p, C.c_size_t, C.c_size_t]
        L.or_normalize_freqs.restype = C.c_int
        L.or_normalize_freqs.argtypes = [u32p, u32p, C.c_size_t, C.c_uint32]
        L.or_predict_fastpath.argtypes = [u16p, C.c_int, C.c_int, C.c_int, u16p]
        L.or_unpredict_fastpath.restype = C.c_long
        L.or_unpredict_fastpath.argtypes = [u16p, C.c_size_t, u16p, C.c_int, C.c_int, C.c_int, u16p]
        L.or_subtract_green.argtypes = [u8p, C.c_size_t, u16p, u16p, u16p]
        L.or_count_colours.restype = C.c_int
        L.or_count_colours.argtypes = [u8p, C.c_size_t]
        L.or_find_lz_rgb.restype = C.c_long
        L.or_find_lz_rgb.argtypes = [u8p, C.c_size_t, C.c_int, C.c_int, u8p, u8p, C.c_int, C.c_int]
        L.or_layer_encode_s0.restype = C.c_long
        L.or_layer_encode_s0.argtypes = [u16p, C.c_size_t, C.c_int, C.c_int, C.c_int, u8p, u8p]
        L.or_encode_tile_s0.restype = C.c_long
        L.or_encode_tile_s0.argtypes = [u8p, C.c_int, C.c_int, u8p, C.c_size_t]
        L.or_tile_bound.restype = C.c_size_t
        L.or_tile_bound.argtypes = [C.c_int, C.c_int]
        L.or_choh_s0.restype = C.c_long
        L.or_choh_s0.argtypes = [u8p, C.c_int, C.c_int, u8p, C.c_size_t, szp]
        L.or_layer_encode.restype = C.c_long
        L.or_layer_encode.argtypes = [u16p, C.c_size_t, C.c_int, C.c_int, C.c_int, C.c_int, u8p, u8p]
        L.or_encode_tile.restype = C.c_long
        L.or_encode_tile.argtypes = [u8p, C.c_int, C.c_int, C.c_int, u8p, C.c_size_t]
        L.or_choh.restype = C.c_long
        L.or_choh.argtypes = [u8p, C.c_int, C.c_int, C.c_int, u8p, C.c_size_t, szp]
        L.or_predict_section.restype = C.c_size_t
        L.or_predict_section.argtypes = [u16p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                         C.c_uint16, u16p]
        L.or_predict_all.argtypes = [u16p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, u16p, u16p]
        L.or_unpredict_all.restype = C.c_long
        L.or_unpredict_all.argtypes = [u16p, C.c_size_t, u16p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, u16p, u16p]
        L.or_choh_bound.restype = C.c_size_t
        L.or_choh_bound.argtypes = [C.c_int, C.c_int]
        L.or_dhoh.restype = C.c_long
        L.or_dhoh.argtypes = [u8p, C.c_size_t, u8p, C.c_size_t, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.or_esym_init.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32]
        _LIB = L
    return _LIB


def ref():
    global _REF
    if _REF is None:
        so = os.path.join(HERE, "_ref", "libref.so")
        if not os.path.exists(so):
            return None
        R = C.CDLL(so)
        R.ref_encode_entropy.restype = C.c_size_t
        R.ref_encode_entropy.argtypes = [u16p, C.c_size_t, C.c_size_t, C.c_uint32, u8p]
        R.ref_decode_entropy.restype = C.c_size_t
        R.ref_decode_entropy.argtypes = [u8p, C.c_size_t, C.c_size_t, u16p, C.c_size_t]
        R.ref_normalize_freqs.argtypes = [u32p, u32p, C.c_size_t, C.c_uint32]
        R.ref_esym_init.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64), u32p, u32p, u32p]
        R.ref_enc_put.restype = C.c_uint64
        R.ref_enc_put.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_int64)]
        R.ref_channelpredict_fastpath.argtypes = [u16p, C.c_int, C.c_int, C.c_int, u16p]
        R.ref_unpredict_all.argtypes = [u16p, C.c_int, C.c_int, C.c_int, C.c_uint16, u16p, u16p]
        R.ref_channelpredict_section.restype = C.c_size_t
        R.ref_channelpredict_section.argtypes = [u16p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                                 C.c_int, C.c_uint16, u16p]
        R.ref_unpredict_map.argtypes = [u16p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, u16p, u16p, u16p]
        R.ref_channelpredict_all.argtypes = [u16p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, u16p, u16p]
        R.ref_subtract_green.argtypes = [u8p, C.c_size_t, u16p, u16p, u16p]
        R.ref_count_colours.restype = C.c_int
        R.ref_count_colours.argtypes = [u8p, C.c_size_t]
        R.ref_find_lz_rgb.restype = C.c_size_t
        R.ref_find_lz_rgb.argtypes = [u8p, C.c_size_t, C.c_int, C.c_int, u8p, u8p, C.c_int, C.c_int]
        R.ref_layer_encode.restype = C.c_size_t
        R.ref_layer_encode.argtypes = [u16p, C.c_size_t, C.c_int, C.c_int, C.c_int, C.c_size_t, u8p, u8p]
        R.ref_encode_tile.restype = C.c_size_t
        R.ref_encode_tile.argtypes = [u8p, C.c_int, C.c_int, C.c_size_t, u8p]
        _REF = R
    return _REF


def ref_bin(name):
    p = os.path.join(HERE, "_ref", name)
    return p if os.path.exists(p) else None


# ------------------------------------------------------------------ numpy-level helpers (oracle)

class OracleError(RuntimeError):
    def __init__(self, code):
        self.code = int(code)
        super().__init__("oracle error %d" % self.code)


def encode_entropy(sym, rng, pb):
    sym = np.ascontiguousarray(sym, dtype=np.uint16)
    L = lib()
    out = np.empty(L.or_entropy_bound(sym.size, rng, pb), dtype=np.uint8)
    r = L.or_encode_entropy(_p(sym, u16p), sym.size, rng, pb, _p(out, u8p))
    if r < 0:
        raise OracleError(r)
    return out[:r].tobytes()


def decode_entropy(data, bp=0):
    """-> (symbols uint16 array, new byte pointer)"""
    buf = np.frombuffer(bytes(data), dtype=np.uint8).copy()
    L = lib()
    n = L.or_peek_count(_p(buf, u8p), buf.size, bp)
    if n < 0:
        raise OracleError(n)
    out = np.empty(max(n, 1), dtype=np.uint16)
    p = C.c_size_t(bp)
    r = L.or_decode_entropy(_p(buf, u8p), buf.size, C.byref(p), _p(out, u16p), n)
    if r < 0:
        raise OracleError(r)
    return out[:r], p.value


def normalize_freqs(freqs, target):
    f = np.ascontiguousarray(freqs, dtype=np.uint32).copy()
    cum = np.zeros(f.size + 1, dtype=np.uint32)
    r = lib().or_normalize_freqs(_p(f, u32p), _p(cum, u32p), f.size, target)
    if r < 0:
        raise OracleError(r)
    return f, cum


def predict_fastpath(plane, depth):
    plane = np.ascontiguousarray(plane, dtype=np.uint16)
    h, w = plane.shape
    out = np.empty_like(plane)
    lib().or_predict_fastpath(_p(plane, u16p), w, h, depth, _p(out, u16p))
    return out


def unpredict_fastpath(res, w, h, depth, backref=None):
    res = np.ascontiguousarray(res, dtype=np.uint16)
    out = np.empty((h, w), dtype=np.uint16)
    br = None if backref is None else np.ascontiguousarray(backref, dtype=np.uint16)
    r = lib().or_unpredict_fastpath(_p(res, u16p), res.size, None if br is None else _p(br, u16p),
                                    w, h, depth, _p(out, u16p))
    if r < 0:
        raise OracleError(r)
    return out


def subtract_green(rgb):
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    n = rgb.size // 3
    G = np.empty(n, np.uint16); R = np.empty(n, np.uint16); B = np.empty(n, np.uint16)
    lib().or_subtract_green(_p(rgb, u8p), n, _p(G, u16p), _p(R, u16p), _p(B, u16p))
    return G, R, B


def encode_tile(rgb, speed=0):
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    h, w, _ = rgb.shape
    L = lib()
    cap = L.or_tile_bound(w, h)
    out = np.empty(cap, np.uint8)
    r = L.or_encode_tile(_p(rgb, u8p), w, h, speed, _p(out, u8p), cap)
    if r < 0:
        raise OracleError(r)
    return out[:r].tobytes()


def choh(rgb, speed=0):
    """-> (file bytes, printed size) exactly as `choh in out W H -sN` (SURVEY Q13 included)."""
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    H, W, _ = rgb.shape
    L = lib()
    cap = L.or_choh_bound(W, H)
    out = np.empty(cap, np.uint8)
    printed = C.c_size_t(0)
    r = L.or_choh(_p(rgb, u8p), W, H, speed, _p(out, u8p), cap, C.byref(printed))
    if r < 0:
        raise OracleError(r)
    return out[:r].tobytes(), printed.value


def predict_section(plane, depth, xt, yt, cx, cy, mask):
    plane = np.ascontiguousarray(plane, dtype=np.uint16)
    h, w = plane.shape
    out = np.empty(w * h, np.uint16)
    k = lib().or_predict_section(_p(plane, u16p), w, h, depth, xt, yt, cx, cy, mask, _p(out, u16p))
    return out[:k].copy()


def predict_all(plane, depth, xt, yt, tile_map):
    plane = np.ascontiguousarray(plane, dtype=np.uint16)
    tm = np.ascontiguousarray(tile_map, dtype=np.uint16)
    h, w = plane.shape
    out = np.empty(w * h, np.uint16)
    lib().or_predict_all(_p(plane, u16p), w, h, depth, xt, yt, _p(tm, u16p), _p(out, u16p))
    return out


def unpredict_all(res, w, h, depth, xt, yt, tile_map, backref=None):
    r = np.ascontiguousarray(res, dtype=np.uint16)
    tm = np.ascontiguousarray(tile_map, dtype=np.uint16)
    br = None if backref is None else np.ascontiguousarray(backref, dtype=np.uint16)
    out = np.empty((h, w), np.uint16)
    k = lib().or_unpredict_all(_p(r, u16p), r.size, None if br is None else _p(br, u16p), w, h, depth, xt, yt,
                               _p(tm, u16p), _p(out, u16p))
    if k < 0:
        raise OracleError(k)
    return out


def layer_encode(plane, depth, speed, nuke=None):
    plane = np.ascontiguousarray(plane, dtype=np.uint16)
    h, w = plane.shape
    n = w * h
    L = lib()
    out = np.empty(L.or_entropy_bound(n, 1 << depth, 31) + 4096, np.uint8)
    nk = None if nuke is None else np.ascontiguousarray(nuke, dtype=np.uint8)
    r = L.or_layer_encode(_p(plane, u16p), n, w, h, depth, speed, None if nk is None else _p(nk, u8p), _p(out, u8p))
    if r < 0:
        raise OracleError(r)
    return out[:r].tobytes()


def dhoh(data):
    buf = np.frombuffer(bytes(data), dtype=np.uint8).copy()
    L = lib()
    Wp, Hp = C.c_int(0), C.c_int(0)
    cap = 3 << 30 if buf.size > 16 else 64
    # read W, H first (header varints) to size the output
    probe = np.empty(1, np.uint8)
    r = L.or_dhoh(_p(buf, u8p), buf.size, _p(probe, u8p), 0, C.byref(Wp), C.byref(Hp))
    if r not in (0, -6):
        raise OracleError(r)
    out = np.empty((Hp.value, Wp.value, 3), np.uint8)
    r = L.or_dhoh(_p(buf, u8p), buf.size, _p(out, u8p), out.size, C.byref(Wp), C.byref(Hp))
    if r < 0:
        raise OracleError(r)
    return out
