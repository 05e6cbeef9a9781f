"""Deterministic "natural-statistic" 8-bit RGB (BASELINE.json configs[4]).

The gradient + noise image of synth.py barely exercises the -s1..-s4 predictor search
(layer_encode.hpp:122-319): every 40-px cell of a linear gradient prefers the same predictor.  This
generator gives the search something to decide between -- piecewise-smooth regions with
irregular hard edges, textured patches, flat runs and short repeating patterns -- while staying
integer-only, so numpy here, the HIP kernel in libhohgpu (hoh_natural_rgb, k_util.hip) and the
committed golden vectors agree byte for byte.

    h(k, a, b)   = splitmix64(salt + (k << 48) + (a << 24) + b),  salt = seed * 0xD6E8FEB86659FD93
    V(k, lg, m)  = bilinear value noise on a grid of spacing 2^lg, node values h(k, gx, gy) & m
    R            = V(1, 7, 1023) + V(2, 4, 127)                    region field (128-px blobs, warped)
    rk           = h(3, R >> 6, ((x >> 9) << 12) | (y >> 9))      region key: contour bands of R,
                                                                  cut again along a 512-px grid
    Lf           = 2 V(4, 8, 255) + V(5, 6, 255) + V(6, 3, 63);  L = (Lf * 79) >> 8   luma field
    T            = V(8, 2, 63) - 32                               fine texture (4-px grid)
    hp           = h(7, x, y)                                     per-pixel noise bits
    nl = (hp & 7) + ((hp >> 3) & 7) - 7          luma noise, shared by the three channels
    nc = +-1 on a quarter of the pixels, per channel   (bits 6+2c, 12+c)
    nb = ((hp >> 16) & 63) - 32                  texture grain
    base = (rk >> 8) & 255; chroma R = ((rk >> 16) & 63) - 32 (0 -> 9), G = 0, B = ((rk >> 22) & 63) - 32
    region type t = rk & 7:
      0      flat                 v = base + ch
      1..3   smooth               v = base + ch + (((L - 128) * gain) >> 2) + nl + nc,  gain = (rk >> 28) & 7
      4..5   textured             v = base + ch + T + (nb >> 1) + nc
      6      ramp                 v = base + ch + (((x & 511) * sx + (y & 511) * sy) >> 7) + (nl >> 1)
      7      4-px checkerboard    v = base + ch + 48 * (((x >> 2) + (y >> 2)) & 1)
    v = clamp(v, 0, 255)

Shifts of negative values are arithmetic (numpy int64 and the kernel's signed 64-bit).  Every
tile of the seeds used here has more than 256 colours and is not grey, so -s0 files decode
(palette and grey tiles are the reference's undecodable / unreproducible cases).
"""
import numpy as np

from .synth import splitmix64

M64 = (1 << 64) - 1
SALT_MUL = 0xD6E8FEB86659FD93


def _salt(seed):
    return np.uint64((seed * SALT_MUL) & M64)


def _h(salt, k, a, b):
    a = np.asarray(a, dtype=np.uint64)
    b = np.asarray(b, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return splitmix64(salt + np.uint64(k << 48) + (a << np.uint64(24)) + b)


def _vnoise(salt, k, lg, m, xs, ys):
    """Value noise at integer pixel coords xs (1-D, columns) x ys (1-D, rows) -> (len(ys), len(xs))."""
    S = 1 << lg
    gx0, gy0 = int(xs.min()) >> lg, int(ys.min()) >> lg
    gx1, gy1 = (int(xs.max()) >> lg) + 1, (int(ys.max()) >> lg) + 1
    gx = np.arange(gx0, gx1 + 1, dtype=np.int64)
    gy = np.arange(gy0, gy1 + 1, dtype=np.int64)
    G = (_h(salt, k, gx[None, :], gy[:, None]) & np.uint64(m)).astype(np.int64)   # [gy][gx]
    ix = (xs >> lg) - gx0
    iy = (ys >> lg) - gy0
    fx = (xs & (S - 1))[None, :]
    fy = (ys & (S - 1))[:, None]
    v00 = G[iy[:, None], ix[None, :]]
    v10 = G[iy[:, None], ix[None, :] + 1]
    v01 = G[iy[:, None] + 1, ix[None, :]]
    v11 = G[iy[:, None] + 1, ix[None, :] + 1]
    top = v00 * (S - fx) + v10 * fx
    bot = v01 * (S - fx) + v11 * fx
    return (top * (S - fy) + bot * fy) >> (2 * lg)


def natural_rgb(W, H, seed=1, row0=0, rows=None, rows_per_chunk=256):
    """Rows [row0, row0 + rows) of the W-wide natural image as a (rows, W, 3) uint8 array."""
    rows = H - row0 if rows is None else rows
    out = np.empty((rows, W, 3), dtype=np.uint8)
    salt = _salt(seed)
    xs = np.arange(W, dtype=np.int64)
    for r0 in range(0, rows, rows_per_chunk):
        ys = np.arange(row0 + r0, row0 + min(rows, r0 + rows_per_chunk), dtype=np.int64)
        X = xs[None, :]
        Y = ys[:, None]
        R = _vnoise(salt, 1, 7, 1023, xs, ys) + _vnoise(salt, 2, 4, 127, xs, ys)
        blk = ((X >> 9) << 12) | (Y >> 9)
        rk = _h(salt, 3, (R >> 6).astype(np.uint64), np.broadcast_to(blk, R.shape).astype(np.uint64))
        Lf = 2 * _vnoise(salt, 4, 8, 255, xs, ys) + _vnoise(salt, 5, 6, 255, xs, ys) + _vnoise(salt, 6, 3, 63, xs, ys)
        L = (Lf * 79) >> 8
        T = _vnoise(salt, 8, 2, 63, xs, ys) - 32
        hp = _h(salt, 7, np.broadcast_to(X, R.shape), np.broadcast_to(Y, R.shape))
        u = lambda v, s, m: ((v >> np.uint64(s)) & np.uint64(m)).astype(np.int64)   # noqa: E731
        t = u(rk, 0, 7)
        base = u(rk, 8, 255)
        chR = u(rk, 16, 63) - 32
        chR = np.where(chR == 0, 9, chR)
        chB = u(rk, 22, 63) - 32
        gain = u(rk, 28, 7)
        sx = u(rk, 32, 63) - 32
        sy = u(rk, 38, 63) - 32
        nl = u(hp, 0, 7) + u(hp, 3, 7) - 7
        nb = u(hp, 16, 63) - 32
        smooth = ((L - 128) * gain) >> 2
        ramp = ((X & 511) * sx + (Y & 511) * sy) >> 7
        checker = 48 * (((X >> 2) + (Y >> 2)) & 1)
        for c, ch in ((0, chR), (1, 0), (2, chB)):
            nc = np.where(u(hp, 6 + 2 * c, 3) == 0, u(hp, 12 + c, 1) * 2 - 1, 0)
            v = base + ch
            v = v + np.select([t == 0, t <= 3, t <= 5, t == 6],
                              [0, smooth + nl + nc, T + (nb >> 1) + nc, ramp + (nl >> 1)],
                              np.broadcast_to(checker, t.shape))
            out[r0:r0 + len(ys), :, c] = np.clip(v, 0, 255).astype(np.uint8)
    return out


def tile_stats(img, tile=256):
    """(palette-candidate tiles, grey tiles) of an image under the reference's tiling."""
    H, W, _ = img.shape
    pal = grey = 0
    for ty in range(H // tile):
        for tx in range(W // tile):
            t = img[ty * tile:(ty + 1) * tile, tx * tile:(tx + 1) * tile].reshape(-1, 3)
            if (t[:, 0] == t[:, 1]).all() and (t[:, 1] == t[:, 2]).all():
                grey += 1
            code = (t[:, 0].astype(np.uint32) << 16) | (t[:, 1].astype(np.uint32) << 8) | t[:, 2]
            if len(np.unique(code)) <= 256:
                pal += 1
    return pal, grey
