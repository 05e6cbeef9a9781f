"""Deterministic synthetic 8-bit RGB input.

Integer-only, so the numpy path here, the HIP generator in libhohgpu (hoh_synth_rgb) and
the committed fixtures all agree byte for byte:

    h     = splitmix64(seed * 0x100000001B3 + (y*W + x)*3 + c)
    base  = (((a_c*x + b_c*y) >> 8) + o_c) & 255            smooth gradient (saw-tooth wrap)
    noise = (h % (k+1)) + ((h >> 16) % (k+1)) - k            triangular, sigma = sqrt(k(k+2)/6)
    v     = clamp(base + noise, 0, 255)

k = 4 gives sigma = 2, the survey's smooth+noise image.  Uniform random bytes are not a valid
workload for the reference.
"""
import numpy as np

A = (37, 53, 29)
B = (23, 31, 47)
O = (10, 80, 160)
M64 = (1 << 64) - 1


def splitmix64(z):
    z = z + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def synth_rgb(W, H, seed=1, noise=4, rows_per_chunk=256):
    """Return a (H, W, 3) uint8 array."""
    out = np.empty((H, W, 3), dtype=np.uint8)
    k = np.uint64(noise + 1)
    salt = np.uint64((seed * 0x100000001B3) & M64)
    xs = np.arange(W, dtype=np.int64)
    with np.errstate(over="ignore"):
        for y0 in range(0, H, rows_per_chunk):
            y1 = min(H, y0 + rows_per_chunk)
            ys = np.arange(y0, y1, dtype=np.int64)[:, None]
            for c in range(3):
                base = (((A[c] * xs[None, :] + B[c] * ys) >> 8) + O[c]) & 255
                idx = ((ys * W + xs[None, :]) * 3 + c).astype(np.uint64)
                h = splitmix64(salt + idx)
                nz = (h % k).astype(np.int64) + ((h >> np.uint64(16)) % k).astype(np.int64) - noise
                out[y0:y1, :, c] = np.clip(base + nz, 0, 255).astype(np.uint8)
    return out
