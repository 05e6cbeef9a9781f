"""Deterministic input generators for the golden vectors (integer-only, numpy-version stable).

Every fixture in golden.json names its generator + parameters; tests regenerate the input and
check the recorded output (bytes for small cases, sha256 + length for large ones).
"""
import numpy as np

from hoh_ans.synth import splitmix64, synth_rgb  # noqa: F401  (re-exported for tests)

M64 = (1 << 64) - 1


def u64_stream(seed, n):
    with np.errstate(over="ignore"):
        idx = np.arange(n, dtype=np.uint64)
        return splitmix64(np.uint64((seed * 0x9E3779B97F4A7C15) & M64) + idx)


def laplace_symbols(seed, n, rng, scale_x16):
    """Two-sided geometric residuals centred on rng//2 (mod rng): |d| ~ floor(-scale*ln(u))."""
    h = u64_stream(seed, n)
    u = ((h >> np.uint64(11)).astype(np.float64) + 0.5) / float(1 << 53)
    mag = np.floor(-(scale_x16 / 16.0) * np.log(u)).astype(np.int64)
    sign = np.where((h & np.uint64(1)) == 1, 1, -1)
    return ((rng // 2 + sign * mag) % rng).astype(np.uint16)


def uniform_symbols(seed, n, rng):
    return (u64_stream(seed, n) % np.uint64(rng)).astype(np.uint16)


def const_symbols(n, value):
    return np.full(n, value, dtype=np.uint16)


def few_symbols(seed, n, rng, k):
    """only k distinct symbols, skewed"""
    h = u64_stream(seed, n)
    pick = (h % np.uint64(k * (k + 1) // 2)).astype(np.int64)
    sym = np.zeros(n, np.int64)
    acc = 0
    for j in range(k):
        acc += k - j
        sym = np.where((pick < acc) & (sym == 0) & (pick >= acc - (k - j)), (j * 37 + 5) % rng, sym)
    return sym.astype(np.uint16)


def make_symbols(spec):
    kind = spec["kind"]
    n, rng = spec["n"], spec["range"]
    if kind == "laplace":
        return laplace_symbols(spec["seed"], n, rng, spec["scale_x16"])
    if kind == "uniform":
        return uniform_symbols(spec["seed"], n, rng)
    if kind == "const":
        return const_symbols(n, spec["value"])
    if kind == "few":
        return few_symbols(spec["seed"], n, rng, spec["k"])
    raise ValueError(kind)


def make_image(spec):
    return synth_rgb(spec["W"], spec["H"], spec["seed"], spec["noise"])


def make_plane(spec):
    img = make_image(spec)
    from oracle import subtract_green  # test infrastructure
    G, R, B = subtract_green(img)
    p = {"G": G, "R": R, "B": B}[spec["plane"]]
    return p.reshape(spec["H"], spec["W"])
