"""Deterministic synthetic inputs shared by the golden generator and the tests.

Pure numpy; no dependence on the oracle or on the product.  Vectors come from
splitmix64 (seed 0x5EED for SpMV x, as SURVEY.md 8(c) prescribes) mapped to
uniform [-1, 1); all-ones vectors would hide gather bugs.
"""
from __future__ import annotations

import hashlib

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(seed: int, n: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        s = (np.uint64(seed) + np.arange(1, n + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15))
        z = s
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(seed: int, n: int) -> np.ndarray:
    """uniform [-1, 1) doubles, 53-bit resolution"""
    u = (splitmix64(seed, n) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    return 2.0 * u - 1.0


def rand_csr(n: int, per_row: int, seed: int, unsorted=True, missing_diag_every=0, diag=4.0):
    """Nonsymmetric random sparse matrix (edge cases for ILU setup).

    Rows hold the diagonal plus up to per_row off-diagonal columns; columns are
    written in a scrambled order when ``unsorted`` (exercises the solver's
    column sort, matrix-utils.cxx:387-481); every ``missing_diag_every``-th row
    omits its diagonal (exercises adjust_zero_diag, matrix-utils.cxx:483-587).
    """
    r = splitmix64(seed, n * (per_row + 2))
    Ap = [0]
    Aj, Ax = [], []
    k = 0
    for i in range(n):
        cols = {}
        for _ in range(per_row):
            c = int(r[k] % np.uint64(n))
            k += 1
            if c != i:
                cols[c] = float((int(r[k % len(r)] >> np.uint64(11)) / 9007199254740992.0) * 2 - 1)
        k += 1
        if not (missing_diag_every and i % missing_diag_every == missing_diag_every - 1):
            cols[i] = diag + (i % 7) * 0.25
        items = sorted(cols.items())
        if unsorted and len(items) > 2:
            items = items[1:] + items[:1]
            items[0], items[-1] = items[-1], items[0]
        for c, v in items:
            Aj.append(c)
            Ax.append(v)
        Ap.append(len(Aj))
    return (np.asarray(Ap, np.int32), np.asarray(Aj, np.int32), np.asarray(Ax, np.float64))


def digest(*arrays) -> str:
    """sha256 over dtype + bytes; every NaN is canonicalised first (x86 and
    gfx950 produce default NaNs of opposite sign, both are "NaN" results)"""
    h = hashlib.sha256()
    for a in arrays:
        a = np.ascontiguousarray(a)
        if a.dtype.kind == "f" and np.isnan(a).any():
            a = np.where(np.isnan(a), np.float64(np.nan), a)
        h.update(str(a.dtype).encode())
        h.update(a.tobytes())
    return h.hexdigest()


def conv_rand(nr: int, nc: int, k: int, seed: int, specials=False):
    """Random CSR for the format conversions (vectorised, any size): each row
    takes 0..k columns drawn with replacement, so rows are unsorted, may repeat
    a column and may be empty.  ``specials`` plants explicit 0.0, -0.0, NaN and
    inf values (bcsr_to_csr keeps only fabs(v) > 0, matrix-utils.cxx:192)."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, k + 1, nr)
    cols = rng.integers(0, nc, (nr, k)).astype(np.int32)
    keep = np.arange(k)[None, :] < lens[:, None]
    Aj = cols[keep]
    Ax = rng.uniform(-1, 1, Aj.size)
    if specials and Aj.size >= 8:
        idx = rng.choice(Aj.size, 4 + Aj.size // 50, replace=False)
        Ax[idx] = np.resize(np.array([0.0, -0.0, np.nan, np.inf]), idx.size)
    Ap = np.zeros(nr + 1, np.int32)
    np.cumsum(lens, out=Ap[1:])
    return Ap, Aj, Ax


def conv_handmade_bcsr():
    """Block CSR inputs the round trip from CSR never produces: block columns
    out of order, repeated block columns (sorted and unsorted rows), zero /
    -0.0 / NaN / inf entries, all-zero blocks, no blocks."""
    rng = np.random.default_rng(2718)

    def mk(nbr, nbc, bs, Bp, Bj, vals=None):
        Bp, Bj = np.asarray(Bp, np.int32), np.asarray(Bj, np.int32)
        Bx = rng.uniform(-1, 1, Bj.size * bs * bs) if vals is None else np.asarray(vals, np.float64)
        return nbr, nbc, bs, Bp, Bj, Bx

    z = rng.uniform(-1, 1, 2 * 9)
    z[[0, 4, 7, 9, 13]] = [0.0, -0.0, np.nan, np.inf, 0.0]
    return {
        "unsorted_blocks": mk(4, 4, 2, [0, 3, 5, 6, 8], [3, 0, 2, 1, 0, 2, 3, 1]),
        "dup_blocks_bs2": mk(3, 3, 2, [0, 3, 4, 6], [1, 0, 1, 2, 0, 0]),
        "dup_blocks_bs1": mk(4, 4, 1, [0, 2, 4, 5, 7], [2, 2, 0, 3, 1, 3, 0]),
        "specials_bs3": mk(2, 3, 3, [0, 1, 2], [2, 0], z),
        "all_zero": mk(2, 2, 2, [0, 1, 2], [1, 0], np.zeros(8)),
        "no_blocks": mk(3, 3, 2, [0, 0, 0, 0], []),
        "rect_bs2": mk(2, 5, 2, [0, 2, 5], [4, 1, 0, 3, 2]),
    }
