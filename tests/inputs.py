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
