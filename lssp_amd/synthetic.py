"""Synthetic inputs of BASELINE.json's configs that are not plain Poisson grids.

thermal_like(): the offline stand-in for SuiteSparse thermal2 that SURVEY.md
8(d) prescribes for config 5 (CG, PC_NON, irregular-row SpMV stress):
an m x m node grid (m = 1108 -> 1,227,664 nodes) with edges to the right and
up plus one diagonal per cell (orientation from splitmix64, seed 20240101),
lognormal(0, 1) edge weights, A = weighted graph Laplacian + 1.0 on the
boundary nodes (SPD), nodes renumbered by a windowed random shuffle
(window 4096).  Rows hold 3-9 entries; nnz = m^2 + 2 * (2m(m-1) + (m-1)^2)
= 8,584,786 at m = 1108 (thermal2: 1,228,045 rows, 8,580,313 nnz).
Columns are sorted ascending in every row (the solver's assemble order).
"""
from __future__ import annotations

import numpy as np

_GOLD = np.uint64(0x9E3779B97F4A7C15)


def _splitmix64(seed: int, n: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + np.arange(1, n + 1, dtype=np.uint64) * _GOLD
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _unit(bits: np.ndarray) -> np.ndarray:
    """(0, 1]: never 0, so log() below is finite"""
    return ((bits >> np.uint64(11)).astype(np.float64) + 1.0) * (1.0 / 9007199254740992.0)


def thermal_like(m: int = 1108, seed: int = 20240101, window: int = 4096):
    """-> (Ap, Aj, Ax) int32/int32/float64 CSR of the SPD thermal2-like matrix"""
    n = m * m
    node = np.arange(n, dtype=np.int64).reshape(m, m)
    # edges: right, up, one diagonal per cell
    ra, rb = node[:, :-1].ravel(), node[:, 1:].ravel()
    ua, ub = node[:-1, :].ravel(), node[1:, :].ravel()
    cells = (m - 1) * (m - 1)
    flip = (_splitmix64(seed, cells) & np.uint64(1)).astype(bool)
    d00, d11 = node[:-1, :-1].ravel(), node[1:, 1:].ravel()
    d01, d10 = node[:-1, 1:].ravel(), node[1:, :-1].ravel()
    da, db = np.where(flip, d01, d00), np.where(flip, d10, d11)
    ea = np.concatenate([ra, ua, da])
    eb = np.concatenate([rb, ub, db])
    ne = ea.size
    # lognormal(0, 1) weights (Box-Muller on two splitmix streams)
    u1 = _unit(_splitmix64(seed + 1, ne))
    u2 = _unit(_splitmix64(seed + 2, ne))
    w = np.exp(np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2))
    # windowed shuffle of the numbering
    keys = _splitmix64(seed + 3, n)
    perm = np.empty(n, np.int64)  # old node -> new row
    for s in range(0, n, window):
        e = min(s + window, n)
        perm[s + np.argsort(keys[s:e], kind="stable")] = np.arange(s, e)
    diag = np.zeros(n)
    np.add.at(diag, ea, w)
    np.add.at(diag, eb, w)
    ii, jj = np.divmod(np.arange(n), m)
    boundary = (ii == 0) | (ii == m - 1) | (jj == 0) | (jj == m - 1)
    diag[boundary] += 1.0
    rows = np.concatenate([perm[ea], perm[eb], perm])
    cols = np.concatenate([perm[eb], perm[ea], perm])
    vals = np.concatenate([-w, -w, diag[np.arange(n)]])
    order = np.lexsort((cols, rows))
    rows, cols, vals = rows[order], cols[order], vals[order]
    Ap = np.zeros(n + 1, np.int64)
    np.cumsum(np.bincount(rows, minlength=n), out=Ap[1:])
    return Ap.astype(np.int32), cols.astype(np.int32), vals.astype(np.float64)
