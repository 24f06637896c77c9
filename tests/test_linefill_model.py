"""Model of the ILU(1) line sweeps' dataflow (lssp_amd/csrc/linefill.hip), CPU only.

A restatement in Python of what k_linef computes: the skewed tiles (j' = j + k,
mirror-symmetric widths), the level map i = v - 2l - p - sigma(p), every
operand's source (own register, DPP neighbour, lane - 16, plane 3 from LDS,
the j-input hj[q + 2][p] and the k-input hk[Q][e] with its forwarded line -1
entry), the publish ranges (rows 0 .. nx, row nx = +0.0), the U sweep as the
mirror of the L tiles and the L sweep's writes into the U rhs stream
(v_U = C(p) - v).  Tiles run one after another in claim order, so a hand-off
entry that is read before it is written shows up as a missing key (NaN).
Bitwise against the oracle's ILU(1) apply on small boxes: the kernel's index
arithmetic is pinned here, independent of the GPU (the GPU tests pin the
kernel itself against the same oracle).
"""
import numpy as np
import pytest

import oracle as O
from test_gpu_parity import _box7

P, NJ, HKS, HJ0 = 8, 16, 18, 2


def sig(p):
    return p >> 2


def widths(m):
    W = (m + 15) // 16
    while True:
        base, extra = m // W, m % W
        if W % 2 == 0 and extra % 2:
            W += 1
            continue
        w = [base] * W
        for q in range(extra // 2):
            w[q] += 1
            w[W - 1 - q] += 1
        if extra % 2:
            w[W // 2] += 1
        return w


def off_grid(j0, nj, k0, np_, ny):
    """build_linefill's LT_SKIP rule: every line of every plane, and line -1
    (forwarded to the k-successor), off the grid."""
    lo, hi = j0 - 1 - (k0 + np_ - 1), j0 + nj - 1 - k0
    return hi < 0 or lo > ny - 1


def model_apply(nx, ny, nz, seed=1, skip=True):
    Ap, Aj, Ax = _box7(nx, ny, nz, seed)
    n = Ap.size - 1
    L, U = O.ilu(O.CSR(n, Ap, Aj, Ax), "iluk", level=1)
    pl = nx * ny
    coef = np.zeros((n, 6))
    for r in range(n):
        for q in range(L.Ap[r], L.Ap[r + 1] - 1):
            off = r - L.Aj[q]
            a = {pl: 0, pl - 1: 1, pl - nx: 2, nx: 3, nx - 1: 4, 1: 5}[off]
            coef[r, a] = L.Ax[q]
    rhs = np.random.default_rng(3).uniform(-1, 1, n)
    m = ny + nz - 1
    wd = widths(m); W = len(wd); S = (nz + P - 1) // P
    js = np.concatenate([[0], np.cumsum(wd)])
    hk, hj = {}, {}
    out = np.full(n, np.nan)
    order = sorted([(K, J) for K in range(S) for J in range(W)], key=lambda t: (t[1] * 36 + t[0] * 13, t[0] * W + t[1]))
    # skipped tiles do not run; their consumers read +0.0 inputs
    skl = {(K, J) for K in range(S) for J in range(W)
           if skip and off_grid(js[J], wd[J], K * P, min(P, nz - K * P), ny)}
    for K, J in order:
        j0, nj, k0, np_ = js[J], wd[J], K * P, min(P, nz - K * P)
        if (K, J) in skl: continue
        T = nx + 2 * (nj - 1) + (np_ - 1) + sig(np_ - 1) + 1; T += T % 2
        kin, jin = K > 0 and (K - 1, J) not in skl, J > 0 and (K, J - 1) not in skl
        kout, jout = K < S - 1, J < W - 1
        def HK(Q, e):
            if not kin: return 0.0
            return hk[(K - 1, J, Q, e)]
        def HJ(qrow, p):  # qrow = q + HJ0
            if not jin: return 0.0
            return hj[(K, J - 1, qrow, p)]
        xp = np.zeros((P, NJ)); bnp = np.zeros((P, NJ)); sep = np.zeros((P, NJ)); bep = np.zeros((P, NJ))
        res = {}
        for v in range(-2, T):
            x = np.zeros((P, NJ)); bn = np.zeros((P, NJ)); be = np.zeros((P, NJ)); se = np.zeros((P, NJ))
            for p in range(P):
                for l in range(NJ):
                    def get(fn, *a):
                        try: return fn(*a)
                        except KeyError: return np.nan
                    # BN
                    if p == 0: bn[p, l] = get(HK, v + 2, 1 + l)
                    elif p == 4: bn[p, l] = res.get((v - 2, 3, l), np.nan)
                    else: bn[p, l] = xp[p - 1, l]
                    # BE
                    if l == 0:
                        if p == 0: be[p, l] = get(HK, v + 2, 0)
                        elif p == 4: be[p, l] = get(HJ, v - 1 + HJ0, 3)
                        else: be[p, l] = get(HJ, v + HJ0, p - 1)
                    else: be[p, l] = bnp[p, l - 1]
                    # SE
                    se[p, l] = get(HJ, v + 1 + HJ0, p) if l == 0 else xp[p, l - 1]
            for p in range(P):
                for l in range(NJ):
                    j = j0 + l - k0 - p
                    i = v - 2 * l - p - sig(p)
                    ok = p < np_ and l < nj and 0 <= j < ny and 0 <= i < nx
                    if ok:
                        r = ((k0 + p) * ny + j) * nx + i
                        c = coef[r]
                        t = rhs[r] - c[0] * bep[p, l]
                        t = t - c[1] * be[p, l]; t = t - c[2] * bn[p, l]; t = t - c[3] * sep[p, l]
                        t = t - c[4] * se[p, l]; t = t - c[5] * xp[p, l]
                        x[p, l] = t; out[r] = t
                    res[(v, p, l)] = x[p, l]
            # publish
            if kout:
                for l in range(nj):
                    i = v - 2 * l - (np_ - 1) - sig(np_ - 1); Q = v - (np_ - 1) - sig(np_ - 1) + 2
                    if 0 <= i <= nx and Q >= 0: hk[(K, J, Q, 1 + l)] = x[np_ - 1, l]
                    if l == 0 and 0 <= i + 1 <= nx and Q >= 0: hk[(K, J, Q, 0)] = se[np_ - 1, 0]
            if jout:
                q = v - 2 * (nj - 1)
                for p in range(np_):
                    if 0 <= q - p - sig(p) <= nx and q + HJ0 >= 0: hj[(K, J, q + HJ0, p)] = x[p, nj - 1]
            bep, sep, bnp, xp = be, se, bn, x
    ref = O.ilu_apply(L, O.CSR(n, np.arange(n + 1, dtype=np.int32), np.arange(n, dtype=np.int32), np.ones(n)), rhs)
    ok_l = np.array_equal(out, ref)
    # U sweep in mirrored coordinates on the L sweep's output, via the OUT=2 stream mapping
    cu = np.zeros((n, 7))
    for r in range(n):
        rs = n - 1 - r
        cu[rs, 6] = U.Ax[U.Ap[r]]
        for q in range(U.Ap[r] + 1, U.Ap[r + 1]):
            off = U.Aj[q] - r
            cu[rs, {pl: 0, pl - 1: 1, pl - nx: 2, nx: 3, nx - 1: 4, 1: 5}[off]] = U.Ax[q]
    ustream = {}
    for K in range(S):
        for J in range(W):
            j0, nj, k0, np_ = js[J], wd[J], K * P, min(P, nz - K * P)
            Kp, Jp = S - 1 - K, W - 1 - J
            for p in range(np_):
                for l in range(nj):
                    j = j0 + l - k0 - p
                    if not (0 <= j < ny): continue
                    for i in range(nx):
                        v = i + 2 * l + p + sig(p)
                        C = nx - 1 + 2 * (nj - 1) + np_ - 1 + sig(p) + sig(np_ - 1 - p)
                        r = ((k0 + p) * ny + j) * nx + i
                        ustream[(Kp, Jp, C - v, np_ - 1 - p, nj - 1 - l)] = out[r]
    # U tiles
    hk.clear(); hj.clear()
    outu = np.full(n, np.nan)
    def u_geom(Kp, Jp):
        K, J = S - 1 - Kp, W - 1 - Jp
        nj, np_ = wd[J], min(P, nz - K * P)
        return m - js[J] - nj, nj, nz - K * P - np_, np_
    sku = {(Kp, Jp) for Kp in range(S) for Jp in range(W) if skip and off_grid(*u_geom(Kp, Jp), ny)}
    for Kp, Jp in order:
        j0, nj, k0, np_ = u_geom(Kp, Jp)
        if (Kp, Jp) in sku: continue
        T = nx + 2 * (nj - 1) + (np_ - 1) + sig(np_ - 1) + 1; T += T % 2
        kin, jin = Kp > 0 and (Kp - 1, Jp) not in sku, Jp > 0 and (Kp, Jp - 1) not in sku
        kout, jout = Kp < S - 1, Jp < W - 1
        def HK(Q, e):
            if not kin: return 0.0
            return hk[(Kp - 1, Jp, Q, e)]
        def HJ(qrow, p):
            if not jin: return 0.0
            return hj[(Kp, Jp - 1, qrow, p)]
        xp = np.zeros((P, NJ)); bnp = np.zeros((P, NJ)); sep = np.zeros((P, NJ)); bep = np.zeros((P, NJ))
        res = {}
        for v in range(-2, T):
            x = np.zeros((P, NJ)); bn = np.zeros((P, NJ)); be = np.zeros((P, NJ)); se = np.zeros((P, NJ))
            for p in range(P):
                for l in range(NJ):
                    def get(fn, *a):
                        try: return fn(*a)
                        except KeyError: return np.nan
                    if p == 0: bn[p, l] = get(HK, v + 2, 1 + l)
                    elif p == 4: bn[p, l] = res.get((v - 2, 3, l), np.nan)
                    else: bn[p, l] = xp[p - 1, l]
                    if l == 0:
                        if p == 0: be[p, l] = get(HK, v + 2, 0)
                        elif p == 4: be[p, l] = get(HJ, v - 1 + HJ0, 3)
                        else: be[p, l] = get(HJ, v + HJ0, p - 1)
                    else: be[p, l] = bnp[p, l - 1]
                    se[p, l] = get(HJ, v + 1 + HJ0, p) if l == 0 else xp[p, l - 1]
            for p in range(P):
                for l in range(NJ):
                    j = j0 + l - k0 - p
                    i = v - 2 * l - p - sig(p)
                    if p < np_ and l < nj and 0 <= j < ny and 0 <= i < nx:
                        rs = ((k0 + p) * ny + j) * nx + i
                        c = cu[rs]
                        t = ustream[(Kp, Jp, v, p, l)] - c[0] * bep[p, l]
                        t = t - c[1] * be[p, l]; t = t - c[2] * bn[p, l]; t = t - c[3] * sep[p, l]
                        t = t - c[4] * se[p, l]; t = t - c[5] * xp[p, l]
                        t = t / c[6]
                        x[p, l] = t; outu[n - 1 - rs] = t
                    res[(v, p, l)] = x[p, l]
            if kout:
                for l in range(nj):
                    i = v - 2 * l - (np_ - 1) - sig(np_ - 1); Q = v - (np_ - 1) - sig(np_ - 1) + 2
                    if 0 <= i <= nx and Q >= 0: hk[(Kp, Jp, Q, 1 + l)] = x[np_ - 1, l]
                    if l == 0 and 0 <= i + 1 <= nx and Q >= 0: hk[(Kp, Jp, Q, 0)] = se[np_ - 1, 0]
            if jout:
                q = v - 2 * (nj - 1)
                for p in range(np_):
                    if 0 <= q - p - sig(p) <= nx and q + HJ0 >= 0: hj[(Kp, Jp, q + HJ0, p)] = x[p, nj - 1]
            bep, sep, bnp, xp = be, se, bn, x
    refu = O.ilu_apply(L, U, rhs)
    return ok_l, np.array_equal(outu, refu)


@pytest.mark.parametrize("nx,ny,nz", [(9, 7, 13), (3, 3, 2), (6, 5, 1), (4, 9, 17), (4, 5, 33)])
@pytest.mark.parametrize("skip", [True, False], ids=["skip-off-grid", "all-tiles"])
def test_linefill_dataflow_model_bitwise_vs_oracle(nx, ny, nz, skip):
    ok_l, ok_u = model_apply(nx, ny, nz, skip=skip)
    assert ok_l and ok_u


def test_off_grid_rule_skips_tiles():
    """The shapes above exercise the rule: (4, 9, 17) and (4, 5, 33) have
    skipped tiles in both sweeps."""
    for nx, ny, nz in ((4, 9, 17), (4, 5, 33)):
        m = ny + nz - 1
        wd = widths(m)
        js = np.concatenate([[0], np.cumsum(wd)])
        S = (nz + P - 1) // P
        n_skip = sum(off_grid(js[J], wd[J], K * P, min(P, nz - K * P), ny) for K in range(S) for J in range(len(wd)))
        assert n_skip > 0
