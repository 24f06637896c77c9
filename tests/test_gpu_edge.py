"""Edge cases of the hot path on the MI355X, checked bit for bit against the
CPU oracle (oracle/lssp_oracle.c, itself pinned to the reference by
tests/test_oracle_golden.py): tiny systems, empty rows, very long rows,
rectangular column spaces, non-finite operands (the SpMV still reads y when
beta = 0, mvops.cxx:42-78, so NaN / Inf in y propagate exactly as in the
reference), diagonal-only and 1x1 factors, and the solvers on 1x1 / diagonal
systems.  No fixture covers these shapes: the oracle is the checker."""
import numpy as np
import pytest

import oracle as O
from inputs import rand_csr, uniform

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    import lssp_amd
    d = lssp_amd.Device(0)
    yield d
    d.close()


def _same(a, b):
    return np.array_equal(np.asarray(a), np.asarray(b), equal_nan=True)


def _csr_rows(rows, n):
    Ap, Aj, Ax = [0], [], []
    for cols in rows:
        for c, v in cols:
            Aj.append(c)
            Ax.append(v)
        Ap.append(len(Aj))
    assert len(Ap) == n + 1
    return np.asarray(Ap, np.int32), np.asarray(Aj, np.int32), np.asarray(Ax, np.float64)


def _empty_rows(n=1000, every=3):
    Ap, Aj, Ax = rand_csr(n, 5, 0xE1, unsorted=False)
    rows = []
    for i in range(n):
        lo, hi = Ap[i], Ap[i + 1]
        rows.append([] if i % every == 1 else list(zip(Aj[lo:hi].tolist(), Ax[lo:hi].tolist())))
    return _csr_rows(rows, n)


def _long_rows(n=6000):
    rng = np.random.default_rng(7)
    rows = []
    for i in range(n):
        k = 20000 if i == 17 else 5000 if i == n - 1 else 4
        cols = np.sort(rng.choice(n, size=k, replace=k > n))  # k > n: repeated columns
        rows.append(list(zip(cols.tolist(), rng.uniform(-1, 1, cols.size).tolist())))
    return _csr_rows(rows, n)


MATS = {
    "1x1": lambda: (np.array([0, 1], np.int32), np.array([0], np.int32), np.array([3.5])),
    "empty_rows": _empty_rows,
    "all_rows_empty": lambda: (np.zeros(65, np.int32), np.zeros(0, np.int32), np.zeros(0)),
    "long_rows": _long_rows,
    "poisson7_5": lambda: (lambda A: (A.Ap, A.Aj, A.Ax))(O.poisson(3, 5)),
}


def _spmv_both(dev, Ap, Aj, Ax, op, alpha, beta, x, y, z0, ncols):
    import lssp_amd
    n = Ap.size - 1
    M = lssp_amd.DMat(dev, Ap, Aj, Ax, ncols=ncols)
    dx, dy, dz = dev.vec(ncols, x), dev.vec(n, y), dev.vec(n, z0)
    if op == 0:
        M.mv_mxy(dx, dz)
    elif op == 1:
        M.mv_amxy(alpha, dx, dz)
    elif op == 2:
        M.mv_amxpby(alpha, dx, beta, dz)
    else:
        M.mv_amxpbyz(alpha, dx, beta, dy, dz)
    got = dz.download()
    A = O.CSR(n, Ap, Aj, Ax)
    zo = z0.copy()
    want = O.spmv(op, A, x, alpha, beta, y=y.copy() if op == 3 else None, z=zo)
    return got, want


@pytest.mark.parametrize("op", [0, 1, 2, 3])
@pytest.mark.parametrize("name", sorted(MATS))
def test_spmv_edge_shapes_bitwise_vs_oracle(dev, name, op):
    Ap, Aj, Ax = MATS[name]()
    n = Ap.size - 1
    x = uniform(0x5EED, n)
    y, z0 = uniform(0xB0B, n), uniform(0xCAFE, n)
    got, want = _spmv_both(dev, Ap, Aj, Ax, op, -0.75, 1.25, x, y, z0, n)
    assert _same(got, want)


def test_spmv_rectangular_column_space(dev):
    n = 777
    Ap, Aj, Ax = rand_csr(n, 6, 0x77, unsorted=True)
    Aj = (Aj.astype(np.int64) * 2 + 1).astype(np.int32)  # columns in [0, 2n)
    x = uniform(1, 2 * n)
    for op in range(4):
        got, want = _spmv_both(dev, Ap, Aj, Ax, op, 0.5, -2.0, x, uniform(2, n), uniform(3, n), 2 * n)
        assert _same(got, want), op


def test_spmv_nonfinite_operands_propagate_like_the_reference(dev):
    A = O.poisson(2, 9)
    n = A.n
    x = uniform(4, n)
    x[5], x[40] = np.inf, -0.0
    y = uniform(5, n)
    y[3], y[60] = np.nan, np.inf  # beta = 0 still reads y: 0 * NaN / 0 * Inf = NaN
    for op, beta in ((3, 0.0), (2, 0.0), (3, -1.0)):
        got, want = _spmv_both(dev, A.Ap, A.Aj, A.Ax, op, 1.0, beta, x, y, y.copy(), n)
        assert _same(got, want), (op, beta)
        assert np.isnan(got).any()


@pytest.mark.parametrize("case", ["1x1", "diagonal", "bj_blk1", "empty_strict_rows"])
def test_ilu_degenerate_factors_bitwise_vs_oracle(dev, case):
    import lssp_amd
    if case == "1x1":
        Ap, Aj, Ax = MATS["1x1"]()
        kw, okw = dict(kind=1, level=0), dict(level=0)
    elif case == "diagonal":
        n = 300
        Ap, Aj, Ax = np.arange(n + 1, dtype=np.int32), np.arange(n, dtype=np.int32), 2.0 + uniform(9, n)
        kw, okw = dict(kind=1, level=0), dict(level=0)
    elif case == "bj_blk1":  # block-Jacobi with 1-row blocks: only diagonals survive
        A = O.poisson(3, 6)
        Ap, Aj, Ax = A.Ap, A.Aj, A.Ax
        kw, okw = dict(kind=1, level=0, blk=1), dict(level=0, blk=1)
    else:  # rows whose strict lower / upper parts are empty, columns unsorted
        Ap, Aj, Ax = rand_csr(500, 2, 0x99, unsorted=True)
        kw, okw = dict(kind=1, level=1), dict(level=1)
    n = Ap.size - 1
    M = lssp_amd.DILU.create(dev, Ap, Aj, Ax, **kw)
    (Lp, Lj, Lx), (Up, Uj, Ux) = M.factors()
    L, U = O.ilu(O.CSR(n, Ap, Aj, Ax), "iluk", **okw)
    assert _same(Lx, L.Ax) and np.array_equal(Lj, L.Aj) and np.array_equal(Lp, L.Ap)
    assert _same(Ux, U.Ax) and np.array_equal(Uj, U.Aj) and np.array_equal(Up, U.Ap)
    rhs = uniform(0x1234, n)
    x = dev.vec(n)
    M.apply(x, dev.vec(n, rhs))
    assert _same(x.download(), O.ilu_apply(L, U, rhs))


@pytest.mark.parametrize("solver", ["BICGSTAB", "CG", "GMRES", "IDRS", "BICGSTABL", "TFQMR"])
@pytest.mark.parametrize("system", ["1x1", "diagonal"])
def test_solvers_on_trivial_systems_bitwise_vs_oracle(dev, solver, system):
    import lssp_amd
    if system == "1x1":
        Ap, Aj, Ax = MATS["1x1"]()
    else:
        n = 200
        Ap, Aj, Ax = np.arange(n + 1, dtype=np.int32), np.arange(n, dtype=np.int32), 1.0 + uniform(11, n) ** 2
    n = Ap.size - 1
    b = uniform(0xB, n)
    sv = getattr(lssp_amd, solver)
    D = lssp_amd.DMat(dev, Ap, Aj, Ax)
    M = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=1, level=0)
    (Lp, Lj, Lx), (Up, Uj, Ux) = M.factors()
    x = dev.vec(n, np.zeros(n))
    r = lssp_amd.solve(dev, D, M, x, dev.vec(n, b), solver=sv, maxit=50, restart=4, bgsl=2, idrs=2,
                       trace_cap=10000)
    o = O.solve(getattr(O, solver), O.CSR(n, Ap, Aj, Ax), b, L=O.CSR(n, Lp, Lj, Lx), U=O.CSR(n, Up, Uj, Ux),
                maxit=50, restart=2 if solver in ("IDRS", "BICGSTABL") else 4, mode=O.TREE)
    assert r.nits == o.nits
    assert _same([r.residual], [o.residual])
    assert _same(r.trace, o.trace)
    assert _same(x.download(), o.x)


@pytest.mark.parametrize("mode", ["tree", "serial"])
@pytest.mark.parametrize("n", [1, 300])
def test_bicgstab_breakdown_without_pc_bitwise_vs_oracle(dev, mode, n):
    """A = 2I, no preconditioner: alpha = (r.r)/(r.2r) = 1/2 exactly, so s = r - alpha v
    is exactly 0 in the first iteration and ||s|| <= 1e-40 stops the run
    (solver-bicgstab.cxx:117-128) inside a batch of queued iterations -- in
    tree mode the ||s|| sum rides with the omega round (FIN_BICG_S_OMEGA)."""
    import lssp_amd
    Ap, Aj, Ax = np.arange(n + 1, dtype=np.int32), np.arange(n, dtype=np.int32), np.full(n, 2.0)
    b = uniform(0xBD, n)
    D = lssp_amd.DMat(dev, Ap, Aj, Ax)
    x = dev.vec(n, np.zeros(n))
    dev.set_reduction(lssp_amd.TREE if mode == "tree" else lssp_amd.SERIAL)
    try:
        r = lssp_amd.solve(dev, D, None, x, dev.vec(n, b), solver=lssp_amd.BICGSTAB, maxit=50, trace_cap=10000)
    finally:
        dev.set_reduction(lssp_amd.TREE)
    o = O.solve(O.BICGSTAB, O.CSR(n, Ap, Aj, Ax), b, maxit=50, mode=O.TREE if mode == "tree" else O.SERIAL)
    assert r.nits == o.nits == 1
    assert _same([r.residual], [o.residual])
    assert _same(r.trace, o.trace)
    assert _same(x.download(), o.x)


def _grid_plus_far_couplings(N=20, seed=5):
    """The 7-pt N^3 grid with two weak couplings per row at offsets +-(N^2+1 ..
    N^2+900): > 255 distinct offsets (no diagonal-id coding) while every 1024-row
    block spans < 16 K columns, so the matrix is served windowed (k_spmv_sell)."""
    import lssp_amd
    Ap, Aj, Ax = lssp_amd.poisson(3, N)
    n = Ap.size - 1
    rng = np.random.default_rng(seed)
    rows = []
    for i in range(n):
        cols = {int(Aj[k]): float(Ax[k]) for k in range(Ap[i], Ap[i + 1])}
        for sgn in (-1, 1):
            c = i + sgn * (N * N + 1 + int(rng.integers(0, 900)))
            if 0 <= c < n and c not in cols:
                cols[c] = -1e-3 * float(rng.random())
        rows.append(sorted(cols.items()))
    return (Ap, Aj, Ax), _csr_rows(rows, n)


def test_windowed_matrix_with_grid_line_sweep_preconditioner(dev):
    """BiCGSTAB in TREE mode with a windowed A and a grid ILU(0) M: the fused
    p / s gather passes move ||s||^2 into t = A sh's third dot, which the
    windowed product does not carry -- k_spmv3 serves that call (ADVICE r05:
    this combination used to fail with EINVAL)."""
    import lssp_amd
    (gp, gj, gx), (Ap, Aj, Ax) = _grid_plus_far_couplings()
    n = Ap.size - 1
    A = lssp_amd.DMat(dev, Ap, Aj, Ax)
    assert A.ndiag == 0 and A.windowed
    M = lssp_amd.DILU.create(dev, gp, gj, gx, kind=lssp_amd.ILUK, level=0)
    assert M.sweep_layout()[0] == 1  # the grid line sweeps
    b = uniform(77, n)
    x = dev.vec(n, np.zeros(n))
    r = lssp_amd.solve(dev, A, M, x, dev.vec(n, b), solver=lssp_amd.BICGSTAB, tol_rel=1e-10, tol_abs=1e-12,
                       tol_rb=0.0, maxit=60, trace_cap=10000)
    (Lp, Lj, Lx), (Up, Uj, Ux) = M.factors()
    o = O.solve(O.BICGSTAB, O.CSR(n, Ap, Aj, Ax), b, L=O.CSR(n, Lp, Lj, Lx), U=O.CSR(n, Up, Uj, Ux),
                rtol=1e-10, atol=1e-12, rbtol=0.0, maxit=60, mode=O.TREE)
    assert r.nits == o.nits
    assert r.residual == o.residual
    assert np.array_equal(r.trace, o.trace)
    assert np.array_equal(x.download(), o.x)
    M.close()
    A.close()
