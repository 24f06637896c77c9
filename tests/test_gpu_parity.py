"""HIP path vs the reference (tests/golden/) and vs the CPU oracle.

All comparisons are bitwise except where a test says otherwise:
  * SpMV, BLAS-1 and ILU setup/apply against the reference's own outputs;
  * solvers in SERIAL reduction mode against the reference's full scalar trace
    (every dot and norm), iteration count, residual and solution;
  * solvers in TREE mode (the fast path) against the oracle restating the same
    canonical reduction order.
"""
import os

import numpy as np
import pytest

import oracle as O
from golden_util import build_matrix, case_id, cases, fx, matches, vec
from inputs import uniform

pytestmark = pytest.mark.gpu

SPMV = cases("spmv")
ILU = cases("ilu")
SOLVE = cases("solve")


@pytest.fixture(scope="module")
def dev():
    import lssp_amd
    d = lssp_amd.Device(0)
    yield d
    d.close()


def _ilu_kw(pc, n):
    if pc["kind"] == "iluk":
        return dict(kind=1, level=pc["level"])
    if pc["kind"] == "ilut":
        return dict(kind=2, tol=pc["tol"], p=pc["p"])
    return dict(kind=1, level=0, blk=(n + pc["nblk"] - 1) // pc["nblk"])


@pytest.mark.parametrize("c", SPMV, ids=[case_id(c) for c in SPMV])
def test_spmv_bitwise_vs_reference(dev, c):
    import lssp_amd
    A = build_matrix(c["mat"])
    M = lssp_amd.DMat(dev, A.Ap, A.Aj, A.Ax)
    x = dev.vec(A.n, uniform(c["xseed"], A.n))
    y = dev.vec(A.n, uniform(c["yseed"], A.n))
    z = dev.vec(A.n, uniform(c["yseed"], A.n))
    a, b = fx(c["alpha"]), fx(c["beta"])
    op = c["op"]
    if op == 0:
        M.mv_mxy(x, z)
    elif op == 1:
        M.mv_amxy(a, x, z)
    elif op == 2:
        M.mv_amxpby(a, x, b, z)
    else:
        M.mv_amxpbyz(a, x, b, y, z)
    assert matches(c["out"], z.download())


@pytest.mark.parametrize("c", ILU, ids=[case_id(c) for c in ILU])
def test_ilu_setup_and_apply_bitwise_vs_reference(dev, c):
    import lssp_amd
    A = build_matrix(c["mat"])
    M = lssp_amd.DILU.create(dev, A.Ap, A.Aj, A.Ax, **_ilu_kw(c["pc"], A.n))
    (Lp, Lj, Lx), (Up, Uj, Ux) = M.factors()
    assert matches(c["L"], Lp, Lj, Lx)
    assert matches(c["U"], Up, Uj, Ux)
    rhs = uniform(c["rhs_seed"], A.n)
    x = dev.vec(A.n)
    r = dev.vec(A.n, rhs)
    M.apply(x, r)
    assert matches(c["apply"], x.download())
    M.apply(r, r)  # x may alias rhs (solver-tri.cxx:48-55 goes through pc->cache)
    assert matches(c["apply"], r.download())


def _solve_inputs(dev, c):
    import lssp_amd
    A = build_matrix(c["mat"])
    Ap, Aj, Ax = lssp_amd.sort_columns(A.Ap, A.Aj, A.Ax)  # lssp.cxx:173
    D = lssp_amd.DMat(dev, Ap, Aj, Ax)
    M = None
    if c["pc"]["kind"] != "none":
        M = lssp_amd.DILU.create(dev, A.Ap, A.Aj, A.Ax, **_ilu_kw(c["pc"], A.n))
    b = dev.vec(A.n, vec(c["b"], A.n))
    x = dev.vec(A.n, np.zeros(A.n) if c["x0"] is None else vec(c["x0"], A.n))
    return A, D, M, x, b


@pytest.mark.parametrize("c", SOLVE, ids=[case_id(c) for c in SOLVE])
def test_solver_serial_mode_trace_bitwise_vs_reference(dev, c):
    """SERIAL reduction mode reproduces the reference run bit for bit."""
    import lssp_amd
    dev.set_reduction(lssp_amd.SERIAL)
    try:
        A, D, M, x, b = _solve_inputs(dev, c)
        r = lssp_amd.solve(dev, D, M, x, b, solver=c["solver"], tol_rel=fx(c["rtol"]), tol_abs=fx(c["atol"]),
                           tol_rb=fx(c["rbtol"]), maxit=c["maxit"], restart=c["restart"],
                           bgsl=c["restart"], idrs=c["restart"], trace_cap=100000)
    finally:
        dev.set_reduction(lssp_amd.TREE)
    assert r.nits == c["nits"]
    assert r.residual == fx(c["residual"])
    assert matches(c["trace"], r.trace)
    assert matches(c["x"], x.download())


TREE_CASES = [c for c in SOLVE if c["mat"].get("N", 0) <= 64 or c["mat"]["type"] == "rand"]
L1_SOLVERS = (O.BICGSAFE, O.CGS, O.GPBICG, O.CR, O.CRS, O.BICRSTAB, O.BICRSAFE, O.GPBICR, O.QMRCGSTAB, O.TFQMR)


@pytest.mark.parametrize("c", TREE_CASES, ids=[case_id(c) for c in TREE_CASES])
def test_solver_tree_mode_bitwise_vs_oracle(dev, c):
    """The fast path: canonical tree reductions, bitwise equal to the oracle's
    restatement of the same order; iteration count within 1 of the reference."""
    import lssp_amd
    A, D, M, x, b = _solve_inputs(dev, c)
    r = lssp_amd.solve(dev, D, M, x, b, solver=c["solver"], tol_rel=fx(c["rtol"]), tol_abs=fx(c["atol"]),
                       tol_rb=fx(c["rbtol"]), maxit=c["maxit"], restart=c["restart"],
                           bgsl=c["restart"], idrs=c["restart"], trace_cap=100000)
    L = U = None
    if M is not None:
        (Lp, Lj, Lx), (Up, Uj, Ux) = M.factors()
        L, U = O.CSR(A.n, Lp, Lj, Lx), O.CSR(A.n, Up, Uj, Ux)
    x0 = None if c["x0"] is None else vec(c["x0"], A.n)
    o = O.solve(c["solver"], A, vec(c["b"], A.n), x0=x0, L=L, U=U, rtol=fx(c["rtol"]), atol=fx(c["atol"]),
                rbtol=fx(c["rbtol"]), maxit=c["maxit"], restart=c["restart"], mode=O.TREE)
    assert r.nits == o.nits
    assert r.residual == o.residual
    assert np.array_equal(r.trace, o.trace)
    # NaN compared as NaN: GMRES-R hitting maxit mid-cycle divides 0/0 in the
    # reference (solver-gmres.cxx:414-418 use a zeroed Hessenberg column)
    assert np.array_equal(x.download(), o.x, equal_nan=True)
    assert abs(r.nits - c["nits"]) <= max(1, c["nits"] // 20)


@pytest.mark.parametrize("n", [1, 255, 256, 257, 4099, 100000, 1 << 20])
def test_dot_norm_tree_and_serial(dev, n):
    import lssp_amd
    xh, yh = uniform(5, n), uniform(6, n)
    x, y = dev.vec(n, xh), dev.vec(n, yh)
    import ctypes
    out = ctypes.c_double()
    for mode in (lssp_amd.TREE, lssp_amd.SERIAL):
        dev.set_reduction(mode)
        assert dev.L.lssp_amd_vec_dot(dev.h, x.ptr, y.ptr, n, ctypes.byref(out)) == 0
        assert out.value == O.dot(xh, yh, mode)
        assert dev.L.lssp_amd_vec_norm(dev.h, x.ptr, n, ctypes.byref(out)) == 0
        assert out.value == np.sqrt(O.dot(xh, xh, mode))
    dev.set_reduction(lssp_amd.TREE)


def test_blas1_bitwise(dev):
    n = 100003
    xh, yh, zh = uniform(1, n), uniform(2, n), uniform(3, n)
    a, b = -0.375, 1.625
    L = dev.L
    x, y, z = dev.vec(n, xh), dev.vec(n, yh), dev.vec(n, zh)
    assert L.lssp_amd_vec_axpby(dev.h, a, x.ptr, b, y.ptr, n) == 0
    assert np.array_equal(y.download(), yh * b + xh * a)          # vector.cxx:98-107
    assert L.lssp_amd_vec_axpbyz(dev.h, a, x.ptr, b, z.ptr, y.ptr, n) == 0
    assert np.array_equal(y.download(), zh * b + xh * a)          # :110-120
    assert L.lssp_amd_vec_axy(dev.h, a, x.ptr, y.ptr, n) == 0
    assert np.array_equal(y.download(), xh * a)                   # :86-95
    assert L.lssp_amd_vec_scale(dev.h, x.ptr, n, b) == 0
    assert np.array_equal(x.download(), xh * b)                   # :141-146
    assert L.lssp_amd_vec_copy(dev.h, y.ptr, z.ptr, n) == 0
    assert np.array_equal(y.download(), zh)
    assert L.lssp_amd_vec_set_value(dev.h, y.ptr, n, 2.5) == 0
    assert np.all(y.download() == 2.5)


@pytest.mark.parametrize("N,kind,kw", [(48, 1, dict(level=0)), (40, 1, dict(level=1)),
                                        (32, 2, dict(tol=1e-4, p=20))])
def test_trisolve_sweeps_and_levels_vs_oracle(dev, N, kind, kw):
    import lssp_amd
    A = O.poisson(3, N)
    M = lssp_amd.DILU.create(dev, A.Ap, A.Aj, A.Ax, kind=kind, **kw)
    if kind == 1 and kw["level"] == 0:
        assert M.levelsL == 3 * N - 2 and M.levelsU == 3 * N - 2
    (Lp, Lj, Lx), (Up, Uj, Ux) = M.factors()
    rhs = uniform(99, A.n)
    r = dev.vec(A.n, rhs)
    x = dev.vec(A.n)
    for which, (P, J, X) in [(0, (Lp, Lj, Lx)), (1, (Up, Uj, Ux))]:
        M.trisolve(which, x, r)
        ref = np.zeros(A.n)
        O.lib().orc_trisolve(which, A.n, O._ptr(P), O._ptr(J), O._ptr(X), O._ptr(ref), O._ptr(rhs))
        assert np.array_equal(x.download(), ref)
    for _ in range(3):  # repeated applies: the sentinel re-arming must hold
        M.apply(x, r)
        assert np.array_equal(x.download(), O.ilu_apply(O.CSR(A.n, Lp, Lj, Lx), O.CSR(A.n, Up, Uj, Ux), rhs))


def _box7(nx, ny, nz, seed):
    """7-pt stencil on an nx x ny x nz box (natural order, i fastest), random
    nonsymmetric diagonally dominant values."""
    rng = np.random.default_rng(seed)
    n = nx * ny * nz
    Ap, Aj, Ax = [0], [], []
    for r in range(n):
        i, j, k = r % nx, r // nx % ny, r // (nx * ny)
        cols = [c for c, ok in ((r - nx * ny, k > 0), (r - nx, j > 0), (r - 1, i > 0), (r, True),
                                (r + 1, i < nx - 1), (r + nx, j < ny - 1), (r + nx * ny, k < nz - 1)) if ok]
        vals = rng.uniform(-1, -0.1, len(cols))
        vals[cols.index(r)] = 7.0 + rng.uniform(0, 1)
        Aj += cols
        Ax += list(vals)
        Ap.append(len(Aj))
    return np.array(Ap, np.int32), np.array(Aj, np.int32), np.array(Ax)


# k_line2's 16-line x 8-plane tiles on boxes with partial tiles in j and k, an
# odd last plane count, slabs with 1..3 planes in the second compute wave
# ((13, 37, 35): 35 = 4 x 8 + 3; (9, 21, 13): 13 = 8 + 5, (20, 17, 6): one tile
# of 6 planes, (11, 16, 4): planes in wave 0 only), 40 x 40 planes, a long thin box
@pytest.mark.parametrize("nx,ny,nz", [(20, 100, 6), (13, 37, 35), (9, 21, 13), (20, 17, 6), (11, 16, 4),
                                      (40, 33, 19), (20, 40, 40), (20, 60, 24)])
def test_line_sweep_tile_shapes_bitwise_vs_oracle(dev, nx, ny, nz):
    import lssp_amd
    tile = (16, 8)
    Ap, Aj, Ax = _box7(nx, ny, nz, nx + ny + nz)
    n = Ap.size - 1
    M = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=1, level=0)
    assert M.sweep_layout() == (True, *tile)
    L, U = O.ilu(O.CSR(n, Ap, Aj, Ax), "iluk", level=0)
    (Lp, Lj, Lx), (Up, Uj, Ux) = M.factors()
    assert np.array_equal(Lx, L.Ax) and np.array_equal(Ux, U.Ax)
    x = dev.vec(n)
    for rep in range(4):  # repeated applies: the shared hand-off buffers must be re-armed exactly
        rhs = uniform(200 + rep, n)
        M.apply(x, dev.vec(n, rhs))
        assert np.array_equal(x.download(), O.ilu_apply(L, U, rhs)), rep
    # the single sweeps (lssp_pc_ilu_solve_lower/upper_matrix, solver-tri.cxx:4-46)
    rhs = uniform(300, n)
    z = dev.vec(n)
    M.trisolve(0, z, dev.vec(n, rhs))
    lo = O.ilu_apply(L, O.CSR(n, np.arange(n + 1, dtype=np.int32), np.arange(n, dtype=np.int32), np.ones(n)), rhs)
    assert np.array_equal(z.download(), lo)
    M.trisolve(1, z, dev.vec(n, rhs))
    up = O.ilu_apply(O.CSR(n, np.arange(n + 1, dtype=np.int32), np.arange(n, dtype=np.int32), np.ones(n)), U, rhs)
    assert np.array_equal(z.download(), up)


# ILU(1) of a 7-point box: skewed line sweeps (linefill.hip).  Boxes with one
# or several j' columns and k-tiles, partial 8-plane tiles (6, 13 = 8 + 5,
# 35 = 4 x 8 + 3, 2), thin lines (nx = 3) and few lines per plane (ny = 3, 4).
@pytest.mark.parametrize("nx,ny,nz", [(20, 17, 6), (13, 37, 35), (9, 21, 13), (40, 33, 19), (3, 3, 2),
                                      (11, 16, 4), (5, 40, 9), (33, 4, 17), (24, 24, 24), (30, 27, 1),
                                      (100, 100, 1)])
def test_line_sweep_ilu1_bitwise_vs_oracle(dev, nx, ny, nz):
    import lssp_amd
    Ap, Aj, Ax = _box7(nx, ny, nz, 7 * nx + ny + nz)
    n = Ap.size - 1
    M = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=1, level=1)
    # 2-D grids of <= 256 lines: one workgroup, lines on lanes (k_lineg); else skewed tiles
    assert M.sweep_layout() == ((2, ny, 1) if nz == 1 else (2, 16, 8))
    L, U = O.ilu(O.CSR(n, Ap, Aj, Ax), "iluk", level=1)
    (Lp, Lj, Lx), (Up, Uj, Ux) = M.factors()
    assert np.array_equal(Lj, L.Aj) and np.array_equal(Lx, L.Ax) and np.array_equal(Ux, U.Ax)
    x = dev.vec(n)
    for rep in range(4):  # repeated applies: the shared hand-off buffers must be re-armed exactly
        rhs = uniform(400 + rep, n)
        M.apply(x, dev.vec(n, rhs))
        assert np.array_equal(x.download(), O.ilu_apply(L, U, rhs)), rep
    rhs = uniform(500, n)
    z = dev.vec(n)
    one = O.CSR(n, np.arange(n + 1, dtype=np.int32), np.arange(n, dtype=np.int32), np.ones(n))
    M.trisolve(0, z, dev.vec(n, rhs))
    assert np.array_equal(z.download(), O.ilu_apply(L, one, rhs))
    M.trisolve(1, z, dev.vec(n, rhs))
    assert np.array_equal(z.download(), O.ilu_apply(one, U, rhs))
    # x aliasing rhs (lssp_pc_ilu_solve may be called in place)
    y = dev.vec(n, rhs)
    M.apply(y, y)
    assert np.array_equal(y.download(), O.ilu_apply(L, U, rhs))


# The one-workgroup 2-D sweeps (linefill.hip k_lineg: ILU(0) of a 5-point grid,
# exam.cxx's configuration, and its ILU(1) pattern) and the tiled sweeps on the
# same 2-D grids (LSSP_AMD_LINEG=0): 1 to 4 waves of lines (a wave with one line,
# the 256-line maximum), nx = 3, repeated applies, both single sweeps, in-place;
# both equal to the oracle bit for bit.
@pytest.mark.parametrize("nx,ny", [(3, 3), (30, 27), (100, 100), (9, 65), (5, 200), (7, 256), (64, 1 + 64 * 3)])
@pytest.mark.parametrize("lineg", ["1", "0"], ids=["one-workgroup", "tiles"])
@pytest.mark.parametrize("level", [0, 1], ids=["ilu0", "ilu1"])
def test_line_sweep_2d_both_paths_bitwise_vs_oracle(dev, nx, ny, lineg, level):
    import lssp_amd
    if level == 0 and ny < 8:
        pytest.skip("not a line-sweep grid for ILU(0) (detect_grid: ny >= 8)")
    Ap, Aj, Ax = _box7(nx, ny, 1, 5 * nx + ny)
    n = Ap.size - 1
    old = os.environ.get("LSSP_AMD_LINEG")
    os.environ["LSSP_AMD_LINEG"] = lineg
    try:
        M = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=1, level=level)
    finally:
        if old is None:
            os.environ.pop("LSSP_AMD_LINEG", None)
        else:
            os.environ["LSSP_AMD_LINEG"] = old
    assert M.sweep_layout() == ((1 + level, ny, 1) if lineg == "1" else (1 + level, 16, 8))
    L, U = O.ilu(O.CSR(n, Ap, Aj, Ax), "iluk", level=level)
    x = dev.vec(n)
    for rep in range(3):
        rhs = uniform(600 + rep, n)
        M.apply(x, dev.vec(n, rhs))
        assert np.array_equal(x.download(), O.ilu_apply(L, U, rhs)), rep
    one = O.CSR(n, np.arange(n + 1, dtype=np.int32), np.arange(n, dtype=np.int32), np.ones(n))
    rhs = uniform(700, n)
    z = dev.vec(n)
    M.trisolve(0, z, dev.vec(n, rhs))
    assert np.array_equal(z.download(), O.ilu_apply(L, one, rhs))
    M.trisolve(1, z, dev.vec(n, rhs))
    assert np.array_equal(z.download(), O.ilu_apply(one, U, rhs))
    y = dev.vec(n, rhs)
    M.apply(y, y)
    assert np.array_equal(y.download(), O.ilu_apply(L, U, rhs))
    M.close()


@pytest.mark.parametrize("seed,n,per_row,missing,blk", [(11, 3000, 6, 0, 0), (12, 2500, 9, 7, 0),
                                                        (13, 4000, 5, 0, 1000), (14, 1999, 4, 5, 333)])
def test_gpu_ilu0_factorization_bitwise_vs_oracle(dev, seed, n, per_row, missing, blk):
    """ILUK numeric factorization runs on the GPU (ilu_factor.hip); random
    unsorted nonsymmetric matrices with missing diagonals and block-Jacobi
    blocks must give the reference's factors bit for bit (oracle pinned to the
    reference by tests/test_oracle_golden.py)."""
    import lssp_amd
    from inputs import rand_csr
    Ap, Aj, Ax = rand_csr(n, per_row, seed, unsorted=True, missing_diag_every=missing)
    for level in (0, 1):
        M = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=lssp_amd.ILUK, level=level, blk=blk)
        (Lp, Lj, Lx), (Up, Uj, Ux) = M.factors()
        L, U = O.ilu(O.CSR(n, Ap, Aj, Ax), "iluk", level=level, blk=blk)
        assert np.array_equal(Lp, L.Ap) and np.array_equal(Lj, L.Aj) and np.array_equal(Lx, L.Ax, equal_nan=True)
        assert np.array_equal(Up, U.Ap) and np.array_equal(Uj, U.Aj) and np.array_equal(Ux, U.Ax, equal_nan=True)
        M.close()


def _scattered(n, seed, maxlen=20, reach=3000):
    """random CSR whose columns scatter within +-reach of the row: rows of 0..maxlen
    entries (empty rows and rows longer than the 12-entry unrolled path included)"""
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, maxlen + 1, n)
    lens[::97] = 0
    Ap = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=Ap[1:])
    Aj = np.empty(Ap[-1], np.int64)
    for r in range(n):
        lo, hi = max(0, r - reach), min(n, r + reach + 1)
        Aj[Ap[r]:Ap[r + 1]] = np.sort(rng.choice(np.arange(lo, hi), lens[r], replace=False))
    Ax = uniform(seed + 7, int(Ap[-1]))
    return O.CSR(n, Ap.astype(np.int32), Aj.astype(np.int32), Ax)


def _jumpy(n, seed):
    """random CSR whose 1024-row blocks read either near their own rows or a
    narrow band around another block's rows (spans of 100..12,000 columns
    that overlap, extend or jump between consecutive blocks; rows of 0..12
    entries): the windowed kernel over many more blocks than CUs"""
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 13, n)
    Ap = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=Ap[1:])
    row = np.repeat(np.arange(n), lens)
    nb = (n + 1023) // 1024
    mode = rng.integers(0, 3, nb)  # 0, 1: near the diagonal; 2: around another block
    target = rng.permutation(nb)
    reach = rng.integers(50, 6000, nb)
    blk = row // 1024
    centre = np.where(mode[blk] == 2, target[blk] * 1024 + 512, row)
    Aj = np.clip(centre + rng.integers(-1, 2, row.size) * rng.integers(0, reach[blk] + 1), 0, n - 1)
    Ax = uniform(seed + 7, int(Ap[-1]))
    return O.CSR(n, Ap.astype(np.int32), Aj.astype(np.int32), Ax)


@pytest.mark.parametrize("which", ["thermal", "thermal-big", "thermal-ring", "scattered", "jumpy", "wide"])
def test_spmv_scattered_bitwise_vs_oracle(dev, which):
    """The uncoded products give the oracle's sums bit for bit (mvops.cxx:42-78,
    118-150) on scattered-column matrices: the thermal-like matrix of config 5
    and random rows of 0..20 entries within +-3000 of the diagonal take the
    windowed-x kernel (k_spmv_win); columns over the whole range ("wide": a
    1024-row block spanning > 16384 columns) take the gathering k_spmv3."""
    import lssp_amd
    from lssp_amd.synthetic import thermal_like
    if which == "thermal":
        Ap, Aj, Ax = thermal_like(m=150, window=512)
        A = O.CSR(Ap.size - 1, Ap, Aj, Ax)
    elif which == "thermal-big":
        Ap, Aj, Ax = thermal_like(m=330, window=4096)  # 108,900 rows: 107 windowed blocks
        A = O.CSR(Ap.size - 1, Ap, Aj, Ax)
    elif which == "thermal-ring":
        # 518,400 rows: 507 windowed blocks, twice the CU count
        Ap, Aj, Ax = thermal_like(m=720, window=2048)
        A = O.CSR(Ap.size - 1, Ap, Aj, Ax)
    elif which == "jumpy":
        A = _jumpy(700000, 29)
    elif which == "wide":
        A = _scattered(40000, 12, maxlen=12, reach=40000)
    else:
        A = _scattered(5000, 11)
    M = lssp_amd.DMat(dev, A.Ap, A.Aj, A.Ax)
    assert M.ndiag == 0
    assert M.windowed == (which != "wide")
    xh, yh = uniform(0x5EED, A.n), uniform(3, A.n)
    x, y, z = dev.vec(A.n, xh), dev.vec(A.n, yh), dev.vec(A.n, yh)
    M.mv_mxy(x, z)
    assert np.array_equal(z.download(), O.spmv(0, A, xh))
    # an x that is not 16-byte aligned (a C caller's x + 1): the windowed
    # kernel stages it with scalar loads instead
    xo = dev.vec(A.n + 1, np.concatenate([[np.nan], xh]))
    import ctypes
    assert dev.L.lssp_amd_mv_mxy(dev.h, M.h, ctypes.c_void_p(xo.ptr.value + 8), z.ptr) == 0
    assert np.array_equal(z.download(), O.spmv(0, A, xh))
    M.mv_amxy(-0.75, x, z)
    assert np.array_equal(z.download(), O.spmv(1, A, xh, alpha=-0.75))
    M.mv_amxpbyz(-1.0, x, 1.0, y, z)
    assert np.array_equal(z.download(), O.spmv(3, A, xh, alpha=-1.0, beta=1.0, y=yh))
    M.mv_amxpby(1.5, x, 0.25, y)
    assert np.array_equal(y.download(), O.spmv(2, A, xh, alpha=1.5, beta=0.25, z=yh.copy()))
    # CG (fused q.p in the SpMV epilogue) in tree mode vs the oracle
    if which in ("thermal", "thermal-big", "thermal-ring", "wide"):
        b = dev.vec(A.n, np.ones(A.n))
        xs = dev.vec(A.n, np.zeros(A.n))
        r = lssp_amd.solve(dev, M, None, xs, b, solver=lssp_amd.CG, maxit=60, trace_cap=100000)
        o = O.solve(lssp_amd.CG, A, np.ones(A.n), maxit=60, mode=O.TREE)
        assert r.nits == o.nits and np.array_equal(r.trace, o.trace, equal_nan=True)
        assert np.array_equal(xs.download(), o.x, equal_nan=True)


def test_spmv_column_coding_chosen_by_structure(dev):
    """Stencil matrices get the 1-byte diagonal-id column stream (5-pt: 5
    offsets, 7-pt: 7), scattered ones keep int32 columns; both bitwise vs the
    oracle (the golden SpMV cases cover both layouts against the reference)."""
    import lssp_amd
    from inputs import conv_rand
    for (Ap, Aj, Ax), want in ((lssp_amd.poisson(2, 40), 5), (lssp_amd.poisson(3, 20), 7),
                               (conv_rand(3000, 3000, 8, 5), 0)):
        n = Ap.size - 1
        M = lssp_amd.DMat(dev, Ap, Aj, Ax)
        assert M.ndiag == want
        xv = uniform(0x5EED, n)
        x, z = dev.vec(n, xv), dev.vec(n)
        M.mv_mxy(x, z)
        ref = O.spmv(0, O.CSR(n, Ap, Aj, Ax), xv)
        assert np.array_equal(z.download().view(np.int64), ref.view(np.int64))


def test_env_selected_paths_bitwise_vs_oracle():
    """The two remaining path selectors, each in a fresh process (they are read
    once): LSSP_AMD_ILU_HOST=1 runs ILUK's numeric factorization on the host
    (ilu_setup.cpp, pc-iluk.cxx:347-409) instead of the GPU, and LSSP_AMD_LINE=0
    gives a 7-pt grid's ILU(0) the general packet sweeps (k_tri_pk6) instead of
    the line sweeps.  Factors and applies are bitwise the oracle's either way,
    and a BiCGSTAB solve on them is bitwise the oracle's tree-mode run."""
    import subprocess
    import sys
    code = r'''
import sys, numpy as np
sys.path.insert(0, "ROOT"); sys.path.insert(0, "ROOT/tests")
import lssp_amd, oracle as O
from inputs import uniform
A = O.poisson(3, 24)
dev = lssp_amd.Device(0)
M = lssp_amd.DILU.create(dev, A.Ap, A.Aj, A.Ax, kind=lssp_amd.ILUK, level=0)
(Lp, Lj, Lx), (Up, Uj, Ux) = M.factors()
L, U = O.ilu(A, "iluk", level=0)
assert np.array_equal(Lj, L.Aj) and np.array_equal(Uj, U.Aj)
assert np.array_equal(Lx.view(np.int64), L.Ax.view(np.int64)) and np.array_equal(Ux.view(np.int64), U.Ax.view(np.int64))
rhs = uniform(5, A.n)
x = dev.vec(A.n)
for _ in range(2):
    M.apply(x, dev.vec(A.n, rhs))
    assert np.array_equal(x.download().view(np.int64), O.ilu_apply(L, U, rhs).view(np.int64))
Ad = lssp_amd.DMat(dev, A.Ap, A.Aj, A.Ax)
xs, b = dev.vec(A.n, np.zeros(A.n)), dev.vec(A.n, np.ones(A.n))
r = lssp_amd.solve(dev, Ad, M, xs, b, solver=lssp_amd.BICGSTAB, trace_cap=1000)
o = O.solve(O.BICGSTAB, A, np.ones(A.n), L=L, U=U, mode=O.TREE)
assert r.nits == o.nits and np.array_equal(r.trace, o.trace) and np.array_equal(xs.download(), o.x)
print("ok", r.nits)
'''.replace("ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    for env in ({"LSSP_AMD_ILU_HOST": "1"}, {"LSSP_AMD_LINE": "0"}, {"LSSP_AMD_ILU_HOST": "1", "LSSP_AMD_LINE": "0"}):
        res = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **env), capture_output=True, text=True,
                             timeout=150)
        assert res.returncode == 0 and "ok" in res.stdout, (env, res.stdout[-2000:], res.stderr[-2000:])


def test_sliced_copy_footprint_and_cap_fallback(dev, monkeypatch):
    """A windowed matrix reports the sliced copy it keeps beside the CSR
    (lssp_amd_mat_bytes); one whose padded copy exceeds the slice-offset cap
    is not windowed and runs on k_spmv3 with the same sums (the cap is lowered
    through LSSP_AMD_SELL_CAP to reach that branch at a small size)."""
    import lssp_amd
    from lssp_amd.synthetic import thermal_like
    Ap, Aj, Ax = thermal_like(m=150, window=512)
    A = O.CSR(Ap.size - 1, Ap, Aj, Ax)
    xh = uniform(0x5EED, A.n)
    ref = O.spmv(0, A, xh)
    M = lssp_amd.DMat(dev, A.Ap, A.Aj, A.Ax)
    csr, aux = M.device_bytes
    assert M.windowed and csr == 4 * (A.n + 1) + 12 * A.nnz
    assert aux >= 10 * A.nnz  # f64 values + 16-bit columns, padded per slice
    monkeypatch.setenv("LSSP_AMD_SELL_CAP", "1000")
    F = lssp_amd.DMat(dev, A.Ap, A.Aj, A.Ax)
    assert not F.windowed and F.device_bytes[1] == 0
    x, z = dev.vec(A.n, xh), dev.vec(A.n)
    F.mv_mxy(x, z)
    assert np.array_equal(z.download(), ref)
    M.mv_mxy(x, z)
    assert np.array_equal(z.download(), ref)


def test_spmv_group_order_bitwise_vs_oracle():
    """The product's column-group block order (kernels.hip, spmv_group_env:
    automatic only for planes of >= 512 blocks, forced here through
    LSSP_AMD_SPMV_ORDER on a 64^3 grid, plane = 16 blocks) and its
    non-temporal vector operands (LSSP_AMD_SPMV_NTV) change which workgroup
    takes which 256-row block, never a sum: every product, fused dot and
    solver trace is bitwise the oracle's, for the full cube and for a slab
    with a ragged last plane (blocks past the last whole plane keep the
    natural order)."""
    import subprocess
    import sys
    code = r'''
import sys, numpy as np
sys.path.insert(0, "ROOT"); sys.path.insert(0, "ROOT/tests")
import lssp_amd, oracle as O
from inputs import uniform
from bench import local_block
dev = lssp_amd.Device(0, reduction=lssp_amd.TREE)
N = 64
for nl in (N ** 3, N * N * 37 + 100):
    Ap, Aj, Ax = local_block(*lssp_amd.poisson(3, N, 0, nl), 0, nl)
    A = O.CSR(nl, Ap, Aj, Ax)
    D = lssp_amd.DMat(dev, Ap, Aj, Ax)
    xh, yh = uniform(11, nl), uniform(12, nl)
    x, y, z = dev.vec(nl, xh), dev.vec(nl, yh), dev.vec(nl)
    D.mv_mxy(x, z)
    assert np.array_equal(z.download().view(np.int64), O.spmv(0, A, xh).view(np.int64))
    D.mv_amxpbyz(0.75, x, -1.25, y, z)
    assert np.array_equal(z.download().view(np.int64), O.spmv(3, A, xh, 0.75, -1.25, yh).view(np.int64))
    L, U = O.ilu(A, "iluk", level=0)
    M = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=lssp_amd.ILUK, level=0)
    for solver, pc in ((lssp_amd.BICGSTAB, True), (lssp_amd.CG, False)):
        xs, b = dev.vec(nl, np.zeros(nl)), dev.vec(nl, np.ones(nl))
        r = lssp_amd.solve(dev, D, M if pc else None, xs, b, solver=solver, tol_rel=0.0, tol_abs=0.0, tol_rb=0.0,
                           maxit=12, trace_cap=200)
        o = O.solve(solver, A, np.ones(nl), L=L if pc else None, U=U if pc else None, rtol=0.0, atol=0.0,
                    rbtol=0.0, maxit=12, mode=O.TREE, trace_cap=200)
        assert r.nits == o.nits == 12 and np.array_equal(r.trace, o.trace)
        assert np.array_equal(xs.download().view(np.int64), o.x.view(np.int64))
    M.close(); D.close()
print("ok")
'''.replace("ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    for env in ({"LSSP_AMD_SPMV_ORDER": "2"}, {"LSSP_AMD_SPMV_ORDER": "4", "LSSP_AMD_SPMV_NTV": "0"},
                {"LSSP_AMD_SPMV_ORDER": "0", "LSSP_AMD_SPMV_NTV": "1"}):
        res = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **env), capture_output=True, text=True,
                             timeout=170)
        assert res.returncode == 0 and "ok" in res.stdout, (env, res.stdout[-2000:], res.stderr[-2000:])
