"""Parity at the FULL sizes of BASELINE.json's configs 3, 4 and 5.

Small grids cannot reach the bugs that live at these sizes: 64-bit stream
offsets (config 4's matrix: 937,951,232 entries, 11.3 GB of column and value
stream, past 2^32 bytes), tens of thousands of packet-schedule levels (config
3's ILUT), and windowed-SpMV blocks whose column spans sit right at the
kernel's 16,384-column LDS limit (config 5).  Every check is bitwise against
the oracle's C restatement of the reference (mvops.cxx:118-150,
solver-tri.cxx:4-60, pc-ilut.cxx:51-286, solver-cg.cxx:8-136,
solver-gmres.cxx:12-255) on the same inputs.

* config 4's matrix (7-pt 512^3) on one GPU: y = A x (the 1-byte diagonal-id
  SpMV) and one ILU(0) apply (line sweeps) on the GPU's own factors;
* config 5 at its full size (thermal-like, m = 1108, window 4096): the
  windowed SpMV with spans measured on the host, then 100 CG iterations in
  TREE mode (the timed mode), trace and x;
* ILUT(1e-4, 20) at 128^3 (config 3's preconditioner, 3,195 levels): the
  factors and one apply, then GMRES(30) for 10 iterations in TREE mode.
"""
import numpy as np
import pytest

import oracle as O
from inputs import uniform

pytestmark = pytest.mark.gpu


def _bits_equal(a, b):
    return a.shape == b.shape and np.array_equal(a.view(np.int64), b.view(np.int64))


def test_config4_matrix_512_spmv_and_ilu0_apply_bitwise():
    import lssp_amd
    N = 512
    dev = lssp_amd.Device(0)
    try:
        Ap, Aj, Ax = lssp_amd.poisson(3, N)
        n, nnz = Ap.size - 1, int(Ap[-1])
        assert n == 134217728 and nnz == 937951232
        assert 12 * nnz > 2 ** 33  # column + value stream past 2^32 bytes (twice over)
        A = lssp_amd.DMat(dev, Ap, Aj, Ax)
        assert A.ndiag == 7
        xh = uniform(0x5EED, n)
        x, y = dev.vec(n, xh), dev.vec(n)
        A.mv_mxy(x, y)
        yg = y.download()
        Ao = O.CSR(n, Ap, Aj, Ax)
        assert _bits_equal(yg, O.spmv(0, Ao, xh))
        del yg
        A.close()
        M = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=lssp_amd.ILUK, level=0)
        assert M.levelsL == 3 * N - 2 and M.levelsU == 3 * N - 2
        del Aj, Ax, Ao
        rhs = uniform(4242, n)
        r = dev.vec(n, rhs)
        M.apply(y, r)
        got = y.download()
        (Lp, Lj, Lx), (Up, Uj, Ux) = M.factors()
        M.close()
        ref = O.ilu_apply(O.CSR(n, Lp, Lj, Lx), O.CSR(n, Up, Uj, Ux), rhs)
        assert _bits_equal(got, ref)
    finally:
        dev.close()


def test_config5_full_size_windowed_cg_tree_bitwise():
    import lssp_amd
    from lssp_amd.synthetic import thermal_like
    Ap, Aj, Ax = thermal_like(m=1108, window=4096)
    n = Ap.size - 1
    assert n == 1227664 and int(Ap[-1]) == 8584786
    # the 1024-row blocks' x spans, staged from lo rounded down to even
    # (capi.cpp build_windows): all within WIN_CAP = 16384, the widest near it
    starts = Ap[0:n:1024]
    ends = Ap[np.minimum(np.arange(1024, n + 1024, 1024), n)]
    spans = np.array([int(Aj[s:e].max()) + 1 - (int(Aj[s:e].min()) & ~1) for s, e in zip(starts, ends)])
    assert spans.max() <= 16384 and spans.max() > 12000, spans.max()
    dev = lssp_amd.Device(0, reduction=lssp_amd.TREE)
    try:
        A = lssp_amd.DMat(dev, Ap, Aj, Ax)
        assert A.ndiag == 0 and A.windowed
        xh = uniform(0x5EED, n)
        x, y = dev.vec(n, xh), dev.vec(n)
        A.mv_mxy(x, y)
        Ao = O.CSR(n, Ap, Aj, Ax)
        assert _bits_equal(y.download(), O.spmv(0, Ao, xh))
        b = dev.vec(n, np.ones(n))
        xs = dev.vec(n, np.zeros(n))
        maxit = 100
        r = lssp_amd.solve(dev, A, None, xs, b, solver=lssp_amd.CG, tol_rel=0.0, tol_abs=0.0, tol_rb=0.0,
                           maxit=maxit, trace_cap=4 * maxit + 16)
        o = O.solve(O.CG, Ao, np.ones(n), rtol=0.0, atol=0.0, rbtol=0.0, maxit=maxit, mode=O.TREE)
        assert r.nits == o.nits == maxit
        assert r.residual == o.residual
        assert _bits_equal(r.trace, o.trace)
        assert _bits_equal(xs.download(), o.x)
    finally:
        dev.close()


def test_ilut_128_factors_apply_and_gmres_tree_bitwise():
    import lssp_amd
    N = 128
    Ao = O.poisson(3, N)
    n = Ao.n
    dev = lssp_amd.Device(0, reduction=lssp_amd.TREE)
    try:
        M = lssp_amd.DILU.create(dev, Ao.Ap, Ao.Aj, Ao.Ax, kind=lssp_amd.ILUT, tol=1e-4, p=20)
        assert M.levelsL == 3195  # SURVEY A4 (the reference's L factor)
        (Lp, Lj, Lx), (Up, Uj, Ux) = M.factors()
        L, U = O.ilu(Ao, "ilut", tol=1e-4, p=20)
        for got, want in ((Lp, L.Ap), (Lj, L.Aj), (Up, U.Ap), (Uj, U.Aj)):
            assert np.array_equal(got, want)
        assert _bits_equal(Lx, L.Ax) and _bits_equal(Ux, U.Ax)
        rhs = uniform(77, n)
        r, x = dev.vec(n, rhs), dev.vec(n)
        for _ in range(2):  # twice: the shadow buffers alternate between applies
            M.apply(x, r)
            assert _bits_equal(x.download(), O.ilu_apply(L, U, rhs))
        A = lssp_amd.DMat(dev, Ao.Ap, Ao.Aj, Ao.Ax)
        b = dev.vec(n, np.ones(n))
        xs = dev.vec(n, np.zeros(n))
        maxit = 10
        res = lssp_amd.solve(dev, A, M, xs, b, solver=lssp_amd.GMRES, restart=30, maxit=maxit, trace_cap=4096)
        o = O.solve(O.GMRES, Ao, np.ones(n), L=L, U=U, maxit=maxit, restart=30, mode=O.TREE)
        assert res.nits == o.nits
        assert res.residual == o.residual
        assert _bits_equal(res.trace, o.trace)
        assert _bits_equal(xs.download(), o.x)
    finally:
        dev.close()


def test_ilu1_line_sweeps_128_and_exam_matrix_bitwise():
    """ILU(1) -- the reference's default level (pc.cxx:3) -- on the skewed line
    sweeps (linefill.hip): 7-pt 128^3 (2 x 763 levels, 144 x 2 tiles) and the
    5-pt 100^2 Laplacian of exam.cxx: factors equal the oracle's, one apply and
    both single sweeps bitwise."""
    import lssp_amd
    dev = lssp_amd.Device(0)
    try:
        for dim, N in ((3, 128), (2, 100)):
            Ap, Aj, Ax = lssp_amd.poisson(dim, N)
            n = Ap.size - 1
            M = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=lssp_amd.ILUK, level=1)
            assert M.sweep_layout() == ((2, 16, 8) if dim == 3 else (2, N, 1))  # 2-D: one workgroup (k_lineg)
            if dim == 3:
                assert M.levelsL == 6 * N - 5
            L, U = O.ilu(O.CSR(n, Ap, Aj, Ax), "iluk", level=1)
            (Lp, Lj, Lx), (Up, Uj, Ux) = M.factors()
            assert _bits_equal(Lx, L.Ax) and _bits_equal(Ux, U.Ax)
            rhs = uniform(777 + dim, n)
            y = dev.vec(n)
            M.apply(y, dev.vec(n, rhs))
            assert _bits_equal(y.download(), O.ilu_apply(L, U, rhs))
            one = O.CSR(n, np.arange(n + 1, dtype=np.int32), np.arange(n, dtype=np.int32), np.ones(n))
            M.trisolve(0, y, dev.vec(n, rhs))
            assert _bits_equal(y.download(), O.ilu_apply(L, one, rhs))
            M.trisolve(1, y, dev.vec(n, rhs))
            assert _bits_equal(y.download(), O.ilu_apply(one, U, rhs))
            M.close()
    finally:
        dev.close()
