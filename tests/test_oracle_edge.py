"""The oracle on the edge shapes of tests/test_gpu_edge.py, pinned against the
reference itself (oracle/_ref/libref.so, built from /root/reference by
oracle/Makefile; skipped where it is absent, e.g. on the GPU box)."""
import numpy as np
import pytest

import oracle as O
from inputs import rand_csr, uniform

pytestmark = pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref/libref.so not built")

import test_gpu_edge as E  # noqa: E402  (the shapes; its GPU tests are not collected from here)


@pytest.mark.parametrize("op", [0, 1, 2, 3])
@pytest.mark.parametrize("name", sorted(E.MATS))
def test_oracle_spmv_edge_shapes_equal_reference(name, op):
    Ap, Aj, Ax = E.MATS[name]()
    n = Ap.size - 1
    A = O.CSR(n, Ap, Aj, Ax)
    x, y, z0 = uniform(0x5EED, n), uniform(0xB0B, n), uniform(0xCAFE, n)
    want = O.ref_spmv(op, A, x, -0.75, 1.25, y=y.copy() if op == 3 else None, z=z0.copy())
    got = O.spmv(op, A, x, -0.75, 1.25, y=y.copy() if op == 3 else None, z=z0.copy())
    assert np.array_equal(got, want, equal_nan=True)


def test_oracle_spmv_nonfinite_equal_reference():
    A = O.poisson(2, 9)
    x = uniform(4, A.n)
    x[5], x[40] = np.inf, -0.0
    y = uniform(5, A.n)
    y[3], y[60] = np.nan, np.inf
    for op, beta in ((3, 0.0), (2, 0.0), (3, -1.0)):
        want = O.ref_spmv(op, A, x, 1.0, beta, y=y.copy(), z=y.copy())
        got = O.spmv(op, A, x, 1.0, beta, y=y.copy(), z=y.copy())
        assert np.array_equal(got, want, equal_nan=True), (op, beta)


@pytest.mark.parametrize("case", ["1x1", "diagonal", "empty_strict_rows"])
def test_oracle_degenerate_factors_equal_reference(case):
    if case == "1x1":
        Ap, Aj, Ax = E.MATS["1x1"]()
        lev = 0
    elif case == "diagonal":
        n = 300
        Ap, Aj, Ax = np.arange(n + 1, dtype=np.int32), np.arange(n, dtype=np.int32), 2.0 + uniform(9, n)
        lev = 0
    else:
        Ap, Aj, Ax = rand_csr(500, 2, 0x99, unsorted=True)
        lev = 1
    A = O.CSR(Ap.size - 1, Ap, Aj, Ax)
    (L, U) = O.ilu(A, "iluk", level=lev)
    (Lr, Ur) = O.ref_ilu(A, "iluk", level=lev)
    for mine, ref in ((L, Lr), (U, Ur)):
        assert np.array_equal(mine.Ap, ref.Ap) and np.array_equal(mine.Aj, ref.Aj)
        assert np.array_equal(mine.Ax, ref.Ax, equal_nan=True)
    rhs = uniform(0x1234, A.n)
    assert np.array_equal(O.ilu_apply(L, U, rhs), O.ref_ilu_apply(A, rhs, "iluk", level=lev), equal_nan=True)


@pytest.mark.parametrize("solver", ["BICGSTAB", "CG", "GMRES", "IDRS", "BICGSTABL", "TFQMR"])
@pytest.mark.parametrize("system", ["1x1", "diagonal"])
def test_oracle_trivial_systems_equal_reference(solver, system):
    if system == "1x1":
        Ap, Aj, Ax = E.MATS["1x1"]()
    else:
        n = 200
        Ap, Aj, Ax = np.arange(n + 1, dtype=np.int32), np.arange(n, dtype=np.int32), 1.0 + uniform(11, n) ** 2
    A = O.CSR(Ap.size - 1, Ap, Aj, Ax)
    b = uniform(0xB, A.n)
    rs = 2 if solver in ("IDRS", "BICGSTABL") else 4
    L, U = O.ilu(A, "iluk", level=0)
    o = O.solve(getattr(O, solver), A, b, L=L, U=U, maxit=50, restart=rs, mode=O.SERIAL)
    r = O.ref_solve(getattr(O, solver), A, b, pc=O.PC_ILUK, level=0, maxit=50, restart=rs)
    assert o.nits == r.nits
    assert np.array_equal([o.residual], [r.residual], equal_nan=True)
    assert np.array_equal(o.trace, r.trace, equal_nan=True)
    assert np.array_equal(o.x, r.x, equal_nan=True)
