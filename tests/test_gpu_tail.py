"""The U sweep's tail product (launch_line_apply_spmv, linesweep.hip k_line2):
BiCGSTAB's v = A ph and t = A sh (solver-bicgstab.cxx:110, :133) computed by
the U sweep's own workgroups as the planes of ph / sh become final.  Every
value must be bitwise the two-step path (the apply, then k_spmv3 with its
fused dots) and the oracle's TREE-order restatement of the driver.

LSSP_AMD_TAIL=2 makes an ineligible call fail instead of falling back, so a
passing run here proves the tail path ran; LSSP_AMD_TAIL=0 is the two-step
path.  Cases (ILU(0), k_line2, and ILU(1), the skewed k_linef sweeps): cubes
with partial tiles in j and k (N = 24, 40), a 2-D 5-point
grid (one plane: every chunk waits for the whole sweep), a block-Jacobi
factor on one rank (plane cuts between tile rows), and a run that converges
mid-batch (the guard skips queued sweeps and tails: the tile counts and chunk
claims must stay consistent for the next solve).
"""
import os

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


def _solve(dev, Ap, Aj, Ax, mode, maxit, blk=0, tol=0.0, level=0):
    import lssp_amd
    n = Ap.size - 1
    old = os.environ.get("LSSP_AMD_TAIL")
    os.environ["LSSP_AMD_TAIL"] = mode
    try:
        A = lssp_amd.DMat(dev, Ap, Aj, Ax)
        M = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=lssp_amd.ILUK, level=level, blk=blk)
        assert M.sweep_layout()[0] == 1 + level  # the ILU(0) / ILU(1) line sweeps
        out = []
        for _ in range(2):  # twice: the counters and claims carry over between solves
            x = dev.vec(n, np.zeros(n))
            b = dev.vec(n, np.ones(n))
            r = lssp_amd.solve(dev, A, M, x, b, solver=lssp_amd.BICGSTAB, tol_rel=tol, tol_abs=tol, tol_rb=tol,
                               maxit=maxit, trace_cap=8 * maxit + 16)
            out.append((r.nits, r.residual, r.trace, x.download()))
        M.close()
        A.close()
        return out
    finally:
        if old is None:
            os.environ.pop("LSSP_AMD_TAIL", None)
        else:
            os.environ["LSSP_AMD_TAIL"] = old


@pytest.mark.parametrize("dim,N,blk,maxit,tol,level", [(3, 24, 0, 30, 0.0, 0), (3, 40, 0, 25, 0.0, 0),
                                                       (2, 100, 0, 40, 0.0, 0), (3, 32, 32 * 32 * 11, 30, 0.0, 0),
                                                       (3, 32, 0, 500, 1e-7, 0), (3, 24, 0, 30, 0.0, 1),
                                                       (3, 40, 0, 500, 1e-7, 1), (2, 100, 0, 40, 0.0, 1)],
                         ids=["cube24", "cube40", "square100", "blockjacobi32", "converges32", "ilu1-cube24",
                              "ilu1-converges40", "ilu1-square100"])
def test_tail_product_bitwise_two_step_and_oracle(dim, N, blk, maxit, tol, level):
    import lssp_amd
    Ap, Aj, Ax = lssp_amd.poisson(dim, N)
    n = Ap.size - 1
    dev = lssp_amd.Device(0, reduction=lssp_amd.TREE)
    # (a 2-D ILU(1) factor runs on one workgroup, k_lineg, which has no tail
    # product: the skewed tiles are selected for it here)
    old = os.environ.get("LSSP_AMD_LINEG")
    os.environ["LSSP_AMD_LINEG"] = "0"
    try:
        fused = _solve(dev, Ap, Aj, Ax, "2", maxit, blk, tol, level)
        plain = _solve(dev, Ap, Aj, Ax, "0", maxit, blk, tol, level)
    finally:
        dev.close()
        if old is None:
            os.environ.pop("LSSP_AMD_LINEG", None)
        else:
            os.environ["LSSP_AMD_LINEG"] = old
    Ao = O.CSR(n, Ap, Aj, Ax)
    L, U = O.ilu(Ao, "iluk", level=level, blk=blk)
    o = O.solve(O.BICGSTAB, Ao, np.ones(n), L=L, U=U, rtol=tol, atol=tol, rbtol=tol, maxit=maxit, mode=O.TREE)
    for f, p in zip(fused, plain):
        assert f[0] == p[0] == o.nits
        assert f[1] == p[1] == o.residual
        assert np.array_equal(f[2].view(np.int64), p[2].view(np.int64))
        assert np.array_equal(f[2], o.trace)
        assert np.array_equal(f[3].view(np.int64), o.x.view(np.int64))
