"""Parity at the benchmark sizes (the headline 216^3 and config 2's 256^3).

* SERIAL reduction mode against the REFERENCE's own first five BiCGSTAB +
  ILUK(0) iterations at 216^3 and 256^3 (tests/golden/large.json, written by
  make_golden_large.py from oracle/_ref/libref.so): every dot and norm the
  driver computed (solver-bicgstab.cxx:86-150), the iteration count, the
  residual and a sha256 of x -- bit for bit.
* TREE mode (the mode bench.py times) against the oracle's restatement of the
  same canonical order at 216^3: trace and x bit for bit.

These are the sizes where a packet, schedule or int32-position bug that small
grids cannot reach would show (10-17 M rows, 70-117 M nonzeros).
"""
import json
import os

import numpy as np
import pytest

import oracle as O
from inputs import digest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "large.json")) as _f:
    LARGE = json.load(_f)["cases"]
GRIDS = [c for c in LARGE if c["pc"]["kind"] == "iluk"]


def _setup(dev, N):
    import lssp_amd
    Ap, Aj, Ax = lssp_amd.poisson(3, N)
    A = lssp_amd.DMat(dev, Ap, Aj, Ax)
    M = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=lssp_amd.ILUK, level=0)
    return (Ap, Aj, Ax), A, M


@pytest.mark.parametrize("c", GRIDS, ids=[f"N{c['N']}" for c in GRIDS])
def test_first_iterations_serial_bitwise_vs_reference(c):
    import lssp_amd
    dev = lssp_amd.Device(0, reduction=lssp_amd.SERIAL)
    try:
        _, A, M = _setup(dev, c["N"])
        n = A.nx
        x = dev.vec(n, np.zeros(n))
        b = dev.vec(n, np.ones(n))
        r = lssp_amd.solve(dev, A, M, x, b, solver=lssp_amd.BICGSTAB, maxit=c["maxit"], trace_cap=4096)
        assert r.nits == c["nits"]
        assert r.residual == float.fromhex(c["residual"])
        assert [v.hex() for v in r.trace] == c["trace"]
        assert digest(x.download()) == c["x_sha256"]
    finally:
        dev.close()


def test_bench_size_tree_bitwise_vs_oracle():
    import lssp_amd
    N, maxit = 216, 5
    dev = lssp_amd.Device(0, reduction=lssp_amd.TREE)
    try:
        (Ap, Aj, Ax), A, M = _setup(dev, N)
        n = A.nx
        x = dev.vec(n, np.zeros(n))
        b = dev.vec(n, np.ones(n))
        r = lssp_amd.solve(dev, A, M, x, b, solver=lssp_amd.BICGSTAB, maxit=maxit, trace_cap=4096)
        xg = x.download()
        del M, A
    finally:
        dev.close()
    Ao = O.CSR(Ap.size - 1, Ap, Aj, Ax)
    L, U = O.ilu(Ao, "iluk", level=0)
    o = O.solve(O.BICGSTAB, Ao, np.ones(Ao.n), L=L, U=U, mode=O.TREE, maxit=maxit)
    assert r.nits == o.nits == maxit
    assert r.residual == o.residual
    assert np.array_equal(r.trace, o.trace)
    assert np.array_equal(xg, o.x)
