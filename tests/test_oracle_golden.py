"""The CPU oracle against the reference's own outputs (tests/golden/).

Every comparison is bitwise.  This is what pins the oracle before it is used
as the checker of the HIP path.
"""
import numpy as np
import pytest

import oracle as O
from golden_util import build_matrix, case_id, cases, fx, matches, stored, vec
from inputs import uniform

SPMV = cases("spmv")
ILU = cases("ilu")
SOLVE = cases("solve")


@pytest.mark.parametrize("c", SPMV, ids=[case_id(c) for c in SPMV])
def test_spmv_matches_reference(c):
    A = build_matrix(c["mat"])
    x = uniform(c["xseed"], A.n)
    y = uniform(c["yseed"], A.n)
    z = O.spmv(c["op"], A, x, fx(c["alpha"]), fx(c["beta"]), y.copy(), y.copy())
    assert matches(c["out"], z)


def _factors(c, A):
    pc = c["pc"]
    if pc["kind"] == "iluk":
        return O.ilu(A, "iluk", level=pc["level"])
    if pc["kind"] == "ilut":
        return O.ilu(A, "ilut", tol=pc["tol"], p=pc["p"])
    return O.ilu(A, "iluk", level=0, blk=(A.n + pc["nblk"] - 1) // pc["nblk"])


@pytest.mark.parametrize("c", ILU, ids=[case_id(c) for c in ILU])
def test_ilu_factors_and_apply_match_reference(c):
    A = build_matrix(c["mat"])
    L, U = _factors(c, A)
    assert (L.nnz, U.nnz) == (c["nnzL"], c["nnzU"])
    assert matches(c["L"], L.Ap, L.Aj, L.Ax)
    assert matches(c["U"], U.Ap, U.Aj, U.Ax)
    assert matches(c["apply"], O.ilu_apply(L, U, uniform(c["rhs_seed"], A.n)))


@pytest.mark.parametrize("c", SOLVE, ids=[case_id(c) for c in SOLVE])
def test_solver_trace_matches_reference(c):
    A = build_matrix(c["mat"])
    b = vec(c["b"], A.n)
    x0 = None if c["x0"] is None else vec(c["x0"], A.n)
    L = U = None
    if c["pc"]["kind"] != "none":
        L, U = _factors(c, A)
    r = O.solve(c["solver"], A, b, x0=x0, L=L, U=U, rtol=fx(c["rtol"]), atol=fx(c["atol"]),
                rbtol=fx(c["rbtol"]), maxit=c["maxit"], restart=c["restart"], mode=O.SERIAL)
    assert r.nits == c["nits"]
    assert r.residual == fx(c["residual"])
    assert matches(c["trace"], r.trace)  # every dot/norm, bit for bit
    assert matches(c["x"], r.x)


def test_tree_mode_same_iterations_as_serial():
    """The GPU's canonical reduction order changes only rounding."""
    A = O.poisson(3, 32)
    L, U = O.ilu(A, "iluk", level=0)
    b = np.ones(A.n)
    s = O.solve(O.BICGSTAB, A, b, L=L, U=U, mode=O.SERIAL)
    t = O.solve(O.BICGSTAB, A, b, L=L, U=U, mode=O.TREE)
    assert abs(s.nits - t.nits) <= 1
    assert t.residual <= 1e-7 * np.sqrt(A.n) or t.residual <= 1e-7 * s.trace[1]
    n = min(len(s.trace), len(t.trace), 12)
    np.testing.assert_allclose(t.trace[:n], s.trace[:n], rtol=1e-9)


def test_tree_reduction_definition():
    """Level-1 256-chunks + level-2 1024 lanes, against a direct numpy restatement."""
    for n in [1, 255, 256, 257, 1000, 65536 + 17, 300000]:
        x = uniform(11, n)
        y = uniform(12, n)
        p = x * y
        C = (n + 255) // 256
        v = np.zeros(C * 256)
        v[:n] = p
        v = v.reshape(C, 4, 64)
        for off in (32, 16, 8, 4, 2, 1):
            v = v[..., :off] + v[..., off:2 * off]
        w = v[..., 0]
        S = (w[:, 0] + w[:, 1]) + (w[:, 2] + w[:, 3])
        K = (C + 1023) // 1024
        S2 = np.zeros(K * 1024)
        S2[:C] = S
        acc = np.zeros(1024)
        for k in range(K):
            acc = acc + S2[k * 1024:(k + 1) * 1024]
        u = acc.reshape(16, 64)
        for off in (32, 16, 8, 4, 2, 1):
            u = u[:, :off] + u[:, off:2 * off]
        u = u[:, 0]
        for off in (8, 4, 2, 1):
            u = u[:off] + u[off:2 * off]
        assert O.dot(x, y, O.TREE) == u[0]
        assert O.dot(x, y, O.SERIAL) == pytest.approx(u[0], rel=1e-12)


def _large():
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "large.json")) as f:
        return json.load(f)["cases"]


def test_oracle_prank_serial_is_the_reference_sequential_sum():
    """SERIAL mode with P ranks is the reference's one sequential sum (the GPU
    ranks continue each other's running sums): the oracle's 8-rank block-Jacobi
    run equals the reference's own nblk = 8 solve at 64^3 (config 4's split)."""
    from inputs import digest
    g = [c for c in _large() if c["pc"]["kind"] == "bj"][0]
    A = O.poisson(3, g["N"])
    nb = g["pc"]["nblk"]
    L, U = O.ilu(A, "iluk", level=0, blk=(A.n + nb - 1) // nb)
    r = O.solve(O.BICGSTAB, A, np.ones(A.n), L=L, U=U, mode=O.SERIAL, nranks=nb, maxit=g["maxit"])
    assert r.nits == g["nits"] and r.residual.hex() == g["residual"]
    assert [v.hex() for v in r.trace] == g["trace"]
    assert digest(r.x) == g["x_sha256"]


def test_oracle_matches_reference_at_bench_size():
    """216^3 (n = 10,077,696): the first five BiCGSTAB + ILU(0) iterations, every
    scalar and x, equal to the reference's (tests/golden/large.json)."""
    from inputs import digest
    g = [c for c in _large() if c["pc"]["kind"] == "iluk" and c["N"] == 216][0]
    A = O.poisson(3, g["N"])
    L, U = O.ilu(A, "iluk", level=0)
    r = O.solve(O.BICGSTAB, A, np.ones(A.n), L=L, U=U, mode=O.SERIAL, maxit=g["maxit"])
    assert r.nits == g["nits"] and r.residual.hex() == g["residual"]
    assert [v.hex() for v in r.trace] == g["trace"]
    assert digest(r.x) == g["x_sha256"]
