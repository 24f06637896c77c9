"""The TIMED mode against the reference at full size: complete solves.

bench.py times the library's TREE reduction order: it is
bitwise equal to the oracle's restatement of that order, and its iterates
differ from the reference's sequential sums in the last bits, which BiCGSTAB
amplifies.  These tests pin what the timed mode must still share
with the reference (tests/golden/full.json, written by make_golden_full.py
from oracle/_ref/libref.so -- the reference compiled from /root/reference)
on the benchmark configurations, solved to the reference's defaults
rtol = atol = rb = 1e-7 (lssp.cxx:11-13), b = 1, x0 = 0:

  * bitwise equality with the oracle's TREE restatement of the same driver
    at full size (nits, residual, every scalar of the history, x), which
    separates "the order of the sums differs" from "the code differs";
  * the iteration count and final residual within the stated tolerances
    NITS_REL / RES_REL of the reference's (the stop test is
    solver-bicgstab.cxx:141-157 / solver-gmres.cxx:206-217);
  * the recomputed true residual ||b - A x|| at most TRUE_FACTOR times the
    reference's own true residual and the stop scale;

and, at 512^3 (config 4's matrix, which the reference cannot run here: 134 M
rows), convergence and the true residual as properties.
"""
import json
import math
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
_path = os.path.join(HERE, "golden", "full.json")
FULL = []
if os.path.exists(_path):
    with open(_path) as _f:
        FULL = json.load(_f)["cases"]

# documented tolerances of the timed (TREE) mode against the reference.  The
# summation order alone moves BiCGSTAB's stop by a few iterations (the
# oracle's TREE restatement of the same driver: 144 vs 145 at 216^3, 161 vs
# 155 at 256^3 -- tests/golden/full.json "tree"): its residual history is
# erratic near the tolerance, and the TREE and sequential scalar histories
# part after ~12 iterations at 1e-6 (lead_agree_* in full.json).  GMRES's
# restarted residual is smooth: its count and residual stay with the reference.
NITS_REL = {4: 0.05, 0: 0.0}   # |nits - ref| <= max(1, ceil(NITS_REL * ref))
RES_REL = {4: 0.5, 0: 1e-6}    # |res - ref| / ref
TRUE_FACTOR = 2.0              # true residual vs max(reference's true residual, stop scale)


def _fx(h):
    return float.fromhex(h)


def _solve_case(c):
    import lssp_amd
    from inputs import digest
    dev = lssp_amd.Device(0, reduction=lssp_amd.TREE)
    try:
        Ap, Aj, Ax = lssp_amd.poisson(3, c["N"])
        n = Ap.size - 1
        A = lssp_amd.DMat(dev, Ap, Aj, Ax)
        if c["pc"]["kind"] == "iluk":
            M = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=lssp_amd.ILUK, level=c["pc"]["level"])
        else:
            M = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=lssp_amd.ILUT, tol=c["pc"]["tol"], p=c["pc"]["p"])
        del Aj, Ax
        b = dev.vec(n, np.ones(n))
        x = dev.vec(n, np.zeros(n))
        r = lssp_amd.solve(dev, A, M, x, b, solver=c["solver"], tol_rel=c["rtol"], tol_abs=c["atol"],
                           tol_rb=c["rbtol"], maxit=5000, restart=c["restart"], trace_cap=200000)
        z = dev.vec(n)
        A.mv_amxpbyz(-1.0, x, 1.0, b, z)
        zh = z.download()
        true_res = math.sqrt(float(np.dot(zh, zh)))
        return r, true_res, n, digest(x.download())
    finally:
        dev.close()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("c", FULL, ids=[c["name"] for c in FULL])
def test_tree_mode_full_solve_vs_reference(c):
    from inputs import digest
    r, true_res, n, xsha = _solve_case(c)
    ref_nits, ref_res, ref_true = c["nits"], _fx(c["residual"]), _fx(c["true_residual"])
    rel = abs(r.residual - ref_res) / ref_res
    tr = c.get("tree")
    print(f"\n{c['name']}: nits {r.nits} (reference {ref_nits}"
          f"{', oracle TREE ' + str(tr['nits']) if tr else ''}), residual {r.residual:.6e} "
          f"(reference {ref_res:.6e}, rel {rel:.3e}), true residual {true_res:.6e} (reference {ref_true:.6e})")
    # the same algorithm in the same order as the oracle's TREE restatement: bit for bit
    if tr:
        assert r.nits == tr["nits"] and r.residual == _fx(tr["residual"])
        assert digest(r.trace) == tr["trace_sha256"] and xsha == tr["x_sha256"]
    # ... and within the stated tolerances of the reference's sequential order
    assert abs(r.nits - ref_nits) <= max(1, math.ceil(NITS_REL[c["solver"]] * ref_nits))
    assert rel <= RES_REL[c["solver"]]
    # the stop scale max(rtol ||r0||, atol, rb ||b||) with r0 = b (x0 = 0)
    scale = max(c["rtol"] * math.sqrt(n), c["atol"], c["rbtol"] * math.sqrt(n))
    assert r.residual <= scale
    assert true_res <= TRUE_FACTOR * max(ref_true, scale)


@pytest.mark.timeout(900)
def test_tree_mode_512_bicgstab_converges():
    """config 4's matrix on one GPU (7-pt 512^3, n = 134,217,728): BiCGSTAB +
    ILU(0) in the timed mode converges to the default tolerances and the
    recomputed true residual is at that scale (the reference does not run at
    this size here; round 2 measured 308 iterations)."""
    c = {"N": 512, "pc": {"kind": "iluk", "level": 0}, "solver": 4, "rtol": 1e-7, "atol": 1e-7,
         "rbtol": 1e-7, "restart": 30}
    r, true_res, n, _ = _solve_case(c)
    scale = 1e-7 * math.sqrt(n)
    print(f"\n512^3: nits {r.nits}, residual {r.residual:.6e} (stop scale {scale:.6e}), true {true_res:.6e}")
    assert 0 < r.nits < 5000 and r.residual <= scale
    assert true_res <= TRUE_FACTOR * scale


SERIAL_CASES = [c for c in FULL if c["solver"] == 4 and c["N"] in (216, 256)]


@pytest.mark.timeout(900)
@pytest.mark.parametrize("c", SERIAL_CASES, ids=[c["name"] for c in SERIAL_CASES])
def test_serial_mode_full_solve_bitwise_reference(c):
    """The reference-exact mode at the benchmark size, to convergence: SERIAL
    reductions (k_dot_serial, the sequential sum of vector.cxx:123-131) make
    the 216^3 BiCGSTAB + ILU(0) solve bit for bit the reference's own complete
    run (tests/golden/full.json from oracle/_ref/libref.so): the iteration count
    (145), the final residual, every one of the 872 dots and norms the driver
    computed (solver-bicgstab.cxx:73-157) and the sha256 of x."""
    import time
    import lssp_amd
    from inputs import digest
    dev = lssp_amd.Device(0, reduction=lssp_amd.SERIAL)
    try:
        Ap, Aj, Ax = lssp_amd.poisson(3, c["N"])
        n = Ap.size - 1
        A = lssp_amd.DMat(dev, Ap, Aj, Ax)
        M = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=lssp_amd.ILUK, level=c["pc"]["level"])
        del Aj, Ax
        b = dev.vec(n, np.ones(n))
        x = dev.vec(n, np.zeros(n))
        t0 = time.perf_counter()
        r = lssp_amd.solve(dev, A, M, x, b, solver=c["solver"], tol_rel=c["rtol"], tol_abs=c["atol"],
                           tol_rb=c["rbtol"], maxit=5000, restart=c["restart"], trace_cap=200000)
        dt = time.perf_counter() - t0
        print(f"\n{c['name']} SERIAL: {r.nits} iterations in {dt:.2f} s = {r.nits / dt:.2f} it/s")
        assert r.nits == c["nits"]
        assert r.residual.hex() == float.fromhex(c["residual"]).hex()
        assert [v.hex() for v in r.trace] == [float.fromhex(h).hex() for h in c["trace"]]
        assert digest(x.download()) == c["x_sha256"]
    finally:
        dev.close()
