#!/usr/bin/env python3
"""Generate tests/golden/full.json: the REFERENCE's complete solves at the
benchmark sizes (oracle/_ref/libref.so, the reference compiled in place).

    make -C oracle all ref && python tests/golden/make_golden_full.py [case ...]

Each case is run to convergence with the reference's defaults rtol = atol = rb
= 1e-7 (lssp.cxx:11-13), b = 1, x0 = 0, and records what the timed (TREE
reduction) mode of the library is pinned against at full size
(tests/test_gpu_refconv.py):

  * nits and the final residual (float.hex) -- the stop test of
    solver-bicgstab.cxx:141-157 / solver-gmres.cxx:206-217;
  * the residual history ||r_k|| (BiCGSTAB: the :149 norm of every iteration;
    GMRES: the |g_{i+1}| estimates are not visible through the API, so the
    history is every norm the driver computed -- restart residuals);
  * ||b - A x|| recomputed in the reference's own SpMV and dot order;
  * the wall time of the reference's solve on this container's CPU (1 core).

Cases: 216^3 BiCGSTAB+ILUK(0) (the headline config,
n = 10,077,696; 145 its), 256^3 BiCGSTAB+ILUK(0) (config 2; 155 its), 256^3
GMRES(30)+ILUT(1e-4, 20) (config 3; 162 its).
"""
from __future__ import annotations

import json
import math
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

import oracle as O  # noqa: E402
from inputs import digest  # noqa: E402

CASES = {
    "bicgstab_iluk0_216": dict(N=216, solver=O.BICGSTAB, pc=O.PC_ILUK, level=0),
    "bicgstab_iluk0_256": dict(N=256, solver=O.BICGSTAB, pc=O.PC_ILUK, level=0),
    "gmres30_ilut_256": dict(N=256, solver=O.GMRES, pc=O.PC_ILUT, ilut_tol=1e-4, ilut_p=20, restart=30),
}


def true_residual(A, x, b):
    """||b - A x|| in the reference's order: lssp_mv_amxpbyz(-1, A, x, 1, b)
    (mvops.cxx:42-78) then lssp_vec_norm (vector.cxx:135-139)."""
    r = np.zeros(A.n)
    O.ref_spmv(3, A, x, alpha=-1.0, beta=1.0, y=np.array(b, dtype=np.float64), z=r)
    return math.sqrt(O.ref_dot(r, r))


def run(name, c):
    A = O.poisson(3, c["N"])
    b = np.ones(A.n)
    t0 = time.time()
    R = O.ref_solve(c["solver"], A, b, pc=c["pc"], level=c.get("level", 0), ilut_tol=c.get("ilut_tol", 1e-3),
                    ilut_p=c.get("ilut_p", -1), maxit=5000, restart=c.get("restart", 30))
    wall = time.time() - t0
    tr = true_residual(A, R.x, b)
    out = {"name": name, "N": c["N"], "n": A.n, "nnz": A.nnz, "solver": c["solver"],
           "pc": {"kind": "iluk" if c["pc"] == O.PC_ILUK else "ilut", "level": c.get("level", 0),
                  "tol": c.get("ilut_tol"), "p": c.get("ilut_p")},
           "restart": c.get("restart", 30), "rtol": 1e-7, "atol": 1e-7, "rbtol": 1e-7,
           "nits": R.nits, "residual": R.residual.hex(), "true_residual": tr.hex(),
           "trace": [float(v).hex() for v in R.trace], "x_sha256": digest(R.x),
           "t_setup_s": round(R.t_setup, 2), "t_solve_s": round(R.t_solve, 2), "wall_s": round(wall, 1)}
    print(f"{name}: nits {R.nits} residual {R.residual:.17e} true {tr:.6e} "
          f"(setup {R.t_setup:.1f} s, solve {R.t_solve:.1f} s)", flush=True)
    return out


def main():
    path = os.path.join(HERE, "full.json")
    have = {}
    if os.path.exists(path):
        with open(path) as f:
            have = {c["name"]: c for c in json.load(f)["cases"]}
    for name in sys.argv[1:] or list(CASES):
        have[name] = run(name, CASES[name])
        with open(path, "w") as f:
            json.dump({"generator": "tests/golden/make_golden_full.py",
                       "source": "oracle/_ref/libref.so (reference compiled in place from /root/reference, "
                                 "g++ -O2), 1 core of this container",
                       "cases": [have[k] for k in CASES if k in have]}, f, indent=1)


if __name__ == "__main__":
    main()
