#!/usr/bin/env python3
"""Generate tests/golden/large.json: the REFERENCE's first iterations at the
benchmark sizes (oracle/_ref/libref.so, the reference compiled in place).

    make -C oracle all ref && python tests/golden/make_golden_large.py

BiCGSTAB + ILUK(0) on the 7-pt Poisson grids 216^3 (the headline config,
n = 10,077,696) and 256^3 (config 2), b = 1, x0 = 0, maxit = 5: every dot and
norm the reference driver computed (solver-bicgstab.cxx:86-150, recorded by
ref_shim.cxx's --wrap of lssp_vec_dot / lssp_vec_norm) as exact float.hex
strings, the iteration count, the residual and a sha256 of x (the vector itself
is 80-134 MB, too large to commit).  Plus block-Jacobi ILU(0) with 8 blocks on
the 64^3 grid solved to convergence (the 8-rank partition of config 4,
pc-iluk.cxx:411-552 with blk = ceil(n/8)).  The GPU tests match these in the
library's SERIAL reduction mode, bit for bit (tests/test_gpu_large.py).
"""
from __future__ import annotations

import json
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


def main():
    cases = []
    for N, maxit in ((216, 5), (256, 5)):
        A = O.poisson(3, N)
        t0 = time.time()
        R = O.ref_solve(O.BICGSTAB, A, np.ones(A.n), pc=O.PC_ILUK, level=0, maxit=maxit)
        cases.append({"solver": O.BICGSTAB, "pc": {"kind": "iluk", "level": 0}, "N": N, "maxit": maxit,
                      "nits": R.nits, "residual": R.residual.hex(), "trace": [float(v).hex() for v in R.trace],
                      "x_sha256": digest(R.x)})
        print(f"N={N} nits {R.nits} residual {R.residual:.17e} ({time.time() - t0:.1f} s)", flush=True)
        del A, R
    N, nblk = 64, 8
    A = O.poisson(3, N)
    R = O.ref_solve_bj(O.BICGSTAB, A, np.ones(A.n), nblk, maxit=5000)
    cases.append({"solver": O.BICGSTAB, "pc": {"kind": "bj", "nblk": nblk}, "N": N, "maxit": 5000,
                  "nits": R.nits, "residual": R.residual.hex(), "trace": [float(v).hex() for v in R.trace],
                  "x_sha256": digest(R.x)})
    print(f"bj N={N} nblk={nblk}: nits {R.nits} residual {R.residual:.17e}", flush=True)
    with open(os.path.join(HERE, "large.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden_large.py",
                   "source": "oracle/_ref/libref.so (reference compiled in place from /root/reference, g++ -O2)",
                   "cases": cases}, f, indent=1)


if __name__ == "__main__":
    main()
