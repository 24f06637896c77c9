#!/usr/bin/env python3
"""Add the ORACLE's tree-order solves to tests/golden/full.json.

    python tests/golden/make_golden_full_tree.py [case ...]

For every case of full.json (the reference's complete solves, written by
make_golden_full.py), run oracle/lssp_oracle.c -- the CPU restatement of the
same drivers -- in TREE reduction mode (the order the
timed GPU path uses) on the same inputs, and store its iteration count,
residual and a per-iteration comparison with the reference's scalar history.
This separates the two things a timed-mode run can differ from the reference
in: the summation order (oracle TREE vs reference: the same algorithm, only
the order of every dot's additions differs) and the implementation (GPU TREE
vs oracle TREE: bitwise, tests/test_gpu_refconv.py).
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


def lead_agree(ref, got, tol):
    """number of leading scalars whose relative deviation is <= tol"""
    k = min(len(ref), len(got))
    dev = np.abs(got[:k] - ref[:k]) / np.maximum(np.abs(ref[:k]), 1e-300)
    bad = np.nonzero(dev > tol)[0]
    return int(bad[0]) if bad.size else k


def main():
    path = os.path.join(HERE, "full.json")
    with open(path) as f:
        doc = json.load(f)
    want = set(sys.argv[1:])
    for c in doc["cases"]:
        if want and c["name"] not in want:
            continue
        A = O.poisson(3, c["N"])
        t0 = time.time()
        if c["pc"]["kind"] == "iluk":
            L, U = O.ilu(A, "iluk", level=c["pc"]["level"])
        else:
            L, U = O.ilu(A, "ilut", tol=c["pc"]["tol"], p=c["pc"]["p"])
        R = O.solve(c["solver"], A, np.ones(A.n), L=L, U=U, rtol=c["rtol"], atol=c["atol"], rbtol=c["rbtol"],
                    maxit=5000, restart=c["restart"], mode=O.TREE)
        ref = np.array([float.fromhex(h) for h in c["trace"]])
        c["tree"] = {"nits": R.nits, "residual": R.residual.hex(), "x_sha256": digest(R.x),
                     "trace_len": int(len(R.trace)), "trace_sha256": digest(R.trace),
                     "lead_agree_1e-12": lead_agree(ref, R.trace, 1e-12),
                     "lead_agree_1e-6": lead_agree(ref, R.trace, 1e-6),
                     "lead_agree_1e-2": lead_agree(ref, R.trace, 1e-2)}
        print(f"{c['name']}: oracle TREE nits {R.nits} (reference {c['nits']}), residual {R.residual:.6e}, "
              f"leading scalars within 1e-12 / 1e-6 / 1e-2: {c['tree']['lead_agree_1e-12']} / "
              f"{c['tree']['lead_agree_1e-6']} / {c['tree']['lead_agree_1e-2']} of {len(ref)} "
              f"({time.time() - t0:.0f} s)", flush=True)
        del A, L, U, R
        with open(path, "w") as f:
            json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
