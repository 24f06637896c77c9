#!/usr/bin/env python3
"""A/B of the U sweep's tail product (GPU box; tuning aid, not a test):
BiCGSTAB it/s with LSSP_AMD_TAIL=1 (the product in the U sweep's tail) and =0
(apply, then the product), alternated in one process, on the 7-pt N^3 grid
with ILU(0) and ILU(1); the traces must be bitwise equal.

    python tools/tail_bench.py [N] [iters] [levels]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lssp_amd  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 216
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    levels = [int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "0,1").split(",")]
    dev = lssp_amd.Device(0)
    Ap, Aj, Ax = lssp_amd.poisson(3, N)
    n = Ap.size - 1
    A = lssp_amd.DMat(dev, Ap, Aj, Ax)
    for level in levels:
        M = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=lssp_amd.ILUK, level=level)
        x = dev.vec(n)
        b = dev.vec(n, np.ones(n))
        out = {"N": N, "level": level, "iters": iters}
        traces = {}
        modes = os.environ.get("TAIL_MODES", "1,0").split(",")
        for rep in range(2):
            for mode in modes:
                os.environ["LSSP_AMD_TAIL"] = mode
                x.upload(np.zeros(n))
                lssp_amd.solve(dev, A, M, x, b, solver=lssp_amd.BICGSTAB, tol_rel=0.0, tol_abs=0.0, tol_rb=0.0,
                               maxit=5)
                x.upload(np.zeros(n))
                dev.sync()
                t0 = time.perf_counter()
                r = lssp_amd.solve(dev, A, M, x, b, solver=lssp_amd.BICGSTAB, tol_rel=0.0, tol_abs=0.0,
                                   tol_rb=0.0, maxit=iters, trace_cap=8 * iters + 16)
                dev.sync()
                dt = time.perf_counter() - t0
                out.setdefault(f"tail{mode}_it_s", []).append(round(iters / dt, 2))
                traces[mode] = r.trace
        if len(traces) > 1:
            out["bitwise"] = bool(np.array_equal(traces["1"], traces["0"]))
        print(json.dumps(out), flush=True)
        M.close()
    os.environ.pop("LSSP_AMD_TAIL", None)
    dev.close()


if __name__ == "__main__":
    main()
