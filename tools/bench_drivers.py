#!/usr/bin/env python3
"""Iterations per second of Krylov drivers on 7-pt Poisson N^3 with ILU(0)
(GPU box; tuning / logging aid).

    python tools/bench_drivers.py [N] [iters] [solver,...]

Each solve runs with zero tolerances, so it performs exactly `iters`
iterations; one JSON line per driver (LSSP_AMD_LIB selects another build).
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    names = (sys.argv[3] if len(sys.argv) > 3 else "bicgsafe,tfqmr,cgs,bicrstab,qmrcgstab,gpbicg").split(",")
    import lssp_amd
    dev = lssp_amd.Device(0)
    Ap, Aj, Ax = lssp_amd.poisson(3, N)
    n = Ap.size - 1
    A = lssp_amd.DMat(dev, Ap, Aj, Ax)
    M = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=lssp_amd.ILUK, level=0)
    b = dev.vec(n, np.ones(n))
    x = dev.vec(n)
    for name in names:
        sv = getattr(lssp_amd, name.upper())
        kw = dict(solver=sv, tol_rel=0.0, tol_abs=0.0, tol_rb=0.0)
        x.upload(np.zeros(n))
        lssp_amd.solve(dev, A, M, x, b, maxit=3, **kw)  # warm-up
        x.upload(np.zeros(n))
        dev.sync()
        t0 = time.perf_counter()
        r = lssp_amd.solve(dev, A, M, x, b, maxit=iters, **kw)
        dev.sync()
        dt = time.perf_counter() - t0
        print(json.dumps({"solver": name, "N": N, "iters": r.nits, "it_per_s": round(r.nits / dt, 2),
                          "ms_per_it": round(dt / max(r.nits, 1) * 1e3, 3),
                          "lib": os.path.basename(os.environ.get("LSSP_AMD_LIB", "default"))}), flush=True)
    dev.close()


if __name__ == "__main__":
    main()
