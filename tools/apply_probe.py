#!/usr/bin/env python3
"""ILU applies for profiling (GPU box; tuning aid): builds the preconditioner of
the 7-pt N^3 grid and runs REPS applies back to back, so rocprofv3 kernel
stats / PMC passes see the sweeps alone.

    python tools/apply_probe.py [N] [ilut|iluk0|iluk1] [reps]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import lssp_amd
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    kind = sys.argv[2] if len(sys.argv) > 2 else "ilut"
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    d = lssp_amd.Device(0)
    Ap, Aj, Ax = lssp_amd.poisson(3, N)
    n = Ap.size - 1
    t0 = time.perf_counter()
    if kind == "ilut":
        M = lssp_amd.DILU.create(d, Ap, Aj, Ax, kind=lssp_amd.ILUT, tol=1e-4, p=20)
    else:
        M = lssp_amd.DILU.create(d, Ap, Aj, Ax, kind=lssp_amd.ILUK, level=int(kind[-1]))
    print(f"setup {time.perf_counter() - t0:.1f} s, levels {M.levelsL} / {M.levelsU}", flush=True)
    r = d.vec(n, np.ones(n))
    x = d.vec(n)
    M.apply(x, r)
    d.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        M.apply_async(x, r)
    d.sync()
    M.check()
    print(f"{reps} applies: {(time.perf_counter() - t0) / reps * 1e3:.3f} ms each", flush=True)


if __name__ == "__main__":
    main()
