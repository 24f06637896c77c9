#!/usr/bin/env python3
"""The 2-D line sweeps: one workgroup (k_lineg, the default for <= 256 lines)
against the tiled sweeps (LSSP_AMD_LINEG=0) on exam.cxx's configurations --
5-point 256^2 ILU(0) (BASELINE configs[0]) and 100^2 ILU(1) (exam.cxx as
shipped) -- plus a 2-D grid at the lane limit.  Per case: apply time (HIP
events, applies queued back to back) and BiCGSTAB it/s (tree, fixed
iterations).  GPU box; tuning/record aid, not a test.

    python tools/lineg_bench.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import lssp_amd  # noqa: E402
from bench_configs import apply_leg, timed_solve  # noqa: E402


def box2(nx, ny):
    """the 5-point Laplacian of an nx x ny grid (CSR, ascending columns)"""
    import numpy as np
    n = nx * ny
    Ap, Aj, Ax = [0], [], []
    for r in range(n):
        i, j = r % nx, r // nx
        for c, ok, v in ((r - nx, j > 0, -1.0), (r - 1, i > 0, -1.0), (r, True, 4.0), (r + 1, i < nx - 1, -1.0),
                         (r + nx, j < ny - 1, -1.0)):
            if ok:
                Aj.append(c)
                Ax.append(v)
        Ap.append(len(Aj))
    return np.array(Ap, np.int32), np.array(Aj, np.int32), np.array(Ax)


def main():
    dev = lssp_amd.Device(0)
    cases = [((256, 256), 0), ((100, 100), 1), ((100, 100), 0), ((256, 256), 1)]
    if "--lines" in sys.argv:  # per-level cost against the number of waves (lines per workgroup)
        cases = [((100, ny), 1) for ny in (64, 128, 192, 256)]
    for (N, NY), level in cases:
        Ap, Aj, Ax = lssp_amd.poisson(2, N) if N == NY else box2(N, NY)
        n = Ap.size - 1
        A = lssp_amd.DMat(dev, Ap, Aj, Ax)
        for lineg in ("1", "0"):
            os.environ["LSSP_AMD_LINEG"] = lineg
            M = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=lssp_amd.ILUK, level=level)
            os.environ.pop("LSSP_AMD_LINEG", None)
            ap = apply_leg(dev, M, n, reps=50)
            timed_solve(dev, A, M, n, lssp_amd.BICGSTAB, 20)
            r, t = timed_solve(dev, A, M, n, lssp_amd.BICGSTAB, 300)
            print(json.dumps({"grid": f"{N}x{NY}", "level": level, "path": "one-workgroup" if lineg == "1" else "tiles",
                              "layout": M.sweep_layout(), "apply_ms": ap["ms"], "levels": [ap["levels_L"], ap["levels_U"]],
                              "bicgstab_it_s": round(r.nits / t, 1)}), flush=True)
            M.close()
        A.close()
    dev.close()


if __name__ == "__main__":
    main()
