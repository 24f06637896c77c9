"""Compute-only projection of bench.py at N GPUs, measured on ONE GPU.

For P in --ranks: rank 0's share of the 216^3 problem (its z-slab of rows,
block-Jacobi ILU(0) of its diagonal block, exactly what bench.py --gpus P
builds on rank 0; the halo columns are dropped, so the SpMV is a little
lighter than the real one) is solved alone for --steps BiCGSTAB iterations.
The time per iteration is a lower bound of bench.py's ms/step at N = P: it
leaves out the per-SpMV halo exchange and the three reduction all-gathers per
iteration that RCCL adds.  One JSON line per P."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import build_local, local_block  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=216)
    ap.add_argument("--ranks", type=str, default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=30)
    args = ap.parse_args()
    import lssp_amd
    dev = lssp_amd.Device(0)
    for P in (int(p) for p in args.ranks.split(",")):
        n, row0, nl, Ap, Aj, Ax = build_local(args.grid, 0, P)
        bp, bj, bx = local_block(Ap, Aj, Ax, row0, nl)
        A = lssp_amd.DMat(dev, bp, bj, bx)
        M = lssp_amd.DILU.create(dev, bp, bj, bx, kind=lssp_amd.ILUK, level=0)
        x, b = dev.vec(nl, np.zeros(nl)), dev.vec(nl, np.ones(nl))

        def run(k):
            return lssp_amd.solve(dev, A, M, x, b, solver=lssp_amd.BICGSTAB, tol_rel=0.0, tol_abs=0.0,
                                  tol_rb=0.0, maxit=k)
        run(3)
        dev.sync()
        t0 = time.perf_counter()
        r = run(args.steps)
        dev.sync()
        dt = (time.perf_counter() - t0) / r.nits
        print(json.dumps({"P": P, "rows_rank0": nl, "levels_L": M.levelsL, "ms_per_iter": round(dt * 1e3, 4),
                          "iters_per_s": round(1.0 / dt, 2)}), flush=True)
        for h in (M, A):
            h.close()
    dev.close()


if __name__ == "__main__":
    main()
