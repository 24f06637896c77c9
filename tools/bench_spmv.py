"""SpMV micro-benchmark (tuning aid): y = A x (k_spmv3) on the 7-pt grid, HIP
events on the library stream."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=216)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--nz", type=int, default=0, help="a z-slab of NZ planes of the grid (block-Jacobi block)")
    ap.add_argument("--thermal", action="store_true", help="config 5's thermal2-like matrix instead")
    ap.add_argument("--window", type=int, default=4096, help="thermal: numbering shuffle window (1: none)")
    args = ap.parse_args()
    import torch
    import lssp_amd
    if args.thermal:
        from lssp_amd.synthetic import thermal_like
        Ap, Aj, Ax = thermal_like(window=args.window)
    elif args.nz:
        from bench import local_block
        nl = args.grid * args.grid * args.nz
        Ap, Aj, Ax = local_block(*lssp_amd.poisson(3, args.grid, 0, nl), 0, nl)
    else:
        Ap, Aj, Ax = lssp_amd.poisson(3, args.grid)
    n = Ap.size - 1
    dev = lssp_amd.Device(0)
    A = lssp_amd.DMat(dev, Ap, Aj, Ax)
    x = dev.vec(n, np.random.default_rng(1).uniform(-1, 1, n))
    y = dev.vec(n)
    for _ in range(5):
        A.mv_mxy(x, y)
    if os.environ.get("LSSP_AMD_PROBE_COPY"):  # PMC calibration: n doubles read, n written
        for _ in range(args.reps):
            dev.L.lssp_amd_vec_copy(dev.h, y.ptr, x.ptr, n)
    s = torch.cuda.ExternalStream(dev.stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(args.reps):
        A.mv_mxy(x, y)
    e1.record(s)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / args.reps
    b = 12 * int(Ap[-1]) + 20 * n + 4
    print(json.dumps({"matrix": f"thermal window {args.window}" if args.thermal else
                      f"poisson {args.grid}^2 x {args.nz}" if args.nz else f"poisson {args.grid}^3",
                      "rows": n, "ndiag": A.ndiag, "ms": round(ms, 5),
                      "GBps": round(b / ms / 1e6, 1), "sum": float(y.download().sum())}))


if __name__ == "__main__":
    main()
