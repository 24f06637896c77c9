"""Micro-benchmark of the ILU triangular sweeps (tuning aid, not a test).

    python tools/bench_trisolve.py --grid 216 [--kind iluk --level 0]
Times lssp_amd_ilu_apply and the single sweeps with HIP events on the
library's stream, for the trisolve variants selected by LSSP_AMD_TRI_MODE /
LSSP_AMD_TRI_BLOCKS_PER_CU (read at context creation).
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=216)
    ap.add_argument("--dim", type=int, default=3)
    ap.add_argument("--kind", default="iluk")
    ap.add_argument("--level", type=int, default=0)
    ap.add_argument("--tol", type=float, default=1e-4)
    ap.add_argument("--p", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--configs", default="0:1,0:2,0:4,2:1,1:1")
    args = ap.parse_args()
    import torch
    import lssp_amd
    Ap, Aj, Ax = lssp_amd.poisson(args.dim, args.grid)
    n = Ap.size - 1
    out = []
    M = None
    for cfg in args.configs.split(","):
        f = cfg.split(":")
        mode, bpc = f[0], f[1]
        os.environ["LSSP_AMD_TRI_MODE"] = mode
        os.environ["LSSP_AMD_TRI_BLOCKS_PER_CU"] = bpc
        os.environ["LSSP_AMD_TRI_DEPTH"] = f[2] if len(f) > 2 else "2"
        os.environ["LSSP_AMD_TRI_PK_ROWS"] = f[3] if len(f) > 3 else "256"
        os.environ["LSSP_AMD_TRI_BP_MULT"] = f[4] if len(f) > 4 else "1"
        os.environ["LSSP_AMD_TRI_DIAG"] = f[5] if len(f) > 5 else "0"  # timing experiments (wrong results)
        dev = lssp_amd.Device(0)
        kind = lssp_amd.ILUK if args.kind == "iluk" else lssp_amd.ILUT
        if M is None:
            M0 = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=kind, level=args.level, tol=args.tol, p=args.p)
            factors = M0.factors()
            levels = (M0.levelsL, M0.levelsU)
            M0.close()
            M = True
        D = lssp_amd.DILU.from_factors(dev, *factors)
        r = dev.vec(n, np.random.default_rng(0).uniform(-1, 1, n))
        x = dev.vec(n)
        s = torch.cuda.ExternalStream(dev.stream)
        D.apply(x, r)
        ref = x.download()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(args.reps):
            D.apply(x, r)
        e1.record(s)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / args.reps
        ok = bool(np.array_equal(x.download(), ref))
        out.append({"mode": int(mode), "blocks_per_cu": int(bpc), "depth": int(os.environ["LSSP_AMD_TRI_DEPTH"]),
                    "rows": int(os.environ["LSSP_AMD_TRI_PK_ROWS"]), "mult": int(os.environ["LSSP_AMD_TRI_BP_MULT"]),
                    "diag": int(os.environ["LSSP_AMD_TRI_DIAG"]), "apply_ms": round(ms, 4),
                    "us_per_level": round(ms * 1e3 / (levels[0] + levels[1]), 3), "stable": ok})
        print(json.dumps(out[-1]), flush=True)
        dev.close()
    print(json.dumps({"n": n, "levels": levels, "nnzL": int(factors[0][0][-1]), "nnzU": int(factors[1][0][-1])}))


if __name__ == "__main__":
    main()
