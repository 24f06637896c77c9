#!/usr/bin/env python3
"""Timing experiments on the line sweeps (tuning aid, not a test; GPU box).

    python tools/line_diag.py [N] [diag,diag,...]

LINE_DIAG_LEVEL=1 times the ILU(1) factor's sweeps instead of ILU(0)'s.
For each LSSP_AMD_LINE_DIAG value (linesweep.hip; results are WRONG when it is
non-zero: 1 storers skip the output stores, 2 loaders skip their DMAs,
4 multiply instead of divide, 8 the poller does not wait for producers,
16 no hand-off stores (only with 8), 32 the apply's L sweep skips its U rhs-stream stores) prints the L sweep, U sweep and apply
times (HIP events on the library's stream).
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 216
    diags = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "0").split(",")]
    import torch
    import lssp_amd
    dev = lssp_amd.Device(0)
    Ap, Aj, Ax = lssp_amd.poisson(3, N)
    n = Ap.size - 1
    level = int(os.environ.get("LINE_DIAG_LEVEL", "0"))  # 1: the ILU(1) line sweeps (linefill.hip)
    M = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=lssp_amd.ILUK, level=level)
    r = dev.vec(n, np.random.default_rng(0).uniform(-1, 1, n))
    x, y = dev.vec(n), dev.vec(n)
    s = torch.cuda.ExternalStream(dev.stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timeit(fn, reps=10):
        for _ in range(2):
            fn()
        e0.record(s)
        for _ in range(reps):
            fn()
        e1.record(s)
        e1.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3

    # bitwise check of the line-sweep apply against the packet sweeps (k_tri_pk6)
    if os.environ.get("LINE_DIAG_NOCHECK"):  # experiment builds that compute wrong values
        return timings(M, r, x, y, diags, timeit, N, dev)
    M.apply(x, r)
    got = x.download()
    os.environ["LSSP_AMD_LINE"] = "0"
    Mp = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=lssp_amd.ILUK, level=level)
    os.environ.pop("LSSP_AMD_LINE")
    Mp.apply(x, r)
    ref = x.download()
    Mp.close()
    print(json.dumps({"N": N, "lib": os.environ.get("LSSP_AMD_LIB", "default"),
                      "bitwise_vs_packet_sweeps": bool(np.array_equal(got.view(np.int64), ref.view(np.int64)))}))
    timings(M, r, x, y, diags, timeit, N, dev)


def timings(M, r, x, y, diags, timeit, N, dev):
    import lssp_amd

    def t(fn):
        try:
            return round(timeit(fn), 1)
        except lssp_amd.LsspError:  # e.g. a variant whose standalone sweep exceeds the LDS
            return None

    for d in diags:
        os.environ["LSSP_AMD_LINE_DIAG"] = str(d)
        out = {"N": N, "diag": d,
               "L_us": t(lambda: M.trisolve(0, y, r)),
               "U_us": t(lambda: M.trisolve(1, x, y)),
               "apply_us": t(lambda: M.apply(x, r)),
               "apply_async_us": t(lambda: M.apply_async(x, r))}
        print(json.dumps(out), flush=True)
    os.environ["LSSP_AMD_LINE_DIAG"] = "0"
    dev.close()


if __name__ == "__main__":
    main()
