#!/usr/bin/env python3
"""Timeline of the U sweep's tail product (GPU box; diagnostics, not a test).

    python tools/tail_timing.py [N] [level]

One BiCGSTAB iteration with LSSP_AMD_TAIL=2 and LSSP_AMD_TAIL_DIAG=1 on the
7-pt N^3 grid; per workgroup of the last U sweep: its start, when it entered
the tail, when its first pair was staged, when it left, the pairs it computed
and the ticks its loader spent waiting for planes (100 MHz clock, us here)."""
import ctypes
import json
import os
import sys

import numpy as np

os.environ["LSSP_AMD_TAIL"] = "2"
os.environ["LSSP_AMD_TAIL_DIAG"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lssp_amd  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 216
    level = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    dev = lssp_amd.Device(0)
    L = dev.L
    L.lssp_amd_debug_words.restype = ctypes.c_int
    L.lssp_amd_debug_words.argtypes = [ctypes.c_void_p, ctypes.c_int]
    Ap, Aj, Ax = lssp_amd.poisson(3, N)
    n = Ap.size - 1
    A = lssp_amd.DMat(dev, Ap, Aj, Ax)
    M = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=lssp_amd.ILUK, level=level)
    for rep in range(3):
        x = dev.vec(n, np.zeros(n))
        b = dev.vec(n, np.ones(n))
        lssp_amd.solve(dev, A, M, x, b, solver=lssp_amd.BICGSTAB, tol_rel=0.0, tol_abs=0.0, tol_rb=0.0, maxit=1)
        dev.sync()
        buf = (ctypes.c_uint * 32768)()
        assert L.lssp_amd_debug_words(buf, 32768) == 0
        w = np.frombuffer(buf, dtype=np.uint32).astype(np.int64)
        tl = w[4096:4096 + 8 * 256].reshape(256, 8)
        start = w[6144:6144 + 256]
        used = tl[:, 1] != 0
        tl, start = tl[used], start[used]
        t00 = start.min()
        us = lambda v: np.round((v - t00) / 100.0, 1)  # noqa: E731
        enter, ready, leave = us(tl[:, 1]), us(tl[:, 2]), us(tl[:, 3])
        worked = tl[:, 4] > 0
        q = lambda v: [float(np.percentile(v, p)) for p in (0, 10, 50, 90, 100)] if len(v) else []  # noqa: E731
        print(json.dumps({"N": N, "level": level, "rep": rep, "wgs": int(used.sum()),
                          "start_us_pct": q(us(start)), "enter_us_pct": q(enter), "leave_us_pct": q(leave),
                          "ready_minus_enter_us_pct": q((ready - enter)[worked]),
                          "pairs_total": int(tl[:, 4].sum()), "pairs_pct": q(tl[worked, 4]),
                          "plane_wait_us_pct": q(tl[worked, 5] / 100.0),
                          "compute_wave_us_per_round_pct": q(tl[worked, 6] / 100.0 / tl[worked, 4]),
                          "loader_wave_us_per_round_pct": q(tl[worked, 7] / 100.0 / tl[worked, 4]),
                          "busy_us_per_pair_pct": q(((leave - ready)[worked] - tl[worked, 5] / 100.0) /
                                                    tl[worked, 4])}), flush=True)
    dev.close()


if __name__ == "__main__":
    main()
