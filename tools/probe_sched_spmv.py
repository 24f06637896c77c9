"""Experiment: SpMV y = A x with x held in a sweep's schedule order (columns
remapped through pos[]), vs natural order.  Schedule order here: z-planes,
within a plane anti-diagonals d = i + j ascending, i ascending (the shape of
the tri_mode 9 schedules).  Bitwise the same y (same per-row order)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import lssp_amd
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 216
    Ap, Aj, Ax = lssp_amd.poisson(3, N)
    n = Ap.size - 1
    r = np.arange(n, dtype=np.int64)
    i, j, k = r % N, (r // N) % N, r // (N * N)
    order = np.lexsort((i, i + j, k))  # position -> row
    pos = np.empty(n, np.int64)
    pos[order] = np.arange(n)
    AjU = pos[Aj].astype(np.int32)
    dev = lssp_amd.Device(0)
    xs = np.random.default_rng(1).uniform(-1, 1, n)
    out = {}
    for name, cols, xv in (("natural", Aj, xs), ("schedule", AjU, xs[order])):
        A = lssp_amd.DMat(dev, Ap, cols, Ax)
        x = dev.vec(n, xv)
        y = dev.vec(n)
        for _ in range(5):
            A.mv_mxy(x, y)
        s = torch.cuda.ExternalStream(dev.stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(50):
            A.mv_mxy(x, y)
        e1.record(s)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / 50
        out[name] = {"ms": round(ms, 5), "GBps": round((12 * int(Ap[-1]) + 20 * n + 4) / ms / 1e6, 1),
                     "y": y.download()}
    same = bool(np.array_equal(out["natural"]["y"], out["schedule"]["y"]))
    print(json.dumps({k: {"ms": v["ms"], "GBps": v["GBps"]} for k, v in out.items()} | {"bitwise": same}))
    dev.close()


if __name__ == "__main__":
    main()
