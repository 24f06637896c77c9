#!/usr/bin/env python3
"""Time the device format conversions (lssp_amd.convert) on 7-pt Poisson N^3
(default 216, BASELINE's matrix) with HIP events on the library's stream.

    python tools/bench_convert.py [N] [bs]

Prints one JSON line per conversion: milliseconds per call (mean of reps, the
host-side size query and output allocation included in the call as a user
sees it) and the algorithmic bytes (each input read once, each output written
once) divided by that time.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 216
    bs = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    import torch
    import lssp_amd
    from lssp_amd import convert as C
    dev = lssp_amd.Device(0)
    Ap, Aj, Ax = lssp_amd.poisson(3, N)
    n, nnz = Ap.size - 1, Aj.size
    dAp, dAj, dAx = dev.idx(n + 1, Ap), dev.idx(nnz, Aj), dev.vec(nnz, Ax)
    s = torch.cuda.ExternalStream(dev.stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timeit(fn, reps=5):
        out = fn()
        for a in out if isinstance(out, tuple) else ():
            if hasattr(a, "free"):
                a.free()
        total = 0.0
        for _ in range(reps):
            e0.record(s)
            out = fn()
            e1.record(s)
            e1.synchronize()
            total += e0.elapsed_time(e1)
            for a in out:
                if hasattr(a, "free"):
                    a.free()
        return total / reps

    Ci, Cj, Cx = C.csr_to_coo(dev, n, nnz, dAp, dAj, dAx)
    m, Bp, Bj, Bx = C.csr_to_bcsr(dev, n, nnz, bs, dAp, dAj, dAx)
    nb = n // bs
    rows = [
        ("csr_to_coo", lambda: C.csr_to_coo(dev, n, nnz, dAp, dAj, dAx), 4 * (n + 1) + 4 * nnz + 24 * nnz),
        ("coo_to_csr", lambda: C.coo_to_csr(dev, n, nnz, Ci, Cj, Cx), 16 * nnz + 4 * (n + 1) + 12 * nnz),
        ("transpose", lambda: C.transpose(dev, n, n, nnz, dAp, dAj, dAx), 2 * (4 * (n + 1) + 12 * nnz)),
        ("csr_to_bcsr", lambda: C.csr_to_bcsr(dev, n, nnz, bs, dAp, dAj, dAx),
         4 * (n + 1) + 12 * nnz + 4 * (nb + 1) + 4 * m + 8 * m * bs * bs),
        ("bcsr_to_csr", lambda: C.bcsr_to_csr(dev, nb, nb, bs, m, Bp, Bj, Bx),
         4 * (nb + 1) + 4 * m + 8 * m * bs * bs + 4 * (n + 1) + 12 * nnz),
    ]
    for name, fn, byts in rows:
        ms = timeit(fn)
        print(json.dumps({"op": name, "N": N, "n": n, "nnz": nnz, "bs": bs if "bcsr" in name else None,
                          "ms": round(ms, 3), "alg_bytes": byts, "alg_GBps": round(byts / ms / 1e6, 1)}),
              flush=True)
    dev.close()


if __name__ == "__main__":
    main()
