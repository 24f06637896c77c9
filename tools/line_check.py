#!/usr/bin/env python3
"""Bitwise check of the line sweeps against the packet sweeps, per sweep (GPU box).

    python tools/line_check.py [N ...]

For each 7-pt N^3 ILU(0): the L sweep, the U sweep and the apply on the line
sweeps vs the same factors on the packet sweeps (LSSP_AMD_LINE=0); prints the
mismatch count and the first mismatching rows as (i, j, k).  Debugging aid.
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import lssp_amd
    sizes = [int(v) for v in sys.argv[1:]] or [24]
    dev = lssp_amd.Device(0)
    for N in sizes:
        Ap, Aj, Ax = lssp_amd.poisson(3, N)
        n = Ap.size - 1
        M = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=lssp_amd.ILUK, level=0)
        os.environ["LSSP_AMD_LINE"] = "0"
        Mp = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=lssp_amd.ILUK, level=0)
        os.environ.pop("LSSP_AMD_LINE")
        r = dev.vec(n, np.random.default_rng(0).uniform(-1, 1, n))
        x = dev.vec(n)
        out = {"N": N, "layout": lssp_amd.device.line_layout(M) if hasattr(lssp_amd.device, "line_layout") else None}
        for name, fn in (("L", lambda m: m.trisolve(0, x, r)), ("U", lambda m: m.trisolve(1, x, r)),
                         ("apply", lambda m: m.apply(x, r))):
            fn(M)
            got = x.download()
            fn(Mp)
            ref = x.download()
            bad = np.flatnonzero(got.view(np.int64) != ref.view(np.int64))
            first = [[int(b % N), int(b // N % N), int(b // (N * N))] for b in bad[:6]]
            out[name] = {"mismatch": int(bad.size), "first_ijk": first}
            if bad.size and os.environ.get("LINE_CHECK_DETAIL"):
                # per (j, k) line: wrong rows' i range
                jk = {}
                for b in bad:
                    key = (int(b // N % N), int(b // (N * N)))
                    lo, hi, c = jk.get(key, (N, -1, 0))
                    jk[key] = (min(lo, int(b % N)), max(hi, int(b % N)), c + 1)
                out[name]["lines"] = sorted([list(k) + list(v) for k, v in jk.items()])[:400]
        print(json.dumps(out), flush=True)
        M.close()
        Mp.close()
    dev.close()


if __name__ == "__main__":
    main()
