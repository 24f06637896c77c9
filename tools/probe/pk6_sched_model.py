#!/usr/bin/env python3
"""Host model of the packet sweep (tuning aid, CPU only): builds ILUT(1e-4, 20)
of the 7-pt N^3 grid with the oracle, cuts the L factor's rows into the packet
schedule the way tri_bp.cpp build_packets6 does (one plane per block, rows by
level, a packet closed at 65 rows -- the EP 24 record slot -- or at the HBM-
operand cap), and runs the packet DAG with tau per packet and a hop latency per
cross-block edge.  At 256^3 it reproduced the kernel (2,546 packets per block
against the trace's 2,550, a block start lag of 25 us against 23.5) and showed
the operand cap of 512 splitting 1,580 levels into 2,546 packets.

    gcc -O2 -shared -fPIC -o /tmp/pk6_sched_model.so tools/probe/pk6_sched_model.c
    python tools/probe/pk6_sched_model.py 128
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import lssp_amd
    import oracle as O
    lib = ctypes.CDLL("/tmp/pk6_sched_model.so")
    P = ctypes.c_void_p
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    Ap, Aj, Ax = lssp_amd.poisson(3, N)
    n = Ap.size - 1
    L, _ = O.ilu(O.CSR(n, Ap, Aj, Ax), "ilut", tol=1e-4, p=20)
    Fp, Fj = np.ascontiguousarray(L.Ap, np.int32), np.ascontiguousarray(L.Aj, np.int32)
    for R, X, RC in ((4096, 512, 65), (4096, 768, 65), (4096, 1024, 65)):
        out = (ctypes.c_double * 4)()
        lib.model2(ctypes.c_int(n), Fp.ctypes.data_as(P), Fj.ctypes.data_as(P), ctypes.c_int(N * N), ctypes.c_int(R),
                   ctypes.c_int(X), ctypes.c_int(RC), ctypes.c_double(0.65), ctypes.c_double(1.0), out)
        print(f"L ring {R} operand cap {X} rows {RC}: packets/block {out[1]:.0f}, span {out[2]:.0f} us, "
              f"block start lag {out[3]:.2f} us", flush=True)


if __name__ == "__main__":
    main()
