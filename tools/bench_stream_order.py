#!/usr/bin/env python3
"""A/B of the streaming kernels' block order (tuning aid, GPU box).

    python tools/bench_stream_order.py [N]

For each configuration a fresh process (the orders are read once per process)
times, at N^3 (7-pt Poisson, default 216): y = A x (k_spmv3, offset ids) and
two BLAS-1 passes (k_ew: axpby, and the BiCGSTAB p update shape via
vec_axpbyz), HIP events on the library's stream, best of 5 x 20 launches;
then 30 BiCGSTAB + ILU(0) iterations (it/s).  Configurations:
LSSP_AMD_SPMV_STREAMS = K (k_spmv3: K streams of consecutive 256-row blocks)
and LSSP_AMD_EW_CHUNKED = 0/1 (k_ew: grid-strided chunks / a contiguous range
of chunks per workgroup).  One JSON line per configuration.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys, time
sys.path.insert(0, {root!r})
import numpy as np, torch, lssp_amd
N = {N}
d = lssp_amd.Device(0)
Ap, Aj, Ax = lssp_amd.poisson(3, N)
n = Ap.size - 1
A = lssp_amd.DMat(d, Ap, Aj, Ax)
x = d.vec(n, np.random.default_rng(0).uniform(-1, 1, n)); y = d.vec(n); z = d.vec(n, np.ones(n))
s = torch.cuda.ExternalStream(d.stream)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
def t(fn, reps=20):
    for _ in range(3): fn()
    best = 1e9
    for _ in range(5):
        e0.record(s)
        for _ in range(reps): fn()
        e1.record(s); e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps * 1e3)
    return round(best, 2)
out = dict(N=N, streams={K}, ew_chunked={C})
out["spmv_us"] = t(lambda: A.mv_mxy(x, y))
out["spmv_tbs"] = round((9 * A.nnz + 20 * n + 4) / (out["spmv_us"] * 1e-6) / 1e12, 3) if hasattr(A, "nnz") else None
L = d.L
out["axpby_us"] = t(lambda: L.lssp_amd_vec_axpby(d.h, 0.5, x.ptr, 0.25, y.ptr, n))
out["axpbyz_us"] = t(lambda: L.lssp_amd_vec_axpbyz(d.h, 0.5, x.ptr, 0.25, y.ptr, z.ptr, n))
M = lssp_amd.DILU.create(d, Ap, Aj, Ax, kind=lssp_amd.ILUK, level=0)
b = d.vec(n, np.ones(n)); xs = d.vec(n, np.zeros(n))
lssp_amd.solve(d, A, M, xs, b, tol_rel=0.0, tol_abs=0.0, tol_rb=0.0, maxit=5)
d.sync(); t0 = time.perf_counter()
r = lssp_amd.solve(d, A, M, xs, b, tol_rel=0.0, tol_abs=0.0, tol_rb=0.0, maxit=40)
d.sync(); out["bicgstab_it_s"] = round(r.nits / (time.perf_counter() - t0), 1)
print(json.dumps(out), flush=True)
d.close()
"""


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 216
    configs = [(8, 0), (16, 0), (32, 0), (64, 0), (128, 0), (256, 0), (8, 0)]
    for K, C in configs:
        env = dict(os.environ, LSSP_AMD_SPMV_STREAMS=str(K), LSSP_AMD_EW_CHUNKED=str(C))
        code = CHILD.format(root=ROOT, N=N, K=K, C=C)
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        print(line[-1] if line else json.dumps({"streams": K, "ew_chunked": C, "error": r.stderr[-400:]}),
              flush=True)


if __name__ == "__main__":
    main()
