import sys, time; sys.path.insert(0, '.')
import numpy as np, lssp_amd
N = int(sys.argv[1]); kind = sys.argv[2] if len(sys.argv) > 2 else "iluk"
d = lssp_amd.Device(0)
Ap, Aj, Ax = lssp_amd.poisson(3, N)
t = time.perf_counter()
M = lssp_amd.DILU.create(d, Ap, Aj, Ax, kind=lssp_amd.ILUK if kind == "iluk" else lssp_amd.ILUT, level=0, tol=1e-4, p=20)
print(kind, N, "setup", round(time.perf_counter() - t, 3), "lib", round(M.setup_seconds, 3), flush=True)
