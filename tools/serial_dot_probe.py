#!/usr/bin/env python3
"""SERIAL-order dot (k_dot_serial) timing on the GPU box: ns per element of the
sequential chain (vector.cxx:123-131) at 1.23 M (config 5) and 10.08 M (216^3)
elements, checked bitwise against the reference order computed on the host
(a plain Python-free loop: numpy's cumulative sum is sequential in float64)."""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lssp_amd  # noqa: E402


def main():
    dev = lssp_amd.Device(0, reduction=lssp_amd.SERIAL)
    for n in (1227664, 10077696):
        rng = np.random.default_rng(n)
        xh, yh = rng.uniform(-1, 1, n), rng.uniform(-1, 1, n)
        want = float(np.cumsum(xh * yh)[-1])  # sequential: s_i = s_{i-1} + x_i y_i from 0.0
        x, y = dev.vec(n, xh), dev.vec(n, yh)
        out = ctypes.c_double()
        L = dev.L
        L.lssp_amd_vec_dot(dev.h, x.ptr, y.ptr, n, ctypes.byref(out))
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            L.lssp_amd_vec_dot(dev.h, x.ptr, y.ptr, n, ctypes.byref(out))
        dt = (time.perf_counter() - t0) / reps
        print(json.dumps({"n": n, "ms_per_dot": round(dt * 1e3, 3), "ns_per_element": round(dt / n * 1e9, 3),
                          "bitwise_vs_sequential_sum": out.value.hex() == want.hex()}), flush=True)
        x.close()
        y.close()
    dev.close()


if __name__ == "__main__":
    main()
