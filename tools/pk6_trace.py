#!/usr/bin/env python3
"""Diagnostics for the packet sweeps (trisolve.hip k_tri_pk6): ILUT(1e-4, 20)
(or ILU(k)) applies at N^3 with LSSP_AMD_PK6_TRACE set; summarises the
per-block and per-packet trace of each sweep.

    python tools/pk6_trace.py [N] [block] [ilut|iluk1]     (GPU box)
"""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(N, blk, kind, path):
    make = ("M = lssp_amd.DILU.create(d, Ap, Aj, Ax, kind=lssp_amd.ILUT, tol=1e-4, p=20)" if kind == "ilut" else
            "M = lssp_amd.DILU.create(d, Ap, Aj, Ax, kind=lssp_amd.ILUK, level=1)")
    code = f"""
import sys, time; sys.path.insert(0, {ROOT!r})
import numpy as np, lssp_amd
d = lssp_amd.Device(0)
Ap, Aj, Ax = lssp_amd.poisson(3, {N})
{make}
n = Ap.size - 1
r = d.vec(n, np.ones(n)); x = d.vec(n)
for _ in range(3):
    M.apply(x, r)
d.sync()
print("levels", M.levelsL, M.levelsU, flush=True)
"""
    env = dict(os.environ, LSSP_AMD_PK6_TRACE=f"{path}:{blk}")
    subprocess.run([sys.executable, "-c", code], env=env, check=True)


def summarise(rec):
    nb = rec["nb"]
    d = np.array(rec["data"], dtype=np.float64)
    blk = d[: 8 * nb].reshape(nb, 8)
    claim, start, end, hits, np_ = blk[:, 0], blk[:, 1], blk[:, 2], blk[:, 3], blk[:, 5]
    tb = rec["tblk"]
    npk = int(np_[tb])
    st = d[8 * nb:8 * nb + 4 * npk].reshape(npk, 4)
    us = lambda v: v / 100.0  # s_memrealtime: 100 MHz  # noqa: E731
    t0 = claim.min()
    print(f"{'U' if rec['upper'] else 'L'} sweep: EP {rec['ep']}, blocks {nb} (B {rec['B']}), grid {rec['grid']}, "
          f"span {us(end.max() - t0):.1f} us, packets per block median {np.median(np_):.0f} "
          f"(max {np_.max():.0f}), sentinel hits {int(hits.sum())} (blocks with any {(hits > 0).sum()})")
    dur = us(end - start)
    lag = us(np.diff(start))
    print(f"  block active median {np.median(dur):.1f} us; start lag between consecutive blocks median "
          f"{np.median(lag):.2f} us (mean {lag.mean():.2f}); last block starts at {us(start.max() - t0):.1f} us")
    per = np.diff(st[:, 0])
    comp = st[:, 1] - st[:, 0]
    lw = st[:, 2]
    print(f"  block {tb}: {npk} packets, period median {np.median(per):.0f} clk (mean {per.mean():.0f}, "
          f"p90 {np.percentile(per, 90):.0f}); compute busy median {np.median(comp):.0f} clk; loader wait "
          f"median {np.median(lw):.0f} clk (p90 {np.percentile(lw, 90):.0f}); loader lands "
          f"{np.median(st[1:, 3] - st[:-1, 0]):.0f} clk after the previous packet's start")


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    blk = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    kind = sys.argv[3] if len(sys.argv) > 3 else "ilut"
    path = os.path.join(ROOT, "gpurun_out", "pk6_trace.jsonl")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    if os.path.exists(path):
        os.remove(path)
    run(N, blk, kind, path)
    with open(path) as f:
        recs = [json.loads(line) for line in f]
    for rec in recs[-2:]:
        summarise(rec)


if __name__ == "__main__":
    main()
