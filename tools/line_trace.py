#!/usr/bin/env python3
"""Diagnostics for the line sweeps (linesweep.hip): run ILU(0) applies at N^3
with LSSP_AMD_LINE_TRACE set and summarise the per-tile / per-step trace.

    python tools/line_trace.py [N] [tile]     (GPU box)
"""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(N, tile, path):
    code = f"""
import sys; sys.path.insert(0, {ROOT!r})
import numpy as np, lssp_amd
d = lssp_amd.Device(0)
Ap, Aj, Ax = lssp_amd.poisson(3, {N})
M = lssp_amd.DILU.create(d, Ap, Aj, Ax, kind=lssp_amd.ILUK, level=0)
n = Ap.size - 1
r = d.vec(n, np.ones(n)); x = d.vec(n)
for _ in range(3):
    M.apply(x, r)
d.sync()
"""
    env = dict(os.environ, LSSP_AMD_LINE_TRACE=f"{path}:{tile}")
    subprocess.run([sys.executable, "-c", code], env=env, check=True)


def summarise(rec):
    nt, W, T = rec["ntiles"], rec["W"], rec["T"]
    d = np.array(rec["data"], dtype=np.float64)
    tiles = d[: 8 * nt].reshape(nt, 8)
    steps = d[8 * nt:8 * nt + 8 * T].reshape(-1, 8)
    claim, start, end, polls = tiles[:, 0], tiles[:, 1], tiles[:, 2], tiles[:, 3]
    t0 = claim.min()
    us = lambda v: (v) / 100.0  # s_memrealtime: 100 MHz  # noqa: E731
    span = us(end.max() - t0)
    dur = us(end - start)
    lag_k = [us(start[t] - start[t - W]) for t in range(W, nt)]
    lag_j = [us(start[t] - start[t - 1]) for t in range(nt) if t % W]
    per = np.diff(steps[:, 0])
    comp = steps[:, 1] - steps[:, 0]
    print(f"{'U' if rec['mirror'] else 'L'} sweep: span {span:.1f} us, tiles {nt} (W {W}), grid {rec['grid']}, "
          f"tile active {np.median(dur):.1f} us (median), re-polls {int(polls.sum())} "
          f"(tiles with any: {(polls > 0).sum()})")
    print(f"  start lag k: median {np.median(lag_k):.2f} us, mean {np.mean(lag_k):.2f}; "
          f"j: median {np.median(lag_j):.2f} us")
    med = lambda c: np.median(steps[steps[:, c] > 0, c]) if (steps[:, c] > 0).any() else 0  # noqa: E731
    print(f"  tile {rec['ttile']}: step period median {np.median(per):.0f} clk (mean {per.mean():.0f}), "
          f"busy (median clk): compute {np.median(comp):.0f}, poller {med(2):.0f}, loader wait {med(3):.0f}, "
          f"loader issue {med(4):.0f}, storer {med(5):.0f}")
    ar = steps[:, 6] - steps[:, 0]
    w1 = steps[:, 7] - steps[:, 0]
    print(f"  compute wave 0: arithmetic done at {np.median(ar):.0f} clk after the step start; "
          f"wave 1 reaches the barrier at {np.median(w1):.0f} clk")
    lim = np.percentile(per, [10, 50, 90, 99])
    print(f"  step period p10/50/90/99: {lim.astype(int).tolist()}")


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 216
    tile = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    if len(sys.argv) > 3:  # LSSP_AMD_LINE_DIAG timing experiment (wrong results)
        os.environ["LSSP_AMD_LINE_DIAG"] = sys.argv[3]
        print(f"LSSP_AMD_LINE_DIAG={sys.argv[3]}")
    path = os.path.join(ROOT, "gpurun_out", "line_trace.jsonl")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    if os.path.exists(path):
        os.remove(path)
    run(N, tile, path)
    with open(path) as f:
        recs = [json.loads(line) for line in f]
    for rec in recs[-2:]:
        summarise(rec)


if __name__ == "__main__":
    main()
