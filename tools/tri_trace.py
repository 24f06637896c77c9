"""Summarise LSSP_AMD_TRI_TRACE dumps of the tri_mode 6 sweep (tuning aid).

Each line of the dump is one sweep: per block [t_claim, t_end, polls, xcc]
in s_memrealtime ticks (100 MHz), then s_memtime cycle sums of the compute
wave (work, barrier) and the loader wave (vmcnt wait, barrier).  Prints, per sweep, the kernel span, block
0's duration (no upstream dependency: warm-up + np steps), the median lag
between the ends of consecutive blocks, the polls and the XCD histogram.
"""
import json
import sys

import numpy as np


def main(path, limit=8):
    for i, line in enumerate(open(path)):
        if i >= limit:
            break
        d = json.loads(line)
        t = np.array(d["blocks"], dtype=np.float64)
        t0, t1, polls, xcc = t[:, 0], t[:, 1], t[:, 2], t[:, 3].astype(int)
        steps = d["npk"] / d["nb"] + 6
        names = ["comp", "cbar", "lwait", "lbar", "lissue", "lprep", "lland"][: t.shape[1] - 4]
        cyc = {k: t[:, 4 + i] / steps for i, k in enumerate(names)}
        base = t0.min()
        us = 0.01  # 100 MHz ticks -> us
        span = (t1.max() - base) * us
        dur = (t1 - t0) * us
        lag = np.diff(t1) * us
        same = xcc[1:] == xcc[:-1]
        print(json.dumps({
            "n": d["n"], "nb": d["nb"], "npk": d["npk"], "grid": d["grid"],
            "span_us": round(span, 1),
            "claim_spread_us": round((t0.max() - base) * us, 1),
            "blk0_us": round(dur[0], 1), "pk_per_blk": round(d["npk"] / d["nb"], 1),
            "end_lag_med_us": round(float(np.median(lag)), 2),
            "end_lag_same_xcd_us": round(float(np.median(lag[same])), 2) if same.any() else None,
            "end_lag_cross_xcd_us": round(float(np.median(lag[~same])), 2) if (~same).any() else None,
            "polls_total": int(polls.sum()), "polls_med": float(np.median(polls)),
            "xcd_hist": np.bincount(xcc, minlength=8).tolist(),
            "cycles_per_step_blk0": {k: round(float(v[0])) for k, v in cyc.items()},
            "cycles_per_step_med": {k: round(float(np.median(v))) for k, v in cyc.items()},
        }))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 8)
