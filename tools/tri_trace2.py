"""Per-step clocks of two consecutive blocks of a tri_mode 9 sweep
(LSSP_AMD_TRI_TRACE2=path:block): where the block-to-block lag goes.
For packet s: producer compute end (block A, step s) -> consumer landing of
packet s (block B, end of step s-1) -> consumer compute end (B, step s)."""
import json
import sys

import numpy as np


def main(path):
    for line in open(path):
        d = json.loads(line)
        t = np.array(d["steps"], dtype=np.float64).reshape(2, 1024, 4) * 0.01  # 100 MHz -> us
        A, B = t[0], t[1]
        n = int((A[:, 0] > 0).sum())
        s = np.arange(60, max(61, n - 60))
        j = s + 8  # index of step s
        vis = B[j - 1, 1] - A[j, 0]       # producer done -> consumer landed (incl. polls)
        land = B[j - 1, 1] - B[j - 1, 2]  # consumer landing phase (after the gathers' wait)
        comp = B[j, 0] - B[j - 1, 1]      # landed -> consumer compute done
        lag = B[j, 0] - A[j, 0]
        step = np.diff(B[8:8 + n, 0])
        polls = np.diff(B[:, 3])[j - 2]
        print(json.dumps({"tb0": d["tb0"], "steps": n, "lag_us": round(float(np.median(lag)), 3),
                          "vis_us": round(float(np.median(vis)), 3), "land_us": round(float(np.median(land)), 3),
                          "comp_us": round(float(np.median(comp)), 3), "step_us": round(float(np.median(step)), 3),
                          "polls_per_step": round(float(np.mean(polls)), 1),
                          "frac_steps_polling": round(float(np.mean(polls > 0)), 3)}))


if __name__ == "__main__":
    main(sys.argv[1])
