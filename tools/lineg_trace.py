#!/usr/bin/env python3
"""Per-level clocks of the one-workgroup 2-D sweep (k_lineg, LSSP_AMD_LINEG_TRACE):
wave 0 lane 0, first sweep, levels < 512: [before the vmcnt wait, after it,
after the barrier, after the level's store].  GPU box; diagnostics only.

    python tools/lineg_trace.py [nx] [ny] [level]
"""
import json
import os
import sys

import numpy as np

path = "/tmp/lineg_trace.jsonl"
os.environ["LSSP_AMD_LINEG_TRACE"] = path
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import lssp_amd  # noqa: E402
from lineg_bench import box2  # noqa: E402


def main():
    nx = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    ny = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    level = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    if os.path.exists(path):
        os.remove(path)
    dev = lssp_amd.Device(0)
    Ap, Aj, Ax = box2(nx, ny)
    n = Ap.size - 1
    M = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=lssp_amd.ILUK, level=level)
    x = dev.vec(n)
    for _ in range(3):
        M.apply(x, dev.vec(n, np.ones(n)))
    dev.sync()
    rec = [json.loads(l) for l in open(path)][-1]
    c = np.array(rec["clk"], dtype=np.int64).reshape(-1, 4)
    V = min(rec["V"], 512)
    c = c[:V]
    per = np.diff(c[:, 0])
    wait = c[:, 1] - c[:, 0]
    bar = c[:, 2] - c[:, 1]
    body = c[:, 3] - c[:, 2]
    q = lambda v: [int(np.percentile(v, p)) for p in (10, 50, 90)]  # noqa: E731
    print(json.dumps({"nx": nx, "ny": ny, "level": level, "V": rec["V"], "NYP": rec["NYP"],
                      "clk_per_level_p10_50_90": q(per[20:]), "vmcnt_wait": q(wait[20:]), "barrier": q(bar[20:]),
                      "issue_compute_store": q(body[20:])}), flush=True)
    dev.close()


if __name__ == "__main__":
    main()
