#!/usr/bin/env python3
"""Per-boundary idle time between consecutive kernels of one stream, from a
rocprofv3 --kernel-trace CSV:

    python tools/kgaps.py run_kernel_trace.csv [--last K]

For the last K dispatches of the busiest queue (the bench's timed steps) it
prints, per (predecessor -> successor) kernel pair, the count and the mean /
median gap from the predecessor's end to the successor's start, the sum of
kernel durations and of gaps -- i.e. how much of ms_per_step is boundaries."""
import argparse
import collections
import csv
import statistics


def short(name):
    name = name.split("(")[0]
    return name if len(name) < 60 else name[:57] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last", type=int, default=2000)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    byq = collections.defaultdict(list)
    for r in rows:
        byq[(r["Agent_Id"], r["Queue_Id"])].append(r)
    q = max(byq.values(), key=len)
    q.sort(key=lambda r: int(r["Start_Timestamp"]))
    q = q[-a.last:]
    gaps = collections.defaultdict(list)
    busy = 0
    for p, s in zip(q, q[1:]):
        g = int(s["Start_Timestamp"]) - int(p["End_Timestamp"])
        gaps[(short(p["Kernel_Name"]), short(s["Kernel_Name"]))].append(g)
    for r in q:
        busy += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    span = int(q[-1]["End_Timestamp"]) - int(q[0]["Start_Timestamp"])
    tot_gap = sum(sum(v) for v in gaps.values())
    print(f"{len(q)} dispatches, span {span / 1e6:.3f} ms, kernels {busy / 1e6:.3f} ms, gaps {tot_gap / 1e6:.3f} ms "
          f"({100 * tot_gap / span:.1f} %)")
    for k, v in sorted(gaps.items(), key=lambda kv: -sum(kv[1])):
        print(f"{len(v):6d} mean {statistics.mean(v) / 1e3:7.2f} us  median {statistics.median(v) / 1e3:7.2f} us  "
              f"sum {sum(v) / 1e6:7.3f} ms  {k[0]} -> {k[1]}")


if __name__ == "__main__":
    main()
