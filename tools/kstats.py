#!/usr/bin/env python3
"""Print a rocprofv3 kernel-stats CSV compactly (both the rocpd2summary
"Duration (Nsec)" layout and rocprofv3's own "TotalDurationNs" one):
    python tools/kstats.py stats.csv [top]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 15
tot_k = "Duration (Nsec)" if rows and "Duration (Nsec)" in rows[0] else "TotalDurationNs"
avg_k = "Average (Nsec)" if rows and "Average (Nsec)" in rows[0] else "AverageNs"
tot = sum(float(r[tot_k]) for r in rows)
for r in rows[:top]:
    print(f'{int(r["Calls"]):6d} {float(r[avg_k]) / 1e3:9.1f}us {float(r[tot_k]) / 1e6:8.2f}ms {r["Name"][:90]}')
print(f"total kernel time {tot / 1e6:.2f} ms")
