#!/usr/bin/env python3
"""Print a rocprofv3 / rocpd2summary kernel-stats CSV compactly:
    python tools/kstats.py stats.csv [top]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 15
tot = sum(float(r["Duration (Nsec)"]) for r in rows)
for r in rows[:top]:
    print(f'{int(r["Calls"]):6d} {float(r["Average (Nsec)"]) / 1e3:9.1f}us {float(r["Duration (Nsec)"]) / 1e6:8.2f}ms '
          f'{r["Name"][:90]}')
print(f"total kernel time {tot / 1e6:.2f} ms")
