#!/usr/bin/env python3
"""Print the top kernels of a rocprofv3 --stats kernel_stats.csv: python tools/kstats.py <csv> [top]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 15
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:top]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f}ms {float(r['Percentage']):5.1f}% n={r['Calls']:>6} "
          f"avg={float(r['AverageNs'])/1e3:8.1f}us {r['Name'][:100]}")
print(f"total {tot/1e6:.2f} ms")
