#!/usr/bin/env python3
"""Top kernels by total time from a rocprofv3 --stats kernel_stats.csv.  usage: tools/kstats.py stats.csv [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f"{float(r['TotalDurationNs']) / 1e6:9.1f} ms {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.1f} us  {r['Name'][:80]}")
print(f"total {tot / 1e6:.1f} ms")
