#!/usr/bin/env python3
"""Per-launch listing of a rocprofv3 kernel trace: every launch of kernels matching a regex after the
N-th launch of a marker kernel, with grid and duration.  usage: trace_launches.py trace.csv regex [skip_before_us]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rx = re.compile(sys.argv[2])
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
skip = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
tot = {}
for r in rows:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    if s < skip or not rx.search(r["Kernel_Name"]):
        continue
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    n = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
    tot[n] = tot.get(n, 0.0) + d
    print(f"{s:12.1f} {d:9.1f} us grid {r['Grid_Size_X']:>8}x{r['Grid_Size_Y']:>4}x{r['Grid_Size_Z']:>4} {n}")
for n, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"total {v / 1e3:9.2f} ms  {n}")
