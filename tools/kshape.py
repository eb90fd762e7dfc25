#!/usr/bin/env python3
"""Per-(kernel, grid) duration summary of a rocprofv3 kernel trace.  usage: tools/kshape.py trace.csv [substr]"""
import collections
import csv
import sys

import numpy as np

sub = sys.argv[2] if len(sys.argv) > 2 else ""
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if sub not in n:
        continue
    d[(n.split("(")[0][5:60], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    v = np.array(v)
    print(f"{k[0]:45s} grid {k[1]:>6s}x{k[2]:>2s}x{k[3]:>2s} n {len(v):5d} med {np.median(v):7.2f} "
          f"p10 {np.percentile(v, 10):7.2f} p90 {np.percentile(v, 90):7.2f} us")
