#!/usr/bin/env python3
"""Roofline kernel cross-check: the bench's live HIP-event average vs the rocprofv3 kernel-trace
durations of the same kernel in the same bench command (microbench launches = the last 400).
usage: tools/roof_check.py kernel_trace.csv bench.json"""
import csv
import json
import statistics
import sys

name = "void gemv_xl_kernel<unsigned short, 64, 2, 1, 1, 2048>"
rows = [r for r in csv.DictReader(open(sys.argv[1])) if r["Kernel_Name"].startswith(name)]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in rows]
b = json.load(open(sys.argv[2]))["roofline"]
print(f"kernel {name[5:]}: {len(d)} launches under rocprofv3 (eager)")
print(f"  microbench (last 400) avg {statistics.mean(d[-400:]):.2f} us | in-frame avg {statistics.mean(d[:-404]):.2f} us "
      f"| all {statistics.mean(d):.2f} us")
print(f"  bench live HIP events avg {b['avg_us']:.2f} us -> {b['achieved']:.0f} GB/s, frac {b['frac']:.3f}, "
      f"PMC traffic {b['traffic']} B/launch vs algorithmic {b['bytes_per_launch']} B")
