#!/usr/bin/env python3
"""FETCH_SIZE per kernel from a rocprofv3 --pmc FETCH_SIZE counter_collection.csv.

Bytes per launch = FETCH_SIZE (KB) x 1024 x 2: the gfx950 correction of MI355X_MICROARCH.md's HBM
section (FETCH_SIZE reports half the bytes of a wide coalesced streaming read).
usage: tools/pmc_summary.py counter_collection.csv [out_summary.txt] [out_traffic.json]"""
import collections
import csv
import json
import sys

vals = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if r.get("Counter_Name", "FETCH_SIZE") != "FETCH_SIZE":
        continue
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    vals[name].append(float(r["Counter_Value"]))
lines = ["kernel, launches, avg FETCH_SIZE KB, x2-corrected bytes/launch"]
for k, v in sorted(vals.items(), key=lambda kv: -sum(kv[1])):
    avg = sum(v) / len(v)
    lines.append(f"{k}, {len(v)}, {avg:.1f}, {int(avg * 1024 * 2)}")
txt = "\n".join(lines)
print(txt)
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write(txt + "\n")
if len(sys.argv) > 3:
    def pick(prefix):
        for k, v in vals.items():
            if k.startswith(prefix):
                return int(sum(v) / len(v) * 1024 * 2), len(v)
        return None, 0
    dec, nd = pick("gemv_xl_kernel<unsigned short, 64, 2, 1, 1")
    bb, nb = pick("gemv_xl_kernel<unsigned short, 64, 2, 1, 4")
    json.dump({"decoder_gate_up": dec, "backbone_gate_up": bb,
               "_note": "HBM-side read bytes per launch = rocprofv3 --pmc FETCH_SIZE (KB) x 1024 x 2 (gfx950 "
                        "wide-stream correction, MI355X_MICROARCH.md HBM section); averaged over every launch of "
                        "the kernel in `CSM_GRAPH=0 python bench.py --no-decode --steps 1 --warmup 0 --frames 8` "
                        "(frames + the roofline microbench). Infinity-Cache hits are counted by FETCH_SIZE.",
               "_launches": {"decoder_gate_up": nd, "backbone_gate_up": nb}}, open(sys.argv[3], "w"), indent=1)
