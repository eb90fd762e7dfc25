#!/usr/bin/env python3
"""Register / LDS / spill summary per kernel instantiation of one HIP source (gfx950).
usage: tools/kres.py <source.hip> [extra hipcc flags]"""
import os
import re
import subprocess
import sys

inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", f"-I{inc}", *sys.argv[2:], "-x", "hip",
       "-c", sys.argv[1], "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
keys = {"VGPRs": "vgpr", "AGPRs": "agpr", "VGPRs Spill": "vspill", "SGPRs Spill": "sspill",
        "Occupancy [waves/SIMD]": "occ", "LDS Size [bytes/block]": "lds"}
cur = None
for line in out.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|"
                  r"LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        if "error" in line:
            print(line)
        continue
    k, v = m.groups()
    if k == "Function Name":
        if cur:
            print(cur)
        cur = v[:64]
    else:
        cur += f" {keys[k]}={v}"
if cur:
    print(cur)
