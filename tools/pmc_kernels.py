#!/usr/bin/env python3
"""Per-kernel summary of tools/pmc.sh passes (rocprofv3 counter_collection.csv + kernel_trace.csv).

For every kernel (name + grid): dispatches, mean duration (kernel trace of the same pass), mean
of each counter per dispatch, and derived:
  hbm_read_B   = FETCH_SIZE (KB) x 1024 x 2  (gfx950 wide-stream correction, MI355X_MICROARCH.md HBM)
  hbm_write_B  = WRITE_SIZE (KB) x 1024
  mfma_util    = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)  (GRBM_GUI_ACTIVE is
                 summed over the 8 XCDs; MFMA_BUSY counts 32 cycles per v_mfma_f32_32x32x16_bf16)
  mfma_tflops  = SQ_VALU_MFMA_BUSY_CYCLES / 32 x 32768 flop / duration  (issued matrix flops,
                 including the exact-split operand passes)
usage: tools/pmc_kernels.py gpurun_out/pmc_<tag> [--top N]"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 25


def kname(r):
    n = r.get("Kernel_Name", "").replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:90]


ctr = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    per = collections.defaultdict(float)  # (dispatch, counter) -> value summed over dims
    names = {}
    for r in csv.DictReader(open(f)):
        key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Counter_Name"])
        per[key] += float(r["Counter_Value"])
        names[key[0]] = kname(r)
    for (d, c), v in per.items():
        ctr[names[d]][c].append(v)
for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        dur[kname(r)].append((float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-3)


def mean(v):
    return sum(v) / len(v) if v else float("nan")


rows = []
for k in set(ctr) | set(dur):
    c = {n: mean(v) for n, v in ctr[k].items()}
    d = mean(dur[k])
    rows.append((d * len(dur[k]) / max(1, len(set(f for f in glob.glob(os.path.join(root, "p*"))))), k, c, d, len(dur[k])))
print("kernel | dispatches/pass | mean us | hbm_read_B | hbm_write_B | mfma_util | mfma_TFLOP/s")
for tot, k, c, d, n in sorted(rows, key=lambda r: -r[0])[:top]:
    rd = c.get("FETCH_SIZE", float("nan")) * 1024 * 2
    wr = c.get("WRITE_SIZE", float("nan")) * 1024
    busy, gui = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0), c.get("GRBM_GUI_ACTIVE", float("nan"))
    util = busy / (1024 * gui / 8) if gui == gui and gui > 0 else float("nan")
    tf = busy / 32 * 32768 / (d * 1e-6) / 1e12 if d == d and d > 0 else float("nan")
    print(f"{k} | {n / 3:.0f} | {d:.2f} | {rd:.0f} | {wr:.0f} | {util:.3f} | {tf:.1f}")
