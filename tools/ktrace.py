#!/usr/bin/env python3
"""Per-frame kernel breakdown from a rocprofv3 ``--kernel-trace`` CSV.

usage: python tools/ktrace.py run_kernel_trace.csv|run_results.db [--last-frames N]

Frames are delimited by ``advance_kernel`` dispatches (one per generated frame).  Only the
last N frames (default: all after the first 5) are summarised, so prompt prefill and
warm-up do not pollute the per-frame numbers.  Reports per-kernel-name time per frame,
launches per frame, mean duration, and the busy fraction of the frame span (1 - gaps).
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last-frames", type=int, default=0)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    if a.trace.endswith(".db"):  # rocprofv3 >= 7 default (rocpd sqlite)
        import sqlite3
        cur = sqlite3.connect(a.trace).execute("select name, start, end from kernels")
        rows = [{"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e} for n, s, e in cur]
    else:
        rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    adv = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("advance_kernel")]
    if len(adv) < 3:
        raise SystemExit("fewer than 3 frames in trace")
    n = a.last_frames or max(1, len(adv) - 5)
    n = min(n, len(adv) - 1)
    lo, hi = adv[-n - 1] + 1, adv[-1] + 1
    sel = rows[lo:hi]
    per = defaultdict(lambda: [0, 0.0])
    busy = 0.0
    for r in sel:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
        k = k.split("(")[0][:90]
        per[k][0] += 1
        per[k][1] += d
        busy += d
    span = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / 1e3
    print(f"frames {n}  span/frame {span / n:.1f} us  busy/frame {busy / n:.1f} us  "
          f"launches/frame {len(sel) / n:.1f}  gap/launch {(span - busy) / len(sel):.2f} us")
    for k, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{t / n:9.1f} us/fr {c / n:7.1f} /fr  avg {t / c:7.2f} us  {k}")


if __name__ == "__main__":
    main()
