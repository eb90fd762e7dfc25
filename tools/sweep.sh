#!/bin/bash
# bench sweep: each line one configuration; stop at the first failure
set -o pipefail
mkdir -p gpurun_out
i=0
while read -r args; do
  [ -z "$args" ] && continue
  i=$((i+1))
  echo "== $args"
  timeout -k 10 240 python -u bench.py --no-cpu-baseline $args > gpurun_out/sweep_$i.json 2> gpurun_out/sweep_$i.err || { echo "failed rc=$?"; tail -20 gpurun_out/sweep_$i.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/sweep_$i.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_us'], d['roofline']['frac'])"
done < "${1:-/dev/stdin}"
