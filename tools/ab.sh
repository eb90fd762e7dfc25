#!/bin/bash
# A/B of environment settings on the B=1 codes-only bench inside one GPU call (box-to-box noise ~3%).
# usage: tools/ab.sh "ENV1=a" "ENV1=b" ...   (each run: 2 steps after 1 warmup)
set -o pipefail
mkdir -p gpurun_out
for cfg in "$@"; do
  for rep in 1 2; do
    env $cfg timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-decode --steps 2 --warmup 1 > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "failed: $cfg"; tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$cfg', 'rep $rep', d['value'], 'fps', d['ms_per_step'], 'ms/step')"
  done
done
