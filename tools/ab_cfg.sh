#!/bin/bash
# A/B of environment settings on one bench configuration inside one GPU call.
# usage: tools/ab_cfg.sh "<bench args>" "ENV1=a" "ENV1=b" ...   (each: 1 step after 1 warmup)
set -o pipefail
mkdir -p gpurun_out
args=$1; shift
for cfg in "$@"; do
  env $cfg timeout -k 10 200 python -u bench.py --no-cpu-baseline $args > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "failed: $cfg"; tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$cfg', d['value'], 'fps', d['ms_per_step'], 'ms/step')"
done
