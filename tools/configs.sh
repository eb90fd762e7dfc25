#!/bin/bash
# One bench line per BASELINE config workload (1 GPU): gpurun_out/cfg_<n>.json
set -o pipefail
mkdir -p gpurun_out
for c in "$@"; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --config $c --steps 1 --warmup 1 > gpurun_out/cfg_$c.json 2> gpurun_out/cfg_$c.err || { echo "config $c failed"; tail -5 gpurun_out/cfg_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/cfg_$c.json')); print('config $c', d['value'], d['unit'], d['ms_per_step'], 'ms/step', d['dtype'])"
done
