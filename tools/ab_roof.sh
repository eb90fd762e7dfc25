#!/bin/bash
# A/B of environment settings: B=1 codes-only frames/s and the bench's live gate/up roofline.
# usage: tools/ab_roof.sh "ENV1=a" "ENV1=b" ...
set -o pipefail
mkdir -p gpurun_out
for cfg in "$@"; do
  env $cfg timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-decode --steps 2 --warmup 1 > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "failed: $cfg"; tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); r=d['roofline']; b=d.get('roofline_backbone',{}); print('$cfg', d['value'], 'fps | dec gate/up', round(r['achieved'],1), r['unit'], 'frac', round(r['frac'],3), '| bb', round(b.get('achieved',0),1))"
done
