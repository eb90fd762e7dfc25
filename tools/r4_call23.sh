#!/bin/bash
# Round 4 call 23: config 3 with the small projections' split-K back (CSM_XS_SMALL_BLOCKS=256
# CSM_XS_SMALL_WAVES=4) vs the new default (no split-K, 8 waves), alternated; then evidence part B's
# kernel traces (configs 4 / 5) and PMC passes (config 4 / config 5 bounded to the frame kernels).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # tag envs
  env $2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 3 --steps 2 --warmup 1 > gpurun_out/r23_$1.json 2> gpurun_out/r23_$1.err || { tail -5 gpurun_out/r23_$1.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r23_$1.json')); print('config 3 $1', d['value'], d['ms_per_step'])"
}
for rep in 1 2; do
  run new$rep "CSM_XS_SMALL_BLOCKS=1" || exit 1
  run old$rep "CSM_XS_SMALL_BLOCKS=256 CSM_XS_SMALL_WAVES=4" || exit 1
done
bash tools/prof.sh r4f_c4 --config 4 --steps 1 --warmup 0 --frames 24 > /dev/null || exit 1
head -16 gpurun_out/prof_r4f_c4/per_frame.txt
bash tools/prof.sh r4f_c5 --config 5 --steps 1 --warmup 0 --frames 24 > /dev/null || exit 1
head -20 gpurun_out/prof_r4f_c5/per_frame.txt
PMC_REGEX='gemm_xs|gemm_wide|attn|embed|advance|gather|sample' PMC_LIMIT=240 bash tools/pmc.sh r4f_c4 --config 4 --frames 8 --no-decode --steps 1 --warmup 0 || exit 1
