#!/bin/bash
# Round 4 call 5: Mimi split-K on every transformer linear -- codec tests, config 3 A/B and trace,
# the B = 1 bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_mimi_gpu.py tests/test_configs_gpu.py tests/test_long_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_mimi_tests5.log 2>&1 || { tail -30 gpurun_out/r4_mimi_tests5.log; exit 1; }
tail -1 gpurun_out/r4_mimi_tests5.log
for v in old new; do
  envs=""; [ $v = old ] && envs="CSM_MIMI_KS_BLOCKS=0 CSM_MIMI_GEMV_M=64"
  env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 3 --steps 1 --warmup 1 > gpurun_out/r5_c3_$v.json 2> gpurun_out/r5_c3_$v.err || { tail -5 gpurun_out/r5_c3_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5_c3_$v.json')); print('config 3 $v', d['value'])"
  env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r5_b1_$v.json 2> gpurun_out/r5_b1_$v.err || { tail -5 gpurun_out/r5_b1_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5_b1_$v.json')); print('B=1 $v', d['value'], d['ms_per_step'])"
done
bash tools/prof.sh r5_c3 --config 3 --steps 1 --warmup 0 --frames 24 > /dev/null || exit 1
head -14 gpurun_out/prof_r5_c3/per_frame.txt
