#!/bin/bash
# Round 4 call 7: split-RVQ encode as one distance GEMM per codebook -- codec / config tests, then config 5
# A/B (CSM_RVQ_GEMM=0: the round-3 tiled kernel) with the per-phase split.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_mimi_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r7_tests.log 2>&1 || { tail -30 gpurun_out/r7_tests.log; exit 1; }
tail -1 gpurun_out/r7_tests.log
for v in gemm tiled gemm; do
  envs=""; [ $v = tiled ] && envs="CSM_RVQ_GEMM=0"
  env $envs timeout -k 10 400 python -u bench.py --no-cpu-baseline --config 5 --steps 2 --warmup 1 --phases > gpurun_out/r7_c5_$v.json 2> gpurun_out/r7_c5_$v.err || { tail -5 gpurun_out/r7_c5_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r7_c5_$v.json')); print('config 5 $v', d['value'], d['phases_s_per_step'])"
done
