#!/bin/bash
# Round 4 call 10: the batched backbone on the streaming GEMM by default (bb_xs) + the refined wave rule --
# batched parity tests, then configs 5 / 4 / 3 against CSM_BB_XS=0.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_kernel_gpu.py tests/test_configs_gpu.py tests/test_quant_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r10_tests.log 2>&1 || { tail -30 gpurun_out/r10_tests.log; exit 1; }
tail -1 gpurun_out/r10_tests.log
for c in 5 4 3; do
  for v in xs wide; do
    envs=""; [ $v = wide ] && envs="CSM_BB_XS=0"
    env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline --config $c --steps 2 --warmup 1 > gpurun_out/r10_c${c}_$v.json 2> gpurun_out/r10_c${c}_$v.err || { tail -5 gpurun_out/r10_c${c}_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r10_c${c}_$v.json')); print('config $c backbone $v', d['value'], d['roofline_backbone']['avg_us'])"
  done
done
