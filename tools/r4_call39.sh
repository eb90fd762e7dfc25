#!/bin/bash
# Round 4 call 39: int4 prefill split-K block target 128 (CSM_GEMM_PREFILL_BLOCKS=1, default) vs 256 (=0): GEMM kernel /
# streaming / config tests, config 5 A/B alternated, then the full GPU suite on the result.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_kernel_gpu.py tests/test_configs_gpu.py tests/test_gemm_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r39_tests.log 2>&1 || { tail -30 gpurun_out/r39_tests.log; exit 1; }
tail -1 gpurun_out/r39_tests.log
run() {  # tag env
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 5 --steps 2 --warmup 1 --phases > gpurun_out/r39_$tag.json 2> gpurun_out/r39_$tag.err || { tail -5 gpurun_out/r39_$tag.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r39_$tag.json')); print('$tag', d['value'], d['ms_per_step'], d.get('phases_s_per_step'))"
}
for rep in 1 2; do run b128_$rep X=0 || exit 1; run b256_$rep CSM_GEMM_PREFILL_BLOCKS=0 || exit 1; done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r39_suite.log 2>&1 || { tail -30 gpurun_out/r39_suite.log; exit 1; }
tail -1 gpurun_out/r39_suite.log
echo RC=0
