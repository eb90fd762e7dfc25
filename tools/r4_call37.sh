#!/bin/bash
# Round 4 call 37: int4 prompt prefill on 256-row blocks for every shape (CSM_GEMM_PREFILL_NBR=256, default) vs the
# per-shape widths (=0): GEMM kernel tests (every projection at 300 rows vs the GEMV), config tests, config 5 A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_kernel_gpu.py tests/test_configs_gpu.py tests/test_gemm_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r37_tests.log 2>&1 || { tail -30 gpurun_out/r37_tests.log; exit 1; }
tail -1 gpurun_out/r37_tests.log
run() {  # tag env
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 5 --steps 2 --warmup 1 --phases > gpurun_out/r37_$tag.json 2> gpurun_out/r37_$tag.err || { tail -5 gpurun_out/r37_$tag.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r37_$tag.json')); print('$tag', d['value'], d['ms_per_step'], d.get('phases_s_per_step'))"
}
for rep in 1 2; do run p256_$rep X=0 || exit 1; run p0_$rep CSM_GEMM_PREFILL_NBR=0 || exit 1; done
run p128 CSM_GEMM_PREFILL_NBR=128 || exit 1
echo RC=0
