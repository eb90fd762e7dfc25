#!/bin/bash
# Round 4 call 26: the arg-max heads at 32 rows without split-K (CSM_XS_HEAD_BLOCKS=1: 33 blocks x 8 waves)
# vs 2 slices (default), on abl hk (HEAD + the knob): batched tests with the knob, config 4 / 3 alternated.
set -o pipefail
mkdir -p gpurun_out
CSM_XS_HEAD_BLOCKS=1 CSM_HIP_LIB=$PWD/abl/libcsm_hip_hk.so timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r26_tests.log 2>&1 || { tail -30 gpurun_out/r26_tests.log; exit 1; }
tail -1 gpurun_out/r26_tests.log
run() {  # cfg tag envs
  env CSM_HIP_LIB=$PWD/abl/libcsm_hip_hk.so $3 timeout -k 10 300 python -u bench.py --no-cpu-baseline --config $1 --steps 2 --warmup 1 > gpurun_out/r26_$2.json 2> gpurun_out/r26_$2.err || { tail -5 gpurun_out/r26_$2.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r26_$2.json')); print('$2', d['value'], d['ms_per_step'])"
}
for rep in 1 2; do
  run 4 c4_hb1_$rep "CSM_XS_HEAD_BLOCKS=1" || exit 1
  run 4 c4_def$rep "CSM_XS_HEAD_BLOCKS=256" || exit 1
done
run 3 c3_hb1 "CSM_XS_HEAD_BLOCKS=1" || exit 1
run 3 c3_def "CSM_XS_HEAD_BLOCKS=256" || exit 1
run 5 c5_hb1 "CSM_XS_HEAD_BLOCKS=1" || exit 1
run 5 c5_def "CSM_XS_HEAD_BLOCKS=256" || exit 1
