#!/bin/bash
# Round 4 call 25: long-context attention (attn_kernel<64>, the backbone) with two key chunks in flight
# (attn2) vs one (cur): attention / prefill parity tests on attn2, configs 5 / 4 alternated with phases.
set -o pipefail
mkdir -p gpurun_out
CSM_HIP_LIB=$PWD/abl/libcsm_hip_attn2.so timeout -k 10 700 python -u -m pytest tests/test_csm_gpu.py tests/test_long_gpu.py tests/test_configs_gpu.py tests/test_gemm_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r25_tests.log 2>&1 || { tail -30 gpurun_out/r25_tests.log; exit 1; }
tail -1 gpurun_out/r25_tests.log
run() {  # cfg tag lib
  CSM_HIP_LIB=$PWD/abl/libcsm_hip_$3.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --config $1 --steps 2 --warmup 1 --phases > gpurun_out/r25_$2.json 2> gpurun_out/r25_$2.err || { tail -5 gpurun_out/r25_$2.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r25_$2.json')); print('$2', d['value'], d['ms_per_step'], d.get('phases_s_per_step'))"
}
for rep in 1 2; do
  run 5 c5_attn2_$rep attn2 || exit 1
  run 5 c5_cur$rep cur || exit 1
done
run 4 c4_attn2 attn2 || exit 1
run 4 c4_cur cur || exit 1
