#!/bin/bash
# Round 4 call 27: gemm_xs at 64 rows with 64-row weight tiles (int4 gate/up, bf16 heads at 64 rows): the
# 128 KB of 8-wave partials reduced one row tile at a time through 8 slots (rh) vs the 4-slot pre-add (hk =
# HEAD + lab knob): batched tests on rh, int4 shapes, config 5 alternated.
set -o pipefail
mkdir -p gpurun_out
CSM_HIP_LIB=$PWD/abl/libcsm_hip_rh.so timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r27_tests.log 2>&1 || { tail -30 gpurun_out/r27_tests.log; exit 1; }
tail -1 gpurun_out/r27_tests.log
for v in rh hk; do
  CSM_HIP_LIB=$PWD/abl/libcsm_hip_$v.so GB_XS=1 GB_ITERS=100 timeout -k 10 300 python -u tools/gemm_bench.py q4 64 > gpurun_out/r27_gb_$v.txt 2>&1 || { tail -5 gpurun_out/r27_gb_$v.txt; exit 1; }
  grep " gate_up .* xs " gpurun_out/r27_gb_$v.txt | sed "s/^/$v /"
done
run() {  # cfg tag lib
  CSM_HIP_LIB=$PWD/abl/libcsm_hip_$3.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --config $1 --steps 2 --warmup 1 > gpurun_out/r27_$2.json 2> gpurun_out/r27_$2.err || { tail -5 gpurun_out/r27_$2.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r27_$2.json')); print('$2', d['value'], d['ms_per_step'])"
}
for rep in 1 2; do
  run 5 c5_rh$rep rh || exit 1
  run 5 c5_hk$rep hk || exit 1
done
