#!/bin/bash
# Round 4 call 6: XCD-aware block placement in gemm_xs / gemm_wide -- batched parity tests, then an A/B
# against the tile-major build (abl/libcsm_hip_nomap.so) on configs 4 and 5 and the decoder shapes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_kernel_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_tests.log 2>&1 || { tail -30 gpurun_out/r6_tests.log; exit 1; }
tail -1 gpurun_out/r6_tests.log
for v in map nomap; do
  lib=""; [ $v = nomap ] && lib=$PWD/abl/libcsm_hip_nomap.so
  CSM_HIP_LIB=$lib GB_XS=1 timeout -k 10 300 python -u tools/gemm_bench.py bf16 32 > gpurun_out/r6_gb_$v.txt 2>&1 || { tail -5 gpurun_out/r6_gb_$v.txt; exit 1; }
  CSM_HIP_LIB=$lib GB_XS=1 timeout -k 10 300 python -u tools/gemm_bench.py q4 64 >> gpurun_out/r6_gb_$v.txt 2>&1 || { tail -5 gpurun_out/r6_gb_$v.txt; exit 1; }
  grep -E " xs |wide" gpurun_out/r6_gb_$v.txt | grep -v "xs-p" | sed "s/^/$v /"
done
for c in 4 5; do
  for v in map nomap map; do
    lib=""; [ $v = nomap ] && lib=$PWD/abl/libcsm_hip_nomap.so
    CSM_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --config $c --steps 2 --warmup 1 > gpurun_out/r6_c${c}_$v.json 2> gpurun_out/r6_c${c}_$v.err || { tail -5 gpurun_out/r6_c${c}_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r6_c${c}_$v.json')); print('config $c $v', d['value'])"
  done
done
