#!/bin/bash
# Round 4 call 4: Mimi split-K GEMMs -- codec GPU tests, config 3 A/B (round-3 behaviour: no split-K,
# 64-row GEMV cutoff) and its kernel trace; gemm_xs reduce-only lab; config-5 phases and a PMC pass
# bounded to the frame kernels.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_mimi_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_mimi_tests.log 2>&1 || { tail -30 gpurun_out/r4_mimi_tests.log; exit 1; }
tail -1 gpurun_out/r4_mimi_tests.log
for v in old new; do
  envs=""; [ $v = old ] && envs="CSM_MIMI_KS_BLOCKS=0 CSM_MIMI_GEMV_M=64"
  env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 3 --steps 1 --warmup 1 > gpurun_out/r4_c3_$v.json 2> gpurun_out/r4_c3_$v.err || { tail -5 gpurun_out/r4_c3_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r4_c3_$v.json')); print('config 3 $v', d['value'])"
done
bash tools/prof.sh r4_c3b --config 3 --steps 1 --warmup 0 --frames 24 > /dev/null || exit 1
head -12 gpurun_out/prof_r4_c3b/per_frame.txt
for v in base xslab16; do
  lib=""; [ $v != base ] && lib=$PWD/abl/libcsm_hip_$v.so
  CSM_HIP_LIB=$lib GB_XS=1 timeout -k 10 300 python -u tools/gemm_bench.py bf16 32 > gpurun_out/lab4_$v.txt 2>&1 || { tail -5 gpurun_out/lab4_$v.txt; exit 1; }
  CSM_HIP_LIB=$lib GB_XS=1 timeout -k 10 300 python -u tools/gemm_bench.py q4 64 >> gpurun_out/lab4_$v.txt 2>&1 || { tail -5 gpurun_out/lab4_$v.txt; exit 1; }
  grep " dec .* xs " gpurun_out/lab4_$v.txt | sed "s/^/$v /"
done
CSM_HIP_LIB=$PWD/abl/libcsm_hip_xsst.so GB_XS=1 GB_ITERS=64 timeout -k 10 300 python -u tools/gemm_bench.py bf16 32 > gpurun_out/lab4_stamps.txt 2>&1 || { tail -5 gpurun_out/lab4_stamps.txt; exit 1; }
CSM_HIP_LIB=$PWD/abl/libcsm_hip_xsst.so GB_XS=1 GB_ITERS=64 timeout -k 10 300 python -u tools/gemm_bench.py q4 64 >> gpurun_out/lab4_stamps.txt 2>&1 || { tail -5 gpurun_out/lab4_stamps.txt; exit 1; }
grep "xs_stamps dec" gpurun_out/lab4_stamps.txt
timeout -k 10 400 python -u bench.py --no-cpu-baseline --config 5 --steps 1 --warmup 1 --phases > gpurun_out/r4_c5_phases.json 2> gpurun_out/r4_c5_phases.err || { tail -5 gpurun_out/r4_c5_phases.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4_c5_phases.json')); print('config 5 phases', d['value'], d['phases_s_per_step'])"
PMC_REGEX='gemm_xs|gemm_wide|attn|embed|advance|gather' PMC_LIMIT=300 bash tools/pmc.sh r4_c5 --config 5 --frames 8 --no-decode --steps 1 --warmup 0 || exit 1
