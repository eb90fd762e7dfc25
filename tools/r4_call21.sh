#!/bin/bash
# Round 4 call 21: the depth decoder's step 1 (2 rows per utterance) on the streaming GEMM (abl s1: the
# projected rows split once by xs_rows_kernel, layer 0's QKV projected from them) vs cur (HEAD: step 1 on
# gemm_wide): batched parity tests on s1, configs 4 / 3 alternated.
set -o pipefail
mkdir -p gpurun_out
CSM_HIP_LIB=$PWD/abl/libcsm_hip_s1.so timeout -k 10 700 python -u -m pytest tests/test_gemm_gpu.py tests/test_configs_gpu.py tests/test_processors_gpu.py tests/test_scoring_gpu.py tests/test_quant_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r21_tests.log 2>&1 || { tail -30 gpurun_out/r21_tests.log; exit 1; }
tail -1 gpurun_out/r21_tests.log
run() {  # args tag lib
  CSM_HIP_LIB=$PWD/abl/libcsm_hip_$3.so timeout -k 10 300 python -u bench.py --no-cpu-baseline $1 --steps 2 --warmup 1 > gpurun_out/r21_$2.json 2> gpurun_out/r21_$2.err || { tail -5 gpurun_out/r21_$2.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r21_$2.json')); print('$2', d['value'], d['ms_per_step'])"
}
for rep in 1 2; do
  run "--config 4" c4_s1_$rep s1 || exit 1
  run "--config 4" c4_cur$rep cur || exit 1
done
run "--config 3" c3_s1 s1 || exit 1
run "--config 3" c3_cur cur || exit 1
CSM_HIP_LIB=$PWD/abl/libcsm_hip_s1.so bash tools/prof.sh r21_c4 --config 4 --steps 1 --warmup 0 --frames 24 > /dev/null || exit 1
head -16 gpurun_out/prof_r21_c4/per_frame.txt
# the decoder's small QKV / o at 32 rows without split-K: CSM_XS_SMALL_BLOCKS=1 (one K slice) with 4 or 8 waves
for v in "CSM_XS_SMALL_BLOCKS=1 CSM_XS_SMALL_WAVES=8" "CSM_XS_SMALL_BLOCKS=1 CSM_XS_SMALL_WAVES=4" "CSM_XS_SMALL_WAVES=4"; do
  env $v CSM_HIP_LIB=$PWD/abl/libcsm_hip_s1.so GB_XS=1 GB_ITERS=100 timeout -k 10 300 python -u tools/gemm_bench.py bf16 32 > gpurun_out/r21_gb.txt 2>&1 || { tail -5 gpurun_out/r21_gb.txt; exit 1; }
  grep " dec .*\(qkv\|o \) .* xs " gpurun_out/r21_gb.txt | sed "s/^/$v: /"
  env $v CSM_HIP_LIB=$PWD/abl/libcsm_hip_s1.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 4 --steps 2 --warmup 1 > gpurun_out/r21_sm.json 2> gpurun_out/r21_sm.err || { tail -5 gpurun_out/r21_sm.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r21_sm.json')); print('config 4 $v', d['value'])"
done
