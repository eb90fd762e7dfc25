#!/bin/bash
# Round 4 call 35: the no-split rule for the decoder's QKV / o extended to 64 rows (CSM_XS_SMALL_M=64: config 5's
# int4 B = 64 and configs 3 / 4's codebook step 1) vs 32 (default): gemm_bench q4 64, batched tests, configs 5 / 4.
set -o pipefail
mkdir -p gpurun_out
for v in 64 32; do
  CSM_XS_SMALL_M=$v timeout -k 10 300 python -u tools/gemm_bench.py q4 64 > gpurun_out/r35_gb_$v.txt 2>&1 || { tail -5 gpurun_out/r35_gb_$v.txt; exit 1; }
  grep "dec qkv *xs \|dec o *xs " gpurun_out/r35_gb_$v.txt | sed "s/^/m$v /"
done
CSM_XS_SMALL_M=64 timeout -k 10 500 python -u -m pytest tests/test_gemm_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r35_tests.log 2>&1 || { tail -30 gpurun_out/r35_tests.log; exit 1; }
tail -1 gpurun_out/r35_tests.log
run() {  # config m tag
  CSM_XS_SMALL_M=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline $1 --steps 2 --warmup 1 > gpurun_out/r35_$3_$2.json 2> gpurun_out/r35_$3_$2.err || { tail -5 gpurun_out/r35_$3_$2.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r35_$3_$2.json')); print('$3 small_m=$2', d['value'], d['ms_per_step'])"
}
for rep in 1 2; do for v in 64 32; do run "--config 5" $v c5 || exit 1; done; done
for rep in 1 2; do for v in 64 32; do run "--config 4" $v c4 || exit 1; done; done
echo RC=0
