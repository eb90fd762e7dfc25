#!/bin/bash
# Round 4 call 16: full GPU suite on the tree's lib (codec GEMMs on fp32 MFMA, 8-wave gemm_wide for
# prompt-sized launches, gemm_xs single-pass 8-slot wave reduction); A/B: gemm_xs reduction (cur vs
# redold = the previous gemm_xs.hip) on decoder shapes and configs 4 / 3; prompt prefill with 8-wave
# gemm_wide (cur vs CSM_GEMM_W8=0) on config 5 with the phase split.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r16_suite.log 2>&1 || { tail -30 gpurun_out/r16_suite.log; exit 1; }
tail -1 gpurun_out/r16_suite.log
for v in cur redold; do
  CSM_HIP_LIB=$PWD/abl/libcsm_hip_$v.so GB_XS=1 GB_ITERS=100 timeout -k 10 300 python -u tools/gemm_bench.py bf16 32 > gpurun_out/r16_gb_$v.txt 2>&1 || { tail -5 gpurun_out/r16_gb_$v.txt; exit 1; }
  grep " xs " gpurun_out/r16_gb_$v.txt | sed "s/^/$v /"
done
run() {  # args tag envs
  env CSM_HIP_LIB=$PWD/abl/libcsm_hip_$3.so $4 timeout -k 10 300 python -u bench.py --no-cpu-baseline $1 --steps 2 --warmup 1 --phases > gpurun_out/r16_$2.json 2> gpurun_out/r16_$2.err || { tail -5 gpurun_out/r16_$2.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r16_$2.json')); print('$2', d['value'], d['ms_per_step'], d.get('phases_s_per_step'))"
}
for rep in 1 2; do
  run "--config 4" c4_cur$rep cur "" || exit 1
  run "--config 4" c4_redold$rep redold "" || exit 1
done
run "--config 3" c3_cur cur "" || exit 1
run "--config 3" c3_redold redold "" || exit 1
for rep in 1 2; do
  run "--config 5" c5_w8_$rep cur "" || exit 1
  run "--config 5" c5_w4_$rep cur "CSM_GEMM_W8=0" || exit 1
done
