#!/bin/bash
# Round 4 call 2: full GPU suite on HEAD; gemm_xs ablation lab (abl/libcsm_hip_xslab<bits>.so, results
# invalid: 1 no MFMA, 2 no activation traffic, 4 no weight traffic, 8 no exchange/epilogue); config-3
# per-frame kernel trace after the round-3 Mimi streaming changes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_suite.log 2>&1 || { tail -30 gpurun_out/r4_suite.log; exit 1; }
tail -1 gpurun_out/r4_suite.log
for v in base xslab1 xslab2 xslab4 xslab6 xslab8 xslab15; do
  lib=""; [ $v != base ] && lib=$PWD/abl/libcsm_hip_$v.so
  CSM_HIP_LIB=$lib GB_XS=1 timeout -k 10 300 python -u tools/gemm_bench.py bf16 32 > gpurun_out/lab_$v.txt 2>&1 || { tail -5 gpurun_out/lab_$v.txt; exit 1; }
  CSM_HIP_LIB=$lib GB_XS=1 timeout -k 10 300 python -u tools/gemm_bench.py q4 64 >> gpurun_out/lab_$v.txt 2>&1 || { tail -5 gpurun_out/lab_$v.txt; exit 1; }
  grep " dec .* xs " gpurun_out/lab_$v.txt | sed "s/^/$v /"
done
bash tools/prof.sh r4_c3 --config 3 --steps 1 --warmup 0 --frames 24 || exit 1
