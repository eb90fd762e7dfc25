#!/bin/bash
# Round 4 call 9: gemm_xs 8 waves per block (CSM_XS_WAVES=8) vs 4 -- decoder shapes, batched parity
# tests under 8 waves, configs 4 / 5 / 3 lines.
set -o pipefail
mkdir -p gpurun_out
for w in 4 8; do
  CSM_XS_WAVES=$w GB_XS=1 timeout -k 10 300 python -u tools/gemm_bench.py bf16 32 64 > gpurun_out/r9_w$w.txt 2>&1 || { tail -5 gpurun_out/r9_w$w.txt; exit 1; }
  CSM_XS_WAVES=$w GB_XS=1 timeout -k 10 300 python -u tools/gemm_bench.py q4 64 >> gpurun_out/r9_w$w.txt 2>&1 || { tail -5 gpurun_out/r9_w$w.txt; exit 1; }
  grep " dec .* xs " gpurun_out/r9_w$w.txt | sed "s/^/w$w /"
done
CSM_XS_WAVES=8 timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_kernel_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r9_tests.log 2>&1 || { tail -30 gpurun_out/r9_tests.log; exit 1; }
tail -1 gpurun_out/r9_tests.log
for c in 5 4 3; do
  for w in 4 8; do
    CSM_XS_WAVES=$w timeout -k 10 300 python -u bench.py --no-cpu-baseline --config $c --steps 2 --warmup 1 > gpurun_out/r9_c${c}_w$w.json 2> gpurun_out/r9_c${c}_w$w.err || { tail -5 gpurun_out/r9_c${c}_w$w.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r9_c${c}_w$w.json')); print('config $c waves $w', d['value'])"
  done
done
