#!/bin/bash
# Round 4 A/B: gemm_xs with 2 vs 4 waves per block (CSM_XS_WAVES): per-projection microbench
# (tools/gemm_bench.py, GB_XS=1), the gemm parity tests under 4 waves, and config 4 / 5 lines.
set -o pipefail
mkdir -p gpurun_out
for w in 2 4; do
  CSM_XS_WAVES=$w GB_XS=1 timeout -k 10 300 python -u tools/gemm_bench.py bf16 32 64 > gpurun_out/xsw${w}_bf16.txt 2>&1 || { tail -5 gpurun_out/xsw${w}_bf16.txt; exit 1; }
  CSM_XS_WAVES=$w GB_XS=1 timeout -k 10 300 python -u tools/gemm_bench.py q4 64 > gpurun_out/xsw${w}_q4.txt 2>&1 || { tail -5 gpurun_out/xsw${w}_q4.txt; exit 1; }
done
grep " dec " gpurun_out/xsw*_bf16.txt gpurun_out/xsw*_q4.txt
CSM_XS_WAVES=4 timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_kernel_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/xsw4_tests.log 2>&1 || { tail -30 gpurun_out/xsw4_tests.log; exit 1; }
tail -2 gpurun_out/xsw4_tests.log
for c in 4 5; do
  for w in 2 4; do
    CSM_XS_WAVES=$w timeout -k 10 300 python -u bench.py --no-cpu-baseline --config $c --steps 2 --warmup 1 > gpurun_out/xsw${w}_cfg$c.json 2> gpurun_out/xsw${w}_cfg$c.err || { tail -5 gpurun_out/xsw${w}_cfg$c.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/xsw${w}_cfg$c.json')); print('config $c waves $w', d['value'], d['roofline']['avg_us'])"
  done
done
