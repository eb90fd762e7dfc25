#!/bin/bash
# Round 4 call 24: the backbone's o (2048 x 2048) back on split-K (cur) vs without (bbo = HEAD, the decoder's
# small-projection rule also covering it): batched tests on cur, configs 4 / 3 alternated; config-5 PMC pass.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r24_tests.log 2>&1 || { tail -30 gpurun_out/r24_tests.log; exit 1; }
tail -1 gpurun_out/r24_tests.log
run() {  # cfg tag lib
  CSM_HIP_LIB=$PWD/abl/libcsm_hip_$3.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --config $1 --steps 2 --warmup 1 > gpurun_out/r24_$2.json 2> gpurun_out/r24_$2.err || { tail -5 gpurun_out/r24_$2.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r24_$2.json')); print('$2', d['value'], d['ms_per_step'])"
}
for rep in 1 2; do
  run 4 c4_cur$rep cur || exit 1
  run 4 c4_bbo$rep bbo || exit 1
done
run 3 c3_cur cur || exit 1
run 3 c3_bbo bbo || exit 1
PMC_REGEX='gemm_xs|gemm_wide|attn|embed|advance|gather' PMC_LIMIT=240 bash tools/pmc.sh r4f_c5 --config 5 --frames 8 --no-decode --steps 1 --warmup 0 || exit 1
