#!/bin/bash
# Round 4 call 17: (1) codec MFMA tile with 4-wide operand loads: bit identity vs the VALU tile, codec /
# config tests, config 5 cur vs mkold (the previous mimi_kernels.hip); (2) the heads' waves per block
# (CSM_XS_HEAD_WAVES 8 = current / 4 / 2: more K slices, the head's bytes over more CUs) on config 4.
set -o pipefail
mkdir -p gpurun_out
for v in 1 0; do
  CSM_MIMI_MFMA=$v timeout -k 10 300 python -u tools/mimi_mfma_check.py gpurun_out/r17_mimi_$v.npz > gpurun_out/r17_mimi_$v.log 2>&1 || { tail -5 gpurun_out/r17_mimi_$v.log; exit 1; }
done
python3 tools/mimi_mfma_check.py --cmp gpurun_out/r17_mimi_1.npz gpurun_out/r17_mimi_0.npz
timeout -k 10 700 python -u -m pytest tests/test_mimi_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r17_tests.log 2>&1 || { tail -30 gpurun_out/r17_tests.log; exit 1; }
tail -1 gpurun_out/r17_tests.log
run() {  # args tag lib envs
  env CSM_HIP_LIB=$PWD/abl/libcsm_hip_$3.so $4 timeout -k 10 300 python -u bench.py --no-cpu-baseline $1 --steps 2 --warmup 1 --phases > gpurun_out/r17_$2.json 2> gpurun_out/r17_$2.err || { tail -5 gpurun_out/r17_$2.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r17_$2.json')); print('$2', d['value'], d['ms_per_step'], d.get('phases_s_per_step'))"
}
for rep in 1 2; do
  run "--config 5" c5_cur$rep cur "" || exit 1
  run "--config 5" c5_mkold$rep mkold "" || exit 1
done
for rep in 1 2; do
  for w in 8 4 2; do run "--config 4" c4_hw${w}_$rep cur "CSM_XS_HEAD_WAVES=$w" || exit 1; done
done
