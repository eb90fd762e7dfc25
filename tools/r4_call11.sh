#!/bin/bash
# Round 4 call 11: 128 x 128-tile codec GEMMs for the long one-shot problems -- codec / config / long tests,
# then configs 5 / 4 and the B = 1 line against CSM_MIMI_T128=0.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_mimi_gpu.py tests/test_configs_gpu.py tests/test_long_gpu.py tests/test_generate_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r11_tests.log 2>&1 || { tail -30 gpurun_out/r11_tests.log; exit 1; }
tail -1 gpurun_out/r11_tests.log
for c in 5 4; do
  for v in t128 t64; do
    envs=""; [ $v = t64 ] && envs="CSM_MIMI_T128=0"
    env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline --config $c --steps 2 --warmup 1 --phases > gpurun_out/r11_c${c}_$v.json 2> gpurun_out/r11_c${c}_$v.err || { tail -5 gpurun_out/r11_c${c}_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r11_c${c}_$v.json')); print('config $c $v', d['value'], d['phases_s_per_step'])"
  done
done
for v in t128 t64; do
  envs=""; [ $v = t64 ] && envs="CSM_MIMI_T128=0"
  env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r11_b1_$v.json 2> gpurun_out/r11_b1_$v.err || { tail -5 gpurun_out/r11_b1_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r11_b1_$v.json')); print('B=1 $v', d['value'], d['ms_per_step'])"
done
timeout -k 10 600 python -u -m pytest tests/test_sampler_filters_gpu.py tests/test_csm_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r11_tests2.log 2>&1 || { tail -30 gpurun_out/r11_tests2.log; exit 1; }
tail -1 gpurun_out/r11_tests2.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 3 --steps 2 --warmup 1 > gpurun_out/r11_c3.json 2> gpurun_out/r11_c3.err || { tail -5 gpurun_out/r11_c3.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r11_c3.json')); print('config 3', d['value'])"
bash tools/prof.sh r11_c3 --config 3 --steps 1 --warmup 0 --frames 24 > /dev/null || exit 1
grep -E "sample_kernel|span" gpurun_out/prof_r11_c3/per_frame.txt
