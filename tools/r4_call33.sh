#!/bin/bash
# Round 4 call 33: wide codec tile with a K-step of 32 (CSM_MIMI_BK=32, default) vs 16: bit identity vs the
# VALU tile, codec / config tests, codec kernel traces for both, config 5 A/B alternated.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/mimi_mfma_check.py gpurun_out/r33_mimi_bk32.npz > gpurun_out/r33_mimi_bk32.log 2>&1 || { tail -5 gpurun_out/r33_mimi_bk32.log; exit 1; }
CSM_MIMI_MFMA=0 timeout -k 10 300 python -u tools/mimi_mfma_check.py gpurun_out/r33_mimi_valu.npz > gpurun_out/r33_mimi_valu.log 2>&1 || { tail -5 gpurun_out/r33_mimi_valu.log; exit 1; }
python3 tools/mimi_mfma_check.py --cmp gpurun_out/r33_mimi_bk32.npz gpurun_out/r33_mimi_valu.npz
timeout -k 10 500 python -u -m pytest tests/test_mimi_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r33_tests.log 2>&1 || { tail -30 gpurun_out/r33_tests.log; exit 1; }
tail -1 gpurun_out/r33_tests.log
for v in 32 16; do
  CSM_MIMI_BK=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof33_mimi_$v -o run -- python3 -u tools/mimi_prof.py 64 5 > gpurun_out/r33_mimi_$v.log 2>&1 || { tail -5 gpurun_out/r33_mimi_$v.log; exit 1; }
  grep "encode\|decode" gpurun_out/r33_mimi_$v.log
done
run() {  # config bk tag
  CSM_MIMI_BK=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline $1 --steps 2 --warmup 1 --phases > gpurun_out/r33_$3_$2.json 2> gpurun_out/r33_$3_$2.err || { tail -5 gpurun_out/r33_$3_$2.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r33_$3_$2.json')); print('$3 bk=$2', d['value'], d['ms_per_step'], d.get('phases_s_per_step'))"
}
for rep in 1 2; do for v in 32 16; do run "--config 5" $v c5 || exit 1; done; done
echo RC=0
