#!/bin/bash
# Round 4 call 31: codec epilogue loads four rows at a time; wide tiles routed by taps and block count.
# Bit identity vs the VALU tile, codec / config tests, codec kernel trace (wide on), configs 5 / 3 A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/mimi_mfma_check.py gpurun_out/r31_mimi_w1.npz > gpurun_out/r31_mimi_w1.log 2>&1 || { tail -5 gpurun_out/r31_mimi_w1.log; exit 1; }
CSM_MIMI_MFMA=0 timeout -k 10 300 python -u tools/mimi_mfma_check.py gpurun_out/r31_mimi_valu.npz > gpurun_out/r31_mimi_valu.log 2>&1 || { tail -5 gpurun_out/r31_mimi_valu.log; exit 1; }
python3 tools/mimi_mfma_check.py --cmp gpurun_out/r31_mimi_w1.npz gpurun_out/r31_mimi_valu.npz
timeout -k 10 500 python -u -m pytest tests/test_mimi_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r31_tests.log 2>&1 || { tail -30 gpurun_out/r31_tests.log; exit 1; }
tail -1 gpurun_out/r31_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof31_mimi -o run -- python3 -u tools/mimi_prof.py 64 5 > gpurun_out/r31_mimi.log 2>&1 || { tail -5 gpurun_out/r31_mimi.log; exit 1; }
grep "encode\|decode" gpurun_out/r31_mimi.log
run() {  # config wide tag
  CSM_MIMI_WIDE=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline $1 --steps 2 --warmup 1 --phases > gpurun_out/r31_$3_$2.json 2> gpurun_out/r31_$3_$2.err || { tail -5 gpurun_out/r31_$3_$2.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r31_$3_$2.json')); print('$3 wide=$2', d['value'], d['ms_per_step'], d.get('phases_s_per_step'))"
}
for rep in 1 2; do for v in 1 0; do run "--config 5" $v c5 || exit 1; done; done
for v in 1 0; do run "--config 3" $v c3 || exit 1; done
echo RC=0
