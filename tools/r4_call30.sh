#!/bin/bash
# Round 4 call 30: codec epilogues with their loads issued before the stores; bit identity of the wide tile,
# the 64 tile and the VALU tile; codec / config tests; codec kernel traces with the wide tiles on / off.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 1 0; do
  CSM_MIMI_WIDE=$v timeout -k 10 300 python -u tools/mimi_mfma_check.py gpurun_out/r30_mimi_w$v.npz > gpurun_out/r30_mimi_w$v.log 2>&1 || { tail -5 gpurun_out/r30_mimi_w$v.log; exit 1; }
done
CSM_MIMI_MFMA=0 timeout -k 10 300 python -u tools/mimi_mfma_check.py gpurun_out/r30_mimi_valu.npz > gpurun_out/r30_mimi_valu.log 2>&1 || { tail -5 gpurun_out/r30_mimi_valu.log; exit 1; }
python3 tools/mimi_mfma_check.py --cmp gpurun_out/r30_mimi_w1.npz gpurun_out/r30_mimi_w0.npz
python3 tools/mimi_mfma_check.py --cmp gpurun_out/r30_mimi_w1.npz gpurun_out/r30_mimi_valu.npz
timeout -k 10 500 python -u -m pytest tests/test_mimi_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r30_tests.log 2>&1 || { tail -30 gpurun_out/r30_tests.log; exit 1; }
tail -1 gpurun_out/r30_tests.log
for v in 1 0; do
  CSM_MIMI_WIDE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof30_mimi_$v -o run -- python3 -u tools/mimi_prof.py 64 5 > gpurun_out/r30_mimi_$v.log 2>&1 || { tail -5 gpurun_out/r30_mimi_$v.log; exit 1; }
  grep "encode\|decode" gpurun_out/r30_mimi_$v.log
done
echo RC=0
