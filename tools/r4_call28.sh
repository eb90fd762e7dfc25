#!/bin/bash
# Round 4 call 28: codec GEMMs of >= 256 columns on BM x 128 tiles (gemm128_mf_kernel, CSM_MIMI_WIDE=1,
# default) vs the 64 x 64 tile (=0): bit-identity of encode codes / decode / streaming decode_step PCM,
# codec + config parity tests, then configs 5 / 3 with the phase split, alternated.
set -o pipefail
mkdir -p gpurun_out
for v in 1 0; do
  CSM_MIMI_WIDE=$v timeout -k 10 300 python -u tools/mimi_mfma_check.py gpurun_out/r28_mimi_$v.npz > gpurun_out/r28_mimi_$v.log 2>&1 || { tail -5 gpurun_out/r28_mimi_$v.log; exit 1; }
done
python3 tools/mimi_mfma_check.py --cmp gpurun_out/r28_mimi_1.npz gpurun_out/r28_mimi_0.npz
timeout -k 10 700 python -u -m pytest tests/test_mimi_gpu.py tests/test_configs_gpu.py tests/test_long_gpu.py tests/test_generate_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r28_tests.log 2>&1 || { tail -30 gpurun_out/r28_tests.log; exit 1; }
tail -1 gpurun_out/r28_tests.log
run() {  # config wide tag
  CSM_MIMI_WIDE=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline $1 --steps 2 --warmup 1 --phases > gpurun_out/r28_$3_$2.json 2> gpurun_out/r28_$3_$2.err || { tail -5 gpurun_out/r28_$3_$2.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r28_$3_$2.json')); print('$3 wide=$2', d['value'], d['ms_per_step'], d.get('phases_s_per_step'))"
}
for rep in 1 2; do for v in 1 0; do run "--config 5" $v c5 || exit 1; done; done
for v in 1 0; do run "--config 3" $v c3 || exit 1; done
echo RC=0
