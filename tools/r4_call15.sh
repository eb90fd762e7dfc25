#!/bin/bash
# Round 4 call 15: codec GEMM tiles on the fp32 matrix cores (gemm64_mf_kernel, CSM_MIMI_MFMA=1, default) vs
# the VALU tile (=0): bit-identity of encode codes / one-shot decode / streaming decode_step PCM between the
# two, codec + config parity tests, then configs 5 / 4 (with phase split) and the B = 1 line, alternated.
set -o pipefail
mkdir -p gpurun_out
for v in 1 0; do
  CSM_MIMI_MFMA=$v timeout -k 10 300 python -u tools/mimi_mfma_check.py gpurun_out/r15_mimi_$v.npz > gpurun_out/r15_mimi_$v.log 2>&1 || { tail -5 gpurun_out/r15_mimi_$v.log; exit 1; }
done
python3 tools/mimi_mfma_check.py --cmp gpurun_out/r15_mimi_1.npz gpurun_out/r15_mimi_0.npz
timeout -k 10 700 python -u -m pytest tests/test_mimi_gpu.py tests/test_configs_gpu.py tests/test_long_gpu.py tests/test_generate_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r15_tests.log 2>&1 || { tail -30 gpurun_out/r15_tests.log; exit 1; }
tail -1 gpurun_out/r15_tests.log
run() {  # config mfma tag
  CSM_MIMI_MFMA=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline $1 --steps 2 --warmup 1 --phases > gpurun_out/r15_$3_$2.json 2> gpurun_out/r15_$3_$2.err || { tail -5 gpurun_out/r15_$3_$2.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r15_$3_$2.json')); print('$3 mfma=$2', d['value'], d['ms_per_step'], d.get('phases_s_per_step'))"
}
for rep in 1 2; do for v in 1 0; do run "--config 5" $v c5 || exit 1; done; done
for v in 1 0; do run "--config 4" $v c4 || exit 1; done
for rep in 1 2; do for v in 1 0; do run "" $v b1 || exit 1; done; done
