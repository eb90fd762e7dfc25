#!/bin/bash
# Round 4 call 34: split-RVQ distance GEMM scored on the fp32 matrix cores (rvq_step_kernel<true>,
# CSM_RVQ_MFMA=1, default) vs the VALU tile (=0): bit identity of codes / PCM on B = 64 x 5 s (4032 latent
# rows: the GEMM path), codec / config tests, a codec kernel trace, config 5 A/B alternated.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 1 0; do
  CSM_RVQ_MFMA=$v timeout -k 10 300 python -u tools/mimi_prof.py 64 5 gpurun_out/r34_rvq_$v.npz > gpurun_out/r34_rvq_$v.log 2>&1 || { tail -5 gpurun_out/r34_rvq_$v.log; exit 1; }
  grep "encode 1\|decode" gpurun_out/r34_rvq_$v.log
done
python3 tools/mimi_mfma_check.py --cmp gpurun_out/r34_rvq_1.npz gpurun_out/r34_rvq_0.npz
timeout -k 10 500 python -u -m pytest tests/test_mimi_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r34_tests.log 2>&1 || { tail -30 gpurun_out/r34_tests.log; exit 1; }
tail -1 gpurun_out/r34_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof34_mimi -o run -- python3 -u tools/mimi_prof.py 64 5 > gpurun_out/r34_mimi.log 2>&1 || { tail -5 gpurun_out/r34_mimi.log; exit 1; }
grep "rvq_step" gpurun_out/prof34_mimi/run_kernel_stats.csv | cut -c1-160
run() {  # config mfma tag
  CSM_RVQ_MFMA=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline $1 --steps 2 --warmup 1 --phases > gpurun_out/r34_$3_$2.json 2> gpurun_out/r34_$3_$2.err || { tail -5 gpurun_out/r34_$3_$2.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r34_$3_$2.json')); print('$3 rvq_mfma=$2', d['value'], d['ms_per_step'], d.get('phases_s_per_step'))"
}
for rep in 1 2; do for v in 1 0; do run "--config 5" $v c5 || exit 1; done; done
echo RC=0
