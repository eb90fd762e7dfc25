#!/bin/bash
# Round 4 call 12 (session 2 start): full GPU suite on the compacted top-k sampler, then config 3
# (B = 32, temperature 0.8 / top-k 50) A/B: sample_kernel with the Gumbel noise drawn for the
# compacted survivors only (new) vs in place over every slot (oldsamp), alternated.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r12_suite.log 2>&1 || { tail -30 gpurun_out/r12_suite.log; exit 1; }
tail -1 gpurun_out/r12_suite.log
for rep in 1 2; do
  for v in new oldsamp; do
    CSM_HIP_LIB=$PWD/abl/libcsm_hip_$v.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 3 --steps 2 --warmup 1 > gpurun_out/r12_c3_$v$rep.json 2> gpurun_out/r12_c3_$v$rep.err || { tail -5 gpurun_out/r12_c3_$v$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r12_c3_$v$rep.json')); print('config 3 $v', d['value'], d['ms_per_step'])"
  done
done
bash tools/prof.sh r12_c3 --config 3 --steps 1 --warmup 0 --frames 24 > /dev/null || exit 1
grep -E "sample_kernel|span" gpurun_out/prof_r12_c3/per_frame.txt
