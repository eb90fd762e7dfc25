#!/bin/bash
# Round 4 call 38: prefill split-K block target sweep (CSM_GEMM_BLOCKS forces the target of EVERY gemm_wide
# launch; only config 5's prefill phase is read).
set -o pipefail
mkdir -p gpurun_out
run() {  # tag env
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 5 --steps 2 --warmup 1 --phases > gpurun_out/r38_$tag.json 2> gpurun_out/r38_$tag.err || { tail -5 gpurun_out/r38_$tag.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r38_$tag.json')); print('$tag', d['value'], d['ms_per_step'], d.get('phases_s_per_step'))"
}
run def1 X=0 || exit 1
run b128 CSM_GEMM_BLOCKS=128 || exit 1
run b512 CSM_GEMM_BLOCKS=512 || exit 1
run b1024 CSM_GEMM_BLOCKS=1024 || exit 1
run def2 X=0 || exit 1
echo RC=0
