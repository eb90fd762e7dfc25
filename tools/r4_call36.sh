#!/bin/bash
# Round 4 call 36: prompt-prefill tile width sweep (CSM_GEMM_NBR = 256 / 128 for every gemm_wide launch vs the
# per-shape default), config 5 with the phase split (the prefill phase is the one read).
set -o pipefail
mkdir -p gpurun_out
run() {  # tag env
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 5 --steps 2 --warmup 1 --phases > gpurun_out/r36_$tag.json 2> gpurun_out/r36_$tag.err || { tail -5 gpurun_out/r36_$tag.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r36_$tag.json')); print('$tag', d['value'], d['ms_per_step'], d.get('phases_s_per_step'))"
}
run def1 X=0 || exit 1
run nbr256 CSM_GEMM_NBR=256 || exit 1
run nbr128 CSM_GEMM_NBR=128 || exit 1
run def2 X=0 || exit 1
run w4 CSM_GEMM_W8=0 || exit 1
echo RC=0
