#!/bin/bash
# Round 4 call 32: knob sweep on the current tree (environment only, no rebuild): streaming-GEMM block
# target, codec wide-tile column threshold, codec split-K block target; configs 5 / 3, default alternated.
set -o pipefail
mkdir -p gpurun_out
run() {  # tag config env...
  local tag=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu-baseline --config $cfg --steps 2 --warmup 1 --phases > gpurun_out/r32_$tag.json 2> gpurun_out/r32_$tag.err || { tail -5 gpurun_out/r32_$tag.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r32_$tag.json')); print('$tag', d['value'], d['ms_per_step'], d.get('phases_s_per_step'))"
}
run c5_def1 5 X=0 || exit 1
run c5_xs192 5 CSM_XS_BLOCKS=192 || exit 1
run c5_xs384 5 CSM_XS_BLOCKS=384 || exit 1
run c5_def2 5 X=0 || exit 1
run c5_wn128 5 CSM_MIMI_WIDE_N=128 || exit 1
run c5_def3 5 X=0 || exit 1
run c3_def1 3 X=0 || exit 1
run c3_ks1024 3 CSM_MIMI_KS_BLOCKS=1024 || exit 1
run c3_wn128 3 CSM_MIMI_WIDE_N=128 || exit 1
run c3_def2 3 X=0 || exit 1
echo RC=0
