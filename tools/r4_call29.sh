#!/bin/bash
# Round 4 call 29: codec kernel traces (B = 64 x 5 s encode x 2 + decode) with the wide tiles on / off.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 1 0; do
  CSM_MIMI_WIDE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mimi_$v -o run -- python3 -u tools/mimi_prof.py 64 5 > gpurun_out/r29_mimi_$v.log 2>&1 || { tail -5 gpurun_out/r29_mimi_$v.log; exit 1; }
  grep "encode\|decode" gpurun_out/r29_mimi_$v.log
done
echo RC=0
