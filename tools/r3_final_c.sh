#!/bin/bash
# Round-3 evidence, part C: PMC passes of configs 4 and 5 on a short run (8 frames, codes only: a
# counter pass serializes every dispatch), per-kernel MFMA busy / FETCH_SIZE / WRITE_SIZE.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/pmc.sh r3_c4 --config 4 --frames 8 --no-decode --steps 1 --warmup 0 > gpurun_out/pmc_c4.log 2>&1 || { tail -5 gpurun_out/pmc_c4.log; exit 1; }
head -14 gpurun_out/pmc_r3_c4/summary.txt
bash tools/pmc.sh r3_c5 --config 5 --frames 8 --no-decode --steps 1 --warmup 0 > gpurun_out/pmc_c5.log 2>&1 || { tail -5 gpurun_out/pmc_c5.log; exit 1; }
head -14 gpurun_out/pmc_r3_c5/summary.txt
