#!/bin/bash
# Round-3 evidence, part B: one bench line per BASELINE workload (configs 4 5 3 + the B = 1 sampled
# lines 6 7), PMC passes of configs 4 and 5 (per-kernel MFMA busy / FETCH_SIZE / WRITE_SIZE).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/configs.sh 4 5 3 6 7 || exit 1
bash tools/pmc.sh r3_c4 --config 4 --steps 1 --warmup 0 > gpurun_out/pmc_c4.log 2>&1 || { tail -5 gpurun_out/pmc_c4.log; exit 1; }
head -12 gpurun_out/pmc_r3_c4/summary.txt
bash tools/pmc.sh r3_c5 --config 5 --steps 1 --warmup 0 > gpurun_out/pmc_c5.log 2>&1 || { tail -5 gpurun_out/pmc_c5.log; exit 1; }
head -12 gpurun_out/pmc_r3_c5/summary.txt
