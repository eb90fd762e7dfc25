#!/bin/bash
# Round-end evidence in one GPU call: the bench line, the rocprofv3 kernel-trace --stats summary of
# the bench command (eager: graph replays cannot be traced on this ROCm build; its dec_frame_kernel
# average must agree with the line's live roofline.avg_us), and the PMC passes of the B = 1 codes
# path (tools/pmc.sh).  Outputs under gpurun_out/final_*.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/final_prof
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || { echo "bench failed rc=$?"; tail -20 gpurun_out/final_bench.err; exit 1; }
cat gpurun_out/final_bench.json
CSM_GRAPH=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final_prof -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/final_prof/bench.json 2> gpurun_out/final_prof/bench.err || { echo "prof failed rc=$?"; tail -20 gpurun_out/final_prof/bench.err; exit 1; }
f=$(find gpurun_out/final_prof -name "*kernel_stats.csv" | head -1)
python3 tools/kstats.py "$f" 20
[ "$1" = "pmc" ] && bash tools/pmc.sh final_b1 --no-decode --frames 8 --steps 1 --warmup 0
exit 0
