#!/bin/bash
# Round-end evidence in one GPU call: the bench line, the rocprofv3 kernel-trace --stats summary of
# the bench command (eager: graph replays cannot be traced on this ROCm build), and a separate
# FETCH_SIZE counter pass for the roofline's traffic field.  Outputs under gpurun_out/final_*.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/final_prof gpurun_out/final_pmc
[ "$1" = "pmc" ] || { timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || { echo "bench failed rc=$?"; tail -20 gpurun_out/final_bench.err; exit 1; }
cat gpurun_out/final_bench.json
CSM_GRAPH=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final_prof -o run -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/final_prof/bench.json 2> gpurun_out/final_prof/bench.err || { echo "prof failed rc=$?"; tail -20 gpurun_out/final_prof/bench.err; exit 1; }
f=$(find gpurun_out/final_prof -name "*kernel_stats.csv" | head -1)
python3 tools/kstats.py "$f" 20; }
# the counter pass prints nothing for minutes (every dispatch is serialized): keep a heartbeat file;
# the folded layer-0 table (15k one-time build launches) is skipped there -- it does not touch gate/up
(while sleep 20; do date >> gpurun_out/final_pmc/heartbeat.txt; done) &
hb=$!
CSM_GRAPH=0 CSM_QKV0_TAB=0 timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/final_pmc -o run -- python3 bench.py --no-cpu-baseline --no-decode --steps 1 --warmup 0 --frames 8 > gpurun_out/final_pmc/bench.json 2> gpurun_out/final_pmc/bench.err || { echo "pmc failed rc=$?"; tail -20 gpurun_out/final_pmc/bench.err; exit 1; }
kill $hb
c=$(find gpurun_out/final_pmc -name "*counter_collection.csv" | head -1)
python3 tools/pmc_summary.py "$c" gpurun_out/final_pmc/summary.txt gpurun_out/final_pmc/pmc_traffic.json | head -8
