#!/bin/bash
# Round-4 end evidence, part A: full GPU suite, the bench line (with cpu_baseline), rocprofv3
# kernel-trace --stats of the bench command (eager), PMC passes of the B = 1 path.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4f_suite.log 2>&1 || { tail -30 gpurun_out/r4f_suite.log; exit 1; }
tail -1 gpurun_out/r4f_suite.log
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 > gpurun_out/r4f_bench.json 2> gpurun_out/r4f_bench.err || { tail -20 gpurun_out/r4f_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4f_bench.json')); print('bench', d['value'], d['roofline']['avg_us'], d['roofline']['frac'], d['roofline_backbone']['avg_us'], d['cpu_baseline']['value'])"
mkdir -p gpurun_out/r4f_prof
CSM_GRAPH=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4f_prof -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/r4f_prof/bench.json 2> gpurun_out/r4f_prof/bench.err || { echo "prof failed rc=$?"; tail -20 gpurun_out/r4f_prof/bench.err; exit 1; }
f=$(find gpurun_out/r4f_prof -name "*kernel_stats.csv" | head -1)
python3 tools/kstats.py "$f" 14
bash tools/pmc.sh r4f_b1 --no-decode --frames 8 --steps 1 --warmup 0 || exit 1
