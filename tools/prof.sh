#!/bin/bash
# Kernel-trace profile of one bench configuration (eager launches: rocprofv3 cannot trace graph replays here).
# usage: tools/prof.sh <tag> <bench args...>
set -o pipefail
tag=$1; shift
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
mkdir -p $out
CSM_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- python3 bench.py --no-cpu-baseline "$@" > $out/bench.json 2> $out/bench.err || { echo "prof failed rc=$?"; tail -20 $out/bench.err; exit 1; }
f=$(find $out -name "*kernel_trace.csv" | head -1)
python3 tools/ktrace.py "$f" > $out/per_frame.txt && head -30 $out/per_frame.txt
