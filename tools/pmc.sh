#!/bin/bash
# rocprofv3 PMC passes (one pass per counter group, each its own run) over one bench configuration,
# eager launches (CSM_GRAPH=0: rocprofv3 cannot trace graph replays here), then a per-kernel summary.
# A counter pass serializes every dispatch and prints nothing for minutes: a heartbeat file under
# gpurun_out/ keeps the run visibly alive.  (The folded layer-0 table stays on: the persistent frame
# decoder needs it, and its build is one launch per codebook.)
# (--roofline-iters 0: no csm_bench_gemv replays, so a kernel's averages are the frame's own launches)
# usage: tools/pmc.sh <tag> <bench args...>      -> gpurun_out/pmc_<tag>/summary.txt
# PMC_REGEX=<regex>: counters only on the kernels it matches (rocprofv3 --kernel-include-regex); the
# rest (weight quantization, context Mimi encode, prefill) run unprofiled, so a config-5 pass stays
# bounded.  PMC_LIMIT: seconds per pass (default 400).
set -o pipefail
tag=$1; shift
export TMPDIR=/tmp
out=gpurun_out/pmc_$tag
mkdir -p $out
(while sleep 20; do date >> $out/heartbeat.txt; done) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
i=0
for pmc in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  CSM_GRAPH=0 timeout -s KILL ${PMC_LIMIT:-400} rocprofv3 --pmc $pmc --kernel-trace ${PMC_REGEX:+--kernel-include-regex "$PMC_REGEX"} --output-format csv -d $out/p$i -o run -- \
    python3 bench.py --no-cpu-baseline --roofline-iters 0 "$@" > $out/p$i.json 2> $out/p$i.err || { echo "pass $i ($pmc) failed rc=$?"; tail -5 $out/p$i.err; exit 1; }
  echo "pass $i done: $pmc"
done
python3 tools/pmc_kernels.py $out > $out/summary.txt && head -40 $out/summary.txt
