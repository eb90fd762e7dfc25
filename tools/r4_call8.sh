#!/bin/bash
# Round 4 call 8: the full GPU suite on HEAD (new: host-sampled frames, tie-heavy filter rows, q4 bb_xs)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r8_suite.log 2>&1 || { tail -40 gpurun_out/r8_suite.log; exit 1; }
tail -2 gpurun_out/r8_suite.log
