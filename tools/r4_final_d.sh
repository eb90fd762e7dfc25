#!/bin/bash
# Round-4 end evidence, part D (final tree after the int4-prefill change): full GPU suite, then the prefill
# split-K block-target sweep (tools/r4_call38.sh).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4fd_suite.log 2>&1 || { tail -30 gpurun_out/r4fd_suite.log; exit 1; }
tail -1 gpurun_out/r4fd_suite.log
bash tools/r4_call38.sh
