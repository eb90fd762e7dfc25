#!/bin/bash
# Round 4 call 22: full GPU suite on the tree's lib (step 1 on the streaming GEMM, the small decoder projections
# without split-K at 8 waves), then evidence part B's config lines, config-5 phases, the fp32 side line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r22_suite.log 2>&1 || { tail -30 gpurun_out/r22_suite.log; exit 1; }
tail -1 gpurun_out/r22_suite.log
bash tools/configs.sh 4 3 5 6 7 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 5 --steps 2 --warmup 1 --phases > gpurun_out/r4f_c5_phases.json 2> gpurun_out/r4f_c5_phases.err || { tail -5 gpurun_out/r4f_c5_phases.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4f_c5_phases.json')); print('config 5 phases', d['value'], d['phases_s_per_step'])"
timeout -k 10 600 python -u bench.py --no-cpu-baseline --dtype float32 --steps 2 --warmup 1 > gpurun_out/r4f_fp32.json 2> gpurun_out/r4f_fp32.err || { tail -20 gpurun_out/r4f_fp32.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4f_fp32.json')); print('fp32', d['value'], d['roofline']['kernel'][:40], d['roofline']['avg_us'])"
