#!/bin/bash
# Round-4 end evidence, part C (final tree after the RVQ change): full GPU suite, smoke(), the bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4fc_suite.log 2>&1 || { tail -30 gpurun_out/r4fc_suite.log; exit 1; }
tail -1 gpurun_out/r4fc_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4fc_smoke.log 2>&1 || { tail -10 gpurun_out/r4fc_smoke.log; exit 1; }
tail -1 gpurun_out/r4fc_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r4fc_bench.json 2> gpurun_out/r4fc_bench.err || { tail -20 gpurun_out/r4fc_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4fc_bench.json')); print('bench', d['value'], d['roofline']['avg_us'], d['roofline']['frac'], d['cpu_baseline']['value'])"
echo RC=0
