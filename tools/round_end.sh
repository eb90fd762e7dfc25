# round-end: full GPU suite, bench line + rocprof stats + PMC passes (tools/final.sh pmc), config lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full.log 2>&1 || { tail -30 gpurun_out/full.log; exit 1; }
tail -1 gpurun_out/full.log
bash tools/final.sh pmc > gpurun_out/final.log 2>&1 || { tail -20 gpurun_out/final.log; exit 1; }
head -1 gpurun_out/final_bench.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('bench', d['value'], d['roofline']['avg_us'], d['roofline']['frac'])"
bash tools/configs.sh 4 5 3 10 8
