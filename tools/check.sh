# full GPU suite + bench line + eager kernel stats of the bench command (gpurun_out/)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full.log 2>&1; tail -2 gpurun_out/full.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_r02.json 2> gpurun_out/bench_r02.err || { tail -5 gpurun_out/bench_r02.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_r02.json')); print(d['value'], d['roofline']['avg_us'])"
export TMPDIR=/tmp
CSM_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kp -o run -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/kp.json 2>&1 || exit 1
python3 tools/kstats.py $(find gpurun_out/kp -name "*kernel_stats.csv" | head -1) 14
