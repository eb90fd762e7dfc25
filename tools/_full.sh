set -e
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_r02.json 2> gpurun_out/bench_r02.err
bash tools/configs.sh 4 5 3 > gpurun_out/cfg.log 2>&1
echo done
