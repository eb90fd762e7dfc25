timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dist_gpu.py > gpurun_out/td.log 2>&1; echo "rc=$?"
