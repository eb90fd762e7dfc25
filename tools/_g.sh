set -e
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gemm_gpu.py tests/test_quant_gpu.py tests/test_configs_gpu.py > gpurun_out/tg.log 2>&1
DT=bf16 timeout -k 10 200 python -u tools/gemm_bench.py bf16 32 64 > gpurun_out/gw_bf16.txt 2>&1
timeout -k 10 200 python -u tools/gemm_bench.py q4 32 64 > gpurun_out/gw_q4.txt 2>&1
