# bb_step: K / V cache rows prefetched before the E1 wait (BB_KV_EARLY) -- tests, then B = 1 bench A/B, alternating
set -o pipefail
mkdir -p gpurun_out
CSM_HIP_LIB=$PWD/lab/libcsm_hip_kv1.so timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_bb_step_gpu.py tests/test_long_gpu.py > gpurun_out/kv_tests.log 2>&1 || { tail -20 gpurun_out/kv_tests.log; exit 1; }
tail -1 gpurun_out/kv_tests.log
bash tools/ab.sh kv0 kv1 kv0 kv1
