# int4 step kernel: the head's two row tiles on separate workgroups (hs1) vs HEAD's kernel (hs0): tests, config 5 A/B
set -o pipefail
mkdir -p gpurun_out
CSM_HIP_LIB=$PWD/lab/libcsm_hip_hs1.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dec_xsd_gpu.py "tests/test_batched_long_gpu.py::test_config5_q4_b64_greedy_125_frames" > gpurun_out/hs_tests.log 2>&1 || { tail -30 gpurun_out/hs_tests.log; exit 1; }
tail -1 gpurun_out/hs_tests.log
bash tools/ab.sh -c 5 hs0 hs1 hs0 hs1
