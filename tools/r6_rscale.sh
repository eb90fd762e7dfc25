# bf16 QKV K halves: row scales published by the half-0 workgroups (rs1) vs computed by each attention wave (rs0)
set -o pipefail
mkdir -p gpurun_out
CSM_HIP_LIB=$PWD/lab/libcsm_hip_rs1.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dec_xsd_gpu.py "tests/test_batched_long_gpu.py::test_config4_shard_b32_greedy_125_frames" > gpurun_out/rs_tests.log 2>&1 || { tail -30 gpurun_out/rs_tests.log; exit 1; }
tail -1 gpurun_out/rs_tests.log
bash tools/ab.sh -c 4 rs0 rs1 rs0 rs1
