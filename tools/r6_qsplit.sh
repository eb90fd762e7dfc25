# bf16 step kernel: QKV K halves on two workgroups (XSD_QSPLIT) -- tests on it, stamps, config 4 A/B; int4 codegen vs HEAD's kernel (base)
set -o pipefail
mkdir -p gpurun_out
CSM_HIP_LIB=$PWD/lab/libcsm_hip_qs1.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dec_xsd_gpu.py "tests/test_batched_long_gpu.py::test_config4_shard_b32_greedy_125_frames" "tests/test_batched_long_gpu.py::test_config3_stream_b32_sampled_64_frames" > gpurun_out/qs_tests.log 2>&1 || { tail -30 gpurun_out/qs_tests.log; exit 1; }
tail -1 gpurun_out/qs_tests.log
for v in qs0 qs1; do
  CSM_HIP_LIB=$PWD/lab/libcsm_hip_$v.so timeout -k 10 150 python -u tools/xsd_stamps.py 32 3 bf16 > gpurun_out/qs_st_$v.log 2>&1 || { tail -5 gpurun_out/qs_st_$v.log; exit 1; }
  echo "$v"; sed -n 1,3p gpurun_out/qs_st_$v.log
done
bash tools/ab.sh -c 4 qs0 qs1 qs0 qs1
bash tools/ab.sh -c 5 base qs1 base qs1
