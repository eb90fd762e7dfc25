# step kernel: attention K / V rows in registers (XSD_KV_REGS) -- tests on it, then stamps + config 4 / 5 lines, alternating
set -o pipefail
mkdir -p gpurun_out
CSM_HIP_LIB=$PWD/lab/libcsm_hip_xkv1.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dec_xsd_gpu.py > gpurun_out/xkv_tests.log 2>&1 || { tail -20 gpurun_out/xkv_tests.log; exit 1; }
tail -1 gpurun_out/xkv_tests.log
for v in xkv0 xkv1; do
  CSM_HIP_LIB=$PWD/lab/libcsm_hip_$v.so timeout -k 10 150 python -u tools/xsd_stamps.py 32 3 bf16 > gpurun_out/xkv_st_$v.log 2>&1 || { tail -5 gpurun_out/xkv_st_$v.log; exit 1; }
  echo "$v"; head -3 gpurun_out/xkv_st_$v.log
done
bash tools/ab.sh -c 4 xkv0 xkv1 xkv0 xkv1
bash tools/ab.sh -c 5 xkv0 xkv1
