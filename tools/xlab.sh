# step-kernel lab variants (lab/libcsm_hip_<v>.so): per-role stamps, bf16 B = 32 and int4 B = 64
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  CSM_HIP_LIB=$PWD/lab/libcsm_hip_$v.so timeout -k 10 150 python -u tools/xsd_stamps.py 32 3 bf16 > gpurun_out/xl_${v}_bf16.log 2>&1 || { tail -5 gpurun_out/xl_${v}_bf16.log; exit 1; }
  CSM_HIP_LIB=$PWD/lab/libcsm_hip_$v.so timeout -k 10 150 python -u tools/xsd_stamps.py 64 3 q4 > gpurun_out/xl_${v}_q4.log 2>&1 || { tail -5 gpurun_out/xl_${v}_q4.log; exit 1; }
  echo "== $v"; head -3 gpurun_out/xl_${v}_bf16.log; head -3 gpurun_out/xl_${v}_q4.log
done
