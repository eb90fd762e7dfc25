# A/B of in-tree variants (abl/libcsm_hip_<v>.so): dec_frame stamps + a short bench line each
set -e
mkdir -p gpurun_out
for v in "$@"; do
  CSM_HIP_LIB=$PWD/abl/libcsm_hip_$v.so timeout -k 10 120 python -u tools/df_stamps.py 6 > gpurun_out/st_$v.log 2>&1
  CSM_HIP_LIB=$PWD/abl/libcsm_hip_$v.so timeout -k 10 200 python -u bench.py --batch 1 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_$v.log 2>&1
  python3 -c "import json; d=json.load(open('gpurun_out/b_$v.log')); print('$v', d['value'], d['roofline']['avg_us'])"
done
