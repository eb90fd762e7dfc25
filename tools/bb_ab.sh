# bb_step variant A/B with stamps: test on the first variant, then bench + stamps per variant
mkdir -p gpurun_out
CSM_HIP_LIB=$PWD/abl/libcsm_hip_$1.so timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_bb_step_gpu.py > gpurun_out/t_bbab.log 2>&1 || { tail -20 gpurun_out/t_bbab.log; exit 1; }
tail -1 gpurun_out/t_bbab.log
for v in "$@"; do
  CSM_HIP_LIB=$PWD/abl/libcsm_hip_$v.so timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bb_$v.json 2> gpurun_out/bb_$v.err || exit 1
  CSM_HIP_LIB=$PWD/abl/libcsm_hip_$v.so timeout -k 10 120 python -u tools/bb_stamps.py 4 > gpurun_out/bbst_$v.txt 2>&1 || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/bb_$v.json')); print('$v', d['value'], d['ms_per_step'], d['roofline_backbone']['avg_us'])"
  grep "WG \|per layer" gpurun_out/bbst_$v.txt
done
