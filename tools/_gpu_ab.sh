set -e
for v in ${TV:-m1}; do
  CSM_HIP_LIB=$PWD/abl/libcsm_hip_$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_dec_frame_gpu.py tests/test_long_gpu.py > gpurun_out/t_$v.log 2>&1 || { echo "tests $v failed"; tail -30 gpurun_out/t_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/t_$v.log)"
done
bash tools/_ab.sh ${AB:-attn m1}
