#!/bin/bash
# Round 4 call 19: abl new = gemm_xs int4 64-row blocks with the tile-split wave layout (TSPLIT) + codec MFMA
# tile staging strided convs along the taps (kcontig); vs cur (HEAD).  Tests on new, codec bit identity,
# int4 decoder shapes, config 5 with the phase split.
set -o pipefail
mkdir -p gpurun_out
export CSM_HIP_LIB_NEW=$PWD/abl/libcsm_hip_new.so
CSM_HIP_LIB=$CSM_HIP_LIB_NEW timeout -k 10 700 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_kernel_gpu.py tests/test_configs_gpu.py tests/test_mimi_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r19_tests.log 2>&1 || { tail -30 gpurun_out/r19_tests.log; exit 1; }
tail -1 gpurun_out/r19_tests.log
for v in 1 0; do
  CSM_HIP_LIB=$CSM_HIP_LIB_NEW CSM_MIMI_MFMA=$v timeout -k 10 300 python -u tools/mimi_mfma_check.py gpurun_out/r19_mimi_$v.npz > gpurun_out/r19_mimi_$v.log 2>&1 || { tail -5 gpurun_out/r19_mimi_$v.log; exit 1; }
done
python3 tools/mimi_mfma_check.py --cmp gpurun_out/r19_mimi_1.npz gpurun_out/r19_mimi_0.npz
for v in new cur; do
  CSM_HIP_LIB=$PWD/abl/libcsm_hip_$v.so GB_XS=1 GB_ITERS=100 timeout -k 10 300 python -u tools/gemm_bench.py q4 64 > gpurun_out/r19_gb_$v.txt 2>&1 || { tail -5 gpurun_out/r19_gb_$v.txt; exit 1; }
  grep " xs " gpurun_out/r19_gb_$v.txt | sed "s/^/$v /"
done
run() {  # args tag lib
  CSM_HIP_LIB=$PWD/abl/libcsm_hip_$3.so timeout -k 10 300 python -u bench.py --no-cpu-baseline $1 --steps 2 --warmup 1 --phases > gpurun_out/r19_$2.json 2> gpurun_out/r19_$2.err || { tail -5 gpurun_out/r19_$2.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r19_$2.json')); print('$2', d['value'], d['ms_per_step'], d.get('phases_s_per_step'))"
}
for rep in 1 2; do
  run "--config 5" c5_new$rep new || exit 1
  run "--config 5" c5_cur$rep cur || exit 1
done
