#!/bin/bash
# Round 4 call 13: (1) full GPU suite on the tree's lib = gemm_xs over fp32 fragment-ordered activations
# split in registers (XS_F32) + short attention with 16-B V rows + compacted top-k sampler; (2) decoder
# shapes xs4 (XS_F32) vs xs6 (producer-split parts); (3) configs 4 / 5 / 3: xs4 vs xs6 vs oldattn
# (xs4 with the previous short attention), alternated.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r13_suite.log 2>&1 || { tail -30 gpurun_out/r13_suite.log; exit 1; }
tail -1 gpurun_out/r13_suite.log
for v in xs4 xs6; do
  CSM_HIP_LIB=$PWD/abl/libcsm_hip_$v.so GB_XS=1 GB_ITERS=100 timeout -k 10 300 python -u tools/gemm_bench.py bf16 32 64 > gpurun_out/r13_gb_$v.txt 2>&1 || { tail -5 gpurun_out/r13_gb_$v.txt; exit 1; }
  CSM_HIP_LIB=$PWD/abl/libcsm_hip_$v.so GB_XS=1 GB_ITERS=100 timeout -k 10 300 python -u tools/gemm_bench.py q4 64 >> gpurun_out/r13_gb_$v.txt 2>&1 || { tail -5 gpurun_out/r13_gb_$v.txt; exit 1; }
  grep " xs " gpurun_out/r13_gb_$v.txt | sed "s/^/$v /"
done
run() {  # config variant tag
  CSM_HIP_LIB=$PWD/abl/libcsm_hip_$2.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --config $1 --steps 2 --warmup 1 > gpurun_out/r13_c$1_$2$3.json 2> gpurun_out/r13_c$1_$2$3.err || { tail -5 gpurun_out/r13_c$1_$2$3.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r13_c$1_$2$3.json')); print('config $1 $2', d['value'], d['ms_per_step'])"
}
for rep in 1 2; do for v in xs4 xs6 oldattn; do run 4 $v $rep || exit 1; done; done
for rep in 1 2; do for v in xs4 xs6; do run 5 $v $rep || exit 1; done; done
for v in xs4 xs6; do run 3 $v 1 || exit 1; done
