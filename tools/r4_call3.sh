#!/bin/bash
# Round 4 call 3: gemm_xs one-block-per-CU (dynamic LDS pad) and reduce-only ablation; config-5 PMC
# pass bounded to the frame kernels (PMC_REGEX) and its per-phase wall split.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base pad xslab16 xslab8; do
  lib=""; envs=""
  case $v in base) ;; pad) envs="CSM_XS_LDS_PAD=98304";; *) lib=$PWD/abl/libcsm_hip_$v.so;; esac
  env CSM_HIP_LIB=$lib $envs GB_XS=1 timeout -k 10 300 python -u tools/gemm_bench.py bf16 32 > gpurun_out/lab3_$v.txt 2>&1 || { tail -5 gpurun_out/lab3_$v.txt; exit 1; }
  env CSM_HIP_LIB=$lib $envs GB_XS=1 timeout -k 10 300 python -u tools/gemm_bench.py q4 64 >> gpurun_out/lab3_$v.txt 2>&1 || { tail -5 gpurun_out/lab3_$v.txt; exit 1; }
  grep " dec .* xs " gpurun_out/lab3_$v.txt | sed "s/^/$v /"
done
for v in base pad; do
  envs=""; [ $v = pad ] && envs="CSM_XS_LDS_PAD=98304"
  env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 4 --steps 2 --warmup 1 > gpurun_out/lab3_c4_$v.json 2> gpurun_out/lab3_c4_$v.err || { tail -5 gpurun_out/lab3_c4_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/lab3_c4_$v.json')); print('config 4 $v', d['value'])"
done
timeout -k 10 400 python -u bench.py --no-cpu-baseline --config 5 --steps 1 --warmup 1 --phases > gpurun_out/r4_c5_phases.json 2> gpurun_out/r4_c5_phases.err || { tail -5 gpurun_out/r4_c5_phases.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4_c5_phases.json')); print('config 5 phases', d['value'], d['phases_s_per_step'])"
PMC_REGEX='gemm_xs|gemm_wide|attn|embed|advance|gather' PMC_LIMIT=300 bash tools/pmc.sh r4_c5 --config 5 --frames 8 --no-decode --steps 1 --warmup 0 || exit 1
