#!/bin/bash
# A/B of abl/libcsm_hip_<v>.so builds (tools/variant.sh) in one GPU call: a short bench line each,
# printing frames/s and the live dec_frame / bb_step (or GEMM) averages.
# usage: tools/ab.sh [-c N] v1 v2 ...   (an entry v@VAR=value also sets an environment variable)
set -o pipefail
mkdir -p gpurun_out
cfg=""
if [ "$1" = "-c" ]; then cfg="--config $2"; shift 2; fi
for ent in "$@"; do
  v=${ent%%@*}; envs=""; tag=$v
  if [ "$ent" != "$v" ]; then envs=${ent#*@}; tag=${v}_${envs//=/}; fi
  lib=$PWD/lab/libcsm_hip_$v.so
  env CSM_HIP_LIB=$lib $envs timeout -k 10 240 python -u bench.py $cfg --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || { echo "$ent failed"; tail -5 gpurun_out/ab_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$tag.json')); print('$ent', d['value'], 'dominant', d['roofline']['avg_us'], 'backbone', d['roofline_backbone']['avg_us'])"
done
