#!/bin/bash
# Round 4 call 14 (measurement only): B = 1 persistent-kernel phase stamps (bb_step, dec_frame), gemm_xs
# phase stamps (lab build -DXS_STAMPS=1) for the decoder / backbone shapes at 32 and 64 rows, and a
# config-4 per-frame kernel trace on HEAD.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/bb_stamps.py 4 > gpurun_out/r14_bb_stamps.txt 2>&1 || { tail -5 gpurun_out/r14_bb_stamps.txt; exit 1; }
cat gpurun_out/r14_bb_stamps.txt
timeout -k 10 200 python -u tools/df_stamps.py 4 > gpurun_out/r14_df_stamps.txt 2>&1 || { tail -5 gpurun_out/r14_df_stamps.txt; exit 1; }
cat gpurun_out/r14_df_stamps.txt
CSM_HIP_LIB=$PWD/abl/libcsm_hip_xsst.so GB_XS=1 GB_ITERS=40 timeout -k 10 300 python -u tools/gemm_bench.py bf16 32 64 > gpurun_out/r14_xs_stamps.txt 2>&1 || { tail -5 gpurun_out/r14_xs_stamps.txt; exit 1; }
CSM_HIP_LIB=$PWD/abl/libcsm_hip_xsst.so GB_XS=1 GB_ITERS=40 timeout -k 10 300 python -u tools/gemm_bench.py q4 64 >> gpurun_out/r14_xs_stamps.txt 2>&1 || { tail -5 gpurun_out/r14_xs_stamps.txt; exit 1; }
grep -E "xs_stamps (dec|bb)" gpurun_out/r14_xs_stamps.txt
bash tools/prof.sh r14_c4 --config 4 --steps 1 --warmup 0 --frames 24 > /dev/null || exit 1
head -24 gpurun_out/prof_r14_c4/per_frame.txt
