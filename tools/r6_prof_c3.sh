# config 3 per-frame kernel trace (streaming decode_step per frame) on the current tree
set -o pipefail
bash tools/prof.sh r6c3 --config 3 --steps 1 --warmup 1 > gpurun_out/prof_r6c3.log 2>&1 || { tail -5 gpurun_out/prof_r6c3.log; exit 1; }
head -40 gpurun_out/prof_r6c3/per_frame.txt
