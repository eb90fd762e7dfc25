# config 5 per-frame kernel trace on the current tree
set -o pipefail
bash tools/prof.sh r6c5 --config 5 --steps 1 --warmup 1 > gpurun_out/prof_r6c5.log 2>&1 || { tail -5 gpurun_out/prof_r6c5.log; exit 1; }
head -36 gpurun_out/prof_r6c5/per_frame.txt
