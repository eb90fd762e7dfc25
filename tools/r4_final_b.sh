#!/bin/bash
# Round-4 end evidence, part B: config lines (configs[2..4] + the sampled B = 1 lines), the fp32 configs[1]
# side line (the reference's random-init arithmetic class), config-4 and config-5 kernel traces and PMC passes
# (config 5 bounded to the frame kernels by PMC_REGEX), config-5 phase split.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/configs.sh 3 4 5 6 7 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 5 --steps 2 --warmup 1 --phases > gpurun_out/r4f_c5_phases.json 2> gpurun_out/r4f_c5_phases.err || { tail -5 gpurun_out/r4f_c5_phases.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4f_c5_phases.json')); print('config 5 phases', d['value'], d['phases_s_per_step'])"
timeout -k 10 600 python -u bench.py --no-cpu-baseline --dtype float32 --steps 2 --warmup 1 > gpurun_out/r4f_fp32.json 2> gpurun_out/r4f_fp32.err || { tail -20 gpurun_out/r4f_fp32.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4f_fp32.json')); print('fp32', d['value'], d['roofline']['kernel'][:40], d['roofline']['avg_us'])"
bash tools/prof.sh r4f_c4 --config 4 --steps 1 --warmup 0 --frames 24 > /dev/null || exit 1
head -16 gpurun_out/prof_r4f_c4/per_frame.txt
bash tools/prof.sh r4f_c5 --config 5 --steps 1 --warmup 0 --frames 24 > /dev/null || exit 1
head -24 gpurun_out/prof_r4f_c5/per_frame.txt
PMC_REGEX='gemm_xs|gemm_wide|attn|embed|advance|gather|sample' PMC_LIMIT=300 bash tools/pmc.sh r4f_c4 --config 4 --frames 8 --no-decode --steps 1 --warmup 0 || exit 1
PMC_REGEX='gemm_xs|gemm_wide|attn|embed|advance|gather' PMC_LIMIT=300 bash tools/pmc.sh r4f_c5 --config 5 --frames 8 --no-decode --steps 1 --warmup 0 || exit 1
