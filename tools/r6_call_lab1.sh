# step-kernel VALU / operand-bytes lab (tools/xlab.sh) + PMC passes of configs 4 / 5 on the step kernels
set -o pipefail
bash tools/xlab.sh xlab0 xlab1 xlab2 || exit 1
PMC_REGEX="dec_step_xs" PMC_LIMIT=300 bash tools/pmc.sh r6c4 --config 4 --frames 8 --steps 1 --warmup 0 > gpurun_out/pmc_r6c4.log 2>&1 || { tail -5 gpurun_out/pmc_r6c4.log; exit 1; }
grep dec_step gpurun_out/pmc_r6c4/summary.txt
PMC_REGEX="dec_step_xs" PMC_LIMIT=300 bash tools/pmc.sh r6c5 --config 5 --frames 8 --steps 1 --warmup 0 > gpurun_out/pmc_r6c5.log 2>&1 || { tail -5 gpurun_out/pmc_r6c5.log; exit 1; }
grep dec_step gpurun_out/pmc_r6c5/summary.txt
