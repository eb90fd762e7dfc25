# PMC passes of configs 4 / 5 with counters on the persistent batched step only (HBM bytes per launch)
set -o pipefail
for c in 4 5; do
  PMC_REGEX="dec_step_xs" PMC_LIMIT=300 bash tools/pmc.sh r6c$c --config $c --frames 8 --steps 1 --warmup 0 > gpurun_out/pmc_r6c$c.log 2>&1 || { tail -5 gpurun_out/pmc_r6c$c.log; exit 1; }
  grep "dec_step\|kernel |" gpurun_out/pmc_r6c$c/summary.txt
done
