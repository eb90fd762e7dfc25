# config 3: the streaming codec's split-K block target (CSM_MIMI_KS_BLOCKS) -- fewer codec blocks beside the step kernel
set -o pipefail
for r in 1 2; do for v in 512 1024 2048; do
  CSM_MIMI_KS_BLOCKS=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 3 --steps 1 --warmup 1 > gpurun_out/mks_$v.json 2> gpurun_out/mks_$v.err || { tail -5 gpurun_out/mks_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/mks_$v.json')); print('config 3 KS_BLOCKS=$v', d['value'])"
done; done
