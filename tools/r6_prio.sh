# config 3 (streaming decode_step overlapping the frames): stream priorities A/B, alternating
set -o pipefail
for r in 1 2; do for v in 0 1; do
  CSM_STREAM_PRIO=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 3 --steps 1 --warmup 1 > gpurun_out/prio_$v.json 2> gpurun_out/prio_$v.err || { tail -5 gpurun_out/prio_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/prio_$v.json')); print('prio=$v', d['value'])"
done; done
