# config 8 (int4 B = 1 stream_generate: decode_step per frame beside the persistent kernels): stream priorities A/B
set -o pipefail
for r in 1 2; do for v in 0 1; do
  CSM_STREAM_PRIO=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 8 --steps 1 --warmup 1 > gpurun_out/p8_$v.json 2> gpurun_out/p8_$v.err || { tail -5 gpurun_out/p8_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/p8_$v.json')); print('config 8 prio=$v', d['value'])"
done; done
