# step kernel with the in-launch sampler (sampled top-k steps): tests, then config 3 A/B (dec_xsd_sample 0 / 1 via env)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dec_xsd_gpu.py "tests/test_batched_long_gpu.py::test_config3_stream_b32_sampled_64_frames" > gpurun_out/xsm_tests.log 2>&1 || { tail -30 gpurun_out/xsm_tests.log; exit 1; }
tail -3 gpurun_out/xsm_tests.log
for r in 1 2; do for v in 0 1; do
  CSM_DEC_XSD_SAMPLE=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 3 --steps 1 --warmup 1 > gpurun_out/xsm_$v.json 2> gpurun_out/xsm_$v.err || { tail -5 gpurun_out/xsm_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/xsm_$v.json')); print('config 3 dec_xsd_sample=$v', d['value'], d['roofline']['avg_us'])"
done; done
