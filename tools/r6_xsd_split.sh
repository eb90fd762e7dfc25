# int4 step kernel with the QKV / o_proj row tiles on separate workgroups: tests, stamps, config 5 / 4 lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dec_xsd_gpu.py "tests/test_batched_long_gpu.py::test_config5_q4_b64_greedy_125_frames" "tests/test_batched_long_gpu.py::test_config4_shard_b32_greedy_125_frames" > gpurun_out/xs_tests.log 2>&1 || { tail -30 gpurun_out/xs_tests.log; exit 1; }
tail -3 gpurun_out/xs_tests.log
timeout -k 10 150 python -u tools/xsd_stamps.py 64 3 q4 > gpurun_out/xs_stamps_q4.log 2>&1 || { tail -5 gpurun_out/xs_stamps_q4.log; exit 1; }
head -6 gpurun_out/xs_stamps_q4.log
for c in 5 4; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --config $c --steps 1 --warmup 1 > gpurun_out/xs_c$c.json 2> gpurun_out/xs_c$c.err || { tail -5 gpurun_out/xs_c$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/xs_c$c.json')); print('config $c', d['value'], d['roofline']['avg_us'])"
done
