# Mimi: transformer attention on the matrix-core tiles + ELU once per element in the encoder:
# parity tests, then encode / decode timing A/B (192 x 5 s = config 5's context encode), bit-identity of ELU_PRE
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_mimi_gpu.py "tests/test_batched_long_gpu.py::test_config5_q4_b64_greedy_125_frames" "tests/test_batched_long_gpu.py::test_config3_stream_b32_sampled_64_frames" > gpurun_out/ma_tests.log 2>&1 || { tail -30 gpurun_out/ma_tests.log; exit 1; }
tail -3 gpurun_out/ma_tests.log
for v in "1 1"; do
  set -- $v
  CSM_MIMI_ATTN_TILES=$1 CSM_MIMI_ELU_PRE=$2 timeout -k 10 200 python -u tools/mimi_prof.py 192 5 /tmp/ma_$1$2.npz > gpurun_out/ma_prof_$1$2.txt 2>&1 || { tail -5 gpurun_out/ma_prof_$1$2.txt; exit 1; }
  echo "tiles=$1 elu_pre=$2"; cat gpurun_out/ma_prof_$1$2.txt
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 5 --steps 1 --warmup 1 --phases > gpurun_out/ma_c5.json 2> gpurun_out/ma_c5.err || { tail -5 gpurun_out/ma_c5.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ma_c5.json')); print('config 5', d['value'], d.get('phases_s_per_step'))"
bash tools/r6_mimi_prof.sh > gpurun_out/ma_kprof.txt 2>&1 || { tail -5 gpurun_out/ma_kprof.txt; exit 1; }
cat gpurun_out/ma_kprof.txt
