# backbone-step check: its tests, then bench with it on / off (gpurun_out/)
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_bb_step_gpu.py tests/test_dec_frame_gpu.py tests/test_long_gpu.py > gpurun_out/t_bb.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|assert" gpurun_out/t_bb.log | head -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_bb1.json 2> gpurun_out/b_bb1.err || exit 1
CSM_BB_STEP=0 timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_bb0.json 2> gpurun_out/b_bb0.err || exit 1
python3 -c "
import json
for v in ('bb1','bb0'):
    d=json.load(open('gpurun_out/b_%s.json'%v)); print(v, d['value'], d['ms_per_step'], d['roofline']['avg_us'])"
