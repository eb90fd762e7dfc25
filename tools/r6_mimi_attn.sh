# Mimi: transformer attention on the matrix-core tiles + ELU once per element in the encoder:
# parity tests, then encode / decode timing A/B (192 x 5 s = config 5's context encode), bit-identity of ELU_PRE
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_mimi_gpu.py tests/test_prefill_attn_gpu.py "tests/test_batched_long_gpu.py::test_config5_q4_b64_greedy_125_frames" > gpurun_out/ma_tests.log 2>&1 || { tail -30 gpurun_out/ma_tests.log; exit 1; }
tail -3 gpurun_out/ma_tests.log
for v in "0 0" "1 0" "1 1"; do
  set -- $v
  CSM_MIMI_ATTN_TILES=$1 CSM_MIMI_ELU_PRE=$2 timeout -k 10 200 python -u tools/mimi_prof.py 192 5 /tmp/ma_$1$2.npz > gpurun_out/ma_prof_$1$2.txt 2>&1 || { tail -5 gpurun_out/ma_prof_$1$2.txt; exit 1; }
  echo "tiles=$1 elu_pre=$2"; cat gpurun_out/ma_prof_$1$2.txt
done
python3 - <<'PY'
import numpy as np
a, b, c = (np.load(f"/tmp/ma_{k}.npz") for k in ("00", "10", "11"))
print("ELU_PRE bit-identical codes", np.array_equal(b["codes"], c["codes"]), "pcm", np.array_equal(b["pcm"], c["pcm"]))
print("tiles vs per-row: codes differing", int((a["codes"] != b["codes"]).sum()), "of", a["codes"].size,
      "pcm max abs diff", float(np.abs(a["pcm"] - b["pcm"]).max()))
PY
timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 5 --steps 1 --warmup 1 --phases > gpurun_out/ma_c5.json 2> gpurun_out/ma_c5.err || { tail -5 gpurun_out/ma_c5.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ma_c5.json')); print('config 5', d['value'], d.get('phases_s_per_step'))"
