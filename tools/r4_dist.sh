#!/bin/bash
# Round 4: the N-rank bench path on the GPU box -- dist GPU tests (self-launch over gloo, RCCL at
# world 1), the default bench line, and the bench line launched by torchrun with 1 rank over RCCL.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r4_dist_tests.log 2>&1 || { tail -40 gpurun_out/r4_dist_tests.log; exit 1; }
tail -3 gpurun_out/r4_dist_tests.log
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/r4_start_bench.json 2> gpurun_out/r4_start_bench.err || { tail -20 gpurun_out/r4_start_bench.err; exit 1; }
cat gpurun_out/r4_start_bench.json
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r4_nccl1_bench.json 2> gpurun_out/r4_nccl1_bench.err || { tail -20 gpurun_out/r4_nccl1_bench.err; exit 1; }
cat gpurun_out/r4_nccl1_bench.json
