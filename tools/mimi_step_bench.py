#!/usr/bin/env python3
"""Streaming codec microbench: reset + F decode_step calls of B utterances (synthetic mimi_202407 weights,
random codes), alone on the GPU -- the per-frame codec cost stream_generate pays.
usage: python tools/mimi_step_bench.py [B] [F]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "csm-mlx_amd"), ROOT]
import numpy as np  # noqa: E402
from csm_mlx.config import MIMI_CONFIGURATION  # noqa: E402
from csm_mlx.mimi import MimiCodec  # noqa: E402
from csm_mlx.weights import synthetic_mimi_weights  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
F = int(sys.argv[2]) if len(sys.argv) > 2 else 125
m = MIMI_CONFIGURATION["mimi_202407"]
codec = MimiCodec(m, max_batch=B, max_frames=F + 8)
codec.load_weights(synthetic_mimi_weights(m))
codes = np.random.default_rng(0).integers(0, 2048, (F, B, 32, 1)).astype(np.int32)
for it in range(2):
    codec.reset_state(B)
    t0 = time.perf_counter()
    for f in range(F):
        codec.decode_step(codes[f])
    dt = time.perf_counter() - t0
    print(f"B={B} decode_step x{F}: {dt * 1e3:.1f} ms, {dt / F * 1e6:.1f} us per step", flush=True)
