#!/usr/bin/env python3
"""Lab: B = 1 real-use rates -- stream_generate (per-frame Mimi decode_step) and sampled generate()
(temperature 0.8, top-k 50) on csm_1b, 10 s, after one warm-up call."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "csm-mlx_amd"), ROOT]
from bench import build_codec, build_model, prompt_ids  # noqa: E402
from csm_mlx.generation import generate, stream_generate  # noqa: E402
from csm_mlx.sampling import make_sampler  # noqa: E402

model = build_model("bf16", 1, device=0)
build_codec(device=0)
ids = prompt_ids(0)
smp = make_sampler(0.8, top_k=50)
print("sampler", smp, flush=True)
for rep in range(3):
    t0 = time.perf_counter()
    n = sum(1 for _ in stream_generate(model, ids, 0, [], max_audio_length_ms=10_000, sampler=smp))
    dt = time.perf_counter() - t0
    print(f"stream_generate sampled: {n} frames in {dt * 1e3:.1f} ms -> {n / dt:.1f} frames/s", flush=True)
for rep in range(4):
    smp = make_sampler(0.8, top_k=50 if rep < 2 else 0)
    t0 = time.perf_counter()
    a = generate(model, ids, 0, [], max_audio_length_ms=10_000, sampler=smp)
    dt = time.perf_counter() - t0
    print(f"generate sampled top_k={smp.top_k}: {a.shape[0] / 1920:.0f} frames in {dt * 1e3:.1f} ms -> {a.shape[0] / 1920 / dt:.1f} frames/s",
          flush=True)
