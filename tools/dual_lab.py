#!/usr/bin/env python3
"""Lab: R engine replicas on one GPU, each generating B/R utterances in its own thread (own HIP
stream), codes only, vs one engine with all B.  usage: python tools/dual_lab.py B R [frames]"""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "csm-mlx_amd"), ROOT]

from bench import build_model, prompt_ids  # noqa: E402
from csm_mlx.generation import generate_codes_batch  # noqa: E402
from csm_mlx.sampling import Sampler  # noqa: E402
from csm_mlx.tokenizers import tokenize_text_segment  # noqa: E402

B, R = int(sys.argv[1]), int(sys.argv[2])
F = int(sys.argv[3]) if len(sys.argv) > 3 else 125
per = B // R
models = [build_model("bf16", per, device=0) for _ in range(R)]
prompts = [[tokenize_text_segment(prompt_ids(g), 0, 32) for g in range(r * per, (r + 1) * per)] for r in range(R)]


def run(r, out):
    h, n, _ = generate_codes_batch(models[r], prompts[r], F, sampler=Sampler(0.0, 0))
    out[r] = int(n.sum())


for rep in range(3):
    out = [0] * R
    ths = [threading.Thread(target=run, args=(r, out)) for r in range(R)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    dt = time.perf_counter() - t0
    print(f"B={B} R={R} rep {rep}: {sum(out)} frames in {dt * 1e3:.1f} ms -> {sum(out) / dt:.1f} frames/s", flush=True)
