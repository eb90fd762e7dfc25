#!/usr/bin/env python3
"""First-call latency after weight load: csm_begin (folded-table builds) + prefill + one frame."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "csm-mlx_amd"), ROOT]
from bench import build_model, prompt_ids  # noqa: E402
from csm_mlx.generation import FrameCache  # noqa: E402
from csm_mlx.sampling import Sampler  # noqa: E402
from csm_mlx.tokenizers import tokenize_text_segment  # noqa: E402

m = build_model(os.environ.get("LAB_DTYPE", "bf16"), 1, device=0)
for rep in range(2):
    t = time.time()
    c = FrameCache(m, 1, Sampler(0.0, 0), [0])
    c.prefill(0, *tokenize_text_segment(prompt_ids(1), 0, 32))
    c.run(1)
    c.codes()
    print(f"call {rep}: first frame incl. table builds {(time.time() - t) * 1e3:.1f} ms", flush=True)
