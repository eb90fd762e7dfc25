#!/usr/bin/env python3
"""Stress the fused decoder attention + o_proj launch (dec_attn_oproj_kernel).

The fused launch must give codes bitwise equal to the two-launch path (same attention arithmetic,
same GEMV K-slicing and reduction order).  Runs csm_1b greedy generation R times per mode and
reports runs whose codes differ from the two-launch reference.

usage: python tools/handoff_stress.py [--reps 5] [--frames 125] [--dtype bf16]
"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "csm-mlx_amd"), ROOT]

import numpy as np  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--frames", type=int, default=125)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--per-frame", action="store_true", help="run(1) per frame with debug reads (test pattern)")
    ap.add_argument("--torch-first", action="store_true", help="import torch first (its HIP runtime wins)")
    a = ap.parse_args()
    if a.torch_first:
        import torch  # noqa: F401
    from csm_mlx import _lib
    from csm_mlx.generation import generate_batch
    from csm_mlx.tokenizers import tokenize_text_segment
    L = _lib.lib()
    model = bench.build_model(a.dtype, a.batch)
    prompts = [tokenize_text_segment(bench.prompt_ids(g), 0, 32) for g in range(a.batch)]

    def run():
        if a.per_frame:
            from csm_mlx.generation import FrameCache
            from csm_mlx.sampling import Sampler
            cache = FrameCache(model, a.batch, Sampler(0.0, 0), list(range(a.batch)))
            for b, (t, m) in enumerate(prompts):
                cache.prefill(b, t, m)
            for _ in range(a.frames):
                cache.run(1)
                cache.debug("c0_logits", (a.batch, 2056))
            hist, n, _ = cache.codes()
            return hist.transpose(1, 0, 2)
        return np.stack([c for c in generate_batch(model, prompts, a.frames * 80, temperature=0.0, decode=False)])

    def opt(k, v):
        _lib.check(L.csm_set_option(model.engine, k.encode(), v))

    opt("fuse_attn", 0)
    ref = run()
    print(f"reference (two launches): codes {ref.shape}", flush=True)
    for name in ("fused",):
        opt("fuse_attn", 1)
        bad = 0
        t0 = time.time()
        for r in range(a.reps):
            got = run()
            if got.shape != ref.shape or not np.array_equal(got, ref):
                bad += 1
                if got.shape == ref.shape:
                    d = np.argwhere(got != ref)[0]
                    print(f"  {name} rep {r}: first diff at {tuple(d)}", flush=True)
                else:
                    print(f"  {name} rep {r}: shape {got.shape}", flush=True)
        print(f"{name}: {bad}/{a.reps} runs differ ({time.time() - t0:.1f} s)", flush=True)


if __name__ == "__main__":
    main()
