#!/usr/bin/env python3
"""Lab: one GPU's batch of B utterances split over E engines, each on its own HIP stream, frames
enqueued asynchronously so the engines' (latency-bound) kernels overlap on the device.  Prints
frames/s for E = 1 and E = E_max at the same total batch, codes-only (no Mimi decode), and checks
that every utterance's codes are identical across the splits.

  python tools/multi_engine.py --batch 32 --engines 1 2 4 --frames 64
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "csm-mlx_amd"), ROOT):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--engines", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import bench
    from csm_mlx.generation import FrameCache
    from csm_mlx.models import CSM, csm_1b
    from csm_mlx.sampling import Sampler
    from csm_mlx.tokenizers import tokenize_text_segment
    from csm_mlx.weights import csm_param_specs, synthetic_csm_weights
    args = csm_1b()
    pool = []  # enough engines for every split: E engines of >= B/E utterances
    for e in sorted(set(a.engines)):
        while len([m for m in pool if m._max_batch >= a.batch // e]) < e:
            pool.append(CSM(args, dtype=a.dtype, max_batch=a.batch // e))
    names = list(csm_param_specs(args))
    for i in range(0, len(names), 16):
        w = list(synthetic_csm_weights(args, 0, names[i:i + 16]).items())
        for m in pool:
            m.load_weights(w, strict=False)
    for m in pool:
        m.load_weights([], strict=True)
    prompts = [tokenize_text_segment(bench.prompt_ids(g), 0, 32) for g in range(a.batch)]
    ref = None
    for E in a.engines:
        per = a.batch // E
        ms = [m for m in pool if m._max_batch >= per][:E]
        best = None
        for _ in range(a.reps):
            caches = []
            for k, m in enumerate(ms):
                c = FrameCache(m, per, Sampler(0.0, 0), [1234 + k * per + b for b in range(per)])
                c.prefill_batch([(b, *prompts[k * per + b]) for b in range(per)])
                caches.append(c)
            for c in caches:
                c.run(1)                     # graphs captured outside the timed loop
            t0 = time.perf_counter()
            left = a.frames - 1
            while left > 0:
                n = min(16, left)
                for c in caches:
                    c.run(n, sync=False)
                left -= n
            for c in caches:
                c.done()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        codes = np.concatenate([c.codes()[0][:, :per] for c in caches], 1)
        if ref is None:
            ref = codes
        same = np.array_equal(codes, ref)
        print(f"E={E} per-engine B={per}: {(a.frames - 1) * a.batch / best:9.1f} frames/s "
              f"({best / (a.frames - 1) * 1e3:.3f} ms per frame step)  codes identical to E={a.engines[0]}: {same}",
              flush=True)


if __name__ == "__main__":
    main()
