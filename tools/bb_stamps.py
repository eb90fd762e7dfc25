#!/usr/bin/env python3
"""Per-hand-off timing of the persistent backbone step (bb_step.hip) from its s_memrealtime stamps
(100 MHz): csm_1b bf16 B=1, a few frames, then the last step's stamps.
usage: python tools/bb_stamps.py [frames] -> per hand-off kind (E1 attention WGs only, E2..E5) the
mean gap on an attention workgroup (0) and a non-attention one (100), and the spread over WGs."""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "csm-mlx_amd"), ROOT]
import numpy as np  # noqa: E402

import bench  # noqa: E402
from csm_mlx import _lib  # noqa: E402
from csm_mlx.generation import FrameCache  # noqa: E402
from csm_mlx.sampling import Sampler  # noqa: E402
from csm_mlx.tokenizers import tokenize_text_segment  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 4
model = bench.build_model("bf16", 1)
L = _lib.lib()
_lib.check(L.csm_set_option(model.engine, b"bb_step_stamps", 1))
cache = FrameCache(model, 1, Sampler(0.0, 0), [0])
cache.prefill(0, *tokenize_text_segment(bench.prompt_ids(0), 0, 32))
for _ in range(frames):
    cache.run(1)
st = np.zeros((256, 128), np.uint64)
_lib.check(L.csm_debug_read(model.engine, b"bb_step_stamps", _lib.ptr(st), st.nbytes, None))
t0 = st[:, 0].astype(np.int64).min()
rel = (st.astype(np.int64) - t0) / 100.0
print(f"kernel span {rel[:, 127].max():.1f} us; start skew {(st[:, 0].astype(np.int64).max() - t0) / 100:.2f} us")
kinds = ["E1", "E2", "E3", "E4", "E5"]
for wg in (0, 100):
    gaps = collections.defaultdict(list)
    prev = 0.0
    for l in range(16):
        for k in range(5):
            slot = 1 + 5 * l + k
            v = rel[wg, slot]
            if v <= 0 or (k == 0 and wg >= 32):
                continue
            gaps[kinds[k]].append(v - prev)
            prev = v
    print(f"WG {wg}: " + ", ".join(f"{k} {np.mean(v):.2f}" for k, v in gaps.items()) + " us (phase before + wait)")
for k in range(1, 5):
    slots = [1 + 5 * l + k for l in range(16)]
    spread = [rel[:, s].max() - rel[:, s].min() for s in slots]
    print(f"{kinds[k]} completion spread over WGs {np.mean(spread):.2f} us")
per_layer = np.diff([rel[100, 1 + 5 * l + 4] for l in range(16)])
print("per layer (us, WG 100):", np.round(per_layer, 1).tolist())
