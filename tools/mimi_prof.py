#!/usr/bin/env python3
"""Codec kernel-trace driver: encode B x S seconds of synthetic PCM twice and decode the codes once
(synthetic mimi_202407 weights), for rocprofv3 --kernel-trace.  usage: python tools/mimi_prof.py [B] [S] [out.npz]
(out.npz: the codes and the decoded PCM, for bit-identity checks between settings)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "csm-mlx_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
from csm_mlx.config import MIMI_CONFIGURATION  # noqa: E402
from csm_mlx.mimi import MimiCodec  # noqa: E402
from csm_mlx.weights import synthetic_mimi_weights  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
S = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
m = MIMI_CONFIGURATION["mimi_202407"]
T = int(24000 * S)
codec = MimiCodec(m, max_batch=B, max_frames=int(12.5 * S) + 8)
codec.load_weights(synthetic_mimi_weights(m))
rng = np.random.default_rng(0)
pcm = (0.1 * rng.standard_normal((B, 1, T))).astype(np.float32)
for it in range(2):
    t0 = time.perf_counter()
    codes = codec.encode(pcm)
    t1 = time.perf_counter()
    print(f"encode {it}: {t1 - t0:.4f} s  codes {codes.shape}", flush=True)
t0 = time.perf_counter()
y = codec.decode(codes)
print(f"decode: {time.perf_counter() - t0:.4f} s  pcm {y.shape}", flush=True)
if len(sys.argv) > 3:
    np.savez(sys.argv[3], codes=codes, pcm=y)
