#!/usr/bin/env python3
"""Bit-identity lab check of the codec GEMM tiles: encode + decode + streaming decode_step of a fixed input
with the current CSM_MIMI_MFMA setting, written to an npz; run once per setting and compare the files.
usage: python tools/mimi_mfma_check.py out.npz   |   python tools/mimi_mfma_check.py --cmp a.npz b.npz"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "csm-mlx_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402

if sys.argv[1] == "--cmp":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    for k in a.files:
        same = a[k].shape == b[k].shape and np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8))
        print(k, a[k].shape, "bit-identical" if same else f"DIFFER max {np.abs(a[k].astype(np.float64) - b[k]).max():.3g}")
    sys.exit(0)
from csm_mlx.config import MIMI_CONFIGURATION  # noqa: E402
from csm_mlx.mimi import MimiCodec  # noqa: E402
from csm_mlx.weights import synthetic_mimi_weights  # noqa: E402
from test_mimi_gpu import _pcm  # noqa: E402

m = MIMI_CONFIGURATION["mimi_202407"]
codec = MimiCodec(m, max_batch=4, max_frames=200)
codec.load_weights(synthetic_mimi_weights(m))
pcm = np.stack([_pcm(24000 * 3 + 480, s) for s in range(4)])
codes = codec.encode(pcm[:, None, :])
y = codec.decode(codes)
codec.reset_state(4)
steps = [codec.decode_step(codes[:, :, t:t + 2]) for t in range(0, 12, 2)]  # streaming: 2 frames per step
out = {"codes": codes, "pcm": y, "pcm_stream": np.concatenate(steps, axis=-1)}
np.savez(sys.argv[1], **out)
print("wrote", sys.argv[1], {k: v.shape for k, v in out.items()})
