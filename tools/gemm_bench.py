#!/usr/bin/env python3
"""Per-projection microbench of the batched MFMA GEMM (csm_bench_gemv: one launch per layer in turn,
HIP events on the engine stream) for csm_1b at a few row counts.
usage: python tools/gemm_bench.py bf16|q4 [M ...]   -> one line per (stack, projection, M)
GB_XS=1: also the streaming matrix-core GEMM over pre-split activations (gemm_xs, which | 8) beside it."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "csm-mlx_amd"), ROOT]
import bench  # noqa: E402
from csm_mlx import _lib  # noqa: E402

dtype = sys.argv[1] if len(sys.argv) > 1 else "bf16"
Ms = [int(a) for a in sys.argv[2:]] or [32, 64]
iters = int(os.environ.get("GB_ITERS", "200"))
model = bench.build_model(dtype, max(Ms) // 2 if max(Ms) > 64 else 64)
L = _lib.lib()
names = ["gate_up", "down", "qkv", "o"]
tot = {}
for M in Ms:
    for stack in (1, 0):
        for kind in range(4):
            for xs in ((0, 8, 24) if os.environ.get("GB_XS") == "1" and M <= 64 else (0,)):
                us, nb = ctypes.c_float(0), ctypes.c_double(0)
                _lib.check(L.csm_bench_gemv(model.engine, stack * 4 + kind + xs, M, iters, ctypes.byref(us),
                                            ctypes.byref(nb)))
                print(f"{dtype} M={M:3d} {'dec' if stack else 'bb '} {names[kind]:7s} { {0: 'wide', 8: 'xs  ', 24: 'xs-p'}[xs] } "
                      f"{us.value:8.2f} us {nb.value / 1e6:8.2f} MB {nb.value / us.value / 1e3:7.0f} GB/s", flush=True)
