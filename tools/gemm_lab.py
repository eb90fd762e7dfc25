#!/usr/bin/env python3
"""Time every csm_1b projection shape (csm_bench_gemv: the production launch, one layer after
another as in a frame) at the given row counts.  usage: python tools/gemm_lab.py [M ...]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "csm-mlx_amd"), ROOT]

from bench import build_model  # noqa: E402
from csm_mlx import _lib  # noqa: E402

Ms = [int(a) for a in sys.argv[1:]] or [32]
model = build_model(os.environ.get("LAB_DTYPE", "bf16"), max(Ms), device=0)
L = _lib.lib()
names = ["gate/up", "down", "qkv", "o"]
tag = os.environ.get("CSM_GEMM", "wk")
for M in Ms:
    for stack in (0, 1):
        for kind in range(4):
            us, nb = ctypes.c_float(0), ctypes.c_double(0)
            _lib.check(L.csm_bench_gemv(model.engine, stack * 4 + kind, M, 200, ctypes.byref(us), ctypes.byref(nb)))
            print(f"{tag:4s} M={M:3d} {'bb ' if stack == 0 else 'dec'} {names[kind]:8s} {us.value:8.2f} us "
                  f"{nb.value / us.value / 1e3:7.0f} GB/s", flush=True)
