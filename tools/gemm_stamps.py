#!/usr/bin/env python3
"""Phase clocks of the batched MFMA GEMM (lab build: tools/variant.sh st gemm_kernels.hip -DGEMM_STAMPS,
run with CSM_HIP_LIB=abl/libcsm_hip_st.so): per projection at M rows, the mean over blocks of
[prologue (first stage staged), K loop, publish + ticket, combine + epilogue (last slice)] in us,
and the launch span (first block start -> last block end).
usage: python tools/gemm_stamps.py bf16|q4 M"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "csm-mlx_amd"), ROOT]
import numpy as np  # noqa: E402

import bench  # noqa: E402
from csm_mlx import _lib  # noqa: E402

dtype, M = sys.argv[1], int(sys.argv[2])
model = bench.build_model(dtype, 64)
L = _lib.lib()
L.csm_gemm_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
names = ["gate_up", "down", "qkv", "o"]
for stack in (1, 0):
    for kind in range(4):
        us, nb = ctypes.c_float(0), ctypes.c_double(0)
        st = np.zeros((1024, 6), np.uint64)
        L.csm_bench_gemv(model.engine, stack * 4 + kind, M, 1, ctypes.byref(us), ctypes.byref(nb))
        L.csm_synchronize(model.engine)
        st[:] = 0
        assert L.csm_gemm_stamps(st.ctypes.data, 1024) == 0
        live = st[:, 0] > 0
        s = st[live].astype(np.int64)
        t0 = s[:, 0].min()
        pro = (s[:, 1] - s[:, 0]) / 100.0
        loop = (s[:, 2] - s[:, 1]) / 100.0
        pub = np.where(s[:, 3] > 0, (s[:, 3] - s[:, 2]) / 100.0, 0.0)
        last = s[:, 4] > 0
        comb = ((s[last, 4] - np.where(s[last, 3] > 0, s[last, 3], s[last, 2])) / 100.0)
        span = (max(s[:, 4].max(), s[:, 3].max(), s[:, 2].max()) - t0) / 100.0
        start_skew = (s[:, 0].max() - t0) / 100.0
        print(f"{dtype} M={M} {'dec' if stack else 'bb '} {names[kind]:7s} blocks {live.sum():4d} span {span:6.2f} "
              f"start-skew {start_skew:5.2f} prologue {pro.mean():5.2f} loop {loop.mean():5.2f} "
              f"pub+ticket {pub.mean():5.2f} combine+epi {comb.mean() if len(comb) else 0:5.2f} us", flush=True)
