#!/usr/bin/env python3
"""Weight-streaming lab: pure streaming reads vs the production GEMV, cache-hot vs HBM-cold.

usage: python tools/lab.py [stream|gemv|all]
Prints us per launch and the effective GB/s for the decoder / backbone GEMV shapes.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "csm-mlx_amd"), ROOT]

from csm_mlx import _lib  # noqa: E402

HOT = 0.0
COLD = 2.0e9  # >> 256 MiB Infinity Cache


def stream(L):
    for nbytes in (2.1e6, 3.1e6, 16.8e6, 33.5e6, 67.1e6):
        for span, sname in ((HOT, "hot"), (COLD, "cold")):
            row = []
            for loads in (1, 4, 16):
                for nt in (0, 1):
                    us = ctypes.c_float(0)
                    _lib.check(L.csm_lab_stream(0, nbytes, span, loads, nt, 200, ctypes.byref(us)))
                    row.append(f"L{loads}{'nt' if nt else '  '} {us.value:6.2f}us {nbytes / us.value / 1e3:5.0f}GB/s")
            print(f"stream {nbytes / 1e6:5.1f}MB {sname:4s} | " + " | ".join(row), flush=True)


def gemv(L):
    shapes = [("dec gate/up", 16384, 1024, 0), ("dec down", 1024, 8192, 1), ("dec qkv", 1536, 1024, 1),
              ("dec o", 1024, 1024, 1), ("bb gate/up", 16384, 2048, 0), ("bb down", 2048, 8192, 1),
              ("bb qkv", 3072, 2048, 1), ("head", 2056, 1024, 1)]
    for M in (1, 4):
        for name, N, K, kind in shapes:
            row = []
            for xl in (0, 1):
                _lib.check(L.csm_set_option(None, b"gemv_xl", xl))
                for span, sname in ((HOT, "hot"), (COLD, "cold")):
                    us = ctypes.c_float(0)
                    _lib.check(L.csm_lab_gemv(0, N, K, M, span, kind, 1, 200, ctypes.byref(us)))
                    row.append(f"{'xl' if xl else 'rg'}-{sname} {us.value:6.2f}us {N * K * 2 / us.value / 1e3:5.0f}GB/s")
            print(f"gemv M={M} {name:12s} {N * K * 2 / 1e6:5.1f}MB | " + " | ".join(row), flush=True)
    _lib.check(L.csm_set_option(None, b"gemv_xl", 1))


def main():
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    L = _lib.lib()
    if what in ("stream", "all"):
        stream(L)
    if what in ("gemv", "all"):
        gemv(L)


if __name__ == "__main__":
    main()
