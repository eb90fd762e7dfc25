"""Launch-floor probe: per-kernel time of dependent near-empty kernels (graph vs eager)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "csm-mlx_amd"), ROOT]
from csm_mlx import _lib  # noqa: E402
from csm_mlx.models import CSM, csm_tiny  # noqa: E402

m = CSM(csm_tiny(), dtype="float32")
L = _lib.lib()
for graph in (1, 0):
    for blocks in (1, 256, 2048):
        us = ctypes.c_float(0)
        _lib.check(L.csm_bench_floor(m.engine, 200, blocks, graph, ctypes.byref(us)))
        print(f"graph={graph} blocks={blocks:5d}: {us.value:.2f} us/kernel", flush=True)
