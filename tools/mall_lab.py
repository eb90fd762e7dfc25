#!/usr/bin/env python3
"""Lab: decoder gate/up and down GEMV time vs the number of layers the microbench rotates over
(working set 1..4 x 33.5 / 16.8 MB): where the Infinity Cache stops holding the decoder."""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) == 1:
    for nl in (1, 2, 3, 4):
        env = dict(os.environ, CSM_BENCH_LAYERS=str(nl))
        subprocess.run([sys.executable, __file__, str(nl)], env=env, check=True)
    sys.exit(0)
sys.path[:0] = [os.path.join(ROOT, "csm-mlx_amd"), ROOT]
from bench import build_model  # noqa: E402
from csm_mlx import _lib  # noqa: E402
model = build_model("bf16", 1, device=0)
L = _lib.lib()
for which, name in ((4, "dec gate/up"), (5, "dec down"), (0, "bb gate/up")):
    us, nb = ctypes.c_float(0), ctypes.c_double(0)
    _lib.check(L.csm_bench_gemv(model.engine, which, 1, 400, ctypes.byref(us), ctypes.byref(nb)))
    print(f"layers={sys.argv[1]} {name:12s} {us.value:7.2f} us  {nb.value / us.value / 1e3:7.0f} GB/s", flush=True)
