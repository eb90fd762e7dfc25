"""Sweep GEMV tilings (G, RPT) for every hot projection shape of csm_1b at batch M (GPU only)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "csm-mlx_amd"), ROOT]
from bench import build_model  # noqa: E402
from csm_mlx import _lib  # noqa: E402


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    model = build_model("bf16", max(M, 1))
    L = _lib.lib()
    names = {0: "bb_gate_up", 1: "bb_down", 2: "bb_qkv", 3: "bb_o", 4: "dec_gate_up", 5: "dec_down", 6: "dec_qkv", 7: "dec_o"}
    res = {}
    for which, nm in names.items():
        for G in (64, 128, 256):
            for R in (2, 4):
                L.csm_set_gemv_config(G, R)
                us, nb = ctypes.c_float(0), ctypes.c_double(0)
                rc = L.csm_bench_gemv(model.engine, which, M, 200, ctypes.byref(us), ctypes.byref(nb))
                if rc != 0:
                    continue
                res[f"{nm} G{G} R{R}"] = (round(us.value, 2), round(nb.value / us.value / 1e3, 1))
        L.csm_set_gemv_config(0, 0)
    for k, v in res.items():
        print(f"{k:24s} {v[0]:8.2f} us {v[1]:8.1f} GB/s", flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
