#!/usr/bin/env python3
"""Per-role timing of the persistent batched decoder step (dec_step_xs.hip) from its s_memrealtime marks
(100 MHz): csm_1b bf16, B utterances (default 32), a few frames; the marks hold the last launch (the last
codebook step of the last frame).
usage: python tools/xsd_stamps.py [B] [frames] [bf16|q4]  -> per layer: when each role's wait ended / it published
(max over the workgroups of that role, us since the first workgroup started), and the kernel span."""
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

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dtype = sys.argv[3] if len(sys.argv) > 3 else "bf16"
model = bench.build_model(dtype, B)
L = _lib.lib()
_lib.check(L.csm_set_option(model.engine, b"dec_xsd_stamps", 1))
cache = FrameCache(model, B, Sampler(0.0, 0), list(range(B)))
for b in range(B):
    cache.prefill(b, *tokenize_text_segment(bench.prompt_ids(b), 0, 32))
for _ in range(frames):
    cache.run(1)
NS = 64
st = np.zeros((256, NS), np.uint64)
_lib.check(L.csm_debug_read(model.engine, b"dec_xsd_stamps", _lib.ptr(st), st.nbytes, None))
s = st.astype(np.int64)
t0 = s[:, 0][s[:, 0] > 0].min()
rel = np.where(s > 0, (s - t0) / 100.0, np.nan)
w = np.arange(256)
isq, iso = w < 48, (w >= 48) & (w < 80)
MR = 64 if dtype == "q4" else 32
print(f"B={B} {dtype}: kernel span {np.nanmax(rel[:, NS - 1]):.1f} us (start skew {np.nanmax(rel[:, 0]):.2f} us)")
names = {1: ("Q waited", isq), 2: ("Q published", isq), 3: ("A K/V staged", None), 4: ("A arrived", None),
         5: ("O waited", iso), 6: ("O published", iso), 7: ("G waited", None), 8: ("G published", None),
         9: ("D waited", None), 10: ("D ticket", None), 11: ("combine published", None)}
prev_end = 0.0
for l in range(4):
    row = [f"L{l} start {np.nanmin(rel[:, 12 * l]):6.1f}"]
    for k, (nm, sel) in names.items():
        col = rel[:, 12 * l + k] if sel is None else rel[sel, 12 * l + k]
        if np.all(np.isnan(col)):
            continue
        row.append(f"{nm} {np.nanmedian(col):6.1f}/{np.nanmax(col):6.1f}")
    print(" | ".join(row))
print("(median/max over the role's workgroups, us since the first workgroup started)")
# layer 1 sub-phases, relative to the role's own wait end (median over its workgroups)
sub = {0: ("Q mma+reduce", isq, 13), 1: ("Q stores issued", isq, 13), 2: ("G mma issued", None, 19),
       3: ("G reduce", None, 19), 4: ("G stores issued", None, 19), 5: ("D mma+reduce", None, 21), 6: ("O mma+reduce", iso, 17),
       7: ("A entered (after stage_kv)", None, 12), 8: ("A polled (wave 0)", None, 12), 9: ("A rows loaded (wave 0)", None, 12)}
for k, (nm, sel, base) in sub.items():
    col = rel[:, 48 + k] - rel[:, base]
    col = col if sel is None else col[sel]
    print(f"  L1 {nm}: {np.nanmedian(col):.2f} us after {'the layer start' if base == 12 else 'its wait'} (max {np.nanmax(col):.2f})")
for nm, a, b_, sel in (("Q publish (drain+barrier)", 49, 14, isq), ("G publish (drain+barrier)", 52, 20, None)):
    col = rel[:, b_] - rel[:, a]
    col = col if sel is None else col[sel]
    print(f"  L1 {nm}: {np.nanmedian(col):.2f} us (max {np.nanmax(col):.2f})")
