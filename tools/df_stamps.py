#!/usr/bin/env python3
"""Per-hand-off timing of the persistent frame decoder (dec_frame.hip) from its s_memrealtime
stamps (100 MHz): csm_1b bf16 B=1, a few frames, then the last frame's stamps.
usage: python tools/df_stamps.py [frames]  -> per hand-off kind: mean gap (us) on WG 0 and the
spread of completion times over the 256 workgroups."""
import collections
import ctypes
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

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 4
model = bench.build_model("bf16", 1)
L = _lib.lib()
_lib.check(L.csm_set_option(model.engine, b"dec_frame_stamps", 1))
cache = FrameCache(model, 1, Sampler(0.0, 0), [0])
cache.prefill(0, *tokenize_text_segment(bench.prompt_ids(0), 0, 32))
for _ in range(frames):
    cache.run(1)
st = np.zeros((256, 1024), np.uint64)
_lib.check(L.csm_debug_read(model.engine, b"dec_frame_stamps", _lib.ptr(st), st.nbytes, None))
t0 = st[:, 1022].astype(np.int64)
end = st[:, 1023].astype(np.int64)
n = int((st[0, :512] > 0).sum())
rel = (st[:, :n].astype(np.int64) - t0.min()) / 100.0        # us since the first WG started
print(f"hand-offs {n}; kernel span {(end.max() - t0.min()) / 100:.1f} us; start skew {(t0.max() - t0.min()) / 100:.2f} us")
# kinds per step: L0 (E3, E4, E5), L1-3 (E1, E3, E4, E5) x3, E6; step 1 has E1 at L0; frame start A0
kinds = ["A0"]
for step in range(1, 32):
    for l in range(4):
        if not (l == 0 and step > 1):
            kinds.append(f"E1.L{l}")
        kinds += [f"E3.L{l}", f"E4.L{l}", f"E5.L{l}"]
    kinds.append("E6")
kinds = kinds[:n]
w0 = rel[0]
gaps = collections.defaultdict(list)
spread = collections.defaultdict(list)
prev = 0.0
for e, k in enumerate(kinds):
    gaps[k.split(".")[0]].append(w0[e] - prev)
    spread[k.split(".")[0]].append(rel[:, e].max() - rel[:, e].min())
    prev = w0[e]
for k in sorted(gaps):
    print(f"{k}: n={len(gaps[k])} mean gap {np.mean(gaps[k]):.2f} us (the phase before it + the wait), "
          f"WG completion spread {np.mean(spread[k]):.2f} us")
step_t = [w0[kinds.index("E6", i)] for i in range(len(kinds)) if kinds[i] == "E6"]
print("per step (us):", np.round(np.diff([0.0] + step_t), 1).tolist()[:8], "...")

# phase marks (WG 0 and the mean over WGs): per layer [attn start, attn end, o published, mlp published]
mk = (st[:, 512:1008].astype(np.int64) - t0.min()) / 100.0
nm = 4 * 4 * 31
mk = mk[:, :nm].reshape(256, 31, 4, 4)
ho = {}
e = 1
for step in range(31):
    for l in range(4):
        if not (l == 0 and step > 0):
            ho[(step, l, "E1")] = e; e += 1
        ho[(step, l, "E3")] = e; e += 1
        ho[(step, l, "E4")] = e; e += 1
        ho[(step, l, "E5")] = e; e += 1
    e += 1
seg = collections.defaultdict(list)
for step in range(1, 31):
    for l in range(4):
        a0, a1, oc, mp = [mk[:, step, l, i] for i in range(4)]
        e3 = rel[:, ho[(step, l, "E3")]]
        e4 = rel[:, ho[(step, l, "E4")]]
        e5 = rel[:, ho[(step, l, "E5")]]
        # previous hand-off completion: E5 of layer l-1, or E6 of the previous step for layer 0
        prev = rel[:, ho[(step, l - 1, "E5")]] if l else rel[:, ho[(step - 1, 3, "E5")] + 1]
        tag = "L0" if l == 0 else "L1-3"
        if l:
            e1 = rel[:, ho[(step, l, "E1")]]
            seg[f"{tag} rms+qkv+publish+E1 wait"].append(np.mean(e1 - prev))
            seg[f"{tag} kv_store -> attn start"].append(np.mean(a0 - e1))
        else:
            seg[f"{tag} table row+kv_store -> attn start"].append(np.mean(a0 - prev))
        seg[f"{tag} attention"].append(np.mean(a1 - a0))
        seg[f"{tag} o_proj+publish"].append(np.mean(oc - a1))
        seg[f"{tag} E3 wait"].append(np.mean(e3 - oc))
        seg[f"{tag} rms+mlp compute+publish"].append(np.mean(mp - e3))
        seg[f"{tag} E4 wait"].append(np.mean(e4 - mp))
        seg[f"{tag} reduce+publish+E5 wait"].append(np.mean(e5 - e4))
    e6 = rel[:, ho[(step, 3, "E5")] + 1]
    seg["head: rms+head+publish+E6 wait"].append(np.mean(e6 - rel[:, ho[(step, 3, "E5")]]))
for k, v in seg.items():
    print(f"  {k}: {np.mean(v):.2f} us (mean over WGs, steps 2-31)")
