"""Teacher-forced scoring throughput (csm_mlx.scoring.score_frames, device cross entropy):
csm_1b bf16 synthetic weights, B utterances x 125 forced frames after a 14-row prompt.
Prints frames/s (scored utterance-frames per second)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "csm-mlx_amd"), ROOT]

import numpy as np  # noqa: E402

from csm_mlx.models import CSM, csm_1b  # noqa: E402
from csm_mlx.scoring import score_frames  # noqa: E402
from csm_mlx.tokenizers import tokenize_text_segment  # noqa: E402
from csm_mlx.weights import bf16_bits, synthetic_csm_weights  # noqa: E402

args = csm_1b()
w = {k: bf16_bits(v) for k, v in synthetic_csm_weights(args, 0).items()}
for B in [int(x) for x in (sys.argv[1:] or ["1", "8"])]:
    model = CSM(args, dtype="bf16", max_batch=B)
    model.load_weights(w)
    rng = np.random.default_rng(1)
    p = [tokenize_text_segment([128000] + list(rng.integers(0, 128000, 12)) + [128001], 0, 32) for _ in range(B)]
    fr = [rng.integers(1, 2048, (125, 32)).astype(np.int32) for _ in range(B)]
    score_frames(model, p, [f[:4] for f in fr], logits=False)           # warm-up
    t = time.perf_counter()
    ce = score_frames(model, p, fr, logits=False)
    dt = time.perf_counter() - t
    print(f"B={B}: {B * 125 / dt:.1f} scored frames/s ({dt * 1e3 / 125:.2f} ms per row), mean CE {ce.mean():.3f}",
          flush=True)
    del model
