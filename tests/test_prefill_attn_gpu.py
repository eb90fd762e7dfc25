"""Prompt-prefill attention on the fp32 matrix cores (attn_prefill_kernel, csm_kernels.hip: one block
per <= 64-row run of one utterance's prompt and kv head, keys in 64-key chunks, S^T = K Q^T and
O^T = V^T P^T on v_mfma_f32_32x32x2f32) against attn_block's per-row kernel on the same engine
(csm_set_option "attn_prefill" 0) and against the oracle (generation.py:108-125 -> models.py
LlamaModel over the prompt rows, attention.py causal SDPA).

Both kernels sum the same fp32 products in different orders, so the bar is h_last within 1e-5 of
max|h| and greedy codes identical (and bit-exact against the oracle).  Lengths cover a 1-row prompt,
runs just under / at / over one 64-row tile and one 64-key chunk, and a 248-row (config 5) prompt;
"split" prefills every prompt in two calls, so the second call's tiles start past position 0 and
attend to keys the first call cached.
"""
import numpy as np
import pytest

from helpers import csm_weights, first_divergence, oracle_batch, oracle_for, tiny_prompt_ids

pytestmark = pytest.mark.gpu

LENS = (1, 15, 16, 17, 63, 64, 65, 130, 248)
FRAMES = 3


def _prompts(K):
    from csm_mlx.tokenizers import tokenize_text_segment
    out = []
    for i, n in enumerate(LENS):
        ids = [998] if n == 1 else tiny_prompt_ids(700 + i, n - 2)
        out.append(tokenize_text_segment(ids, 0, K))
    return out


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_prefill_attention_tiles_vs_per_row(dtype):
    from csm_mlx import _lib
    from csm_mlx.generation import FrameCache
    from csm_mlx.models import CSM
    from csm_mlx.sampling import Sampler
    args, w = csm_weights("tiny")
    K = args.n_audio_codebooks
    B = len(LENS)
    model = CSM(args, dtype=dtype, max_batch=B)
    model.load_weights(w)
    prompts = _prompts(K)
    L = _lib.lib()
    D = model.backbone.args.hidden_size

    def run(tiles, how):
        _lib.check(L.csm_set_option(model.engine, b"attn_prefill", 1 if tiles else 0))
        cache = FrameCache(model, B, Sampler(0.0, 0), [0] * B)
        if how == "batch":
            cache.prefill_batch([(b, t, m) for b, (t, m) in enumerate(prompts)])
        elif how == "single":
            for b, (t, m) in enumerate(prompts):
                cache.prefill(b, t, m)
        else:  # split: two calls per prompt, the second appending after the first's rows
            for b, (t, m) in enumerate(prompts):
                k = max(1, t.shape[0] // 2)
                cache.prefill(b, t[:k], m[:k])
                if k < t.shape[0]:
                    cache.prefill(b, t[k:], m[k:])
        h = cache.debug("h_last", (B, D))
        cache.run(FRAMES)
        hist, n, _ = cache.codes()
        return h, hist[:FRAMES], n

    ref_h, ref_c, ref_n = run(False, "batch")
    runs = {how: run(True, how) for how in ("batch", "single", "split")}
    _lib.check(L.csm_set_option(model.engine, b"attn_prefill", 1))
    del model
    scale = np.abs(ref_h).max(axis=1)
    for how, (h, c, n) in runs.items():
        err = (np.abs(h - ref_h).max(axis=1) / scale).max()
        assert err <= 1e-5, f"{how}: h_last {err:.2e} x max|h| from the per-row attention"
        assert np.array_equal(c, ref_c) and np.array_equal(n, ref_n), f"{how}: codes differ from the per-row attention"
    ref = oracle_batch(oracle_for(args, w, bf16=(dtype == "bf16")), prompts, FRAMES)
    for b in range(B):
        assert ref_n[b] == FRAMES and first_divergence(runs["batch"][1][:, b], ref[b][0]) is None, f"utterance {b} vs oracle"


def test_prefill_attention_tiles_csm_1b_gqa4():
    """csm_1b's layout (32 query heads over 8 kv heads, G = 4, hd 64: all four waves of attn_prefill_kernel
    busy, which the tiny backbone's G = 2 never reaches) with single-prompt prefills long enough for the tile
    path (70 and 130 rows: 2 and 3 tiles, the last partial): tiles vs the per-row attention on the same engine
    (h_last within 1e-5 of max|h|, codes identical) and codes bit-exact against the oracle."""
    from csm_mlx import _lib
    from csm_mlx.generation import FrameCache
    from csm_mlx.models import CSM
    from csm_mlx.sampling import Sampler
    from csm_mlx.tokenizers import tokenize_text_segment
    from helpers import prompt_ids
    args, w = csm_weights("1b")
    K = args.n_audio_codebooks
    prompts = [tokenize_text_segment(prompt_ids(900 + i, n - 2), 0, K) for i, n in enumerate((70, 130))]
    B = len(prompts)
    model = CSM(args, dtype="bf16", max_batch=B)
    model.load_weights(w)
    L = _lib.lib()
    D = model.backbone.args.hidden_size

    def run(tiles):
        _lib.check(L.csm_set_option(model.engine, b"attn_prefill", 1 if tiles else 0))
        cache = FrameCache(model, B, Sampler(0.0, 0), [0] * B)
        for b, (t, m) in enumerate(prompts):
            cache.prefill(b, t, m)
        h = cache.debug("h_last", (B, D))
        cache.run(2)
        hist, n, _ = cache.codes()
        return h, hist[:2], n

    ref_h, ref_c, ref_n = run(False)
    h, c, n = run(True)
    del model
    err = (np.abs(h - ref_h).max(axis=1) / np.abs(ref_h).max(axis=1)).max()
    assert err <= 1e-5, f"h_last {err:.2e} x max|h| from the per-row attention"
    assert np.array_equal(c, ref_c) and np.array_equal(n, ref_n), "codes differ from the per-row attention"
    ref = oracle_batch(oracle_for(args, w, bf16=True), prompts, 2)
    for b in range(B):
        assert first_divergence(c[:, b], ref[b][0]) is None, f"utterance {b} vs oracle"
