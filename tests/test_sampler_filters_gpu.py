"""mlx_lm make_sampler's filters beyond top-k on the GPU sampler (sample_filtered_kernel): top_p,
min_p and min_tokens_to_keep, alone and chained with top_k (README.md:49 "temp, top_p, min_p,
min_tokens_to_keep, top_k"; cli/generate.py:168-174).  Sampled codes bit-exact against the oracle's
restatement of the filter chain (oracle/csm_oracle.py filter_keep) and of the counter-based RNG, at
csm_1b B = 1 and B = 8 and on the tiny model."""
import numpy as np
import pytest

from helpers import csm_weights, first_divergence, oracle_batch, oracle_for, prompt_ids, tiny_prompt_ids

pytestmark = pytest.mark.gpu

FILTERS = [dict(top_p=0.9), dict(min_p=0.05, min_tokens_to_keep=2), dict(top_k=200, top_p=0.8, min_p=0.02),
           dict(top_p=0.3, min_tokens_to_keep=5)]


def _run(model, prompts, frames, smp, seeds):
    from csm_mlx.generation import generate_codes_batch
    hist, n, _ = generate_codes_batch(model, prompts, frames, sampler=smp, seeds=seeds)
    return [hist[: n[b], b].copy() for b in range(len(prompts))]


def _check(args, w, model, prompts, frames, flt, bf16):
    from csm_mlx.sampling import make_sampler
    smp = make_sampler(0.8, **flt)
    seeds = [900 + b for b in range(len(prompts))]
    got = _run(model, prompts, frames, smp, seeds)
    ref = oracle_batch(oracle_for(args, w, bf16=bf16), prompts, frames, temperature=0.8, top_k=smp.top_k,
                       seeds=seeds, top_p=smp.top_p, min_p=smp.min_p, min_keep=smp.min_tokens_to_keep)
    for b in range(len(prompts)):
        assert first_divergence(got[b], ref[b][0]) is None, f"{flt}: utterance {b} differs at frame " \
                                                            f"{first_divergence(got[b], ref[b][0])}"


@pytest.mark.parametrize("flt", FILTERS)
def test_tiny_filters(flt):
    from csm_mlx.models import CSM
    from csm_mlx.tokenizers import tokenize_text_segment
    args, w = csm_weights("tiny")
    model = CSM(args, dtype="float32", max_batch=3)
    model.load_weights(w)
    K = args.n_audio_codebooks
    prompts = [tokenize_text_segment(tiny_prompt_ids(50 + b, 3 + b), 0, K) for b in range(3)]
    _check(args, w, model, prompts, 5, flt, bf16=False)


@pytest.mark.parametrize("B", [1, 8])
def test_csm_1b_filters(B):
    """B = 1: the launch path (the persistent frame decoder keeps to temperature / top-k); B = 8: the
    matrix-core projections.  Every filter set, 3 frames."""
    from csm_mlx.models import CSM
    from csm_mlx.tokenizers import tokenize_text_segment
    args, w = csm_weights("1b")
    model = CSM(args, dtype="bf16", max_batch=B)
    model.load_weights(w)
    prompts = [tokenize_text_segment(prompt_ids(60 + b, 10 + b % 3), 0, 32) for b in range(B)]
    for flt in FILTERS:
        _check(args, w, model, prompts, 3, flt, bf16=True)
    del model
