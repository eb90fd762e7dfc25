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


TIE_FILTERS = [dict(top_k=5, min_p=0.3), dict(top_k=5, top_p=0.6), dict(min_p=0.1, min_tokens_to_keep=3),
               dict(top_p=0.5), dict(top_k=7, top_p=0.9, min_p=0.05, min_tokens_to_keep=2)]


def _tie_row(rng, V):
    """A c0 logits row built to stress the filter boundaries: values from a small set (exact ties,
    several at the top-k boundary), pairs one float32 ulp apart (their lp = l - lse can round equal)."""
    base = np.float32(rng.choice([0.0, 0.5, 1.0, 2.0, 2.0, 3.0], V))
    top = np.float32(4.0)
    idx = rng.choice(V, 9, replace=False)
    base[idx[:3]] = top                                    # a three-way tie at the maximum
    base[idx[3]] = np.nextafter(top, np.float32(5.0))      # one ulp above it
    base[idx[4:6]] = np.float32(3.5)
    base[idx[6]] = np.nextafter(np.float32(3.5), np.float32(0.0))
    base[idx[7:]] = np.float32(2.0)
    return base.astype(np.float32)


@pytest.mark.parametrize("flt", TIE_FILTERS)
def test_filter_boundaries_on_tied_rows(flt):
    """The kept set at the filter boundaries (ties at the top-k value, near-equal log-probabilities):
    a logits processor replaces every utterance's c0 logits by a synthetic tie-heavy row, the GPU's
    sample_filtered_kernel picks c0, and the pick must equal the oracle's Gumbel-max over
    ``filter_keep`` with the same counter-based noise (step = frame * K) -- 4 utterances x 6 frames,
    each a different row and seed, so a differing kept set shows as a differing pick.  Parity is against
    the oracle's restatement; against mlx_lm it is unpinned (not importable, no sampler fixture)."""
    from csm_mlx.generation import generate_codes_batch
    from csm_mlx.models import CSM
    from csm_mlx.sampling import make_sampler
    from csm_mlx.tokenizers import tokenize_text_segment
    from oracle.csm_oracle import sample_one
    args, w = csm_weights("tiny")
    B, frames, K, V = 4, 6, args.n_audio_codebooks, args.n_audio_vocab
    model = CSM(args, dtype="float32", max_batch=B)
    model.load_weights(w)
    rows = {}

    def proc(hist, logits):
        f = 0 if hist.size == 0 else hist.shape[0]
        rng = np.random.default_rng(7000 + 31 * f + sum(flt.get(k, 0) * 100 for k in ("top_k",)))
        out = np.stack([_tie_row(rng, V) for _ in range(B)])
        rows[f] = out.copy()
        return out

    smp = make_sampler(0.8, **flt)
    seeds = [4242 + 17 * b for b in range(B)]
    prompts = [tokenize_text_segment(tiny_prompt_ids(80 + b, 3 + b), 0, K) for b in range(B)]
    hist, n, _ = generate_codes_batch(model, prompts, frames, sampler=smp, seeds=seeds, logits_processors=[proc])
    del model
    checked = 0
    for b in range(B):
        for f in range(int(n[b])):
            exp = sample_one(rows[f][b], 0.8, smp.top_k, seeds[b], f * K, top_p=smp.top_p, min_p=smp.min_p,
                             min_keep=smp.min_tokens_to_keep)
            assert int(hist[f, b, 0]) == exp, f"{flt}: utterance {b} frame {f}: GPU c0 {hist[f, b, 0]} vs oracle {exp}"
            checked += 1
    assert checked >= B * 2
