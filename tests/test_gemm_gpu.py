"""GPU parity of the batched matrix-core path (gemm_kernels.hip: bf16 or int4 weights, activations
split into three bf16 parts -- fp32-exact products -- split-K slices) taken by every bf16 / int4
projection once a launch has >= 8 rows (B >= 8 utterances, decoder step 1 at B >= 4, prompt prefill
of >= 8 rows).

The bar is the greedy bar of the GEMV paths, with no exception: codes bit-exact against the oracle
run with bf16-rounded (or int4-dequantized) weights and fp32 activations, every utterance, every
frame; logits within 2e-3 (bf16) / 1e-3 (int4) x max|logit|.
"""
import numpy as np
import pytest

from helpers import csm_weights, first_divergence, oracle_batch, oracle_for, prompt_ids, tiny_prompt_ids

pytestmark = pytest.mark.gpu


def _model(args, weights, dtype, max_batch):
    from csm_mlx.models import CSM
    m = CSM(args, dtype=dtype, max_batch=max_batch)
    m.load_weights(weights)
    return m


def _batch_vs_oracle(args, w, id_sets, frames, rtol, dtype="bf16", logits_of=None):
    """logits_of: utterances whose logits are compared every frame (codes: all of them)."""
    from csm_mlx.generation import FrameCache
    from csm_mlx.sampling import Sampler
    from csm_mlx.tokenizers import tokenize_text_segment
    K, V = args.n_audio_codebooks, args.n_audio_vocab
    Vp = (V + 7) // 8 * 8
    B = len(id_sets)
    model = _model(args, w, dtype, B)
    o = oracle_for(args, w, bf16=(dtype == "bf16"), q4=(dtype == "q4"))
    prompts = [tokenize_text_segment(ids, 0, K) for ids in id_sets]
    cache = FrameCache(model, B, Sampler(0.0, 0), [0] * B)
    for b, (t, m) in enumerate(prompts):
        cache.prefill(b, t, m)
    logs = []
    for _ in range(frames):
        cache.run(1)
        logs.append((cache.debug("c0_logits", (B, Vp))[:, :V], cache.debug("ci_logits", (K - 1, B, Vp))[:, :, :V]))
    hist, n, _ = cache.codes()
    del model
    ref = oracle_batch(o, prompts, frames, collect_logits=True)
    bad = []
    for b in range(B):
        ref_codes, ref_logs = ref[b]
        div = first_divergence(hist[: n[b], b], ref_codes)
        if div is not None or n[b] != len(ref_codes):
            f = div if div is not None else min(n[b], len(ref_codes))
            bad.append(f"utterance {b}: first divergence at frame {f} ({n[b]} vs {len(ref_codes)} frames)")
            continue
        if logits_of is not None and b not in logits_of:
            continue
        for f in range(len(ref_codes)):
            for got, want in ((logs[f][0][b], ref_logs[f][0]), (logs[f][1][:, b], ref_logs[f][1])):
                err = np.abs(got - want).max()
                assert err <= rtol * np.abs(want).max(), f"utterance {b} frame {f}: logits err {err:.3e}"
    assert not bad, "; ".join(bad)


@pytest.mark.parametrize("B", [4, 8, 12, 33])
def test_tiny_bf16_batched_mfma(B):
    """B = 4: only decoder step 1 (M = 8 rows) on MFMA; 8 / 12: every projection; 33: two batch tiles."""
    args, w = csm_weights("tiny")
    id_sets = [tiny_prompt_ids(100 + b, 2 + b % 7) for b in range(B)]
    _batch_vs_oracle(args, w, id_sets, 6, 2e-3)


@pytest.mark.parametrize("dtype", ["bf16", "q4"])
def test_tiny_f1280_streaming_gemm_stage_coverage(dtype):
    """A decoder MLP of width 1280 (the engine takes multiples of 256): the streaming GEMM's down
    projection has K = 1280 = 20 stages of 64, which an 8-wave block does not divide (the shape rule now
    picks 4 waves; the 8-wave block once skipped 4 of the 20 stages).  B = 8 greedy, 5 frames, bit-exact
    against the oracle.  q4: the int4 GEMV (decoder step 1's rows, the head at B = 1) also takes K = 1280
    (a 64-lane group with lanes 40..63 idle; round 5 refused the shape)."""
    import dataclasses
    from csm_mlx.models import csm_tiny
    from csm_mlx.weights import synthetic_csm_weights
    args = dataclasses.replace(csm_tiny(), decoder_name="tiny_f1280")
    w = synthetic_csm_weights(args, 0)
    id_sets = [tiny_prompt_ids(700 + b, 2 + b % 5) for b in range(8)]
    _batch_vs_oracle(args, w, id_sets, 5, 2e-3 if dtype == "bf16" else 1e-3, dtype=dtype)


@pytest.mark.parametrize("B", [9, 33])
def test_tiny_q4_batched_mfma(B):
    """int4 weights on the matrix cores: nibbles as exact bf16 operands, per-group scale / bias fold."""
    args, w = csm_weights("tiny")
    id_sets = [tiny_prompt_ids(300 + b, 2 + b % 5) for b in range(B)]
    _batch_vs_oracle(args, w, id_sets, 6, 1e-3, dtype="q4")


@pytest.mark.parametrize("B", [8, 32, 64])
def test_csm_1b_bf16_batched_mfma(B):
    """csm_1b bf16 at B = 8 (split-K slices: backbone QKV / o / down, decoder QKV / o / down, heads),
    32 (configs[3]'s per-GPU shard: one 32-row tile) and 64 (MT = 2 tiles, decoder step 1 at 128 rows
    in two chunks): 4 frames, every utterance bit-exact.  Prompts of 3 lengths (ragged positions)."""
    args, w = csm_weights("1b")
    id_sets = [prompt_ids(200 + b, 10 + b % 3) for b in range(B)]
    _batch_vs_oracle(args, w, id_sets, 4, 2e-3, logits_of={0, B // 2, B - 1})


@pytest.mark.parametrize("B", [8, 64])
def test_csm_1b_q4_batched_mfma(B):
    """configs[4]'s int4 g64 engine at B = 8 and 64: 4 frames, every utterance bit-exact against the
    oracle on the dequantized weights."""
    args, w = csm_weights("1b")
    id_sets = [prompt_ids(400 + b, 10 + b % 3) for b in range(B)]
    _batch_vs_oracle(args, w, id_sets, 4, 1e-3, dtype="q4", logits_of={0, B - 1})


@pytest.mark.parametrize("dtype", ["bf16", "q4"])
def test_batched_prefill_matches_per_utterance(dtype):
    """csm_prefill_batch (every prompt's rows in one pass per projection, ragged lengths) against
    csm_prefill per utterance: identical greedy codes, logits within fp32 summation-order noise."""
    from csm_mlx.generation import FrameCache
    from csm_mlx.sampling import Sampler
    from csm_mlx.tokenizers import tokenize_text_segment
    args, w = csm_weights("tiny")
    K, V = args.n_audio_codebooks, args.n_audio_vocab
    Vp = (V + 7) // 8 * 8
    B = 12
    prompts = [tokenize_text_segment(tiny_prompt_ids(300 + b, 2 + (5 * b) % 11), 0, K) for b in range(B)]
    out = []
    for batched in (False, True):
        model = _model(args, w, dtype, B)
        cache = FrameCache(model, B, Sampler(0.0, 0), [0] * B)
        if batched:
            cache.prefill_batch([(b, t, m) for b, (t, m) in enumerate(prompts)])
        else:
            for b, (t, m) in enumerate(prompts):
                cache.prefill(b, t, m)
        logs = []
        for _ in range(4):
            cache.run(1)
            logs.append(cache.debug("c0_logits", (B, Vp))[:, :V].copy())
        hist, n, _ = cache.codes()
        out.append((hist.copy(), n.copy(), logs))
        del cache, model
    (h0, n0, l0), (h1, n1, l1) = out
    assert np.array_equal(n0, n1) and np.array_equal(h0, h1)
    for a, b in zip(l0, l1):
        assert np.abs(a - b).max() <= 1e-4 * np.abs(a).max()


def test_csm_1b_bf16_batch_composition_invariance():
    """An utterance's greedy codes do not depend on which other prompts share its batch: the same
    csm_1b bf16 prompt alone (B = 1: persistent backbone step + frame decoder, fp32 GEMV sums) and
    as utterance 5 of a B = 32 batch prefilled in one csm_prefill_batch pass (matrix-core GEMMs whose
    split-K slice count follows the batch's total row count) -- 6 frames, codes identical, c0 logits
    within the bf16 bar.  (Summation order differs between the two; greedy codes are the bar.)"""
    from csm_mlx.generation import FrameCache
    from csm_mlx.sampling import Sampler
    from csm_mlx.tokenizers import tokenize_text_segment
    args, w = csm_weights("1b")
    K, V = args.n_audio_codebooks, args.n_audio_vocab
    Vp = (V + 7) // 8 * 8
    B, frames, j = 32, 6, 5
    prompts = [tokenize_text_segment(prompt_ids(700 + b, 8 + b % 5), 0, K) for b in range(B)]
    model = _model(args, w, "bf16", B)
    out = []
    for batch in ([prompts[j]], prompts):
        cache = FrameCache(model, len(batch), Sampler(0.0, 0), [0] * len(batch))
        if len(batch) > 1:
            cache.prefill_batch([(b, t, m) for b, (t, m) in enumerate(batch)])
        else:
            cache.prefill(0, *batch[0])
        logs = []
        for _ in range(frames):
            cache.run(1)
            logs.append(cache.debug("c0_logits", (len(batch), Vp))[:, :V].copy())
        hist, n, _ = cache.codes()
        b = 0 if len(batch) == 1 else j
        out.append((hist[: n[b], b].copy(), [l[b] for l in logs]))
        del cache
    del model
    (c1, l1), (c32, l32) = out
    assert len(c1) == frames and first_divergence(c1, c32) is None, "codes depend on the batch composition"
    for a, b in zip(l1, l32):
        assert np.abs(a - b).max() <= 2e-3 * np.abs(a).max()


@pytest.mark.parametrize("B,dtype,bb", [(8, "bf16", 0), (24, "bf16", 0), (24, "q4", 0), (24, "bf16", 1), (24, "q4", 1)])
def test_streaming_decoder_matches_wide_gemm(B, dtype, bb):
    """The batched depth decoder at codebook steps >= 2 on the streaming matrix-core GEMM over
    pre-split activations (gemm_xs.hip; option gemm_xs, on by default) against the same frames on
    gemm_wide_kernel: identical greedy codes, ci logits within fp32 summation-order noise (both sum
    exact fp32 products), 4 frames, csm_1b bf16 and int4; bb=1 also runs the backbone's projections
    on it (option bb_xs, on by default since round 4; bb=0 keeps it on gemm_wide)."""
    from csm_mlx import _lib
    from csm_mlx.generation import FrameCache
    from csm_mlx.sampling import Sampler
    from csm_mlx.tokenizers import tokenize_text_segment
    args, w = csm_weights("1b")
    K, V = args.n_audio_codebooks, args.n_audio_vocab
    Vp = (V + 7) // 8 * 8
    prompts = [tokenize_text_segment(prompt_ids(900 + b, 9 + b % 4), 0, K) for b in range(B)]
    model = _model(args, w, dtype, B)
    L = _lib.lib()
    out = []
    for on in (0, 1):
        _lib.check(L.csm_set_option(model.engine, b"gemm_xs", on))
        _lib.check(L.csm_set_option(model.engine, b"bb_xs", on * bb))
        cache = FrameCache(model, B, Sampler(0.0, 0), [0] * B)
        cache.prefill_batch([(b, t, m) for b, (t, m) in enumerate(prompts)])
        logs = []
        for _ in range(4):
            cache.run(1)
            logs.append(cache.debug("ci_logits", (K - 1, B, Vp))[:, :, :V].copy())
        hist, n, _ = cache.codes()
        out.append((hist.copy(), n.copy(), logs))
        del cache
    _lib.check(L.csm_set_option(model.engine, b"gemm_xs", 1))
    _lib.check(L.csm_set_option(model.engine, b"bb_xs", 1))
    del model
    (h0, n0, l0), (h1, n1, l1) = out
    assert np.array_equal(n0, n1) and np.array_equal(h0, h1), "streaming decoder codes differ from gemm_wide"
    for a, b in zip(l0, l1):
        assert np.abs(a - b).max() <= 1e-4 * np.abs(a).max()
