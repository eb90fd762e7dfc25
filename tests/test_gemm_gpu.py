"""GPU parity of the batched matrix-core path (gemm_kernels.hip: bf16 or int4 weights, split-bf16
activations on MFMA, split-K slices) -- taken by every bf16 / int4 projection once a launch has
>= 8 rows (B >= 8 utterances, decoder step 1 at B >= 4, prompt prefill of >= 8 rows).

Greedy codes must be bit-exact against the oracle run with bf16-rounded (or int4-dequantized)
weights and fp32 activations, logits within 2e-3 / 1e-3 x max|logit| -- the bar of the GEMV paths;
a code may differ only at a near-tie (the oracle's logits of the two codes closer than that bar),
after which the utterance is no longer compared.
"""
import numpy as np
import pytest

from helpers import csm_weights, first_divergence, oracle_for, prompt_ids, tiny_prompt_ids

pytestmark = pytest.mark.gpu


def _model(args, weights, dtype, max_batch):
    from csm_mlx.models import CSM
    m = CSM(args, dtype=dtype, max_batch=max_batch)
    m.load_weights(weights)
    return m


def _batch_vs_oracle(args, w, id_sets, frames, rtol, dtype="bf16", check=None):
    from csm_mlx.generation import FrameCache
    from csm_mlx.sampling import Sampler
    from csm_mlx.tokenizers import tokenize_text_segment
    from oracle.csm_oracle import text_frame
    K, V = args.n_audio_codebooks, args.n_audio_vocab
    Vp = (V + 7) // 8 * 8
    B = len(id_sets)
    model = _model(args, w, dtype, B)
    o = oracle_for(args, w, bf16=(dtype == "bf16"), q4=(dtype == "q4"))
    cache = FrameCache(model, B, Sampler(0.0, 0), [0] * B)
    for b, ids in enumerate(id_sets):
        cache.prefill(b, *tokenize_text_segment(ids, 0, K))
    logs = []
    for _ in range(frames):
        cache.run(1)
        logs.append((cache.debug("c0_logits", (B, Vp))[:, :V], cache.debug("ci_logits", (K - 1, B, Vp))[:, :, :V]))
    hist, n, _ = cache.codes()
    for b, ids in enumerate(id_sets):
        if check is not None and b not in check:
            continue
        ref, ref_logs = o.generate_codes(*text_frame(ids, K), frames, collect_logits=True)
        div = first_divergence(hist[: n[b], b], ref)
        upto = len(ref_logs) if div is None else div
        if div is not None:
            # accepted only as a near-tie: the oracle's logits for the two codes at the first diverging
            # codebook differ by less than the logit tolerance (later frames then legitimately differ)
            k = int(np.argmax(hist[div, b] != ref[div]))
            lo = ref_logs[div][0] if k == 0 else ref_logs[div][1][k - 1]
            gap = abs(float(lo[ref[div][k]]) - float(lo[hist[div, b][k]]))
            assert gap <= rtol * np.abs(lo).max(), (
                f"utterance {b} diverges at frame {div} codebook {k}: {hist[div, b][k]} vs {ref[div][k]}, "
                f"oracle logit gap {gap:.3e}")
        else:
            assert n[b] == len(ref), f"utterance {b}: {n[b]} frames vs oracle {len(ref)}"
        for f in range(upto):
            for got, want in ((logs[f][0][b], ref_logs[f][0]), (logs[f][1][:, b], ref_logs[f][1])):
                err = np.abs(got - want).max()
                assert err <= rtol * np.abs(want).max(), f"utterance {b} frame {f}: logits err {err:.3e}"
    del model


@pytest.mark.parametrize("B", [4, 8, 12, 33])
def test_tiny_bf16_batched_mfma(B):
    """B = 4: only decoder step 1 (M = 8 rows) on MFMA; 8 / 12: every projection; 33: two batch tiles."""
    args, w = csm_weights("tiny")
    id_sets = [tiny_prompt_ids(100 + b, 2 + b % 7) for b in range(B)]
    _batch_vs_oracle(args, w, id_sets, 5, 2e-3)


def test_csm_1b_bf16_batched_mfma():
    """csm_1b at B = 8: split-K slices (backbone QKV / o / down, decoder QKV / o / down) + heads."""
    args, w = csm_weights("1b")
    id_sets = [prompt_ids(200 + b, 4 + b) for b in range(8)]
    _batch_vs_oracle(args, w, id_sets, 2, 2e-3)


def test_csm_1b_bf16_batched_mfma_two_tiles():
    """csm_1b at B = 40: 64-row batch tiles (MT = 2, 2-stage prefetch ring), split-K up to 16 slices
    combined in one launch, the step-1 decoder at M = 80 (two batch chunks); utterances from both
    tiles and both chunks are compared (all 40 run in the batch)."""
    args, w = csm_weights("1b")
    id_sets = [prompt_ids(500 + b, 3 + b % 9) for b in range(40)]
    _batch_vs_oracle(args, w, id_sets, 2, 2e-3, check={0, 17, 31, 39})


@pytest.mark.parametrize("B", [9, 33])
def test_tiny_q4_batched_mfma(B):
    """int4 weights on the matrix cores: dequantized while staging, split hi/lo (3 products)."""
    args, w = csm_weights("tiny")
    id_sets = [tiny_prompt_ids(300 + b, 2 + b % 5) for b in range(B)]
    _batch_vs_oracle(args, w, id_sets, 4, 1e-3, dtype="q4")


def test_csm_1b_q4_batched_mfma():
    args, w = csm_weights("1b")
    id_sets = [prompt_ids(400 + b, 4 + b) for b in range(8)]
    _batch_vs_oracle(args, w, id_sets, 2, 1e-3, dtype="q4")
