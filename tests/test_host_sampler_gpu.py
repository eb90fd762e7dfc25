"""``sampler=`` with an arbitrary callable (the reference CLI passes mlx_lm's make_sampler callable,
/root/reference/csm_mlx/cli/generate.py:168-174, :197-199): the frame runs with every code chosen on
the host -- csm_frame_c0_logits, then csm_frame_host_step per codebook, which feeds the host's codes
forward and returns the next codebook's logits.  Checked against the oracle's frame loop with the same
callable (oracle/csm_oracle.py ``frame(sampler=)``), and an arg-max callable against the GPU greedy
graph path, bit for bit."""
import numpy as np
import pytest

from helpers import csm_weights, first_divergence, oracle_for, prompt_ids, tiny_prompt_ids

pytestmark = pytest.mark.gpu


def third_largest(logits):
    """A deterministic non-greedy sampler: the index of each row's third-largest logit."""
    x = np.asarray(logits, np.float32)
    return np.argsort(-x, axis=-1, kind="stable")[:, 2]


def argmax_sampler(logits):
    return np.argmax(np.asarray(logits, np.float32), axis=-1)


def _gpu_codes(model, prompts, frames, sampler):
    from csm_mlx.generation import generate_codes_batch, _resolve_sampler
    hist, n, _ = generate_codes_batch(model, prompts, frames, sampler=_resolve_sampler(0.8, sampler))
    return [hist[: n[b], b].copy() for b in range(len(prompts))]


def test_host_sampler_matches_oracle_tiny():
    from csm_mlx.models import CSM
    from csm_mlx.tokenizers import tokenize_text_segment
    args, w = csm_weights("tiny")
    model = CSM(args, dtype="float32", max_batch=2)
    model.load_weights(w)
    K = args.n_audio_codebooks
    ids = [tiny_prompt_ids(70 + b, 3 + b) for b in range(2)]
    prompts = [tokenize_text_segment(i, 0, K) for i in ids]
    got = _gpu_codes(model, prompts, 6, third_largest)
    o = oracle_for(args, w)
    for b in range(2):
        ref = o.generate_codes(*prompts[b], 6, sampler=third_largest)
        assert first_divergence(got[b], ref) is None, f"utterance {b}: differs at {first_divergence(got[b], ref)}"


@pytest.mark.parametrize("which,dtype,B", [("tiny", "float32", 2), ("1b", "bf16", 1)])
def test_host_argmax_sampler_equals_greedy_graph(which, dtype, B):
    """An arg-max callable on the host picks exactly what the GPU greedy path picks (first max)."""
    from csm_mlx.models import CSM
    from csm_mlx.sampling import Sampler
    from csm_mlx.tokenizers import tokenize_text_segment
    args, w = csm_weights(which)
    model = CSM(args, dtype=dtype, max_batch=B)
    model.load_weights(w)
    K = args.n_audio_codebooks
    ids = [tiny_prompt_ids(90 + b, 4) if which == "tiny" else prompt_ids(90 + b) for b in range(B)]
    prompts = [tokenize_text_segment(i, 0, K) for i in ids]
    frames = 5 if which == "tiny" else 3
    host = _gpu_codes(model, prompts, frames, argmax_sampler)
    greedy = _gpu_codes(model, prompts, frames, Sampler(0.0, 0))
    for b in range(B):
        assert np.array_equal(host[b], greedy[b]), f"utterance {b}"
    del model


def test_stream_generate_with_host_sampler():
    """stream_generate(sampler=callable) streams the host-sampled frames through decode_step."""
    from csm_mlx.generation import stream_generate
    from csm_mlx.models import CSM
    from csm_mlx.tokenizers import set_audio_tokenizer
    from csm_mlx.config import MIMI_CONFIGURATION
    from csm_mlx.mimi import MimiCodec
    from csm_mlx.weights import synthetic_mimi_weights
    args, w = csm_weights("tiny")
    model = CSM(args, dtype="float32", max_batch=1)
    model.load_weights(w)
    mc = MIMI_CONFIGURATION["tiny"]
    codec = MimiCodec(mc, max_batch=2)
    codec.load_weights(synthetic_mimi_weights(mc, 0))
    set_audio_tokenizer(codec, mc.n_q)
    chunks = list(stream_generate(model, tiny_prompt_ids(5, 4), 0, [], 4 * 80, sampler=third_largest))
    assert 1 <= len(chunks) <= 4 and all(c.shape == (mc.frame_size,) for c in chunks)
