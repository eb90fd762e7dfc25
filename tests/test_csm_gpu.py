"""GPU parity: the HIP frame engine (through the C ABI) against the numpy oracle.

Greedy codes must be bit-exact; logits must agree within a relative tolerance
of 2e-4 x max|logit| (fp32 weights) / 2e-3 (bf16 weights vs a bf16-rounded
oracle, activations fp32 on both sides).  On a code mismatch the test reports
the first diverging frame and the oracle's top-2 logit margin there.
"""
import numpy as np
import pytest

from helpers import csm_weights, first_divergence, oracle_for, prompt_ids, tiny_prompt_ids

pytestmark = pytest.mark.gpu


def _model(args, weights, dtype, max_batch=1):
    from csm_mlx.models import CSM
    m = CSM(args, dtype=dtype, max_batch=max_batch)
    m.load_weights(weights)
    return m


@pytest.fixture(scope="module")
def tiny():
    return csm_weights("tiny")


def _oracle_frames(o, ids, frames, K, temperature=0.0, top_k=0, seed=0):
    from oracle.csm_oracle import text_frame
    t, m = text_frame(ids, K)
    return o.generate_codes(t, m, frames, temperature=temperature, top_k=top_k, seed=seed, collect_logits=True)


def _engine_frames(model, ids, frames, temperature=0.0, top_k=0, seed=0):
    from csm_mlx.generation import FrameCache
    from csm_mlx.sampling import Sampler
    from csm_mlx.tokenizers import tokenize_text_segment
    t, m = tokenize_text_segment(ids, 0, model.n_audio_codebooks)
    cache = FrameCache(model, 1, Sampler(temperature, top_k), [seed])
    cache.prefill(0, t, m)
    logs = []
    V = model.n_audio_vocab
    Vp = (V + 7) // 8 * 8
    K = model.n_audio_codebooks
    for _ in range(frames):
        cache.run(1)
        c0 = cache.debug("c0_logits", (1, Vp))[0, :V]
        ci = cache.debug("ci_logits", (K - 1, 1, Vp))[:, 0, :V]
        logs.append((c0, ci))
    hist, n, done = cache.codes()
    return hist[:, 0], n[0], logs


def _compare(eng, orc, frames, rtol):
    hist, n_e, logs_e = eng
    codes_o, logs_o = orc
    # emitted frames agree (EOS semantics) and codes are bit-exact
    F = len(codes_o)
    assert n_e == F, f"engine emitted {n_e} frames, oracle {F}"
    div = first_divergence(hist[:F], codes_o)
    if div is not None:
        c0o = logs_o[div][0]
        top = np.sort(c0o)[-2:]
        pytest.fail(f"codes diverge at frame {div}: engine {hist[div]} oracle {codes_o[div]}; "
                    f"oracle c0 top-2 margin {top[1]-top[0]:.3e}")
    for f in range(min(len(logs_e), len(logs_o))):
        for a, b in ((logs_e[f][0], logs_o[f][0]), (logs_e[f][1], logs_o[f][1])):
            scale = np.abs(b).max()
            err = np.abs(a - b).max()
            assert err <= rtol * scale, f"frame {f}: logits max err {err:.3e} vs scale {scale:.3e}"


@pytest.mark.parametrize("dtype", ["float32", "bf16"])
def test_tiny_greedy_parity(tiny, dtype):
    args, w = tiny
    model = _model(args, w, dtype)
    o = oracle_for(args, w, bf16=(dtype == "bf16"))
    ids = tiny_prompt_ids(1)
    frames = 12
    eng = _engine_frames(model, ids, frames)
    orc = _oracle_frames(o, ids, frames, args.n_audio_codebooks)
    _compare(eng, orc, frames, 2e-4 if dtype == "float32" else 2e-3)


def test_tiny_topk_sampling_parity(tiny):
    """Temperature + top-k: the GPU Gumbel sampler and the oracle restatement of the same
    counter-based RNG must pick identical codes."""
    args, w = tiny
    model = _model(args, w, "float32")
    o = oracle_for(args, w)
    ids = tiny_prompt_ids(2)
    eng = _engine_frames(model, ids, 8, temperature=0.8, top_k=5, seed=1234)
    orc = _oracle_frames(o, ids, 8, args.n_audio_codebooks, temperature=0.8, top_k=5, seed=1234)
    _compare(eng, orc, 8, 2e-4)


@pytest.mark.parametrize("top_k", [50, 0])
def test_csm_1b_topk_sampling_parity(top_k):
    """configs[2] sampler at csm_1b size (V = 2051: nine logits per thread, a 4-digit radix select of
    the top-50 threshold, or no top-k): codes identical to the oracle's restatement of the RNG."""
    args, w = csm_weights("1b")
    model = _model(args, w, "float32")
    o = oracle_for(args, w)
    ids = prompt_ids(5)
    eng = _engine_frames(model, ids, 2, temperature=0.8, top_k=top_k, seed=77)
    orc = _oracle_frames(o, ids, 2, args.n_audio_codebooks, temperature=0.8, top_k=top_k, seed=77)
    _compare(eng, orc, 2, 2e-4)
    del model


def test_tiny_batched_ragged_prompts(tiny):
    """B utterances with different prompt lengths == each utterance run alone."""
    from csm_mlx.generation import generate_codes_batch
    from csm_mlx.sampling import Sampler
    from csm_mlx.tokenizers import tokenize_text_segment
    from oracle.csm_oracle import text_frame
    args, w = tiny
    K = args.n_audio_codebooks
    model = _model(args, w, "float32", max_batch=3)
    o = oracle_for(args, w)
    id_sets = [tiny_prompt_ids(10, 3), tiny_prompt_ids(11, 9), tiny_prompt_ids(12, 6)]
    prompts = [tokenize_text_segment(ids, 0, K) for ids in id_sets]
    hist, n, _ = generate_codes_batch(model, prompts, 6, sampler=Sampler(0.0, 0))
    for b, ids in enumerate(id_sets):
        t, m = text_frame(ids, K)
        ref = o.generate_codes(t, m, 6)
        assert n[b] == len(ref)
        assert first_divergence(hist[: n[b], b], ref) is None, f"utterance {b} diverges"


def test_generate_frame_appends_rows(tiny):
    """generate_frame with explicit feedback rows == the graph-driven frame loop."""
    from csm_mlx.generation import generate_frame, make_frame_cache
    from csm_mlx.tokenizers import tokenize_text_segment
    args, w = tiny
    K = args.n_audio_codebooks
    model = _model(args, w, "float32")
    o = oracle_for(args, w)
    ids = tiny_prompt_ids(3)
    t, m = tokenize_text_segment(ids, 0, K)
    cache = make_frame_cache(model, 1, temperature=0.0)
    out = []
    inp, msk = t[None], m[None]
    for _ in range(4):
        s = generate_frame(model, inp, temperature=0.0, token_mask=msk, cache=cache)
        out.append(s[0])
        inp = np.concatenate([s, np.zeros((1, 1), np.int32)], 1)[:, None, :]
        msk = np.concatenate([np.ones((1, K), bool), np.zeros((1, 1), bool)], 1)[:, None, :]
    from oracle.csm_oracle import text_frame
    ref = o.generate_codes(*text_frame(ids, K), 4)
    assert first_divergence(np.stack(out), ref) is None


def test_window_guard():
    """generation.py:132-137: prompt length >= 2048 - frames raises ValueError."""
    from csm_mlx.generation import _check_window
    from csm_mlx.models import CSM, csm_tiny
    m = CSM(csm_tiny(), dtype="float32")
    with pytest.raises(ValueError, match="Inputs too long"):
        _check_window(m, 2048 - 125, 125)
    _check_window(m, 2048 - 126, 125)


@pytest.mark.parametrize("dtype", ["float32", "bf16"])
def test_csm_1b_first_frames(dtype):
    """csm_1b-shaped run (seeded synthetic weights), config-2 prompt, first 3 frames."""
    args, w = csm_weights("1b")
    model = _model(args, w, dtype)
    o = oracle_for(args, w, bf16=(dtype == "bf16"))
    ids = prompt_ids(1)
    eng = _engine_frames(model, ids, 3)
    orc = _oracle_frames(o, ids, 3, args.n_audio_codebooks)
    _compare(eng, orc, 3, 2e-4 if dtype == "float32" else 2e-3)
    del model


@pytest.mark.parametrize("which,dtype", [("tiny", "float32"), ("tiny", "bf16"), ("1b", "bf16")])
def test_folded_layer0_qkv_table_matches_gemv(tiny, which, dtype):
    """Decoder steps >= 2 gather layer 0's (RoPE'd q, k | v) from the table built at csm_begin by the
    same QKV GEMV: codes must be bit-identical to running the GEMV every step."""
    from csm_mlx import _lib
    from csm_mlx.generation import generate_codes_batch
    from csm_mlx.sampling import Sampler
    from csm_mlx.tokenizers import tokenize_text_segment
    args, w = tiny if which == "tiny" else csm_weights("1b")
    model = _model(args, w, dtype, max_batch=2)
    K = args.n_audio_codebooks
    ids = [tiny_prompt_ids(40 + b, 3 + b) if which == "tiny" else prompt_ids(40 + b) for b in range(2)]
    prompts = [tokenize_text_segment(i, 0, K) for i in ids]
    L = _lib.lib()
    frames = 12 if which == "tiny" else 6
    _lib.check(L.csm_set_option(model.engine, b"qkv0_tab", 0))
    ref, n_ref, _ = generate_codes_batch(model, prompts, frames, sampler=Sampler(0.0, 0))
    _lib.check(L.csm_set_option(model.engine, b"qkv0_tab", 1))
    got, n_got, _ = generate_codes_batch(model, prompts, frames, sampler=Sampler(0.0, 0))
    assert np.array_equal(n_got, n_ref)
    assert np.array_equal(got, ref), f"first diff at {np.argwhere(got != ref)[0]}"
    del model


def test_eos_first_frame_stops_generation(tiny):
    """generation.py:151-152 / :163-165: an all-zero frame is EOS -- it is not appended, and with no
    samples generate() returns zeros((0,)).  Zeroed heads make every logit 0, so the first-max greedy
    pick is code 0 in every codebook (the reference's argmax tie rule) for every utterance."""
    from csm_mlx.generation import generate, generate_codes_batch
    from csm_mlx.sampling import Sampler
    from csm_mlx.tokenizers import tokenize_text_segment
    args, w = tiny
    w = dict(w)
    for k in ("codebook0_head.weight", "audio_head"):
        w[k] = np.zeros_like(w[k])
    model = _model(args, w, "float32", max_batch=3)
    o = oracle_for(args, w)
    from oracle.csm_oracle import text_frame
    ref = o.generate_codes(*text_frame(tiny_prompt_ids(7, 4), args.n_audio_codebooks), 10)
    assert len(ref) == 0
    prompts = [tokenize_text_segment(tiny_prompt_ids(7 + b, 3 + b), 0, args.n_audio_codebooks) for b in range(3)]
    hist, n, _ = generate_codes_batch(model, prompts, 10, sampler=Sampler(0.0, 0))
    assert n.tolist() == [0, 0, 0]
    audio = generate(model, text=tiny_prompt_ids(7, 4), speaker=0, context=[], max_audio_length_ms=800, temperature=0.0)
    assert audio.shape == (0,) and audio.dtype == np.float32
    del model


def test_eos_per_utterance_in_batch(tiny):
    """Batched EOS: with the ci heads zeroed and only c0-head row 0 non-zero, a frame is all-zero
    (EOS) exactly when that row's logit is positive for the utterance's backbone state -- so some
    utterances stop at different frames while the others keep generating.  Every utterance must match
    its own oracle run (codes and frame count)."""
    from csm_mlx.generation import generate_codes_batch
    from csm_mlx.sampling import Sampler
    from csm_mlx.tokenizers import tokenize_text_segment
    from oracle.csm_oracle import text_frame
    args, w = tiny
    w = dict(w)
    rng = np.random.default_rng(3)
    c0 = np.zeros_like(w["codebook0_head.weight"])
    c0[0] = rng.normal(0, 1.0, c0.shape[1]).astype(c0.dtype)
    w["codebook0_head.weight"] = c0
    w["audio_head"] = np.zeros_like(w["audio_head"])
    K = args.n_audio_codebooks
    B, F = 8, 6
    model = _model(args, w, "float32", max_batch=B)
    o = oracle_for(args, w)
    ids = [tiny_prompt_ids(90 + b, 2 + b % 5) for b in range(B)]
    hist, n, _ = generate_codes_batch(model, [tokenize_text_segment(i, 0, K) for i in ids], F, sampler=Sampler(0.0, 0))
    lens = []
    for b in range(B):
        ref = o.generate_codes(*text_frame(ids[b], K), F)
        lens.append(len(ref))
        assert n[b] == len(ref), f"utterance {b}: {n[b]} frames vs oracle {len(ref)}"
        assert np.array_equal(hist[: n[b], b], np.asarray(ref).reshape(-1, K))
    assert 0 < sum(1 for x in lens if x < F) < B, f"want a mix of stopped / running utterances, got {lens}"
    del model
