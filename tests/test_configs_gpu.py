"""BASELINE.json configs at csm_1b size, end to end through the drop-in API, against the oracle.

* configs[2]: ``stream_generate_batch`` at B = 32, temperature 0.8, top-k 50 (matrix-core
  projections, the GPU sampler, the overlapped per-frame Mimi ``decode_step`` loop): codes
  bit-exact against the oracle's restatement of the engine's counter-based RNG, every streamed
  chunk within 1e-4 RMS of the Mimi oracle's ``decode_step``.
* configs[4]: int4 g64 (``nn.quantize``) engine, B = 4, three 5 s context Segments per utterance
  (Mimi-encoded, L = 248 rows: a 248-row matrix-core prefill) + the text row: first frames
  bit-exact against the oracle on the dequantized weights.
"""
import numpy as np
import pytest

from helpers import csm_weights, first_divergence, oracle_batch, oracle_for, prompt_ids

pytestmark = pytest.mark.gpu


def _codec(batch):
    from csm_mlx.config import MIMI_CONFIGURATION
    from csm_mlx.mimi import MimiCodec
    from csm_mlx.tokenizers import set_audio_tokenizer
    from csm_mlx.weights import synthetic_mimi_weights
    mc = MIMI_CONFIGURATION["mimi_202407"]
    mw = synthetic_mimi_weights(mc, 0)
    codec = MimiCodec(mc, max_batch=batch)
    codec.load_weights(mw)
    set_audio_tokenizer(codec, 32)
    return codec, mc, mw


def _engine_codes(model, B):
    import ctypes
    from csm_mlx import _lib
    L = _lib.lib()
    F = ctypes.c_int(0)
    _lib.check(L.csm_read_codes(model.engine, None, None, None, ctypes.byref(F)))
    hist = np.zeros((F.value, B, model.n_audio_codebooks), np.int32)
    n = np.zeros(B, np.int32)
    _lib.check(L.csm_read_codes(model.engine, _lib.ptr(hist), _lib.ptr(n), None, None))
    return hist, n


def test_config2_stream_generate_batch_sampled():
    from csm_mlx.generation import stream_generate_batch
    from csm_mlx.models import CSM
    from csm_mlx.tokenizers import tokenize_text_segment
    from oracle.mimi_oracle import OracleMimi
    B, frames = 32, 3
    args, w = csm_weights("1b")
    model = CSM(args, dtype="bf16", max_batch=B)
    model.load_weights(w)
    codec, mc, mw = _codec(B)
    prompts = [tokenize_text_segment(prompt_ids(1000 + b), 0, 32) for b in range(B)]
    seeds = [1234 + b for b in range(B)]
    chunks = [pcm.copy() for pcm, _ in stream_generate_batch(model, prompts, frames * 80, temperature=0.8,
                                                             top_k=50, seeds=seeds)]
    hist, n = _engine_codes(model, B)
    del model
    assert len(chunks) == frames and all(c.shape == (B, 1920) for c in chunks)
    ref = oracle_batch(oracle_for(args, w, bf16=True), prompts, frames, temperature=0.8, top_k=50, seeds=seeds)
    bad = [b for b in range(B) if n[b] != frames or first_divergence(hist[:frames, b], ref[b][0]) is not None]
    assert not bad, f"sampled codes differ for utterances {bad}"
    om = OracleMimi(mc, mw)
    om.reset_state()
    codes = np.stack([ref[b][0] for b in range(B)])                  # (B, F, K)
    for f in range(frames):
        want = om.decode_step(np.ascontiguousarray(codes[:, f, :, None]))[:, 0]
        rms = np.sqrt(np.mean((chunks[f].astype(np.float64) - want) ** 2, axis=1))
        assert rms.max() <= 1e-4, f"frame {f}: chunk RMS error {rms.max():.3e}"


def test_config4_q4_context_segments():
    from csm_mlx.generation import generate_codes_batch
    from csm_mlx.models import CSM
    from csm_mlx.sampling import Sampler
    from csm_mlx.segment import Segment
    from csm_mlx.tokenizers import tokenize_segments_batch, tokenize_text_segment
    from oracle.mimi_oracle import OracleMimi
    import bench
    B, frames = 4, 2
    args, w = csm_weights("1b")
    model = CSM(args, dtype="q4", max_batch=B)     # bench.py --config 5: float weights quantized on load
    model.load_weights(w)
    codec, mc, mw = _codec(3 * B)
    segs = [Segment(s % 2, prompt_ids(10_000 + 10 * g + s), bench.context_audio(g, s)) for g in range(B) for s in range(3)]
    enc = tokenize_segments_batch(segs, n_audio_codebooks=32)
    prompts = []
    for g in range(B):
        parts = enc[3 * g:3 * g + 3] + [tokenize_text_segment(prompt_ids(g), 0, 32)]
        prompts.append((np.concatenate([t for t, _ in parts]), np.concatenate([m for _, m in parts])))
    assert all(t.shape[0] == 248 for t, _ in prompts)
    hist, n, _ = generate_codes_batch(model, prompts, frames, sampler=Sampler(0.0, 0))
    del model
    # the GPU Mimi encode of a context segment == the Mimi oracle's (the prompt both sides consume)
    seg_codes = OracleMimi(mc, mw).encode(segs[0].audio[None, None])[0]
    assert np.array_equal(enc[0][0][len(segs[0].text):-1, :32], seg_codes.T)
    ref = oracle_batch(oracle_for(args, w, q4=True), prompts, frames)
    for b in range(B):
        assert n[b] == frames and first_divergence(hist[:frames, b], ref[b][0]) is None, f"utterance {b}"


def test_config5_multi_group_prefill():
    """configs[4] at its real prefill shape: B = 9 prompts of 248 Mimi-encoded context rows = 2,232
    rows, more than one csm_prefill_batch group holds (<= 2,048 rows: groups of 8 + 1), and again with
    the group cap lowered to 500 rows (5 groups of <= 2 utterances) -- the per-group h_last and row
    tables bench.py --config 5 runs (B = 64: 8 groups).  Both against csm_prefill per utterance
    (h_last within the int4 bar, the first 2 frames' codes identical) and against the oracle on the
    dequantized weights for utterances 0, 7 (last of group 1) and 8 (group 2 alone)."""
    import ctypes
    from csm_mlx import _lib
    from csm_mlx.generation import FrameCache
    from csm_mlx.models import CSM
    from csm_mlx.sampling import Sampler
    from csm_mlx.segment import Segment
    from csm_mlx.tokenizers import tokenize_segments_batch, tokenize_text_segment
    import bench
    B, frames = 9, 2
    args, w = csm_weights("1b")
    model = CSM(args, dtype="q4", max_batch=B)
    model.load_weights(w)
    _codec(3 * B)
    segs = [Segment(s % 2, prompt_ids(10_000 + 10 * g + s), bench.context_audio(g, s)) for g in range(B) for s in range(3)]
    enc = tokenize_segments_batch(segs, n_audio_codebooks=32)
    prompts = []
    for g in range(B):
        parts = enc[3 * g:3 * g + 3] + [tokenize_text_segment(prompt_ids(g), 0, 32)]
        prompts.append((np.concatenate([t for t, _ in parts]), np.concatenate([m for _, m in parts])))
    assert sum(t.shape[0] for t, _ in prompts) > 2048
    L = _lib.lib()
    D = model.backbone.args.hidden_size

    def run(mode):
        _lib.check(L.csm_set_option(model.engine, b"prefill_rows", 500 if mode == "cap500" else 0))
        cache = FrameCache(model, B, Sampler(0.0, 0), [0] * B)
        if mode == "single":
            for b, (t, m) in enumerate(prompts):
                cache.prefill(b, t, m)
        else:
            cache.prefill_batch([(b, t, m) for b, (t, m) in enumerate(prompts)])
        h = cache.debug("h_last", (B, D))
        cache.run(frames)
        hist, n, _ = cache.codes()
        return h, hist[:frames], n

    h1, c1, n1 = run("single")
    h2, c2, n2 = run("default")
    h3, c3, n3 = run("cap500")
    _lib.check(L.csm_set_option(model.engine, b"prefill_rows", 0))
    del model
    for h, c, n, tag in ((h2, c2, n2, "2 groups"), (h3, c3, n3, "5 groups")):
        err = np.abs(h - h1).max(axis=1) / np.abs(h1).max(axis=1)
        assert err.max() <= 1e-3, f"{tag}: h_last differs from per-utterance prefill ({err.max():.2e})"
        assert np.array_equal(c, c1) and np.array_equal(n, n1), f"{tag}: codes differ from per-utterance prefill"
    sel = [0, 7, 8]
    ref = oracle_batch(oracle_for(args, w, q4=True), [prompts[b] for b in sel], frames)
    for j, b in enumerate(sel):
        assert n1[b] == frames and first_divergence(c2[:, b], ref[j][0]) is None, f"utterance {b} vs oracle"
