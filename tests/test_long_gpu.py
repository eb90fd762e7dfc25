"""GPU parity past one 64-key attention chunk, against committed oracle fixtures
(tests/golden/make_golden.py):

* configs[1] at full length -- csm_1b B = 1 greedy, 125 frames from the 14-row prompt, so the
  backbone attention reaches S = 139 keys (three chunks of the online-softmax loop, the clamped
  prefetch of the last one) -- fp32 weights and bf16 weights, through the graph-replayed frame loop;
* a tiny model with a 236-row prompt (text / 100 audio rows / text / 100 audio rows / text): a
  multi-chunk prefill (236 rows at once) and decode at S = 236..275;
* configs[0] plumbing -- ``generate()`` of the (unverified) "[0]Hello from Sesame." ids, 10 s,
  greedy, then Mimi decode to PCM, against the oracle's codes and the Mimi oracle's waveform.

Greedy codes bit-exact; logits within 2e-4 (fp32) / 2e-3 (bf16) x max|logit|; waveform <= 1e-4 RMS.
"""
import os

import numpy as np
import pytest

from helpers import csm_weights, first_divergence

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _fixture(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def _model(args, w, dtype):
    from csm_mlx.models import CSM
    m = CSM(args, dtype=dtype, max_batch=1)
    m.load_weights(w)
    return m


def _run_collect(model, tokens, mask, n_frames, keep, ci_cbs=None):
    """Frame loop (one graph replay per frame) with the logits of frames ``keep`` read back."""
    from csm_mlx.generation import FrameCache
    from csm_mlx.sampling import Sampler
    K, V = model.n_audio_codebooks, model.n_audio_vocab
    Vp = (V + 7) // 8 * 8
    cache = FrameCache(model, 1, Sampler(0.0, 0), [0])
    cache.prefill(0, tokens, mask)
    c0s, cis = [], []
    for f in range(n_frames):
        cache.run(1)
        if f in keep:
            c0s.append(cache.debug("c0_logits", (1, Vp))[0, :V])
            ci = cache.debug("ci_logits", (K - 1, 1, Vp))[:, 0, :V]
            cis.append(ci if ci_cbs is None else ci[[c - 1 for c in ci_cbs]])
    hist, n, _ = cache.codes()
    return hist[: n[0], 0], np.stack(c0s), np.stack(cis)


def _check(codes, c0, ci, ref_codes, ref_c0, ref_ci, rtol):
    div = first_divergence(codes, ref_codes)
    assert div is None, f"codes diverge at frame {div}: {codes[div]} vs {ref_codes[div]}"
    assert len(codes) == len(ref_codes)
    for i in range(len(ref_c0)):
        for got, want in ((c0[i], ref_c0[i]), (ci[i], ref_ci[i])):
            err = np.abs(got - want).max()
            assert err <= rtol * np.abs(want).max(), f"kept frame #{i}: logits err {err:.3e}"


@pytest.mark.parametrize("dtype", ["float32", "bf16"])
def test_csm_1b_125_frames_vs_fixture(dtype):
    from csm_mlx.tokenizers import tokenize_text_segment
    z = _fixture("csm_1b_greedy_125.npz")
    tag = "fp32" if dtype == "float32" else "bf16"
    args, w = csm_weights("1b")
    model = _model(args, w, dtype)
    t, m = tokenize_text_segment(z["ids"].tolist(), 0, 32)
    codes, c0, ci = _run_collect(model, t, m, 125, set(z["frames"].tolist()), z["ci_codebooks"].tolist())
    _check(codes, c0, ci, z[f"{tag}_codes"], z[f"{tag}_c0"], z[f"{tag}_ci"], 2e-4 if tag == "fp32" else 2e-3)
    del model


@pytest.mark.parametrize("dtype", ["float32", "bf16"])
def test_tiny_long_prompt_vs_fixture(dtype):
    z = _fixture("tiny_long_prompt.npz")
    tag = "fp32" if dtype == "float32" else "bf16"
    assert z["tokens"].shape[0] >= 200
    args, w = csm_weights("tiny")
    model = _model(args, w, dtype)
    codes, c0, ci = _run_collect(model, z["tokens"], z["mask"], 40, set(z["frames"].tolist()))
    _check(codes, c0, ci, z[f"{tag}_codes"], z[f"{tag}_c0"], z[f"{tag}_ci"], 2e-4 if tag == "fp32" else 2e-3)
    del model


def test_config0_generate_plumbing():
    """configs[0]: generate(csm, "[0]Hello from Sesame." (fixture ids), 0, [], 10000, temperature=0)
    -> codes of all 125 frames == the oracle's; PCM == the Mimi oracle's decode of them."""
    from csm_mlx.config import MIMI_CONFIGURATION
    from csm_mlx.generation import generate, generate_codes_batch
    from csm_mlx.mimi import MimiCodec
    from csm_mlx.sampling import Sampler
    from csm_mlx.tokenizers import set_audio_tokenizer, tokenize_text_segment
    from csm_mlx.weights import synthetic_mimi_weights
    from oracle.mimi_oracle import OracleMimi
    z = _fixture("config0_plumbing.npz")
    args, w = csm_weights("1b")
    model = _model(args, w, "float32")
    mc = MIMI_CONFIGURATION["mimi_202407"]
    mw = synthetic_mimi_weights(mc, 0)
    codec = MimiCodec(mc, max_batch=1)
    codec.load_weights(mw)
    set_audio_tokenizer(codec, 32)
    ids = z["ids"].tolist()
    hist, n, _ = generate_codes_batch(model, [tokenize_text_segment(ids, 0, 32)], 125, sampler=Sampler(0.0, 0))
    assert n[0] == len(z["codes"]) == 125
    assert first_divergence(hist[:125, 0], z["codes"]) is None
    audio = generate(model, ids, 0, [], 10_000, temperature=0.0)
    assert audio.shape == (int(z["n_samples"]),) == (125 * 1920,) and audio.dtype == np.float32
    ref = OracleMimi(mc, mw).decode(np.ascontiguousarray(z["codes"].T[None]))[0, 0]
    np.testing.assert_allclose(ref[:1920], z["pcm_head"], rtol=0, atol=1e-6)   # the oracle is pinned too
    rms = float(np.sqrt(np.mean((audio.astype(np.float64) - ref) ** 2)))
    assert rms <= 1e-4, f"waveform RMS error {rms:.3e}"
    del model


def test_csm_1b_q4_stream_generate_125_frames():
    """The reference demo's path (run_streaming_csm_mlx.py:811-818, :844-852): nn.quantize(model, 64, 4), then
    stream_generate -- here csm_1b int4 g64 at B = 1, configs[1]'s utterance, greedy, 10 s -- against
    tests/golden/csm_1b_q4_stream_125.npz (the oracle on the dequantized weights + the Mimi oracle's decode_step):
    codes bit-exact over all 125 frames (the fixture stores every code's top-2 margin; none may part), c0 / ci
    logits at frames 0 / 64 / 124 within 1e-3 x max|logit| (read from a frame-loop run of the same engine),
    every streamed chunk's RMS / mean / projections within what 1e-4 RMS allows, whole chunks <= 1e-4 RMS."""
    from csm_mlx import nn, stream_generate
    from csm_mlx.config import MIMI_CONFIGURATION
    from csm_mlx.mimi import MimiCodec
    from csm_mlx.tokenizers import set_audio_tokenizer, tokenize_text_segment
    from csm_mlx.weights import synthetic_mimi_weights
    z = _fixture("csm_1b_q4_stream_125.npz")
    from csm_mlx.models import CSM
    args, w = csm_weights("1b")
    model = CSM(args, dtype="bf16", max_batch=1)
    nn.quantize(model, group_size=64, bits=4)      # before the load: the fp32 weights quantize on the device,
    model.load_weights(w)                          # as the oracle's quantize -> dequantize of the same weights
    mc = MIMI_CONFIGURATION["mimi_202407"]
    codec = MimiCodec(mc, max_batch=1)
    codec.load_weights(synthetic_mimi_weights(mc, 0))
    set_audio_tokenizer(codec, 32)
    ids = z["ids"].tolist()
    chunks = [np.asarray(c, np.float32) for c in stream_generate(model, ids, 0, [], 10_000, temperature=0.0)]
    t, m = tokenize_text_segment(ids, 0, 32)
    codes, c0, ci = _run_collect(model, t, m, 125, set(z["frames"].tolist()), z["ci_codebooks"].tolist())
    del model
    _check(codes, c0, ci, z["codes"], z["c0"], z["ci"], 1e-3)
    assert len(chunks) == len(z["codes"]) == 125
    bad = []
    for f, y in enumerate(chunks):
        y = y.astype(np.float64)
        if abs(np.sqrt(np.mean(y ** 2)) - z["rms"][f]) > 1e-4 or abs(y.mean() - z["mean"][f]) > 1e-4 or \
                np.abs(y @ z["proj_vec"].T - z["proj"][f]).max() > 1e-4 * np.sqrt(1920):
            bad.append(f)
    for f, ref in zip(z["pcm_frames"], z["pcm"]):
        err = float(np.sqrt(np.mean((chunks[int(f)].astype(np.float64) - ref) ** 2)))
        if err > 1e-4:
            bad.append((int(f), err))
    assert not bad, f"streamed chunks off the Mimi oracle: {bad[:10]}"
