"""The persistent batched depth-decoder step (dec_step_xs.hip: the 4 decoder layers of a codebook step
>= 2 for 1..32 bf16 rows in ONE launch, flag / counter hand-offs between 256 resident workgroups, every
projection on the matrix cores) against the streaming launch path it replaces (run_dec_xs: ~20 launches
per step) and against the oracle.

Both paths compute exact fp32 products of the bf16 weights with fp32 activations and accumulate in
fp32, in different orders: greedy codes must be identical to the launch path and to the oracle, c0 / ci
logits within the bf16 bar; the step must run for every codebook step >= 2 of every frame, be
deterministic run to run, and leave no hand-off timeout behind (generation.py:72-89 at batch B)."""
import numpy as np
import pytest

from helpers import csm_weights, first_divergence, oracle_batch, oracle_for, prompt_ids

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def model_1b():
    from csm_mlx.models import CSM
    args, w = csm_weights("1b")
    model = CSM(args, dtype="bf16", max_batch=32)
    model.load_weights(w)
    yield args, w, model
    del model


def _epoch(model):
    from csm_mlx import _lib
    ep = np.zeros(1, np.uint32)
    _lib.check(_lib.lib().csm_debug_read(model.engine, b"dec_xsd_epoch", _lib.ptr(ep), 4, None))
    return int(ep[0])


def _run(model, prompts, frames, sampler):
    from csm_mlx.generation import FrameCache
    K, V = model.n_audio_codebooks, model.n_audio_vocab
    Vp = (V + 7) // 8 * 8
    B = len(prompts)
    cache = FrameCache(model, B, sampler, [1234 + b for b in range(B)])
    for b, (t, m) in enumerate(prompts):
        cache.prefill(b, t, m)
    logs = []
    for _ in range(frames):
        cache.run(1)
        logs.append(cache.debug("ci_logits", (K - 1, B, Vp))[:, :, :V])
    hist, n, _ = cache.codes()
    return hist, n, logs


def _ab(model, prompts, frames, sampler):
    from csm_mlx import _lib
    L = _lib.lib()
    _lib.check(L.csm_set_option(model.engine, b"dec_xsd", 0))
    ref = _run(model, prompts, frames, sampler)
    _lib.check(L.csm_set_option(model.engine, b"dec_xsd", 1))
    e0 = _epoch(model)
    got = _run(model, prompts, frames, sampler)
    K = model.n_audio_codebooks
    assert _epoch(model) - e0 == frames * (K - 2), "the persistent step did not run every codebook step >= 2"
    _lib.check(L.csm_synchronize(model.engine))
    return ref, got


@pytest.mark.parametrize("B", [8, 19, 32])
def test_dec_xsd_matches_launch_path_greedy(model_1b, B):
    """B = 8 (the smallest batch on the streaming path), 19 (rows 19..31 of the tile idle), 32 (a full
    tile: configs[3]'s per-GPU shard): 5 frames, codes identical, ci logits within 2e-3 x max."""
    from csm_mlx.sampling import Sampler
    from csm_mlx.tokenizers import tokenize_text_segment
    args, w, model = model_1b
    prompts = [tokenize_text_segment(prompt_ids(500 + b, 10 + b % 3), 0, args.n_audio_codebooks) for b in range(B)]
    (rh, rn, rl), (gh, gn, gl) = _ab(model, prompts, 5, Sampler(0.0, 0))
    assert np.array_equal(rn, gn)
    for b in range(B):
        d = first_divergence(gh[: gn[b], b], rh[: rn[b], b])
        assert d is None, f"utterance {b}: codes differ from the launch path at frame {d}"
    for f, (a, r) in enumerate(zip(gl, rl)):
        err = np.abs(a - r).max(axis=-1)
        tol = 2e-3 * np.abs(r).max(axis=-1)
        assert (err <= tol).all(), f"frame {f}: ci logits differ (max {err.max():.3e})"


def test_dec_xsd_matches_oracle_and_is_deterministic(model_1b):
    """B = 32 greedy, 4 frames: every utterance bit-exact against the oracle (bf16-rounded weights, fp32
    activations); a second run gives identical codes."""
    from csm_mlx.generation import generate_codes_batch
    from csm_mlx.sampling import Sampler
    from csm_mlx.tokenizers import tokenize_text_segment
    args, w, model = model_1b
    B = 32
    prompts = [tokenize_text_segment(prompt_ids(600 + b, 10 + b % 3), 0, args.n_audio_codebooks) for b in range(B)]
    h1, n1, _ = generate_codes_batch(model, prompts, 4, sampler=Sampler(0.0, 0))
    h2, n2, _ = generate_codes_batch(model, prompts, 4, sampler=Sampler(0.0, 0))
    assert np.array_equal(h1, h2) and np.array_equal(n1, n2)
    ref = oracle_batch(oracle_for(args, w, bf16=True), prompts, 4)
    for b in range(B):
        want = ref[b][0] if isinstance(ref[b], tuple) else ref[b]
        d = first_divergence(h1[: n1[b], b], want)
        assert d is None and n1[b] == len(want), f"utterance {b}: first divergence {d}"


def test_dec_xsd_sampled_matches_launch_path(model_1b):
    """configs[2]'s sampler (temperature 0.8, top-k 50) at B = 32: the head and sample_kernel stay launches
    after the persistent step, the step reads the sampler's single published code per row; 4 frames,
    codes identical to the launch path."""
    from csm_mlx.sampling import Sampler
    from csm_mlx.tokenizers import tokenize_text_segment
    args, w, model = model_1b
    B = 32
    prompts = [tokenize_text_segment(prompt_ids(700 + b, 10 + b % 3), 0, args.n_audio_codebooks) for b in range(B)]
    (rh, rn, _), (gh, gn, _) = _ab(model, prompts, 4, Sampler(0.8, 50))
    assert np.array_equal(rn, gn)
    for b in range(B):
        d = first_divergence(gh[: gn[b], b], rh[: rn[b], b])
        assert d is None, f"utterance {b}: sampled codes differ from the launch path at frame {d}"


@pytest.fixture(scope="module")
def model_1b_q4():
    from csm_mlx.models import CSM
    args, w = csm_weights("1b")
    model = CSM(args, dtype="q4", max_batch=64)
    model.load_weights(w)
    yield args, w, model
    del model


@pytest.mark.parametrize("B", [8, 40, 64])
def test_dec_xsd_q4_matches_launch_path_and_oracle(model_1b_q4, B):
    """The int4 kernel (nn.quantize'd decoder, two 32-row tiles: configs[4]'s B = 64): nibbles as exact
    bf16 operands, the per-group scale / bias fold over the producers' half-group sums.  4 frames greedy:
    codes identical to the launch path and to the oracle on the dequantized weights, ci logits within
    1e-3 x max of the launch path."""
    from csm_mlx.sampling import Sampler
    from csm_mlx.tokenizers import tokenize_text_segment
    args, w, model = model_1b_q4
    prompts = [tokenize_text_segment(prompt_ids(800 + b, 10 + b % 3), 0, args.n_audio_codebooks) for b in range(B)]
    (rh, rn, rl), (gh, gn, gl) = _ab(model, prompts, 4, Sampler(0.0, 0))
    assert np.array_equal(rn, gn)
    for b in range(B):
        d = first_divergence(gh[: gn[b], b], rh[: rn[b], b])
        assert d is None, f"utterance {b}: codes differ from the launch path at frame {d}"
    for f, (a, r) in enumerate(zip(gl, rl)):
        err = np.abs(a - r).max(axis=-1)
        assert (err <= 1e-3 * np.abs(r).max(axis=-1)).all(), f"frame {f}: ci logits differ (max {err.max():.3e})"
    if B == 64:
        ref = oracle_batch(oracle_for(args, w, q4=True), prompts, 4)
        for b in range(B):
            d = first_divergence(gh[: gn[b], b], ref[b][0])
            assert d is None and gn[b] == len(ref[b][0]), f"utterance {b}: first divergence {d} vs the oracle"


def test_dec_xsd_timeout_reported_and_recovered(model_1b):
    """A raised hand-off timeout flag: every wait of the step kernel gives up (bounded spins, the grid
    drains), the frame raises, and the flags / tickets / epoch are reset so the next frames are exact
    again (codes identical to the launch path)."""
    from csm_mlx import _lib
    from csm_mlx.sampling import Sampler
    from csm_mlx.tokenizers import tokenize_text_segment
    args, w, model = model_1b
    L = _lib.lib()
    B = 16
    prompts = [tokenize_text_segment(prompt_ids(900 + b, 10 + b % 3), 0, args.n_audio_codebooks) for b in range(B)]
    _lib.check(L.csm_set_option(model.engine, b"dec_xsd", 1))
    _lib.check(L.csm_set_option(model.engine, b"inject_handoff_error", 1))
    with pytest.raises(_lib.CsmHipError, match="hand-off wait timed out"):
        _run(model, prompts, 2, Sampler(0.0, 0))
    _lib.check(L.csm_synchronize(model.engine))
    (rh, rn, _), (gh, gn, _) = _ab(model, prompts, 3, Sampler(0.0, 0))
    assert np.array_equal(rn, gn)
    for b in range(B):
        assert first_divergence(gh[: gn[b], b], rh[: rn[b], b]) is None, f"utterance {b} after the reset"


@pytest.mark.parametrize("B", [32, 64])
def test_dec_xsd_in_launch_sampler_matches_sample_kernel(model_1b_q4, B):
    """Sampled steps (temperature 0.8, top-k 50) with the sampler inside the step's launch (role_s: the
    radix-select threshold and Gumbel-max of sample_kernel on 512 threads) against the same kernel with
    sample_kernel launched after it (option dec_xsd_sample 0): 4 frames of int4 rows, codes identical."""
    from csm_mlx import _lib
    from csm_mlx.sampling import Sampler
    from csm_mlx.tokenizers import tokenize_text_segment
    args, w, model = model_1b_q4
    L = _lib.lib()
    prompts = [tokenize_text_segment(prompt_ids(950 + b, 10 + b % 3), 0, args.n_audio_codebooks) for b in range(B)]
    _lib.check(L.csm_set_option(model.engine, b"dec_xsd", 1))
    _lib.check(L.csm_set_option(model.engine, b"dec_xsd_sample", 0))
    ref = _run(model, prompts, 4, Sampler(0.8, 50))
    _lib.check(L.csm_set_option(model.engine, b"dec_xsd_sample", 1))
    got = _run(model, prompts, 4, Sampler(0.8, 50))
    _lib.check(L.csm_synchronize(model.engine))
    assert np.array_equal(ref[1], got[1])
    for b in range(B):
        d = first_divergence(got[0][: got[1][b], b], ref[0][: ref[1][b], b])
        assert d is None, f"utterance {b}: in-launch sampled codes differ at frame {d}"
