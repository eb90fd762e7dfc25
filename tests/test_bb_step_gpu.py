"""The persistent backbone step (bb_step.hip: the 16 backbone blocks + final norm of a batch-1 bf16
decode row in ONE launch, tagged-granule hand-offs between 256 resident workgroups) against the
per-projection launch path it replaces and against the oracle.

Codes must be identical to the launch path and to the oracle (fp32-accumulation paths over the same
bf16 weights, summed in different orders); c0 logits (a function of h_last) within the bf16 bar; the
step must run for every frame, be deterministic and leave no hand-off timeout behind.  A prompt past
512 positions exercises the attention's multi-pass key loop (8 waves x 64 keys per pass)."""
import numpy as np
import pytest

from helpers import csm_weights, first_divergence, oracle_for, prompt_ids

pytestmark = pytest.mark.gpu


def _run(model, prompt, frames):
    from csm_mlx.generation import FrameCache
    from csm_mlx.sampling import Sampler
    V = model.n_audio_vocab
    Vp = (V + 7) // 8 * 8
    cache = FrameCache(model, 1, Sampler(0.0, 0), [0])
    cache.prefill(0, *prompt)
    logs = []
    for _ in range(frames):
        cache.run(1)
        logs.append(cache.debug("c0_logits", (1, Vp))[0, :V])
    hist, n, _ = cache.codes()
    return hist[: n[0], 0], logs


def _epoch(L, model):
    from csm_mlx import _lib
    ep = np.zeros(1, np.uint32)
    _lib.check(L.csm_debug_read(model.engine, b"bb_step_epoch", _lib.ptr(ep), 4, None))
    return int(ep[0])


@pytest.fixture(scope="module")
def model_1b():
    from csm_mlx.models import CSM
    args, w = csm_weights("1b")
    model = CSM(args, dtype="bf16")
    model.load_weights(w)
    yield args, w, model
    del model


def _compare(model, prompt, frames, check_oracle=None):
    from csm_mlx import _lib
    L = _lib.lib()
    _lib.check(L.csm_set_option(model.engine, b"bb_step", 0))
    ref, ref_logs = _run(model, prompt, frames)
    _lib.check(L.csm_set_option(model.engine, b"bb_step", 1))
    e0 = _epoch(L, model)
    got, got_logs = _run(model, prompt, frames)
    # the prompt prefill yields the first frame's h_last; every later frame runs one backbone step
    assert _epoch(L, model) - e0 == (frames - 1) * 80, "the persistent backbone step did not run every frame"
    assert first_divergence(got, ref) is None, f"bb_step codes differ from the launch path at {first_divergence(got, ref)}"
    for f, (a, b) in enumerate(zip(got_logs, ref_logs)):
        assert np.abs(a - b).max() <= 2e-3 * np.abs(b).max(), f"frame {f}: c0 logits differ"
    return got


def test_bb_step_matches_launch_path_and_oracle(model_1b):
    from csm_mlx.generation import generate_codes_batch
    from csm_mlx.sampling import Sampler
    from csm_mlx.tokenizers import tokenize_text_segment
    args, w, model = model_1b
    prompt = tokenize_text_segment(prompt_ids(31), 0, 32)
    got = _compare(model, prompt, 12)
    h1, n1, _ = generate_codes_batch(model, [prompt], 40, sampler=Sampler(0.0, 0))
    h2, n2, _ = generate_codes_batch(model, [prompt], 40, sampler=Sampler(0.0, 0))
    assert np.array_equal(h1, h2) and np.array_equal(n1, n2)
    assert first_divergence(h1[:12, 0], got) is None
    orc = oracle_for(args, w, bf16=True).generate_codes(*prompt, 12)
    assert first_divergence(got, orc) is None


def test_bb_step_long_context(model_1b):
    from csm_mlx.tokenizers import tokenize_text_segment
    args, w, model = model_1b
    rng = np.random.default_rng(7)
    ids = [int(t) for t in rng.integers(1000, 120000, 600)]  # 600 text rows: keys span two passes
    prompt = tokenize_text_segment(ids, 0, 32)
    _compare(model, prompt, 4)


def test_handoff_timeout_reported_by_every_frame_entry(model_1b):
    """A raised hand-off timeout flag of the persistent kernels surfaces as an error from the
    teacher-forced frame and from both halves of the processor-split frame (not only from a later
    generate): csm_frame_forced / csm_frame_c0_logits / csm_frame_finish check it."""
    from csm_mlx import _lib
    from csm_mlx.generation import FrameCache
    from csm_mlx.sampling import Sampler
    from csm_mlx.tokenizers import tokenize_text_segment
    args, w, model = model_1b
    L = _lib.lib()
    K, V = args.n_audio_codebooks, args.n_audio_vocab
    prompt = tokenize_text_segment(prompt_ids(31), 0, K)
    codes = np.ones((1, K), np.int32)
    logits = np.zeros((1, V), np.float32)
    for entry in ("forced", "c0", "finish"):
        cache = FrameCache(model, 1, Sampler(0.0, 0), [0])
        cache.prefill(0, *prompt)
        cache.run(1)                                      # the next frame starts with a backbone step
        if entry == "finish":
            _lib.check(L.csm_frame_c0_logits(model.engine, _lib.ptr(logits)))
        _lib.check(L.csm_set_option(model.engine, b"inject_handoff_error", 1))
        with pytest.raises(_lib.CsmHipError, match="hand-off wait timed out"):
            if entry == "forced":
                _lib.check(L.csm_frame_forced(model.engine, _lib.ptr(codes), None, None, None))
            elif entry == "c0":
                _lib.check(L.csm_frame_c0_logits(model.engine, _lib.ptr(logits)))
            else:
                _lib.check(L.csm_frame_finish(model.engine, _lib.ptr(logits), None))
        _lib.check(L.csm_synchronize(model.engine))       # the flag was consumed by the report


@pytest.fixture(scope="module")
def model_1b_q4():
    from csm_mlx.models import CSM
    args, w = csm_weights("1b")
    model = CSM(args, dtype="q4")
    model.load_weights(w)
    yield args, w, model
    del model


def test_bb_step_q4_matches_launch_path_and_oracle(model_1b_q4):
    """The int4 persistent backbone step (bb_step_q4_kernel: nn.quantize'd weights read as nibbles + group
    affine words, the bf16 kernel's hand-offs) against the int4 GEMV launch path on the same engine (codes
    identical, c0 logits within 2e-3 x max) and the oracle on the dequantized weights (codes), 12 frames;
    deterministic run to run."""
    from csm_mlx.generation import generate_codes_batch
    from csm_mlx.sampling import Sampler
    from csm_mlx.tokenizers import tokenize_text_segment
    args, w, model = model_1b_q4
    prompt = tokenize_text_segment(prompt_ids(31), 0, 32)
    got = _compare(model, prompt, 12)
    h1, n1, _ = generate_codes_batch(model, [prompt], 40, sampler=Sampler(0.0, 0))
    h2, n2, _ = generate_codes_batch(model, [prompt], 40, sampler=Sampler(0.0, 0))
    assert np.array_equal(h1, h2) and np.array_equal(n1, n2)
    assert first_divergence(h1[:12, 0], got) is None
    orc = oracle_for(args, w, q4=True).generate_codes(*prompt, 12)
    assert first_divergence(got, orc) is None


def test_bb_step_q4_long_context(model_1b_q4):
    from csm_mlx.tokenizers import tokenize_text_segment
    args, w, model = model_1b_q4
    rng = np.random.default_rng(7)
    prompt = tokenize_text_segment([int(t) for t in rng.integers(1000, 120000, 600)], 0, 32)
    _compare(model, prompt, 4)
