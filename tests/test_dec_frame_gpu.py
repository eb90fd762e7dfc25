"""The persistent frame decoder (dec_frame.hip: codebook0_head + the 31 depth-decoder steps of a
batch-1 greedy bf16 frame in ONE launch, tagged-granule hand-offs between 256 resident workgroups)
against the per-projection launch path it replaces and against the oracle.

Codes must be identical to the launch path and to the oracle (both are fp32-accumulation paths over
the same bf16 weights); logits within the bf16 bar; the decoder must be deterministic run to run and
leave no hand-off timeout behind.  (tests/test_long_gpu.py's 125-frame bf16 fixture runs on it too.)"""
import numpy as np
import pytest

from helpers import csm_weights, first_divergence, oracle_for, prompt_ids

pytestmark = pytest.mark.gpu


def _run(model, prompt, frames):
    from csm_mlx.generation import FrameCache
    from csm_mlx.sampling import Sampler
    V, K = model.n_audio_vocab, model.n_audio_codebooks
    Vp = (V + 7) // 8 * 8
    cache = FrameCache(model, 1, Sampler(0.0, 0), [0])
    cache.prefill(0, *prompt)
    logs = []
    for _ in range(frames):
        cache.run(1)
        logs.append((cache.debug("c0_logits", (1, Vp))[0, :V], cache.debug("ci_logits", (K - 1, 1, Vp))[:, 0, :V]))
    hist, n, _ = cache.codes()
    return hist[: n[0], 0], logs


@pytest.mark.parametrize("dtype", ["bf16", "q4"])
def test_dec_frame_matches_launch_path_and_oracle(dtype):
    """q4: dec_frame_kernel<true> (an nn.quantize'd engine: int4 nibbles + group affine words for every
    decoder projection, codebook0_head and the projection; audio_head bf16) against the int4 GEMV launch
    path and the oracle on the dequantized weights."""
    from csm_mlx import _lib
    from csm_mlx.generation import generate_codes_batch
    from csm_mlx.models import CSM
    from csm_mlx.sampling import Sampler
    from csm_mlx.tokenizers import tokenize_text_segment
    args, w = csm_weights("1b")
    model = CSM(args, dtype=dtype)
    model.load_weights(w)
    L = _lib.lib()
    prompt = tokenize_text_segment(prompt_ids(31), 0, 32)
    _lib.check(L.csm_set_option(model.engine, b"dec_frame", 0))
    ref, ref_logs = _run(model, prompt, 12)
    _lib.check(L.csm_set_option(model.engine, b"dec_frame", 1))
    ep0 = np.zeros(1, np.uint32)
    _lib.check(L.csm_debug_read(model.engine, b"dec_frame_epoch", _lib.ptr(ep0), 4, None))
    got, got_logs = _run(model, prompt, 12)
    ep1 = np.zeros(1, np.uint32)
    _lib.check(L.csm_debug_read(model.engine, b"dec_frame_epoch", _lib.ptr(ep1), 4, None))
    assert int(ep1[0]) - int(ep0[0]) == 12 * 498, "the persistent frame decoder did not run every frame"
    assert first_divergence(got, ref) is None, f"dec_frame codes differ from the launch path at {first_divergence(got, ref)}"
    for f, ((c0a, cia), (c0b, cib)) in enumerate(zip(got_logs, ref_logs)):
        for a, b in ((c0a, c0b), (cia, cib)):
            assert np.abs(a - b).max() <= 2e-3 * np.abs(b).max(), f"frame {f}: logits differ"
    # deterministic, graph-replayed multi-frame loop (csm_run_frames of 16 frames per call)
    h1, n1, _ = generate_codes_batch(model, [prompt], 40, sampler=Sampler(0.0, 0))
    h2, n2, _ = generate_codes_batch(model, [prompt], 40, sampler=Sampler(0.0, 0))
    assert np.array_equal(h1, h2) and np.array_equal(n1, n2)
    assert first_divergence(h1[:12, 0], got) is None
    orc = oracle_for(args, w, bf16=(dtype == "bf16"), q4=(dtype == "q4")).generate_codes(*prompt, 12)
    assert first_divergence(got, orc) is None
    del model


@pytest.mark.parametrize("top_k,dtype", [(0, "bf16"), (50, "bf16"), (0, "q4"), (50, "q4")])
def test_dec_frame_sampled_matches_launch_path_and_oracle(top_k, dtype):
    """The reference's default sampler (temperature 0.8, generation.py:102, :51-54; top_k 0) and
    config 3's top-k 50 at batch 1 on the persistent frame decoder: every head hands all its logits
    to every workgroup, which runs sample_kernel's top-k radix select + Gumbel-max.  12 frames: codes
    identical to the launch path (sample_kernel) and to the oracle's restatement of the counter-based
    RNG; the decoder ran every frame (same 498 hand-offs as greedy)."""
    from csm_mlx import _lib
    from csm_mlx.generation import FrameCache, generate_codes_batch
    from csm_mlx.models import CSM
    from csm_mlx.sampling import Sampler
    from csm_mlx.tokenizers import tokenize_text_segment
    args, w = csm_weights("1b")
    model = CSM(args, dtype=dtype)
    model.load_weights(w)
    L = _lib.lib()
    prompt = tokenize_text_segment(prompt_ids(33), 0, 32)
    smp, seed, frames = Sampler(0.8, top_k), 4242, 12

    def run():
        h, n, _ = generate_codes_batch(model, [prompt], frames, sampler=smp, seeds=[seed])
        return h[: n[0], 0].copy()
    _lib.check(L.csm_set_option(model.engine, b"dec_frame", 0))
    ref = run()
    _lib.check(L.csm_set_option(model.engine, b"dec_frame", 1))
    ep0 = np.zeros(1, np.uint32)
    _lib.check(L.csm_debug_read(model.engine, b"dec_frame_epoch", _lib.ptr(ep0), 4, None))
    got = run()
    ep1 = np.zeros(1, np.uint32)
    _lib.check(L.csm_debug_read(model.engine, b"dec_frame_epoch", _lib.ptr(ep1), 4, None))
    assert int(ep1[0]) - int(ep0[0]) == frames * 498, "the persistent frame decoder did not run every sampled frame"
    assert len(got) == frames and first_divergence(got, ref) is None, \
        f"sampled dec_frame codes differ from the launch path at {first_divergence(got, ref)}"
    assert np.array_equal(run(), got)                                     # deterministic per seed
    orc = oracle_for(args, w, bf16=(dtype == "bf16"), q4=(dtype == "q4")).generate_codes(
        *prompt, frames, temperature=0.8, top_k=top_k, seed=seed)
    assert first_divergence(got, orc) is None
    del model


