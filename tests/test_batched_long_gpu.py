"""Batched configs at full length against committed oracle fixtures (tests/golden/make_golden.py):

* configs[3]'s per-GPU shard -- csm_1b bf16 B = 32 greedy, all 125 frames (the backbone's batched
  attention past one 64-key chunk), codes of every utterance up to its EOS, c0 logits and the ci logits
  of codebooks 1 / 16 / 31 at frames 0 / 64 / 100 / 124 for four utterances that run all 125 frames,
  and the c0 logits of each early utterance's EOS frame;
* configs[2] -- B = 32, temperature 0.8, top-k 50, ``stream_generate_batch`` over all 125 frames: codes
  (the oracle's restatement of the engine's counter-based RNG) and, per (utterance, frame) before its
  EOS, the streamed chunk's RMS, mean and projections on four seeded unit vectors against the Mimi
  oracle's ``decode_step``, plus whole chunks (utterance 0's first 8, each ending utterance's last 4
  before its EOS frame).

* configs[4] -- csm_1b int4 B = 64 with Mimi-encoded 3-segment contexts (248-row prompts), 125 greedy
  frames from the GPU-encoded prompts, utterances 0-7 and 56-63 against the oracle on the dequantized weights
  (plain seed-0 weights: no early EOS).

The first two run on the EOS-capable rig of the seed-0 weights (tests/helpers.py eos_rig), so utterances end at
different frames (per-utterance EOS at B > 1, generation.py:139-161).  Bars: codes and frame counts
bit-exact; logits within 2e-3 x max|logit|; chunks within 1e-4 RMS (statistics: within what a 1e-4
RMS error allows)."""
import os

import numpy as np
import pytest

from helpers import eos_weights, first_divergence

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NEAR_TIE = 1e-5   # oracle top-2 logit margin / max|logit| below which a code is a tie at fp32 resolution


def _fixture(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def _prompts():
    from csm_mlx.tokenizers import tokenize_text_segment
    from helpers import prompt_ids
    return [tokenize_text_segment(prompt_ids(1 if g == 0 else 1000 + g), 0, 32) for g in range(32)]


def _model(args, w, B):
    from csm_mlx.models import CSM
    m = CSM(args, dtype="bf16", max_batch=B)
    m.load_weights(w)
    return m


def _check_codes(hist, n, z):
    ref_n = z["n_frames"]
    assert (ref_n < z["codes"].shape[1]).any(), "the fixture has no utterance that ends early"
    bad = []
    for b in range(len(ref_n)):
        want = z["codes"][b, : ref_n[b]]
        got = hist[: n[b], b]
        div = first_divergence(got, want)
        if div is not None or n[b] != ref_n[b]:
            bad.append(f"utterance {b}: {n[b]} vs {ref_n[b]} frames, first divergence {div}")
    assert not bad, "; ".join(bad)


def test_config4_shard_b32_greedy_125_frames():
    from csm_mlx.generation import FrameCache
    from csm_mlx.sampling import Sampler
    z = _fixture("config4_b32_greedy_125.npz")
    args, w = eos_weights("1b")
    B, K, V = 32, args.n_audio_codebooks, args.n_audio_vocab
    Vp = (V + 7) // 8 * 8
    model = _model(args, w, B)
    cache = FrameCache(model, B, Sampler(0.0, 0), [0] * B)
    cache.prefill_batch([(b, t, m) for b, (t, m) in enumerate(_prompts())])
    keep = {int(f): i for i, f in enumerate(z["frames"])}
    ref_n = z["n_frames"]
    eos_at = {int(ref_n[b]): [] for b in z["eos_utts"]}
    for b in z["eos_utts"]:
        eos_at[int(ref_n[b])].append(int(b))
    cis = [c - 1 for c in z["ci_codebooks"]]
    errs = []
    for f in range(125):
        cache.run(1)
        if f in keep or f in eos_at:
            c0 = cache.debug("c0_logits", (B, Vp))[:, :V]
        if f in keep:
            ci = cache.debug("ci_logits", (K - 1, B, Vp))[:, :, :V]
            i = keep[f]
            for j, b in enumerate(z["logit_utts"]):            # (utterances that run all 125 frames)
                for got, want in ((c0[b], z["c0"][i, j]), (ci[cis, b], z["ci"][i, j])):
                    err = float(np.abs(got - want).max())
                    if err > 2e-3 * float(np.abs(want).max()):
                        errs.append(f"frame {f} utterance {b}: logits err {err:.3e}")
        for b in eos_at.get(f, []):
            j = list(z["eos_utts"]).index(b)
            err = float(np.abs(c0[b] - z["eos_c0"][j]).max())
            if err > 2e-3 * float(np.abs(z["eos_c0"][j]).max()):
                errs.append(f"EOS frame {f} utterance {b}: c0 logits err {err:.3e}")
    hist, n, _ = cache.codes()
    del model
    _check_codes(hist, n, z)
    assert not errs, "; ".join(errs[:10])


def test_config3_stream_b32_sampled_64_frames():
    from csm_mlx.generation import stream_generate_batch
    from test_configs_gpu import _codec, _engine_codes
    z = _fixture("config3_b32_stream_125.npz")
    args, w = eos_weights("1b")
    B, frames = 32, int(z["codes"].shape[1])
    model = _model(args, w, B)
    _codec(B)
    chunks = [pcm.copy() for pcm, _ in stream_generate_batch(model, _prompts(), frames * 80, temperature=0.8,
                                                             top_k=50, seeds=[1234 + g for g in range(B)])]
    hist, n = _engine_codes(model, B)
    del model
    _check_codes(hist, n, z)
    ref_n = z["n_frames"]
    assert len(chunks) >= int(ref_n.max())
    vec = z["proj_vec"]
    bad = []
    for f in range(int(ref_n.max())):
        y = chunks[f].astype(np.float64)
        for b in range(B):
            if f >= ref_n[b]:
                continue
            rms = float(np.sqrt(np.mean(y[b] ** 2)))
            if abs(rms - z["rms"][b, f]) > 1e-4 or abs(float(y[b].mean()) - z["mean"][b, f]) > 1e-4 or \
                    np.abs(y[b] @ vec.T - z["proj"][b, f]).max() > 1e-4 * np.sqrt(1920):
                bad.append(f"utterance {b} frame {f}")
    for b in z["pcm_utts"]:
        ref, st = z[f"pcm_{b}"], int(z[f"pcm_start_{b}"])
        got = np.stack([chunks[st + f][b] for f in range(len(ref))]) if len(ref) else ref
        err = float(np.sqrt(np.mean((got.astype(np.float64) - ref) ** 2))) if len(ref) else 0.0
        if err > 1e-4:
            bad.append(f"utterance {b}: chunk RMS error {err:.3e}")
    assert not bad, "; ".join(bad[:10])


# Codes where the engine, summing the same fp32 products in another order, takes the other side of an oracle
# top-2 logit near-tie: an exact allow-list of (utterance, frame, codebook), each also required to carry a stored
# oracle margin < NEAR_TIE.  Any other divergence fails.
C5_FRAME_TIES = set()


def _c5_expected(z, u, gpu_tokens):
    """The fixture run the GPU-encoded prompt of pinned utterance u must be compared with: the oracle's prompt,
    or -- where the GPU encode took the other side of a context RVQ near-tie (oracle margin < rvq_tie) -- the
    fixture's variant prompt for exactly that code.  Returns (codes, n_frames, margins, flip or None)."""
    if np.array_equal(gpu_tokens, z["tokens"][u]):
        return z["codes"][u], int(z["n_frames"][u]), z["margin"][u], None
    for v in np.nonzero(z["var_of"][:, 0] == u)[0]:
        if np.array_equal(gpu_tokens, z["var_tokens"][v]):
            flip = tuple(int(x) for x in z["var_of"][v]) + (float(z["var_margin"][v]),)
            assert flip[-1] < float(z["rvq_tie"])
            return z["var_codes"][v], int(z["var_n_frames"][v]), z["var_frame_margin"][v], flip
    rows = np.unique(np.argwhere(gpu_tokens != z["tokens"][u])[:, 0]).tolist()
    listed = [tuple(int(x) for x in r) + (float(m),) for r, m in zip(z["rvq_near"], z["rvq_near_margin"]) if r[0] == u]
    raise AssertionError(f"pinned utterance {int(z['utts'][u])}: the GPU-encoded prompt differs from the oracle's at rows "
                         f"{rows} and matches no near-tie variant (context codes with RVQ margin < 1e-5: {listed})")


def test_config5_q4_b64_greedy_125_frames():
    """configs[4] at full length: B = 64 int4 (nn.quantize) prompts of 3 Mimi-encoded context Segments (the GPU
    codec, as bench.py --config 5) + the text row, 248 rows each through csm_prefill_batch (the matrix-core
    prefill and its attention), 125 greedy frames FROM THE GPU-ENCODED PROMPTS.  16 utterances -- 0-7 and 56-63,
    both 32-row tiles of the 64-row int4 GEMMs -- against tests/golden/config5_q4_b16_greedy_125.npz (the codec
    and CSM oracles on the dequantized weights):

    * every GPU-encoded prompt equals the oracle's, or -- only at a context code whose oracle RVQ margin is below
      the fixture's rvq_tie (3e-6 of the latent: the oracle's own latents move 1.2-1.4e-6 between two BLAS call
      shapes) -- the fixture's variant prompt that takes the runner-up code there (the oracle's other outcome,
      with its own 125 frames);
    * codes and frame counts bit-exact against the matching oracle run, except at the (utterance, frame,
      codebook) codes of C5_FRAME_TIES, each of which must carry an oracle top-2 logit margin < NEAR_TIE (then
      that utterance is compared up to it);
    * c0 / ci logits of the first and last pinned utterance at frames 0 / 64 / 124 within 1e-3 x max|logit|
      (the int4 bar of test_gemm_gpu.py) where that utterance's prompt is the oracle's."""
    import bench
    from csm_mlx.generation import FrameCache
    from csm_mlx.models import CSM
    from csm_mlx.sampling import Sampler
    from helpers import csm_weights
    from test_configs_gpu import _codec
    z = _fixture("config5_q4_b16_greedy_125.npz")
    args, w = csm_weights("1b")
    B, K, V = 64, args.n_audio_codebooks, args.n_audio_vocab
    Vp = (V + 7) // 8 * 8
    model = CSM(args, dtype="q4", max_batch=B)
    model.load_weights(w)
    _codec(3 * B)
    mine = list(range(B))
    prompts = bench.context_prompts(mine, bench.context_segments(mine))
    utts = [int(g) for g in z["utts"]]
    exp, flips = {}, []
    for u, g in enumerate(utts):
        assert np.array_equal(prompts[g][1], z["masks"][u]), f"utterance {g}: prompt masks differ"
        assert np.array_equal(prompts[g][0][:, K], z["tokens"][u][:, K]), f"utterance {g}: text rows differ"
        exp[g] = _c5_expected(z, u, prompts[g][0])
        if exp[g][3] is not None:
            flips.append((g,) + exp[g][3][1:])
    print("config 5 context codes the GPU encode takes at an RVQ near-tie (utterance, segment, codebook, frame, "
          "oracle margin):", flips, flush=True)
    cache = FrameCache(model, B, Sampler(0.0, 0), [0] * B)
    cache.prefill_batch([(b, t, m) for b, (t, m) in enumerate(prompts)])
    keep = {int(f): i for i, f in enumerate(z["frames"])}
    logit_utts = [(j, utts[int(u)]) for j, u in enumerate(z["logit_utts"]) if exp[utts[int(u)]][3] is None]
    assert logit_utts, "no logit utterance ran the oracle's own prompt"
    cis = [c - 1 for c in z["ci_codebooks"]]
    errs = []
    for f in range(125):
        cache.run(1)
        if f in keep:
            c0 = cache.debug("c0_logits", (B, Vp))[:, :V]
            ci = cache.debug("ci_logits", (K - 1, B, Vp))[:, :, :V]
            for j, g in logit_utts:
                for got, want in ((c0[g], z["c0"][j, keep[f]]), (ci[cis, g], z["ci"][j, keep[f]])):
                    err = float(np.abs(got - want).max())
                    if err > 1e-3 * float(np.abs(want).max()):
                        errs.append(f"frame {f} utterance {g}: logits err {err:.3e}")
    hist, n, _ = cache.codes()
    del model
    bad, ties = [], []
    for g in utts:
        codes, nb, margin, _ = exp[g]
        div = first_divergence(hist[: n[g], g], codes[:nb])
        if div is None and n[g] == nb:
            continue
        if div is not None and div < min(n[g], nb):
            k = int(np.argmax(hist[div, g] != codes[div]))
            ties.append((g, div, k, float(margin[div, k])))
            if (g, div, k) in C5_FRAME_TIES and margin[div, k] < NEAR_TIE:
                continue
        bad.append(f"utterance {g}: {n[g]} vs {nb} frames, first divergence {div}" +
                   (f" (codebook {ties[-1][2]}, oracle margin {ties[-1][3]:.2e})" if ties and ties[-1][0] == g else ""))
    print("config 5 codes that part from the oracle (utterance, frame, codebook, oracle margin):", ties, flush=True)
    assert not bad, "; ".join(bad)
    assert not errs, "; ".join(errs[:10])


def test_generate_loop_polls_eos_one_chunk_behind():
    """generate_codes_batch's frame loop (csm_run_frames_ahead: each chunk enqueued before the previous
    chunk's EOS poll returns) on the config-4 fixture's early-ending utterances alone (EOS at frames 5-102,
    so the whole batch ends and the loop leaves early), then on all 32: codes and frame counts equal the
    fixture's, whatever frames ran past the batch's end."""
    from csm_mlx.generation import generate_codes_batch
    from csm_mlx.sampling import Sampler
    z = _fixture("config4_b32_greedy_125.npz")
    args, w = eos_weights("1b")
    prompts = _prompts()
    early = [int(b) for b in z["eos_utts"]]
    for utts in (early, list(range(32))):
        model = _model(args, w, len(utts))
        hist, n, cache = generate_codes_batch(model, [prompts[b] for b in utts], 125, sampler=Sampler(0.0, 0))
        ran = cache.frames
        del cache, model
        if utts is early:
            assert ran < 125, "the loop did not leave after every utterance ended"
        for j, b in enumerate(utts):
            nb = int(z["n_frames"][b])
            assert n[j] == nb, f"utterance {b}: {n[j]} vs {nb} frames"
            assert first_divergence(hist[: n[j], j], z["codes"][b, :nb]) is None, f"utterance {b}: codes differ"
