"""GPU parity of teacher-forced scoring (csm_frame_forced) against the oracle's whole-sequence
restatement of compute_loss (trainer.py:203-318): one causal backbone call, one causal decoder call
over (B*(S-1), K+1) rows.  fp32 weights; losses within 1e-4 relative."""
import numpy as np
import pytest

from helpers import csm_weights, oracle_for

pytestmark = pytest.mark.gpu


def _batch(args, seed=0):
    """Two utterances padded to one length: (text prompt, scored audio) and
    (text, unscored context audio, text, scored audio); loss masks on the scored audio rows."""
    from csm_mlx.tokenizers import tokenize_text_segment
    rng = np.random.default_rng(seed)
    K = args.n_audio_codebooks

    def audio(n):
        t = np.zeros((n, K + 1), np.int32)
        t[:, :K] = rng.integers(0, 64, (n, K))
        m = np.zeros((n, K + 1), bool)
        m[:, :K] = True
        return t, m
    rows = []
    t1, m1 = tokenize_text_segment([998, 5, 6, 7, 999], 0, K)
    a1, am1 = audio(6)
    rows.append((np.concatenate([t1, a1]), np.concatenate([m1, am1]), np.r_[np.zeros(len(t1)), np.ones(6)]))
    t2, m2 = tokenize_text_segment([998, 11, 999], 1, K)
    c2, cm2 = audio(2)
    t3, m3 = tokenize_text_segment([998, 12, 13, 999], 0, K)
    a2, am2 = audio(8)
    toks = np.concatenate([t2, c2, t3, a2])
    rows.append((toks, np.concatenate([m2, cm2, m3, am2]), np.r_[np.zeros(len(toks) - 8), np.ones(8)]))
    S = max(len(r[0]) for r in rows)
    T = np.zeros((2, S, K + 1), np.int32)
    M = np.zeros((2, S, K + 1), bool)
    LM = np.zeros((2, S, K + 1), bool)
    for b, (t, m, lm) in enumerate(rows):
        T[b, : len(t)], M[b, : len(t)] = t, m
        LM[b, : len(t)] = lm[:, None].astype(bool)
    return {"tokens": T, "masks": M, "loss_masks": LM, "first_codebook_weight_multiplier": 1.5}


def _batch_multiseg(args, seed=1):
    """tokenize_segments_with_loss_mask layout (tokenizers.py:105-145): per utterance alternating
    speaker segments [text rows, audio rows + EOS zero row], loss masks ones except the segments of a
    masked speaker (1) -- text rows and a masked speaker's rows follow the first scored row."""
    from csm_mlx.tokenizers import tokenize_text_segment
    rng = np.random.default_rng(seed)
    K = args.n_audio_codebooks

    def audio(n):
        t = np.zeros((n + 1, K + 1), np.int32)
        t[:n, :K] = rng.integers(0, 64, (n, K))
        m = np.zeros((n + 1, K + 1), bool)
        m[:, :K] = True
        return t, m
    utts = []
    for spec in ([(0, 3, 5), (1, 2, 4), (0, 4, 3)], [(1, 2, 2), (0, 3, 6)]):
        toks, msks, lms = [], [], []
        for spk, n_txt, n_aud in spec:
            t, m = tokenize_text_segment([998] + [int(x) for x in rng.integers(0, 990, n_txt)] + [999], spk, K)
            a, am = audio(n_aud)
            seg_t, seg_m = np.concatenate([t, a]), np.concatenate([m, am])
            toks.append(seg_t)
            msks.append(seg_m)
            lms.append(np.full(seg_t.shape, spk != 1))
        utts.append((np.concatenate(toks), np.concatenate(msks), np.concatenate(lms)))
    S = max(len(u[0]) for u in utts)
    T = np.zeros((2, S, K + 1), np.int32)
    M = np.zeros((2, S, K + 1), bool)
    LM = np.zeros((2, S, K + 1), bool)
    for b, (t, m, lm) in enumerate(utts):
        T[b, : len(t)], M[b, : len(t)], LM[b, : len(t)] = t, m, lm
    return {"tokens": T, "masks": M, "loss_masks": LM, "first_codebook_weight_multiplier": 1.0}


@pytest.mark.parametrize("per_sample,mismatch", [(False, False), (True, False), (False, True)])
def test_compute_loss_multi_segment_matches_oracle(per_sample, mismatch):
    """Text rows (and masked-speaker segments) after the first scored row: utterance 0 is scored on
    its own (text rows appended to the backbone with their own masks); utterance 1 (masked speaker
    first, one scored segment last) takes the batched path -- both paths in one call."""
    from csm_mlx.models import CSM
    from csm_mlx.scoring import _split, compute_loss
    from oracle.csm_oracle import compute_loss_ref
    args, w = csm_weights("tiny")
    model = CSM(args, dtype="float32", max_batch=2)
    model.load_weights(w)
    batch = _batch_multiseg(args)
    K = args.n_audio_codebooks
    assert _split(batch["tokens"], batch["masks"], batch["loss_masks"], K)[1] == [False, True]
    got = compute_loss(model, batch, per_sample=per_sample, cause_mismatch=mismatch)
    ref = compute_loss_ref(oracle_for(args, w), batch, per_sample=per_sample, cause_mismatch=mismatch)
    assert np.all(np.isfinite(got)) and np.shape(got) == np.shape(ref)
    np.testing.assert_allclose(got, ref, rtol=1e-4)


@pytest.mark.parametrize("per_sample,mismatch", [(False, False), (True, False), (False, True)])
def test_compute_loss_matches_oracle(per_sample, mismatch):
    from csm_mlx.models import CSM
    from csm_mlx.scoring import compute_loss
    from oracle.csm_oracle import compute_loss_ref
    args, w = csm_weights("tiny")
    model = CSM(args, dtype="float32", max_batch=2)
    model.load_weights(w)
    batch = _batch(args)
    got = compute_loss(model, batch, per_sample=per_sample, cause_mismatch=mismatch)
    ref = compute_loss_ref(oracle_for(args, w), batch, per_sample=per_sample, cause_mismatch=mismatch)
    assert np.all(np.isfinite(got)) and np.shape(got) == np.shape(ref)
    np.testing.assert_allclose(got, ref, rtol=1e-4)


def test_score_frames_greedy_codes_are_argmax():
    """Forcing the greedy generator's own codes reproduces its logits: arg-max of every scored
    row equals the forced code."""
    from csm_mlx.generation import generate_batch
    from csm_mlx.models import CSM
    from csm_mlx.scoring import score_frames
    from csm_mlx.tokenizers import tokenize_text_segment
    args, w = csm_weights("tiny")
    model = CSM(args, dtype="float32", max_batch=2)
    model.load_weights(w)
    p = [tokenize_text_segment([998, 21, 22, 999], 0, args.n_audio_codebooks)]
    codes = generate_batch(model, p, 8 * 80, temperature=0.0, decode=False)[0]
    logits = score_frames(model, p, [codes])
    assert np.array_equal(logits[0, : len(codes)].argmax(-1), codes)


def test_device_cross_entropy_matches_logits():
    """score_frames(logits=False) (forced_ce_kernel) equals the host cross entropy of the logits."""
    from csm_mlx.models import CSM
    from csm_mlx.scoring import cross_entropy, score_frames
    from csm_mlx.tokenizers import tokenize_text_segment
    args, w = csm_weights("tiny")
    model = CSM(args, dtype="float32", max_batch=3)
    model.load_weights(w)
    rng = np.random.default_rng(5)
    K = args.n_audio_codebooks
    p = [tokenize_text_segment([998, 30 + b, 999], 0, K) for b in range(3)]
    fr = [rng.integers(0, 64, (n, K)).astype(np.int32) for n in (5, 7, 6)]
    lg = score_frames(model, p, fr)
    ce = score_frames(model, p, fr, logits=False)
    for b in range(3):
        n = len(fr[b])
        np.testing.assert_allclose(ce[b, :n], cross_entropy(lg[b, :n], fr[b]), rtol=1e-5, atol=1e-5)


def test_csm_1b_device_cross_entropy():
    """forced_ce_kernel at csm_1b's vocabulary (V = 2051: nine logits per thread) against the host
    cross entropy of the same logits; bf16 weights, B = 2, 4 forced rows."""
    from csm_mlx.models import CSM
    from csm_mlx.scoring import cross_entropy, score_frames
    from csm_mlx.tokenizers import tokenize_text_segment
    from helpers import prompt_ids
    args, w = csm_weights("1b")
    model = CSM(args, dtype="bf16", max_batch=2)
    model.load_weights(w)
    rng = np.random.default_rng(6)
    p = [tokenize_text_segment(prompt_ids(s), 0, 32) for s in (1, 2)]
    fr = [rng.integers(0, 2051, (4, 32)).astype(np.int32) for _ in range(2)]
    lg = score_frames(model, p, fr)
    ce = score_frames(model, p, fr, logits=False)
    for b in range(2):
        np.testing.assert_allclose(ce[b], cross_entropy(lg[b], fr[b]), rtol=1e-5, atol=1e-4)
