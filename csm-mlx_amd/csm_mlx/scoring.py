"""Teacher-forced scoring -- the forward half of ``CSMTrainer.compute_loss``
(/root/reference/csm_mlx/finetune/trainer.py:203-318).

The reference runs the backbone over the whole (B, S-1) sequence, then the decoder over
(B*(S-1), 33) rows [h_t, E_0(c_0), ..., E_31(c_31)] of the next frame, and takes the cross entropy
of every code.  On the GPU the same numbers come out of the frame engine run in teacher-forcing
mode: the prompt prefix is prefilled, then every scored row is one ``csm_frame_forced`` call (the
backbone consumes the previous row, codebook0_head and the 31 decoder steps store their logits and
feed the *given* codes forward, exactly the causal inputs compute_loss builds).  The cross entropy
of every forced code is reduced on the GPU (``forced_ce_kernel``: B*K floats leave the device per
row); only ``cause_mismatch`` (targets differ from the fed codes) copies logits to the host.  The
masked means are taken on the host.

Layouts: per utterance, rows before the first row with a loss are any prompt (text and context
audio, prefilled).  When every later row is a full audio row (audio columns unmasked, text column
masked; trailing all-masked rows are padding) the whole batch is scored together.  Otherwise
(multi-segment conversations: text rows or partially masked rows after the first scored row, as
``tokenize_segments_with_loss_mask`` builds them) that utterance is scored on its own: every row
t >= r0 is a forced frame predicting row t, and a row the engine cannot feed back as
``[codes, 0]`` / ``[1]*K + [0]`` is appended to the backbone with its own tokens and mask by
``csm_prefill`` -- the backbone input compute_loss builds for it (trainer.py:232-239).
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np

from . import _lib
from .generation import FrameCache, _check_window
from .sampling import Sampler


def cross_entropy(logits: np.ndarray, targets: np.ndarray) -> np.ndarray:
    """mlx.nn.losses.cross_entropy(reduction="none"): logsumexp(logits) - logits[target], fp32."""
    lg = logits.astype(np.float32)
    mx_ = lg.max(-1, keepdims=True)
    lse = (np.log(np.exp(lg - mx_).sum(-1, dtype=np.float32)) + mx_[..., 0]).astype(np.float32)
    picked = np.take_along_axis(lg, targets[..., None].astype(np.int64), -1)[..., 0]
    return (lse - picked).astype(np.float32)


def score_frames(model, prompts: Sequence[Tuple[np.ndarray, np.ndarray]], frames: Sequence[np.ndarray],
                 logits: bool = True):
    """Teacher-forced scoring of B utterances: prompt b (tokens (L_b, K+1), mask) followed by the
    audio frames ``frames[b]`` (F_b, K).  F = max F_b; row f of utterance b predicts frames[b][f]
    (rows past F_b are padding).  Returns logits (B, F, K, V) float32, or with ``logits=False`` the
    cross entropy of every forced code (B, F, K), reduced on the GPU (no logits leave the device)."""
    B, K, V = len(prompts), model.n_audio_codebooks, model.n_audio_vocab
    F = max((len(f) for f in frames), default=0)
    for t, _ in prompts:
        _check_window(model, t.shape[0], F)
    forced = np.zeros((F, B, K), np.int32)
    for b, fr in enumerate(frames):
        fr = np.asarray(fr, np.int32).reshape(-1, K)
        forced[: len(fr), b] = fr
    cache = FrameCache(model, B, Sampler(0.0, 0), [0] * B)
    for b, (t, m) in enumerate(prompts):
        cache.prefill(b, t, m)
    L = _lib.lib()
    if not logits:
        ce = np.zeros((F, B, K), np.float32)
        for f in range(F):
            codes = np.ascontiguousarray(forced[f])
            _lib.check(L.csm_frame_forced(model.engine, _lib.ptr(codes), None, None, _lib.ptr(ce[f])))
        return np.ascontiguousarray(ce.transpose(1, 0, 2))
    out = np.zeros((B, F, K, V), np.float32)
    c0 = np.zeros((B, V), np.float32)
    ci = np.zeros((K - 1, B, V), np.float32)
    for f in range(F):
        codes = np.ascontiguousarray(forced[f])
        _lib.check(L.csm_frame_forced(model.engine, _lib.ptr(codes), _lib.ptr(c0), _lib.ptr(ci), None))
        out[:, f, 0] = c0
        out[:, f, 1:] = ci.transpose(1, 0, 2)
    return out


def _standard_row(mask_row: np.ndarray, K: int) -> bool:
    """A row the engine feeds back itself after a forced frame: audio columns on, text column off."""
    return bool(mask_row[:K].all()) and not bool(mask_row[K])


def _split(tokens: np.ndarray, masks: np.ndarray, loss_masks: np.ndarray, K: int):
    """Per utterance: first scored row r0 (>= 1) and whether the rows from r0 on are full audio rows
    followed only by trailing padding (the batched path)."""
    B, S, _ = tokens.shape
    scored = (masks[:, :, :K] & loss_masks[:, :, :K]).any(-1)          # (B, S)
    r0, simple = [], []
    for b in range(B):
        rows = np.nonzero(scored[b, 1:])[0]
        r = int(rows[0]) + 1 if len(rows) else S
        tail = masks[b, r:]
        full = tail[:, :K].all(-1) & ~tail[:, K]
        empty = ~tail.any(-1)
        ok = bool((full | empty).all()) and not (len(full) and np.any(np.diff(empty.astype(int)) < 0))
        r0.append(r)
        simple.append(ok)
    return r0, simple


def _score_utterance(model, tokens: np.ndarray, masks: np.ndarray, r0: int, logits: bool):
    """One utterance of any layout: rows [0, r0) prefilled, then a forced frame per row t >= r0 (its
    c0 / ci predictions from h_{t-1}); rows that are not full audio rows are appended to the backbone
    with their own mask.  Returns (S - r0, K, V) logits or (S - r0, K) cross entropies."""
    S, n_cb = tokens.shape
    K, V = n_cb - 1, model.n_audio_vocab
    L = _lib.lib()
    cache = FrameCache(model, 1, Sampler(0.0, 0), [0])
    cache.prefill(0, tokens[:r0], masks[:r0])
    out = np.zeros((S - r0, K, V) if logits else (S - r0, K), np.float32)
    c0 = np.zeros((1, V), np.float32)
    ci = np.zeros((K - 1, 1, V), np.float32)
    for t in range(r0, S):
        codes = np.ascontiguousarray(tokens[t, :K][None], np.int32)
        if logits:
            _lib.check(L.csm_frame_forced(model.engine, _lib.ptr(codes), _lib.ptr(c0), _lib.ptr(ci), None))
            out[t - r0, 0] = c0[0]
            out[t - r0, 1:] = ci[:, 0]
        else:
            ce = np.zeros((1, K), np.float32)
            _lib.check(L.csm_frame_forced(model.engine, _lib.ptr(codes), None, None, _lib.ptr(ce)))
            out[t - r0] = ce[0]
        if t + 1 < S and not _standard_row(masks[t], K):
            cache.prefill(0, tokens[t:t + 1], masks[t:t + 1])   # row t with its own mask
    return out


def compute_loss(model, batch: Dict[str, np.ndarray], *, per_sample: bool = False, cause_mismatch: bool = False,
                 **kwargs):
    """trainer.py:203-318 on the GPU frame engine (teacher forcing); returns the scalar loss, or the
    (B,) per-sample losses with ``per_sample``.  Masked means divide by the mask sums as the
    reference does (0/0 gives nan)."""
    tokens = np.asarray(batch["tokens"], np.int32)
    masks = np.asarray(batch["masks"]).astype(bool)
    loss_masks = np.asarray(batch["loss_masks"]).astype(bool)
    w0 = np.float32(batch["first_codebook_weight_multiplier"])
    B, S, n_cb = tokens.shape
    K = n_cb - 1
    r0, simple = _split(tokens, masks, loss_masks, K)
    batched = [b for b in range(B) if simple[b]]
    # targets / loss masks on the reference's shifted grid (row t = 1..S-1 predicts row t)
    tgt = tokens[:, 1:, :K]                                              # :220-221
    lm = masks[:, 1:, :K] & loss_masks[:, 1:, :K]                        # :263-265
    ce = np.zeros((B, S - 1, K), np.float32)
    if cause_mismatch:   # targets differ from the fed codes (:266-269): cross entropy from the logits
        tgt = np.concatenate([tgt[:, 1:], tgt[:, :1]], axis=1)
    res = {}
    if batched:
        prompts = [(tokens[b, : r0[b]], masks[b, : r0[b]]) for b in batched]
        frames = [tokens[b, r0[b]:, :K] for b in batched]
        got = score_frames(model, prompts, frames, logits=cause_mismatch)  # (b, F, K[, V])
        res.update({b: got[j] for j, b in enumerate(batched)})
    for b in range(B):
        if not simple[b]:
            res[b] = _score_utterance(model, tokens[b], masks[b], r0[b], cause_mismatch)
    for b in range(B):
        n = S - r0[b]
        if n > 0:
            if cause_mismatch:
                ce[b, r0[b] - 1:] = cross_entropy(res[b][:n], tgt[b, r0[b] - 1:])
            else:        # targets are the fed codes: cross entropy reduced on the GPU
                ce[b, r0[b] - 1:] = res[b][:n]
    ce = np.where(lm, ce, np.float32(0))
    lmf = lm.astype(np.float32)
    with np.errstate(invalid="ignore", divide="ignore"):
        if per_sample:
            c0 = ce[:, :, 0].sum(-1) / lmf[:, :, 0].sum(-1) * w0
            total = c0 / np.float32(K)
            for i in range(1, K):
                total = total + (ce[:, :, i].sum(-1) / lmf[:, :, i].sum(-1)) / np.float32(K)
        else:
            c0 = ce[:, :, 0].sum() / lmf[:, :, 0].sum() * w0
            total = c0 / np.float32(K)
            for i in range(1, K):
                total = total + (ce[:, :, i].sum() / lmf[:, :, i].sum()) / np.float32(K)
    return np.asarray(total, np.float32)
