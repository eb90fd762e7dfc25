"""Prompt framing + Mimi codec access -- drop-in for /root/reference/csm_mlx/tokenizers.py.

Frame layout (tokenizers.py:43-102): every prompt row is (K+1) ids; text rows
carry the text id in the last column (mask only there), audio rows carry the K
codes in columns 0..K-1 (mask there) and each audio segment ends with an all-zero
EOS frame.

Assets: the reference downloads the Llama-3.2 tokenizer and the Mimi checkpoint
by name (tokenizers.py:17, :29).  Offline, ``get_text_tokenizer`` / ``get_audio_tokenizer``
only look in the local Hugging Face cache; synthetic runs register a codec with
``set_audio_tokenizer`` and pass pre-tokenized ids (a list of ints) as ``text``.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Union

import numpy as np

from .config import TOKENIZERS
from .segment import Segment

_audio_tokenizers = {}


def set_audio_tokenizer(codec, n_audio_codebooks: Optional[int] = None):
    """Register the process-wide codec for ``n_audio_codebooks`` (replaces the hub download)."""
    _audio_tokenizers[n_audio_codebooks or codec.m.n_q] = codec


def get_audio_tokenizer(n_audio_codebooks: int):
    """tokenizers.py:14-21."""
    if n_audio_codebooks in _audio_tokenizers:
        return _audio_tokenizers[n_audio_codebooks]
    from huggingface_hub import hf_hub_download
    from .config import MIMI_CONFIGURATION
    from .mimi import MimiCodec
    try:
        path = hf_hub_download(**TOKENIZERS["audio"], local_files_only=True)
    except Exception as ex:  # noqa: BLE001
        raise RuntimeError("Mimi weights are not in the local HF cache (offline); register a codec with "
                           "csm_mlx.tokenizers.set_audio_tokenizer(...)") from ex
    import dataclasses
    m = dataclasses.replace(MIMI_CONFIGURATION["mimi_202407"], n_q=n_audio_codebooks)
    codec = MimiCodec(m)
    codec.load_pytorch_weights(path)
    _audio_tokenizers[n_audio_codebooks] = codec
    return codec


_text_tokenizer = None


def _with_bos_eos_template(tok):
    """tokenizers.py:29-39: BOS/EOS TemplateProcessing around every encode (single and pair)."""
    from tokenizers.processors import TemplateProcessing
    bos, eos = tok.bos_token, tok.eos_token
    tok._tokenizer.post_processor = TemplateProcessing(
        single=f"{bos}:0 $A:0 {eos}:0",
        pair=f"{bos}:0 $A:0 {eos}:0 {bos}:1 $B:1 {eos}:1",
        special_tokens=[(f"{bos}", tok.bos_token_id), (f"{eos}", tok.eos_token_id)],
    )
    return tok


def set_text_tokenizer(tok):
    """Register a text tokenizer (a transformers fast tokenizer with bos/eos tokens) in place of the
    hub download; the reference's BOS/EOS template is applied to it."""
    global _text_tokenizer
    _text_tokenizer = _with_bos_eos_template(tok)
    return _text_tokenizer


def get_text_tokenizer():
    """tokenizers.py:24-40 (BOS/EOS template around every encode).  Offline: a registered tokenizer
    (``set_text_tokenizer``) or the local HF cache."""
    global _text_tokenizer
    if _text_tokenizer is None:
        from transformers import AutoTokenizer
        try:
            tok = AutoTokenizer.from_pretrained(TOKENIZERS["text"]["repo_id"], local_files_only=True)
        except Exception as ex:  # noqa: BLE001
            raise RuntimeError("the Llama-3.2 tokenizer is not in the local HF cache (offline); register one "
                               "with csm_mlx.tokenizers.set_text_tokenizer(...) or pass pre-tokenized ids "
                               "(a list of ints) as `text`") from ex
        _text_tokenizer = _with_bos_eos_template(tok)
    return _text_tokenizer


def tokenize_text_segment(text: Union[str, Sequence[int]], speaker: int, n_audio_codebooks: int = 32):
    """tokenizers.py:43-58 -> (n, K+1) int32 tokens, (n, K+1) bool mask."""
    if isinstance(text, str):
        ids = get_text_tokenizer().encode(f"[{speaker}]{text}")
    else:
        ids = [int(t) for t in text]
    n = len(ids)
    tokens = np.zeros((n, n_audio_codebooks + 1), np.int32)
    mask = np.zeros((n, n_audio_codebooks + 1), bool)
    tokens[:, -1] = ids
    mask[:, -1] = True
    return tokens, mask


def audio_codes_to_frames(codes_kt: np.ndarray):
    """tokenizers.py:73-85: (K, T) codes + EOS zero frame -> (T+1, K+1) rows, mask cols 0..K-1."""
    K, T = codes_kt.shape
    c = np.concatenate([codes_kt.astype(np.int32), np.zeros((K, 1), np.int32)], axis=1)
    tokens = np.zeros((T + 1, K + 1), np.int32)
    mask = np.zeros((T + 1, K + 1), bool)
    tokens[:, :-1] = c.T
    mask[:, :-1] = True
    return tokens, mask


def tokenize_audio(audio, *, n_audio_codebooks: int = 32):
    """tokenizers.py:61-85: Mimi.encode (1,1,N) -> (K,T) codes, then frame rows."""
    codec = get_audio_tokenizer(n_audio_codebooks)
    codes = codec.encode(np.asarray(audio, np.float32)[None, None])[0]
    return audio_codes_to_frames(codes)


def tokenize_segment(segment: Segment, *, n_audio_codebooks: int = 32):
    """tokenizers.py:88-102."""
    t_tok, t_mask = tokenize_text_segment(segment.text, segment.speaker, n_audio_codebooks)
    a_tok, a_mask = tokenize_audio(segment.audio, n_audio_codebooks=n_audio_codebooks)
    return np.concatenate([t_tok, a_tok], 0).astype(np.int32), np.concatenate([t_mask, a_mask], 0).astype(bool)


def tokenize_segments_batch(segments: List[Segment], *, n_audio_codebooks: int = 32):
    """Batched context encode: every segment's audio goes through ONE Mimi.encode launch
    (same-length audio only; ragged lengths fall back to per-segment encodes)."""
    codec = get_audio_tokenizer(n_audio_codebooks)
    audios = [np.asarray(s.audio, np.float32) for s in segments]
    if len({len(a) for a in audios}) == 1 and audios:
        rows = getattr(codec, "encode_rows", None)  # (a registered stand-in codec may only have encode)
        codes = rows(audios) if rows else codec.encode(np.stack(audios)[:, None, :])
    else:
        codes = [codec.encode(a[None, None])[0] for a in audios]
    out = []
    for seg, c in zip(segments, codes):
        t_tok, t_mask = tokenize_text_segment(seg.text, seg.speaker, n_audio_codebooks)
        a_tok, a_mask = audio_codes_to_frames(np.asarray(c))
        out.append((np.concatenate([t_tok, a_tok], 0), np.concatenate([t_mask, a_mask], 0)))
    return out


def tokenize_segments_with_loss_mask(segments: List[Segment], *, n_audio_codebooks: int = 32,
                                     mask_speaker_ids: Sequence[int], max_audio_length_ms: Optional[int]):
    """tokenizers.py:105-145 (the fine-tuning batch layout that ``scoring.compute_loss`` scores):
    every segment's rows concatenated, loss mask ones except the rows of segments whose speaker is in
    ``mask_speaker_ids``, all three truncated to max_audio_length_ms / 80 rows."""
    parts = [tokenize_segment(seg, n_audio_codebooks=n_audio_codebooks) for seg in segments]
    tokens = np.concatenate([t for t, _ in parts], 0).astype(np.int32)
    masks = np.concatenate([m for _, m in parts], 0).astype(bool)
    loss_masks = np.ones_like(tokens)
    pos = 0
    for (t, _), seg in zip(parts, segments):
        if seg.speaker in mask_speaker_ids:
            loss_masks[pos:pos + t.shape[0]] = 0
        pos += t.shape[0]
    if max_audio_length_ms is not None:
        n = int(max_audio_length_ms / 80)
        tokens, masks, loss_masks = tokens[:n], masks[:n], loss_masks[:n]
    return tokens, masks, loss_masks


def decode_audio(audio_tokens, *, n_audio_codebooks: int = 32) -> np.ndarray:
    """tokenizers.py:148-150: (B, K, F) codes -> (B, 1, F*1920) PCM."""
    return get_audio_tokenizer(n_audio_codebooks).decode(np.asarray(audio_tokens, np.int32))
