"""Frame generation -- drop-in for /root/reference/csm_mlx/generation.py.

``generate_frame`` / ``generate`` / ``stream_generate`` keep the reference
signatures (generation.py:21-31, 95-105, 181-191) plus the ``sampler=`` keyword
the reference README/CLI pass (README.md:49; cli/generate.py:197-199).  The
frame step itself runs as two captured HIP graphs inside libcsm_hip.so
(csm-mlx_amd/csrc/csm_engine.hip); the host only assembles prompts, polls EOS
flags every ``chunk`` frames and hands the code history to the Mimi decoder,
which reads it straight from device memory.

``generate_batch`` is the batched extension used by bench.py: B independent
utterances share every weight read (the reference is batch-1 only,
generation.py:156).
"""
from __future__ import annotations

import ctypes
import os
from typing import Any, Callable, Generator, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from .models import CSM
from .sampling import HostSampler, Sampler
from .segment import Segment
from .tokenizers import decode_audio, get_audio_tokenizer, tokenize_segment, tokenize_text_segment

default_stream = None  # MLX stream placeholder (generation.py:19); the engine owns its HIP stream


def _resolve_sampler(temperature: float, sampler, top_k: int = 0):
    """A Sampler descriptor (runs on the GPU), or any other callable wrapped as a HostSampler (runs
    on the host for every codebook: csm_frame_host_step)."""
    if sampler is not None:
        if isinstance(sampler, (Sampler, HostSampler)):
            return sampler
        if callable(sampler):
            return HostSampler(sampler)
        raise TypeError(f"sampler must be a csm_mlx.sampling.Sampler or a callable, got {type(sampler).__name__}")
    return Sampler(float(temperature), int(top_k))


def _seed_list(seed, B: int) -> np.ndarray:
    if seed is None:
        base = int.from_bytes(os.urandom(8), "little")
        return np.array([(base + b) & ((1 << 64) - 1) for b in range(B)], np.uint64)
    if np.ndim(seed) == 0:
        return np.array([(int(seed) + b) & ((1 << 64) - 1) for b in range(B)], np.uint64)
    s = np.asarray(seed, np.uint64).reshape(-1)
    if len(s) != B:
        raise ValueError("need one seed per utterance")
    return s


class FrameCache:
    """Replaces the per-layer mlx_lm ``KVCache`` list: a batch slot in the engine
    (KV caches, positions, code history live on the GPU).

    The engine holds ONE active generation per model: creating a FrameCache (or calling
    ``generate`` / ``stream_generate`` / ``score_frames``, which create one) starts a new batch and
    overwrites the KV caches.  An older FrameCache of the same model then raises on every call
    instead of silently reading the new state (the reference's KVCache lists are independent
    objects; here the caches live in the engine)."""

    def __init__(self, model: CSM, batch_size: int, sampler: Sampler, seeds=None):
        self.model = model
        self.B = batch_size
        self.sampler = sampler
        self.seeds = _seed_list(seeds, batch_size)
        self.L = _lib.lib()
        _lib.check(self.L.csm_begin(model.engine, batch_size, _lib.ptr(self.seeds), sampler.temp, sampler.top_k))
        if not sampler.greedy and sampler.filtered:
            _lib.check(self.L.csm_set_sampler_filters(model.engine, sampler.top_p, sampler.min_p,
                                                      sampler.min_tokens_to_keep))
        model._generation = getattr(model, "_generation", 0) + 1
        self._gen = model._generation
        self.frames = 0

    def _check(self):
        if getattr(self.model, "_generation", 0) != self._gen:
            raise RuntimeError("this FrameCache was superseded: a newer generation started on the same model "
                               "(the engine holds one active generation per model)")

    def prefill(self, b: int, tokens: np.ndarray, mask: np.ndarray):
        self._check()
        t = np.ascontiguousarray(tokens, np.int32)
        m = np.ascontiguousarray(mask, np.uint8)
        _lib.check(self.L.csm_prefill(self.model.engine, b, t.shape[0], _lib.ptr(t), _lib.ptr(m)))

    def prefill_batch(self, items: Sequence[Tuple[int, np.ndarray, np.ndarray]]):
        """prefill for several utterances in one pass per <= max_seq_len rows (csm_prefill_batch):
        items = (b, tokens, mask) with distinct b."""
        self._check()
        if not items:
            return
        utts = np.array([b for b, _, _ in items], np.int32)
        Ts = np.array([t.shape[0] for _, t, _ in items], np.int32)
        toks = np.ascontiguousarray(np.concatenate([np.asarray(t, np.int32) for _, t, _ in items]), np.int32)
        msks = np.ascontiguousarray(np.concatenate([np.asarray(m, np.uint8) for _, _, m in items]), np.uint8)
        _lib.check(self.L.csm_prefill_batch(self.model.engine, len(items), _lib.ptr(utts), _lib.ptr(Ts),
                                            _lib.ptr(toks), _lib.ptr(msks)))

    def run(self, nframes: int, sync: bool = True) -> bool:
        """Enqueue nframes frame graphs; with sync, wait and return whether every utterance is done
        (without, return False at once: the caller polls ``done()``, which waits for the frames)."""
        self._check()
        done = ctypes.c_int(0)
        _lib.check(self.L.csm_run_frames(self.model.engine, nframes, ctypes.byref(done) if sync else None))
        self.frames += nframes
        return bool(done.value)

    def run_ahead(self, nframes: int) -> Optional[bool]:
        """Enqueue nframes frames and return whether every utterance had hit EOS by the end of the
        PREVIOUS chunk run this way (None for the first): the EOS poll one chunk behind, so the GPU never
        waits on the host (csm_run_frames_ahead)."""
        self._check()
        prev = ctypes.c_int(-1)
        _lib.check(self.L.csm_run_frames_ahead(self.model.engine, nframes, ctypes.byref(prev)))
        self.frames += nframes
        return None if prev.value < 0 else bool(prev.value)

    def run_processed(self, processors: Sequence[Callable], c0_history: Optional[list]) -> bool:
        """One frame with host ``logits_processors`` applied to the c0 logits (generation.py:42-61):
        the engine stops after codebook0_head, each processor maps (stack(c0_history) or zeros((0,)),
        logits (B, V)) -> logits, and the frame finishes on the GPU from the processed logits.
        Appends this frame's c0 (B, 1) to ``c0_history``; returns whether every utterance is done."""
        self._check()
        V = self.model.n_audio_vocab
        logits = np.zeros((self.B, V), np.float32)
        _lib.check(self.L.csm_frame_c0_logits(self.model.engine, _lib.ptr(logits)))
        hist = np.stack(c0_history, 0) if c0_history else np.zeros((0,), np.int32)
        for proc in processors:
            logits = np.ascontiguousarray(np.asarray(proc(hist, logits), np.float32).reshape(self.B, V))
        done = ctypes.c_int(0)
        _lib.check(self.L.csm_frame_finish(self.model.engine, _lib.ptr(logits), ctypes.byref(done)))
        self.frames += 1
        if c0_history is not None:
            c0_history.append(self.last_codes()[:, :1].copy())
        return bool(done.value)

    def run_host_sampled(self, sampler: HostSampler, processors: Sequence[Callable] = (),
                         c0_history: Optional[list] = None) -> bool:
        """One frame whose every code comes from a host sampler callable (the reference's sampler=,
        applied per codebook): c0 logits -> processors -> sampler -> csm_frame_host_step, which feeds
        the codes forward and returns the next codebook's logits, K times.  Returns whether every
        utterance is done."""
        self._check()
        V, K = self.model.n_audio_vocab, self.model.n_audio_codebooks
        logits = np.zeros((self.B, V), np.float32)
        _lib.check(self.L.csm_frame_c0_logits(self.model.engine, _lib.ptr(logits)))
        hist = np.stack(c0_history, 0) if c0_history else np.zeros((0,), np.int32)
        for proc in processors:
            logits = np.ascontiguousarray(np.asarray(proc(hist, logits), np.float32).reshape(self.B, V))
        done = ctypes.c_int(0)
        for i in range(K):
            raw = np.asarray(sampler(logits)).reshape(self.B)
            if raw.size and (raw.min() < 0 or raw.max() >= V):   # no silent clamp: -1 -> 0 would read as EOS
                raise ValueError(f"sampler returned a code outside [0, {V}): {raw.min()} .. {raw.max()}")
            codes = np.ascontiguousarray(raw, np.int32)
            if i == 0 and c0_history is not None:
                c0_history.append(codes[:, None].copy())
            out = np.zeros((self.B, V), np.float32)
            _lib.check(self.L.csm_frame_host_step(self.model.engine, _lib.ptr(codes),
                                                  _lib.ptr(out) if i + 1 < K else None, ctypes.byref(done)))
            logits = out
        self.frames += 1
        return bool(done.value)

    def codes(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """(history [F,B,K], n_frames [B], done [B])."""
        self._check()
        F = ctypes.c_int(0)
        _lib.check(self.L.csm_read_codes(self.model.engine, None, None, None, ctypes.byref(F)))
        hist = np.zeros((F.value, self.B, self.model.n_audio_codebooks), np.int32)
        n = np.zeros(self.B, np.int32)
        d = np.zeros(self.B, np.uint8)
        _lib.check(self.L.csm_read_codes(self.model.engine, _lib.ptr(hist), _lib.ptr(n), _lib.ptr(d), None))
        return hist, n, d

    def done(self) -> np.ndarray:
        self._check()
        d = np.zeros(self.B, np.uint8)
        _lib.check(self.L.csm_read_codes(self.model.engine, None, None, _lib.ptr(d), None))
        return d.astype(bool)

    def last_codes(self) -> np.ndarray:
        self._check()
        out = np.zeros((self.B, self.model.n_audio_codebooks), np.int32)
        _lib.check(self.L.csm_debug_read(self.model.engine, b"codes", _lib.ptr(out), out.nbytes, None))
        return out

    def debug(self, what: str, shape) -> np.ndarray:
        self._check()
        out = np.zeros(shape, np.float32)
        _lib.check(self.L.csm_debug_read(self.model.engine, what.encode(), _lib.ptr(out), out.nbytes, None))
        return out


def make_frame_cache(model: CSM, batch_size: int = 1, *, temperature: float = 0.8, sampler=None, seed=None):
    return FrameCache(model, batch_size, _resolve_sampler(temperature, sampler), seed)


def generate_frame(model: CSM, tokens, *, temperature: float = 0.8, token_mask=None,
                   logits_processors: Optional[List[Callable]] = None, cache: Optional[FrameCache] = None,
                   stream: Any = default_stream, c0_history: Optional[list] = None, sampler=None, seed=None):
    """generation.py:21-92.  tokens (B, T, K+1); returns codes (B, K) int32.

    The rows are appended to the backbone KV held by ``cache`` (a fresh one when None),
    then one frame (c0 + 31 decoder steps) runs on the GPU.  With ``logits_processors`` the frame
    pauses after codebook0_head for them (``FrameCache.run_processed``)."""
    tokens = np.asarray(tokens, np.int32)
    mask = np.ones_like(tokens, dtype=bool) if token_mask is None else np.asarray(token_mask).astype(bool)
    B = tokens.shape[0]
    if cache is None:
        cache = make_frame_cache(model, B, temperature=temperature, sampler=sampler, seed=seed)
    else:
        # the sampler is fixed when the cache starts its batch (csm_begin); the reference applies the
        # temperature of every call (generation.py:51-54), so a different one cannot be honoured
        want = _resolve_sampler(temperature, sampler)
        if want != cache.sampler:
            raise ValueError(f"generate_frame's sampler {want} differs from the cache's {cache.sampler}; "
                             f"create the cache with make_frame_cache(model, temperature=..., sampler=...)")
    for b in range(B):
        cache.prefill(b, tokens[b], mask[b])
    if isinstance(cache.sampler, HostSampler):
        cache.run_host_sampled(cache.sampler, logits_processors or (), c0_history)
        return cache.last_codes()
    if logits_processors:
        cache.run_processed(logits_processors, c0_history)
        return cache.last_codes()
    cache.run(1)
    codes = cache.last_codes()
    if c0_history is not None:
        c0_history.append(codes[:, :1].copy())
    return codes


def build_prompt(model: CSM, text, speaker: int, context: Sequence[Segment]):
    """generation.py:108-125 -> (L, K+1) tokens, mask."""
    K = model.n_audio_codebooks
    toks, masks = [], []
    for seg in context:
        t, m = tokenize_segment(seg, n_audio_codebooks=K)
        toks.append(t)
        masks.append(m)
    t, m = tokenize_text_segment(text, speaker, K)
    toks.append(t)
    masks.append(m)
    return np.concatenate(toks, 0).astype(np.int32), np.concatenate(masks, 0).astype(bool)


def _check_window(model: CSM, L: int, max_audio_frames: int):
    max_seq_len = model.max_seq_len - max_audio_frames                         # generation.py:131-137
    if L >= max_seq_len:
        raise ValueError(f"Inputs too long ({L}), must be below max_seq_len - max_audio_frames: {max_seq_len}")


def _mark(timings: Optional[dict], key: str, t0: float, model: Optional[CSM] = None) -> float:
    """Phase timer (bench.py --phases): wait for the engine, add the elapsed wall time to timings[key]."""
    import time
    if timings is None:
        return t0
    if model is not None:
        _lib.check(_lib.lib().csm_synchronize(model.engine))
    t = time.perf_counter()
    timings[key] = timings.get(key, 0.0) + (t - t0)
    return t


def generate_codes_batch(model: CSM, prompts: Sequence[Tuple[np.ndarray, np.ndarray]], max_audio_frames: int, *,
                         sampler: Sampler, seeds=None, chunk: int = 8,
                         logits_processors: Optional[List[Callable]] = None, timings: Optional[dict] = None):
    """Run the frame loop for B prompts.  Returns (hist [F,B,K], n_frames [B], cache).  With
    ``logits_processors`` every frame pauses after codebook0_head for them (generation.py:44-49).
    ``timings`` (optional dict): wall seconds of the prompt prefill and of the frames are added to
    its "prefill" / "frames" entries (the engine is synchronized at each boundary)."""
    import time
    B = len(prompts)
    for t, _ in prompts:
        _check_window(model, t.shape[0], max_audio_frames)
    t0 = time.perf_counter()
    cache = FrameCache(model, B, sampler, seeds)
    if B > 1:   # every prompt's rows through one pass of each projection (weights streamed once)
        cache.prefill_batch([(b, t, m) for b, (t, m) in enumerate(prompts)])
    else:
        cache.prefill(0, *prompts[0])
    t0 = _mark(timings, "prefill", t0, model)
    left = max_audio_frames
    if isinstance(sampler, HostSampler):  # a sampler callable: every code from the host, frame by frame
        c0_history_h: list = []
        for _ in range(max_audio_frames):
            if cache.run_host_sampled(sampler, logits_processors or (), c0_history_h):
                break
        left = 0
    elif logits_processors:
        c0_history: list = []                                                    # generation.py:128
        for _ in range(max_audio_frames):
            if cache.run_processed(logits_processors, c0_history):
                break
        left = 0
    ahead = os.environ.get("CSM_EOS_AHEAD", "1") != "0"   # lab: 0 = poll each chunk after it ends (A/B)
    while left > 0:
        n = min(chunk if ahead else 2 * chunk, left)
        ended = cache.run_ahead(n) if ahead else cache.run(n)   # EOS poll (generation.py:151); ahead: of the
        left -= n                                               # previous chunk, while this one runs
        if ended:                           # (this chunk's frames then change no returned code)
            break
    hist, n_frames, _ = cache.codes()
    _mark(timings, "frames", t0, model)
    return hist, n_frames, cache


def _decode_batch(model: CSM, hist: np.ndarray, n_frames: np.ndarray) -> List[np.ndarray]:
    """Mimi decode per group of equal-length utterances (a shorter utterance must not see
    frames generated after its EOS)."""
    K = model.n_audio_codebooks
    codec = get_audio_tokenizer(K)
    out: List[Optional[np.ndarray]] = [None] * len(n_frames)
    for F in sorted(set(int(f) for f in n_frames)):
        idx = [b for b in range(len(n_frames)) if n_frames[b] == F]
        if F == 0:
            for b in idx:
                out[b] = np.zeros((0,), np.float32)
            continue
        codes = np.ascontiguousarray(hist[:F, idx].transpose(1, 2, 0))          # (b, K, F)
        pcm = codec.decode(codes)
        for j, b in enumerate(idx):
            out[b] = pcm[j, 0]
    return out


def generate(model: CSM, text, speaker: int, context: List[Segment], max_audio_length_ms: float = 90_000, *,
             temperature: float = 0.8, logits_processors: Optional[List[Callable]] = None,
             stream: Any = default_stream, sampler=None, seed=None) -> np.ndarray:
    """generation.py:95-178: returns the (F*1920,) float32 waveform (or zeros((0,)) + warning)."""
    max_audio_frames = int(max_audio_length_ms / 80)
    prompt = build_prompt(model, text, speaker, context)
    smp = _resolve_sampler(temperature, sampler)
    hist, n_frames, _ = generate_codes_batch(model, [prompt], max_audio_frames, sampler=smp, seeds=seed,
                                             logits_processors=logits_processors)
    if n_frames[0] == 0:
        print("[WARN] No samples generated.")
        return np.zeros((0,), dtype=np.float32)
    return _decode_batch(model, hist, n_frames)[0]


def generate_batch(model: CSM, prompts: Sequence[Tuple[np.ndarray, np.ndarray]], max_audio_length_ms: float = 10_000,
                   *, temperature: float = 0.0, top_k: int = 0, sampler=None, seeds=None, decode: bool = True,
                   with_codes: bool = False, timings: Optional[dict] = None):
    """Batched extension: B prompts (tokens, mask) -> list of waveforms (or codes if decode=False;
    (codes, waveforms) with ``with_codes``).  ``timings``: per-phase wall seconds (prefill, frames,
    decode) added to the dict."""
    import time
    smp = _resolve_sampler(temperature, sampler, top_k)
    hist, n_frames, _ = generate_codes_batch(model, prompts, int(max_audio_length_ms / 80), sampler=smp, seeds=seeds,
                                             timings=timings)
    codes = [hist[: n_frames[b], b] for b in range(len(prompts))]
    if not decode:
        return codes
    t0 = time.perf_counter()
    pcm = _decode_batch(model, hist, n_frames)
    _mark(timings, "decode", t0)
    return (codes, pcm) if with_codes else pcm


def _overlapped_frames(cache: "FrameCache", codec, max_audio_frames: int):
    """The streaming loop of generation.py:232-256 with frame f+1 computing on the engine's stream
    while the codec decodes frame f on its own: enqueue f+1, decode + yield f, then wait for f+1 and
    test EOS (an all-done frame is not decoded or yielded, as the reference breaks before its
    decode_step).  Yields (pcm (B, 1920), done (B,)) in frame order."""
    prev = None  # (codes, done) of the last finished, not yet decoded frame
    for _ in range(max_audio_frames):
        cache.run(1, sync=False)
        if prev is not None:
            yield codec.decode_step(prev[0])[:, 0], prev[1]
        d = cache.done()                                                           # waits for the frame
        if d.all():
            prev = None
            break                                                                  # EOS (generation.py:239)
        prev = (cache.last_codes(), d)
    if prev is not None:
        yield codec.decode_step(prev[0])[:, 0], prev[1]


def _host_sampled_frames(cache: "FrameCache", codec, max_audio_frames: int, sampler: HostSampler, processors):
    """The streaming loop with a host sampler callable (every code from the host; nothing to overlap):
    EOS is tested before the frame is decoded (generation.py:237-251)."""
    c0_history: list = []
    for _ in range(max_audio_frames):
        if cache.run_host_sampled(sampler, processors or (), c0_history):
            break
        yield codec.decode_step(cache.last_codes())[:, 0], cache.done()


def _processed_frames(cache: "FrameCache", codec, max_audio_frames: int, processors):
    """The streaming loop with host logits processors: each frame pauses after codebook0_head, so
    there is nothing to overlap; EOS is tested before the frame is decoded (generation.py:237-251)."""
    c0_history: list = []
    for _ in range(max_audio_frames):
        if cache.run_processed(processors, c0_history):
            break
        yield codec.decode_step(cache.last_codes())[:, 0], cache.done()


def stream_generate_batch(model: CSM, prompts: Sequence[Tuple[np.ndarray, np.ndarray]],
                          max_audio_length_ms: float = 10_000, *, temperature: float = 0.8, top_k: int = 0,
                          sampler=None, seeds=None) -> Generator[Tuple[np.ndarray, np.ndarray], None, None]:
    """Batched extension of ``stream_generate`` (generation.py:181-258): per frame yields
    (pcm (B, 1920) float32 from the codec's streaming ``decode_step``, done (B,) bool).  An
    utterance's rows after its EOS frame are not audio (its ``done`` flag is set)."""
    max_audio_frames = int(max_audio_length_ms / 80)
    for t, _ in prompts:
        _check_window(model, t.shape[0], max_audio_frames)
    smp = _resolve_sampler(temperature, sampler, top_k)
    B = len(prompts)
    codec = get_audio_tokenizer(model.n_audio_codebooks)
    cache = FrameCache(model, B, smp, seeds)
    cache.prefill_batch([(b, t, m) for b, (t, m) in enumerate(prompts)])
    codec.reset_state(B)
    try:
        if isinstance(smp, HostSampler):
            yield from _host_sampled_frames(cache, codec, max_audio_frames, smp, None)
        else:
            yield from _overlapped_frames(cache, codec, max_audio_frames)
    finally:
        codec.reset_state(B)


def stream_generate(model: CSM, text, speaker: int, context: List[Segment], max_audio_length_ms: float = 90_000,
                    *, temperature: float = 0.8, logits_processors: Optional[List[Callable]] = None,
                    stream: Any = default_stream, sampler=None, seed=None) -> Generator[np.ndarray, None, None]:
    """generation.py:181-258: yields (1920,) float32 PCM per generated frame.

    Codec streaming state is per call (the reference resets a process-global Mimi,
    generation.py:224-225, :258)."""
    max_audio_frames = int(max_audio_length_ms / 80)
    t, m = build_prompt(model, text, speaker, context)
    _check_window(model, t.shape[0], max_audio_frames)
    smp = _resolve_sampler(temperature, sampler)
    codec = get_audio_tokenizer(model.n_audio_codebooks)
    cache = FrameCache(model, 1, smp, seed)
    cache.prefill(0, t, m)
    codec.reset_state(1)
    try:
        if isinstance(smp, HostSampler):
            frames = _host_sampled_frames(cache, codec, max_audio_frames, smp, logits_processors)
        elif logits_processors:
            frames = _processed_frames(cache, codec, max_audio_frames, logits_processors)
        else:
            frames = _overlapped_frames(cache, codec, max_audio_frames)
        for pcm, _ in frames:
            yield pcm[0]
    finally:
        codec.reset_state(1)
