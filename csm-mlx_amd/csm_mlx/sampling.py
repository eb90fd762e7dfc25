"""Sampler descriptors (mlx_lm ``make_sampler`` surface used by the reference CLI/README:
/root/reference/csm_mlx/cli/generate.py:168-174, README.md:49).

The sampler runs on the GPU inside the frame graph, so a sampler is a
descriptor (temperature, top_k, top_p, min_p, min_tokens_to_keep): greedy is first-max argmax; otherwise Gumbel-max over
``logits * (1/temp)`` restricted to the entries mlx_lm's filter chain keeps
(top_k -> top_p -> min_p on the log-probabilities; ties at the k-th value kept),
driven by a counter-based splitmix64 stream keyed by (seed, frame*K + codebook,
vocab id).  The filter chain's restatement is oracle/csm_oracle.py
``filter_keep``; the GPU side is ``sample_filtered_kernel`` (csm_kernels.hip).

An arbitrary callable (``sampler=fn``, as the reference CLI passes mlx_lm's sampler) is honoured too,
on the host: ``HostSampler`` wraps it, and every frame then hands each codebook's logits (B, V) to
``fn`` and feeds the codes it returns forward (csm_frame_host_step; 32 host round trips per frame,
so a compatibility path, not the fast one).
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class Sampler:
    temp: float = 0.0
    top_k: int = 0
    top_p: float = 0.0
    min_p: float = 0.0
    min_tokens_to_keep: int = 1

    @property
    def greedy(self) -> bool:
        return self.temp == 0

    @property
    def filtered(self) -> bool:
        """top_p / min_p active (mlx_lm make_sampler: top_p in (0, 1), min_p != 0)."""
        return 0.0 < self.top_p < 1.0 or self.min_p != 0.0


def make_sampler(temp: float = 0.0, top_p: float = 0.0, min_p: float = 0.0, min_tokens_to_keep: int = 1,
                 top_k: int = 0, xtc_probability: float = 0.0, **_unused) -> Sampler:
    """mlx_lm.sample_utils.make_sampler (as cli/generate.py:168-174 calls it) as a GPU sampler
    descriptor.  XTC sampling has no GPU counterpart and raises."""
    if xtc_probability:
        raise NotImplementedError("XTC sampling does not run on the GPU sampler")
    if not (0.0 <= top_p <= 1.0) or not (0.0 <= min_p <= 1.0) or int(min_tokens_to_keep) < 1:
        raise ValueError("top_p and min_p must lie in [0, 1], min_tokens_to_keep >= 1")
    return Sampler(float(temp), int(top_k), float(top_p), float(min_p), int(min_tokens_to_keep))


@dataclass(frozen=True)
class HostSampler:
    """A sampler callable run on the host for every codebook: fn(logits (B, V) float32) -> codes (B,)
    or (B, 1) ints.  (mlx_lm samplers take log-probabilities; ``logprobs=True`` hands fn
    logits - logsumexp(logits) instead.)"""
    fn: object
    logprobs: bool = False
    temp: float = 1.0        # the engine's sampler is unused on this path (every code comes from fn)
    top_k: int = 0
    top_p: float = 0.0
    min_p: float = 0.0
    min_tokens_to_keep: int = 1

    greedy = False
    filtered = False

    def __call__(self, logits):
        import numpy as np
        x = np.asarray(logits, np.float32)
        if self.logprobs:
            m = x.max(axis=-1, keepdims=True)
            x = x - (m + np.log(np.exp(x - m).sum(axis=-1, keepdims=True)))
        return np.asarray(self.fn(x)).reshape(x.shape[0]).astype(np.int32)

