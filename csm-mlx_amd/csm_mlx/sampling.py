"""Sampler descriptors (mlx_lm ``make_sampler`` surface used by the reference CLI/README:
/root/reference/csm_mlx/cli/generate.py:168-174, README.md:49).

The sampler runs on the GPU inside the frame graph, so a sampler is a
descriptor (temperature, top_k) rather than an arbitrary callable: greedy is
first-max argmax; otherwise Gumbel-max over ``logits * (1/temp)`` restricted to
the top-k logits (ties at the k-th value kept), driven by a counter-based
splitmix64 stream keyed by (seed, frame*K + codebook, vocab id).
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class Sampler:
    temp: float = 0.0
    top_k: int = 0

    @property
    def greedy(self) -> bool:
        return self.temp == 0


def make_sampler(temp: float = 0.0, top_p: float = 0.0, min_p: float = 0.0, min_tokens_to_keep: int = 1,
                 top_k: int = 0, **_unused) -> Sampler:
    if top_p not in (0.0, 1.0) or min_p != 0.0:
        raise NotImplementedError("only temperature and top_k sampling run on the GPU sampler")
    return Sampler(float(temp), int(top_k))
