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
and so is ``make_sampler(xtc_probability=...)`` (XTC has no GPU counterpart: the chain runs there),
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
                 top_k: int = 0, xtc_probability: float = 0.0, xtc_threshold: float = 0.0,
                 xtc_special_tokens=(), seed: int = 0, **_unused):
    """mlx_lm.sample_utils.make_sampler (as cli/generate.py:168-174 calls it) as a GPU sampler
    descriptor.  XTC ("exclude top choices", which the reference CLI never passes) has no GPU
    counterpart: with ``xtc_probability > 0`` and ``temp > 0`` the whole chain runs on the host as a
    ``HostSampler`` (``xtc_chain``); at ``temp == 0`` mlx_lm ignores XTC and so does this."""
    if not (0.0 <= top_p <= 1.0) or not (0.0 <= min_p <= 1.0) or int(min_tokens_to_keep) < 1:
        raise ValueError("top_p and min_p must lie in [0, 1], min_tokens_to_keep >= 1")
    if not (0.0 <= xtc_probability <= 1.0) or not (0.0 <= xtc_threshold <= 0.5):
        raise ValueError("xtc_probability must lie in [0, 1] and xtc_threshold in [0, 0.5]")
    if xtc_probability > 0.0 and temp != 0:
        return HostSampler(xtc_chain(float(temp), float(top_p), float(min_p), int(min_tokens_to_keep), int(top_k),
                                     float(xtc_probability), float(xtc_threshold), tuple(xtc_special_tokens), seed),
                           logprobs=True)
    return Sampler(float(temp), int(top_k), float(top_p), float(min_p), int(min_tokens_to_keep))


def xtc_chain(temp, top_p, min_p, min_tokens_to_keep, top_k, xtc_probability, xtc_threshold,
              xtc_special_tokens=(), seed: int = 0):
    """mlx_lm's make_sampler chain with XTC, on host log-probabilities (B, V): top_k (exactly k kept),
    top_p (cumulative ascending probability > 1 - top_p), min_p (log p >= log p_max + log min_p, the
    first ``min_tokens_to_keep`` by rank always kept), then XTC as mlx_lm's ``apply_xtc`` -- ONE
    uniform draw per call (for the whole batch) decides whether XTC applies, and the floor is ONE
    minimum over the whole (B, V) array of the probabilities above ``xtc_threshold`` (``.min()`` with
    no axis); every token whose probability exceeds that floor is removed (special tokens exempt) --
    then a categorical draw of ``logprobs / temp``.  At B = 1 the per-call and per-row forms agree; at
    B > 1 this keeps mlx_lm's batch-global form.  Restated from mlx_lm's published sample_utils (not in
    /root/reference, which never enables XTC): parity unpinned; the arithmetic is pinned on hand-worked
    rows in tests/test_abi_cpu.py."""
    import numpy as np
    rng = np.random.default_rng(seed)
    special = np.asarray(list(xtc_special_tokens), np.int64)

    def fn(lp):
        x = mlx_filter(lp, top_k, top_p, min_p, min_tokens_to_keep)
        ninf = -np.inf
        p = np.exp(x - x.max(axis=-1, keepdims=True))
        p /= p.sum(axis=-1, keepdims=True)
        floor = np.where(p > xtc_threshold, p, np.inf).min()          # batch-global, as mlx_lm
        mask = p > floor
        if special.size:
            mask[:, special] = False
        if not rng.random() > xtc_probability:                          # one draw per call
            x = np.where(mask, ninf, x)
        g = -np.log(-np.log(rng.random(x.shape)))
        return np.argmax(x / temp + g, axis=-1)
    return fn


def mlx_filter(lp, top_k, top_p, min_p, min_tokens_to_keep):
    """mlx_lm's top_k -> top_p -> min_p on host log-probabilities (B, V): the removed entries -inf
    (float64; top_k keeps exactly k, as mlx's argpartition)."""
    import numpy as np
    x = np.array(lp, np.float64)
    ninf = -np.inf
    if top_k > 0 and top_k < x.shape[-1]:
        drop = np.argpartition(-x, top_k - 1, axis=-1)[:, top_k:]
        np.put_along_axis(x, drop, ninf, axis=-1)
    if 0.0 < top_p < 1.0:
        order = np.argsort(x, axis=-1, kind="stable")
        cum = np.cumsum(np.take_along_axis(np.exp(x), order, axis=-1), axis=-1)
        cp = np.empty_like(cum)
        np.put_along_axis(cp, order, cum, axis=-1)
        x = np.where(cp > 1 - top_p, x, ninf)
    if min_p != 0.0:
        order = np.argsort(-x, axis=-1, kind="stable")
        srt = np.take_along_axis(x, order, axis=-1)
        rem = srt < srt[:, :1] + np.log(min_p)
        rem[:, :min_tokens_to_keep] = False
        rm = np.empty_like(rem)
        np.put_along_axis(rm, order, rem, axis=-1)
        x = np.where(rm, ninf, x)
    return x


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

