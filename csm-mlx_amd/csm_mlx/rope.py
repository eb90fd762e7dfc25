"""RoPE cos/sin tables uploaded to the engine (computed once on the host, float32).

``llama3_rope_table`` restates ``Llama3ScaledRoPE.rope_init`` / ``apply_scaling`` /
``build_rope_cache`` (/root/reference/csm_mlx/attention.py:57-117) exactly as the
reference evaluates it: float32 frequencies, per-frequency scaling rule with
wavelength thresholds old_context_len/high (2048) and old_context_len/low (8192),
a [max_seq_len, dim/2, 2] cache of (cos, sin).  The reference passes only
``base`` and ``scale_factor`` (attention.py:201-205), so low/high/old_context
keep their defaults 1 / 4 / 8192.

``mimi_rope_table`` is the same table for moshi_mlx ``nn.RoPE(head_dim,
traditional=True, base=max_period)`` (no scaling) used by the codec transformer.
"""
from __future__ import annotations

import math

import numpy as np

F32 = np.float32


def _freqs(dim: int, base: float) -> np.ndarray:
    expo = (np.arange(0, dim, 2, dtype=F32)[: dim // 2] / F32(dim)).astype(F32)
    return (F32(1.0) / np.power(F32(base), expo, dtype=F32)).astype(F32)


def llama3_scaled_theta(dim, base, scale_factor, low_freq_factor=1.0, high_freq_factor=4.0, old_context_len=8192):
    freqs = _freqs(dim, base)
    low_wl = old_context_len / low_freq_factor
    high_wl = old_context_len / high_freq_factor
    out = np.empty_like(freqs)
    for i, f in enumerate(freqs):
        wl = F32(2 * math.pi) / f
        if wl < high_wl:
            out[i] = f
        elif wl > low_wl:
            out[i] = f / F32(scale_factor)
        else:
            smooth = (F32(old_context_len) / wl - F32(low_freq_factor)) / F32(high_freq_factor - low_freq_factor)
            out[i] = (F32(1) - smooth) * f / F32(scale_factor) + smooth * f
    return out


def table_from_theta(theta: np.ndarray, n_pos: int) -> np.ndarray:
    idx = np.outer(np.arange(n_pos, dtype=F32), theta).astype(F32)
    return np.ascontiguousarray(np.stack([np.cos(idx), np.sin(idx)], axis=-1).astype(F32))


def llama3_rope_table(args, max_seq_len: int = 2048) -> np.ndarray:
    factor = float(args.rope_scaling.get("factor", 1.0)) if args.rope_scaling else 1.0
    theta = llama3_scaled_theta(args.head_dim, args.rope_theta, factor)
    return table_from_theta(theta, max_seq_len)


def mimi_rope_table(m, n_pos: int) -> np.ndarray:
    hd = m.dimension // m.num_heads
    return table_from_theta(_freqs(hd, m.max_period), n_pos)
