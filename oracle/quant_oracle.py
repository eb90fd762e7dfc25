"""CPU ORACLE -- numpy restatement of MLX affine quantization (nn.quantize, group 64, 4 bits).

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module; the product path
(csm-mlx_amd/) never does.

What it restates.  The reference quantizes the whole CSM with
``nn.quantize(model, group_size, bits)`` (/root/reference/run_streaming_csm_mlx.py:811-818,
README.md:108-111).  That call swaps every ``nn.Linear`` for
``QuantizedLinear`` and every ``nn.Embedding`` for ``QuantizedEmbedding``; the raw
``audio_head`` array (models.py:65-67) and the RMSNorm weights are not modules of those
types and stay full precision.  The arithmetic lives in the un-vendored dependency
``mlx>=0.22.1`` (pyproject.toml:13): ``mx.quantize`` (affine, per group of ``group_size``
consecutive input elements of a row):

    w_max, w_min = max/min of the group
    scale = max((w_max - w_min) / (2^bits - 1), 1e-7)
    scale = scale if |w_min| > |w_max| else -scale
    edge  = w_min if |w_min| > |w_max| else w_max
    q0    = round(edge / scale)
    scale = edge / q0 if q0 != 0 else scale          (zero maps to the integer -q0 exactly)
    bias  = edge if q0 != 0 else 0
    q     = clip(round((w - bias) / scale), 0, 2^bits - 1)      packed 8 per uint32, element j
                                                                at bits 4*(j % 8) of word j // 8
    dequantize: w_hat = scale * q + bias

``round`` is round-half-to-even (``std::rint``).  This is recalled from mlx's
``quantize`` (mlx/ops.cpp), not verifiable offline: **parity unpinned** against MLX
itself.  The reference ships no quantized fixture.  The build's one addition,
documented in DESIGN.md: scale and bias are rounded to bf16 (the dtype of the
released bf16 checkpoint, in which MLX computes and stores them) before ``q`` is
computed, so the device stores 2 x bf16 per group (0.5625 B/param).  The property
MLX's own tests assert (python/tests/test_quantized.py: |w - w_hat| <= |scale|) is
checked in tests/test_quant_cpu.py.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


def _bf16_round(a: np.ndarray) -> np.ndarray:
    u = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)
    r = ((u + np.uint32(0x7FFF) + ((u >> np.uint32(16)) & np.uint32(1))) >> np.uint32(16)) << np.uint32(16)
    return r.view(np.float32)


def affine_quantize(w: np.ndarray, group_size: int = 64, bits: int = 4):
    """(packed uint32 (N, K*bits/32), scales f32 (N, K/g), biases f32 (N, K/g)); scales/biases hold bf16 values."""
    if bits != 4:
        raise ValueError("only 4-bit affine quantization is restated")
    w = np.ascontiguousarray(w, dtype=F32)
    N, K = w.shape
    if K % group_size:
        raise ValueError(f"last dim {K} not divisible by group size {group_size}")
    n_bins = F32((1 << bits) - 1)
    g = w.reshape(N, K // group_size, group_size)
    w_max = g.max(-1)
    w_min = g.min(-1)
    mask = np.abs(w_min) > np.abs(w_max)
    scale = np.maximum((w_max - w_min) / n_bins, F32(1e-7)).astype(F32)
    scale = np.where(mask, scale, -scale).astype(F32)
    edge = np.where(mask, w_min, w_max).astype(F32)
    q0 = np.rint(edge / scale).astype(F32)
    nz = q0 != 0
    with np.errstate(divide="ignore", invalid="ignore"):
        scale = np.where(nz, edge / np.where(nz, q0, F32(1)), scale).astype(F32)
    bias = np.where(nz, edge, F32(0)).astype(F32)
    scale = _bf16_round(scale)
    bias = _bf16_round(bias)
    q = np.clip(np.rint((g - bias[..., None]) / scale[..., None]), 0, n_bins).astype(np.uint32)
    q = q.reshape(N, K // 8, 8)
    packed = np.zeros((N, K // 8), np.uint32)
    for j in range(8):
        packed |= q[:, :, j] << np.uint32(4 * j)
    return packed, scale, bias


def unpack(packed: np.ndarray) -> np.ndarray:
    N, W = packed.shape
    q = np.empty((N, W, 8), np.uint32)
    for j in range(8):
        q[:, :, j] = (packed >> np.uint32(4 * j)) & np.uint32(15)
    return q.reshape(N, W * 8)


def dequantize(packed: np.ndarray, scales: np.ndarray, biases: np.ndarray, group_size: int = 64) -> np.ndarray:
    """mx.dequantize: scale * q + bias per group (fp32)."""
    q = unpack(packed).astype(F32)
    N, K = q.shape
    s = np.repeat(scales.astype(F32), group_size, axis=1)
    b = np.repeat(biases.astype(F32), group_size, axis=1)
    return (s * q + b).astype(F32)


def quantized_names(names):
    """Parameters nn.quantize replaces: every Linear / Embedding weight (not audio_head, not norms)."""
    out = []
    for n in names:
        if n == "audio_head" or n.endswith("norm.weight") or n.endswith("layernorm.weight"):
            continue
        if n.endswith(".weight"):
            out.append(n)
    return out


def quantize_dequantize_weights(weights: dict, group_size: int = 64) -> dict:
    """The fp32 weights an nn.quantize'd CSM computes with: w_hat for every quantized parameter."""
    out = dict(weights)
    for n in quantized_names(list(weights)):
        p, s, b = affine_quantize(np.asarray(weights[n], F32), group_size)
        out[n] = dequantize(p, s, b, group_size)
    return out
