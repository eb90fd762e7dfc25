"""``MimiCodec`` -- the GPU Mimi codec (drop-in for moshi_mlx ``Mimi`` as the reference uses it).

Methods mirror the calls the reference makes (/root/reference/csm_mlx/tokenizers.py:16-19, 70,
150; generation.py:225, 251, 258): ``load_pytorch_weights``, ``encode``, ``decode``,
``decode_step``, ``reset_state``.  All compute runs in libcsm_hip.so (mimi_* C ABI); codec
weights are kept in fp32 (waveform parity target 1e-4 RMS).
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Iterable, Optional, Tuple, Union

import numpy as np

from . import _lib
from .config import MimiArgs
from .rope import mimi_rope_table


def _dims(m: MimiArgs) -> _lib.MimiDims:
    r = (ctypes.c_int * 8)(*list(m.ratios) + [0] * (8 - len(m.ratios)))
    return _lib.MimiDims(m.channels, m.dimension, m.n_filters, len(m.ratios), r, m.kernel_size,
                         m.residual_kernel_size, m.last_kernel_size, m.compress, m.num_heads, m.num_layers,
                         m.dim_feedforward, m.context, m.n_q, m.bins, m.codebook_dim, m.downsample_stride,
                         m.norm_eps, 1 if m.gelu == "erf" else 0, 0 if m.attn_mode == "mlx" else 1)


class MimiCodec:
    def __init__(self, m: MimiArgs, *, device: Optional[int] = None, max_batch: int = 1, max_frames: int = 1200):
        from .models import default_device
        self.m = m
        self.device = default_device() if device is None else device
        self.max_batch = max_batch
        self.max_frames = max_frames
        L = _lib.lib()
        h = ctypes.c_void_p()
        _lib.check(L.mimi_create(ctypes.byref(_dims(m)), self.device, max_batch, max_frames, ctypes.byref(h)))
        self._h = h
        n_pos = 2 * max_frames * m.downsample_stride + 64
        t = mimi_rope_table(m, n_pos)
        _lib.check(L.mimi_set_rope_table(h, _lib.ptr(t), t.shape[0], t.shape[1] * 2))
        self._stream_B = None

    def __del__(self):
        try:
            if getattr(self, "_h", None) is not None:
                _lib.lib().mimi_destroy(self._h)
                self._h = None
        except Exception:
            pass

    # ------------------------------------------------------------------ weights
    def load_weights(self, weights: Union[Dict[str, np.ndarray], Iterable[Tuple[str, np.ndarray]]], strict=True):
        L = _lib.lib()
        items = weights.items() if isinstance(weights, dict) else weights
        for name, arr in items:
            a, dt = _lib.host_tensor(arr)
            rc = L.mimi_load_tensor(self._h, name.encode(), _lib.ptr(a), dt, _lib.shape_arr(a.shape), a.ndim)
            if rc != 0 and not strict:
                continue
            _lib.check(rc)
        if strict:
            _lib.check(L.mimi_weights_ready(self._h))
        return self

    def load_pytorch_weights(self, path: str):
        """Kyutai PyTorch checkpoint (safetensors), as moshi_mlx ``Mimi.load_pytorch_weights``
        (tokenizers.py:19).  Weight-normalised convs (weight_g / weight_v) are folded to plain
        weights, ``in_projs.0`` / ``out_projs.0`` spellings are aliased, unknown keys ignored."""
        from safetensors import safe_open
        raw = {}
        with safe_open(path, framework="pt") as f:
            for k in f.keys():
                raw[k] = f.get_tensor(k).float().numpy()
        out = {}
        for k, v in raw.items():
            if k.endswith(".weight_g"):
                continue
            if k.endswith(".weight_v"):
                g = raw[k[:-1] + "g"]
                norm = np.sqrt((v.astype(np.float64) ** 2).sum(axis=tuple(range(1, v.ndim)), keepdims=True))
                k, v = k[:-2], (g * v / norm).astype(np.float32)
            k = k.replace(".self_attn.in_projs.0.weight", ".self_attn.in_proj_weight")
            k = k.replace(".self_attn.out_projs.0.weight", ".self_attn.out_proj.weight")
            out[k] = v
        self.load_weights(out, strict=False)
        _lib.check(_lib.lib().mimi_weights_ready(self._h))
        return self

    # ------------------------------------------------------------------ codec
    def encode(self, pcm: np.ndarray) -> np.ndarray:
        """(B, 1, N) or (B, N) float32 -> (B, n_q, Tf) int32."""
        x = np.asarray(pcm, np.float32)
        if x.ndim == 3:
            x = x[:, 0, :]
        B, N = x.shape
        out = []
        for b0 in range(0, B, self.max_batch):
            xb = np.ascontiguousarray(x[b0: b0 + self.max_batch])
            nb = xb.shape[0]
            Tf = int(np.ceil(N / self.m.frame_size)) + 2
            codes = np.zeros((nb, self.m.n_q, Tf), np.int32)
            got = ctypes.c_int(0)
            _lib.check(_lib.lib().mimi_encode(self._h, nb, N, _lib.ptr(xb), _lib.ptr(codes), ctypes.byref(got)))
            out.append(codes.reshape(-1)[: nb * self.m.n_q * got.value].reshape(nb, self.m.n_q, got.value))
        return np.concatenate(out, 0)

    def encode_rows(self, rows) -> np.ndarray:
        """Same-length 1-D float32 clips -> (B, n_q, Tf) int32, as ``encode(np.stack(rows))`` without the
        stacking copy (each clip is uploaded into its slot: mimi_encode_rows)."""
        xs = [np.ascontiguousarray(r, np.float32).reshape(-1) for r in rows]
        if not xs or len({x.shape[0] for x in xs}) != 1:
            raise ValueError("encode_rows: same-length clips only")
        N = xs[0].shape[0]
        out = []
        for b0 in range(0, len(xs), self.max_batch):
            part = xs[b0: b0 + self.max_batch]
            nb = len(part)
            ptrs = (ctypes.c_void_p * nb)(*[x.ctypes.data for x in part])
            Tf = int(np.ceil(N / self.m.frame_size)) + 2
            codes = np.zeros((nb, self.m.n_q, Tf), np.int32)
            got = ctypes.c_int(0)
            _lib.check(_lib.lib().mimi_encode_rows(self._h, nb, N, None, ptrs, _lib.ptr(codes), ctypes.byref(got)))
            out.append(codes.reshape(-1)[: nb * self.m.n_q * got.value].reshape(nb, self.m.n_q, got.value))
        return np.concatenate(out, 0)

    def decode(self, codes: np.ndarray) -> np.ndarray:
        """(B, n_q, F) int32 -> (B, 1, F*frame_size) float32.  Resets streaming state (moshi_mlx)."""
        c = np.asarray(codes, np.int32)
        B, K, F = c.shape
        if K != self.m.n_q:
            raise ValueError(f"expected {self.m.n_q} codebooks, got {K}")
        out = []
        for b0 in range(0, B, self.max_batch):
            cb = np.ascontiguousarray(c[b0: b0 + self.max_batch])
            nb = cb.shape[0]
            pcm = np.zeros((nb, F * self.m.frame_size), np.float32)
            _lib.check(_lib.lib().mimi_decode(self._h, nb, F, _lib.ptr(cb), 0, 0, _lib.ptr(pcm), 0))
            out.append(pcm)
        self._stream_B = None
        return np.concatenate(out, 0)[:, None, :]

    def reset_state(self, batch_size: int = 1):
        _lib.check(_lib.lib().mimi_reset_state(self._h, batch_size))
        self._stream_B = batch_size

    def decode_step(self, codes: np.ndarray) -> np.ndarray:
        """One frame: (B, n_q, 1) or (B, n_q) -> (B, 1, frame_size)."""
        c = np.asarray(codes, np.int32)
        if c.ndim == 3:
            c = c[:, :, 0]
        B = c.shape[0]
        if self._stream_B != B:
            self.reset_state(B)
        c = np.ascontiguousarray(c)
        pcm = np.zeros((B, self.m.frame_size), np.float32)
        _lib.check(_lib.lib().mimi_decode_step(self._h, B, _lib.ptr(c), _lib.ptr(pcm)))
        return pcm[:, None, :]
