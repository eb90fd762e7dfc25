"""CPU ORACLE -- numpy fp32 restatement of the Mimi codec used by the reference.

TEST INFRASTRUCTURE ONLY (see csm_oracle.py header for the import rule).

The reference calls moshi-mlx ``Mimi(mimi_202407(n_q))`` (un-vendored dependency,
``moshi-mlx>=0.2.3``, /root/reference/pyproject.toml:14) at:
  * encode       /root/reference/csm_mlx/tokenizers.py:61-85  (``Mimi.encode``)
  * decode       /root/reference/csm_mlx/tokenizers.py:148-150 (``Mimi.decode``)
  * decode_step  /root/reference/csm_mlx/generation.py:224-258 (``decode_step``, ``reset_state``)

moshi-mlx is absent here; this file restates its published algorithm (SEANet
causal convs, 8-layer transformer, split RVQ), as recalled from moshi-mlx 0.2.x:
  - causal StreamingConv1d: left pad (k_eff - stride) (+ right "extra" padding
    for a partial last frame), ``constant`` padding except the replicate-padded
    downsample;  ConvTranspose trims (k - stride) samples on the right;
  - transformer: LayerNorm(eps 1e-5) pre-norm, fused in_proj, RoPE
    ``traditional=True`` (interleaved pairs) base 10000, LayerScale, FFN with
    ``gelu_approx`` (tanh);  attention ``attn_mode``:
      "mlx"    -- moshi_mlx ``Attention.__call__``: no mask inside a call, keys =
                  the last ``t + min(context, past)`` positions;
      "causal" -- Kyutai PyTorch / transformers: causal with a 250-step window;
  - EuclideanCodebook.encode: argmin over ``|c|^2/2 - x.c`` (first minimum).
The architecture (attention modes aside) is cross-checked against the
independent in-container ``transformers.MimiModel`` (tests/test_oracle_mimi.py,
causal mode, permuted q/k for rotate_half RoPE, gelu_pytorch_tanh).
Against moshi-mlx itself this file is **parity unpinned**.
"""
from __future__ import annotations

import math
from typing import Dict

import numpy as np

F32 = np.float32


def elu(x):
    return np.where(x > 0, x, np.expm1(np.minimum(x, 0))).astype(F32)


def gelu(x, mode="tanh"):
    x = x.astype(F32)
    if mode == "tanh":
        c = F32(math.sqrt(2.0 / math.pi))
        return (F32(0.5) * x * (F32(1) + np.tanh(c * (x + F32(0.044715) * x * x * x)))).astype(F32)
    from scipy.special import erf
    return (0.5 * x * (1 + erf(x / math.sqrt(2)))).astype(F32)


def extra_padding(length: int, k_eff: int, stride: int, padding_total: int) -> int:
    n_frames = (length - k_eff + padding_total) / stride + 1
    ideal = (math.ceil(n_frames) - 1) * stride + (k_eff - padding_total)
    return ideal - length


def conv1d(x, w, b, stride=1, dil=1, pad_mode="constant"):
    """Causal StreamingConv1d forward (non-streaming). x (B,Cin,T), w (Cout,Cin,k)."""
    B, Cin, T = x.shape
    Cout, _, k = w.shape
    k_eff = (k - 1) * dil + 1
    pt = k_eff - stride
    ep = extra_padding(T, k_eff, stride, pt)
    if pad_mode == "replicate":
        x = np.concatenate([np.repeat(x[:, :, :1], pt, axis=2), x, np.repeat(x[:, :, -1:], ep, axis=2)], axis=2)
    else:
        x = np.pad(x, ((0, 0), (0, 0), (pt, ep)))
    Tp = x.shape[2]
    Tout = (Tp - k_eff) // stride + 1
    idx = np.arange(Tout)[:, None] * stride + np.arange(k)[None, :] * dil      # (Tout, k)
    cols = x[:, :, idx]                                                         # (B, Cin, Tout, k)
    cols = cols.transpose(0, 2, 1, 3).reshape(B, Tout, Cin * k)
    y = np.matmul(cols, w.reshape(Cout, Cin * k).T).transpose(0, 2, 1)
    if b is not None:
        y = y + b[None, :, None]
    return y.astype(F32)


def conv_transpose1d(x, w, b, stride, groups=1):
    """Causal StreamingConvTranspose1d: full transposed conv then trim (k - stride) on the right.
    x (B,Cin,T); w (Cin, Cout/groups, k)."""
    B, Cin, T = x.shape
    _, cpg, k = w.shape
    Cout = cpg * groups
    full = np.zeros((B, Cout, (T - 1) * stride + k), F32)
    if groups == 1:
        contrib = np.einsum("bct,cok->botk", x, w, optimize=True)                  # (B,Cout,T,k)
    else:
        assert cpg == 1 and groups == Cin
        contrib = x[:, :, :, None] * w[:, 0, :][None, :, None, :]                    # (B,C,T,k)
    for j in range(k):
        full[:, :, j: j + (T - 1) * stride + 1: stride] += contrib[:, :, :, j]
    y = full[:, :, : full.shape[2] - (k - stride)]
    if b is not None:
        y = y + b[None, :, None]
    return y.astype(F32)


def layer_norm(x, w, b, eps):
    x = x.astype(F32)
    mu = x.mean(-1, keepdims=True, dtype=F32)
    var = ((x - mu) ** 2).mean(-1, keepdims=True, dtype=F32)
    return ((x - mu) / np.sqrt(var + F32(eps)) * w + b).astype(F32)


def rope_traditional(x, offset, base):
    """mlx nn.RoPE(traditional=True): rotate (x[2i], x[2i+1]) by pos * base^(-2i/d). x (B,H,T,hd)."""
    B, H, T, hd = x.shape
    inv = (F32(1.0) / np.power(F32(base), (np.arange(0, hd, 2, dtype=F32) / F32(hd)), dtype=F32)).astype(F32)
    pos = (np.arange(T, dtype=F32) + F32(offset))
    ang = np.outer(pos, inv).astype(F32)
    c, s = np.cos(ang)[None, None], np.sin(ang)[None, None]
    xs = x.reshape(B, H, T, hd // 2, 2)
    x0, x1 = xs[..., 0], xs[..., 1]
    return np.stack([x0 * c - x1 * s, x0 * s + x1 * c], -1).reshape(B, H, T, hd).astype(F32)


class TransformerRef:
    def __init__(self, w, prefix, m):
        self.w, self.p, self.m = w, prefix, m

    def new_cache(self):
        return [{"k": None, "v": None, "offset": 0} for _ in range(self.m.num_layers)]

    def attn(self, l, x, cache):
        m, w = self.m, self.w
        p = f"{self.p}.transformer.layers.{l}.self_attn"
        B, T, d = x.shape
        H = m.num_heads
        hd = d // H
        qkv = np.matmul(x, w[f"{p}.in_proj_weight"].T).astype(F32).reshape(B, T, 3, H, hd)
        q, k, v = (qkv[:, :, i].transpose(0, 2, 1, 3) for i in range(3))
        off = cache["offset"]
        q = rope_traditional(q, off, m.max_period)
        k = rope_traditional(k, off, m.max_period)
        K = k if cache["k"] is None else np.concatenate([cache["k"], k], axis=2)
        Vv = v if cache["v"] is None else np.concatenate([cache["v"], v], axis=2)
        cache["k"], cache["v"], cache["offset"] = K, Vv, off + T
        S = K.shape[2]
        s = np.matmul(q, K.transpose(0, 1, 3, 2)).astype(F32) * F32(hd ** -0.5)
        qpos = off + np.arange(T)[:, None]
        kpos = np.arange(S)[None, :]
        if m.attn_mode == "mlx":
            keep = np.broadcast_to(kpos >= S - (T + min(m.context, S - T)), (T, S))
        else:
            keep = (kpos <= qpos) & (qpos - kpos < m.context)
        s = np.where(keep, s, F32(-np.inf))
        s = s - s.max(-1, keepdims=True)
        pr = np.exp(s)
        pr = pr / pr.sum(-1, keepdims=True)
        o = np.matmul(pr.astype(F32), Vv).astype(F32).transpose(0, 2, 1, 3).reshape(B, T, d)
        return np.matmul(o, w[f"{p}.out_proj.weight"].T).astype(F32)

    def __call__(self, x_bct, cache):
        """conv layout in/out (B,C,T)."""
        m, w = self.m, self.w
        x = x_bct.transpose(0, 2, 1).astype(F32)
        for l in range(m.num_layers):
            p = f"{self.p}.transformer.layers.{l}"
            n1 = layer_norm(x, w[f"{p}.norm1.weight"], w[f"{p}.norm1.bias"], m.norm_eps)
            x = (x + w[f"{p}.layer_scale_1.scale"] * self.attn(l, n1, cache[l])).astype(F32)
            n2 = layer_norm(x, w[f"{p}.norm2.weight"], w[f"{p}.norm2.bias"], m.norm_eps)
            h = gelu(np.matmul(n2, w[f"{p}.linear1.weight"].T).astype(F32), m.gelu)
            x = (x + w[f"{p}.layer_scale_2.scale"] * np.matmul(h, w[f"{p}.linear2.weight"].T).astype(F32)).astype(F32)
        return x.transpose(0, 2, 1)


class OracleMimi:
    def __init__(self, m, weights: Dict[str, np.ndarray]):
        from csm_mlx.weights import mimi_layout, mimi_codebook   # layout tables only
        self.m = m
        self.w = {k: np.asarray(v, F32) for k, v in weights.items()}
        self.enc_layout, self.dec_layout = mimi_layout(m)
        self.enc_tr = TransformerRef(self.w, "encoder_transformer", m)
        self.dec_tr = TransformerRef(self.w, "decoder_transformer", m)
        self.cb_first = [mimi_codebook(self.w, "rvq_first", 0)]
        self.cb_rest = [mimi_codebook(self.w, "rvq_rest", k) for k in range(m.n_q - 1)]
        self.reset_state()

    # ------------------------------------------------------------------ SEANet
    def _res(self, p, meta, x):
        w = self.w
        y = conv1d(elu(x), w[f"{p}.block.1.conv.conv.weight"], w[f"{p}.block.1.conv.conv.bias"], 1, meta["dil"])
        y = conv1d(elu(y), w[f"{p}.block.3.conv.conv.weight"], w[f"{p}.block.3.conv.conv.bias"])
        return (x + y).astype(F32)

    def _seanet(self, layout, x):
        w = self.w
        for kind, p, meta in layout:
            if kind == "conv":
                if meta["elu"]:
                    x = elu(x)
                x = conv1d(x, w[f"{p}.conv.conv.weight"], w[f"{p}.conv.conv.bias"], meta["stride"], meta["dil"])
            elif kind == "convtr":
                x = conv_transpose1d(elu(x), w[f"{p}.convtr.convtr.weight"], w[f"{p}.convtr.convtr.bias"], meta["stride"])
            else:
                x = self._res(p, meta, x)
        return x

    # ------------------------------------------------------------------ RVQ
    @staticmethod
    def vq_encode(x_btd, cb):
        """moshi_mlx EuclideanCodebook.encode: argmin(|c|^2/2 - x.c), first minimum."""
        c2 = (cb * cb).sum(-1, dtype=F32) / F32(2)
        dot = np.matmul(x_btd, cb.T).astype(F32)
        return np.argmin(c2 - dot, axis=-1)

    @staticmethod
    def vq_margin(x_btd, cb, ref_norm=None):
        """Sensitivity margin of the nearest-code choice (test bookkeeping, not part of the codec): with
        d_j = |c_j|^2/2 - x.c_j, best j1 and runner-up j2, (d_j2 - d_j1) / (|h| |c_j1 - c_j2|), |h| =
        ref_norm (the quantizer's projected latent at that frame; default |x|).  Perturbing the latent by
        delta moves the gap by at most |delta| |c_j1 - c_j2|, so a choice can flip under another summation
        order of the latent only where this is below that order's relative error |delta| / |h|.
        Returns (margin (B,T), runner-up index (B,T))."""
        d = ((cb * cb).sum(-1, dtype=F32) / F32(2) - np.matmul(x_btd, cb.T).astype(F32)).astype(np.float64)
        order = np.argsort(d, axis=-1, kind="stable")
        j1, j2 = order[..., 0], order[..., 1]
        gap = np.take_along_axis(d, j2[..., None], -1)[..., 0] - np.take_along_axis(d, j1[..., None], -1)[..., 0]
        hn = np.linalg.norm(x_btd.astype(np.float64), axis=-1) if ref_norm is None else ref_norm
        den = hn * np.linalg.norm(cb[j1].astype(np.float64) - cb[j2].astype(np.float64), axis=-1)
        return gap / np.maximum(den, 1e-30), j2

    def rvq_encode(self, q, x_bct, cbs, margins=None, force=None):
        """margins: a list that receives each codebook's (margin, runner-up) (vq_margin); force: {(b, t, k)}
        of codes to take as the runner-up instead of the nearest code (the other outcome of a near-tie,
        for the parity tests' variant prompts); the residual chain then continues from that choice."""
        w = self.w
        h = np.matmul(w[f"quantizer.{q}.input_proj.weight"][:, :, 0], x_bct).astype(F32)   # (B,cd,T)
        r = h.transpose(0, 2, 1).copy()
        hn = np.linalg.norm(r.astype(np.float64), axis=-1)
        codes = []
        for k, cb in enumerate(cbs):
            idx = self.vq_encode(r, cb)
            if margins is not None or force:
                mg, j2 = self.vq_margin(r, cb, hn)
                if margins is not None:
                    margins.append((mg, j2))
                for (b, t, kk) in (force or ()):
                    if kk == k:
                        idx[b, t] = j2[b, t]
            r = (r - cb[idx]).astype(F32)
            codes.append(idx)
        return np.stack(codes, axis=1).astype(np.int32)                                      # (B,nq,T)

    def _rvq_decode(self, q, codes_bkt, cbs):
        w = self.w
        acc = np.zeros((codes_bkt.shape[0], codes_bkt.shape[2], cbs[0].shape[1]), F32)
        for k in range(codes_bkt.shape[1]):
            acc = (acc + cbs[k][np.clip(codes_bkt[:, k], 0, self.m.bins - 1)]).astype(F32)
        return np.matmul(w[f"quantizer.{q}.output_proj.weight"][:, :, 0], acc.transpose(0, 2, 1)).astype(F32)

    def quantizer_decode(self, codes):
        y = self._rvq_decode("rvq_first", codes[:, :1], self.cb_first)
        if codes.shape[1] > 1:
            y = y + self._rvq_decode("rvq_rest", codes[:, 1:], self.cb_rest)
        return y.astype(F32)

    def upsample(self, x):
        return conv_transpose1d(x, self.w["upsample.convtr.convtr.convtr.weight"], None,
                                self.m.downsample_stride, groups=x.shape[1])

    # ------------------------------------------------------------------ public
    def encode(self, pcm_b1n: np.ndarray, with_margins: bool = False, force=()) -> np.ndarray:
        """Mimi.encode: (B,1,N) -> (B,n_q,Tf) int32.  with_margins: also return each code's RVQ margin
        (B,n_q,Tf) (vq_margin); force: codes (b, codebook, t) taken as the runner-up (rvq_encode)."""
        x = self._seanet(self.enc_layout, pcm_b1n.astype(F32))
        x = self.enc_tr(x, self.enc_tr.new_cache())
        x = conv1d(x, self.w["downsample.conv.conv.conv.weight"], None, self.m.downsample_stride, 1, "replicate")
        self.debug_latent = x
        ms = [] if with_margins else None
        sem = self.rvq_encode("rvq_first", x, self.cb_first, ms, {(b, t, 0) for b, k, t in force if k == 0})
        ac = self.rvq_encode("rvq_rest", x, self.cb_rest, ms, {(b, t, k - 1) for b, k, t in force if k > 0})
        codes = np.concatenate([sem, ac], axis=1)
        if with_margins:
            return codes, np.stack([m for m, _ in ms], axis=1)
        return codes

    def decode(self, codes_bkf: np.ndarray) -> np.ndarray:
        """Mimi.decode: (B,n_q,F) -> (B,1,F*frame_size)."""
        x = self.upsample(self.quantizer_decode(codes_bkf))
        x = self.dec_tr(x, self.dec_tr.new_cache())
        return self._seanet(self.dec_layout, x)

    def reset_state(self):
        self._tr_cache = self.dec_tr.new_cache()
        self._qhist = None
        self._hist = None
        self._emitted = 0

    def decode_step(self, codes_bk1: np.ndarray, window: int = 0) -> np.ndarray:
        """Mimi.decode_step on one frame (B,n_q,1) -> (B,1,frame_size).

        The causal convs (upsample, SEANet) are evaluated on the whole history,
        which equals their streaming state machine exactly; the transformer keeps
        a real KV cache so the "mlx" attention mode sees the keys streaming sees.
        window > 0: the SEANet decoder runs on the last `window` frames of history
        only (its receptive field is < 5 frames, so for window >= 8 the new frame's
        samples are the same values up to BLAS summation order -- checked in
        tests/test_oracle_cpu.py); linear instead of quadratic in the frames."""
        q = self.quantizer_decode(codes_bk1)
        self._qhist = q if self._qhist is None else np.concatenate([self._qhist, q], axis=2)
        s = self.m.downsample_stride
        new = self.upsample(self._qhist[:, :, -2:])[:, :, -s:]   # (depthwise k = 2 s: the last two frames)
        y = self.dec_tr(new, self._tr_cache)
        self._hist = y if self._hist is None else np.concatenate([self._hist, y], axis=2)
        fs = self.m.frame_size
        if window > 0:
            pcm = self._seanet(self.dec_layout, self._hist[:, :, -window * s:])
            out = pcm[:, :, -fs:]
        else:
            pcm = self._seanet(self.dec_layout, self._hist)
            out = pcm[:, :, self._emitted: self._emitted + fs]
        self._emitted += fs
        return out
