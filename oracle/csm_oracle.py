"""CPU ORACLE -- numpy fp32 restatement of the reference CSM hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module; the product path
(csm-mlx_amd/) never does.

Parity status: the reference (MLX, mlx-lm, moshi-mlx) cannot be imported or run
in this container (ModuleNotFoundError, no network) and
ships no tests, fixtures or golden vectors, so this restatement is
**parity unpinned** against the reference itself.  It follows the reference
sources line by line as a spec:

  * frame step            /root/reference/csm_mlx/generation.py:21-92
  * generate loop / EOS   /root/reference/csm_mlx/generation.py:95-178
  * embeddings            /root/reference/csm_mlx/models.py:79-92
  * Llama-3 scaled RoPE   /root/reference/csm_mlx/attention.py:10-177
  * GQA attention         /root/reference/csm_mlx/attention.py:180-253
  * Llama block / RMSNorm mlx_lm.models.llama (TransformerBlock, MLP) as wired
                          by /root/reference/csm_mlx/models.py:50-77
  * LoRA / DoRA adapters  mlx_lm.tuner LoRALinear / DoRALinear / LoRAEmbedding /
                          DoRAEmbedding forwards (unfused), as wrapped by
                          /root/reference/csm_mlx/finetune/utils.py:16-108

Sampling with temperature cannot reproduce MLX's RNG; it restates the build's
own counter-based Gumbel-max sampler (``gumbel_u``) so GPU sampled codes can be
checked bit-for-bit against this file.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import numpy as np

F32 = np.float32


# ----------------------------------------------------------------------------- RoPE
def llama3_rope_theta(dim: int, base: float, scale_factor: float, low_freq_factor: float = 1.0,
                      high_freq_factor: float = 4.0, old_context_len: int = 8192) -> np.ndarray:
    """attention.py:57-79 (rope_init) + :94-117 (apply_scaling), in float32 as MLX does."""
    expo = (np.arange(0, dim, 2, dtype=F32)[: dim // 2] / F32(dim)).astype(F32)
    freqs = (F32(1.0) / np.power(F32(base), expo, dtype=F32)).astype(F32)
    low_freq_wavelen = old_context_len / low_freq_factor
    high_freq_wavelen = old_context_len / high_freq_factor
    out = []
    for freq in freqs:
        wavelen = F32(2 * math.pi) / freq                      # mx float32 scalar math
        if wavelen < high_freq_wavelen:
            out.append(freq)
        elif wavelen > low_freq_wavelen:
            out.append(freq / F32(scale_factor))
        else:
            smooth = (F32(old_context_len) / wavelen - F32(low_freq_factor)) / F32(high_freq_factor - low_freq_factor)
            out.append((F32(1) - smooth) * freq / F32(scale_factor) + smooth * freq)
    return np.array(out, dtype=F32)


def rope_cache(theta: np.ndarray, max_seq_len: int = 2048) -> np.ndarray:
    """attention.py:81-92 -> (max_seq_len, dim//2, 2) = [cos, sin]."""
    seq = np.arange(max_seq_len, dtype=F32)
    idx_theta = np.outer(seq, theta).astype(F32)
    return np.stack([np.cos(idx_theta), np.sin(idx_theta)], axis=-1).astype(F32)


def rope_apply(x: np.ndarray, cache: np.ndarray, offset: int) -> np.ndarray:
    """attention.py:119-177: interleaved pairs (2i, 2i+1), fp32.  x: (B, T, H, hd)."""
    b, t, h, hd = x.shape
    if offset + t > cache.shape[0]:
        raise ValueError("RoPE position beyond the cached 2048-position table (attention.py:152)")
    c = cache[offset: offset + t].reshape(1, t, 1, hd // 2, 2)
    xs = x.astype(F32).reshape(b, t, h, hd // 2, 2)
    x0, x1 = xs[..., 0], xs[..., 1]
    out = np.stack([x0 * c[..., 0] - x1 * c[..., 1], x1 * c[..., 0] + x0 * c[..., 1]], axis=-1)
    return out.reshape(b, t, h, hd).astype(F32)


# ----------------------------------------------------------------------------- blocks
def rms_norm(x: np.ndarray, w: np.ndarray, eps: float) -> np.ndarray:
    """mlx fast.rms_norm: x * rsqrt(mean(x^2) + eps) * w, fp32 internally."""
    x = x.astype(F32)
    ms = np.mean(x * x, axis=-1, keepdims=True, dtype=F32)
    return (x * (F32(1) / np.sqrt(ms + F32(eps))) * w).astype(F32)


def linear(x: np.ndarray, w: np.ndarray) -> np.ndarray:
    """nn.Linear without bias: y = x @ W.T with W (out, in)."""
    return np.matmul(x, w.T).astype(F32)


def adapted_linear(x: np.ndarray, w: np.ndarray, ad: Optional[dict]) -> np.ndarray:
    """mlx_lm LoRALinear / DoRALinear forward, unfused (finetune/utils.py:33-50 wraps the layer):
    LoRA  y = x W^T + scale (x A) B;  DoRA  y = (m / ||W + scale B^T A^T||_row) (x W^T + scale (x A) B).
    ad: {"a": (in, r), "b": (r, out), "scale": s, "m": (out,) or None}."""
    y = linear(x, w)
    if ad is None:
        return y
    z = (y + F32(ad["scale"]) * np.matmul(np.matmul(x, ad["a"]), ad["b"])).astype(F32)
    if ad.get("m") is not None:
        wf = w + (F32(ad["scale"]) * ad["b"].T) @ ad["a"].T
        z = (ad["m"] / np.linalg.norm(wf, axis=1).astype(F32)).astype(F32) * z
    return z.astype(F32)


def adapted_embedding(idx: np.ndarray, w: np.ndarray, ad: Optional[dict]) -> np.ndarray:
    """mlx_lm LoRAEmbedding / DoRAEmbedding forward: y = E[i] + scale A[i] B, DoRA rows rescaled
    by m[i] / ||E[i] + scale A[i] B||."""
    y = w[idx]
    if ad is None:
        return y
    z = (y + np.matmul(ad["a"][idx], F32(ad["scale"]) * ad["b"])).astype(F32)
    if ad.get("m") is not None:
        z = (ad["m"][idx] / np.linalg.norm(z, axis=-1).astype(F32))[..., None] * z
    return z.astype(F32)


def silu(x):
    return (x / (F32(1) + np.exp(-x))).astype(F32)


def sdpa(q, k, v, scale, causal_offset: Optional[int]):
    """softmax(q k^T * scale + mask) v; q (B,H,T,hd), k/v (B,H,S,hd); causal iff T>1."""
    s = np.matmul(q, np.swapaxes(k, -1, -2)).astype(F32) * F32(scale)
    T, S = q.shape[2], k.shape[2]
    if causal_offset is not None and T > 1:
        qi = np.arange(T)[:, None] + causal_offset
        kj = np.arange(S)[None, :]
        s = np.where(kj <= qi, s, F32(-np.inf))
    s = s - s.max(-1, keepdims=True)
    p = np.exp(s)
    p = p / p.sum(-1, keepdims=True)
    return np.matmul(p.astype(F32), v).astype(F32)


class KVCacheRef:
    """mlx_lm KVCache semantics: append at offset, return the [:offset] view."""

    def __init__(self):
        self.k = None
        self.v = None
        self.offset = 0

    def update_and_fetch(self, k, v):
        self.k = k if self.k is None else np.concatenate([self.k, k], axis=2)
        self.v = v if self.v is None else np.concatenate([self.v, v], axis=2)
        self.offset = self.k.shape[2]
        return self.k, self.v


class LlamaRef:
    """mlx_lm LlamaModel with embed_tokens=Identity and the reference Attention patched in."""

    def __init__(self, w: Dict[str, np.ndarray], prefix: str, args, adapters: Optional[Dict[str, dict]] = None):
        self.w, self.p, self.a = w, prefix, args
        self.adapters = adapters or {}
        rs = args.rope_scaling
        theta = llama3_rope_theta(args.head_dim, args.rope_theta, rs.get("factor", 1.0),
                                  1.0, 4.0, 8192)   # attention.py:201-205 passes only base/scale_factor
        self.rope = rope_cache(theta, 2048)

    def attention(self, i, x, cache: KVCacheRef):
        a, w, p = self.a, self.w, f"{self.p}.layers.{i}.self_attn"
        b, t, _ = x.shape
        hd, H, Hkv = a.head_dim, a.num_attention_heads, a.num_key_value_heads
        q = self.lin(x, f"{p}.q_proj").reshape(b, t, H, hd)
        k = self.lin(x, f"{p}.k_proj").reshape(b, t, Hkv, hd)
        v = self.lin(x, f"{p}.v_proj").reshape(b, t, Hkv, hd)
        off = cache.offset
        q = rope_apply(q, self.rope, off)
        k = rope_apply(k, self.rope, off)
        q, k, v = (np.swapaxes(z, 1, 2) for z in (q, k, v))
        k, v = cache.update_and_fetch(k, v)
        rep = H // Hkv
        k = np.repeat(k, rep, axis=1)
        v = np.repeat(v, rep, axis=1)
        o = sdpa(q, k, v, hd ** -0.5, off)
        o = np.swapaxes(o, 1, 2).reshape(b, t, H * hd)
        return self.lin(o, f"{p}.o_proj")

    def lin(self, x, path):
        return adapted_linear(x, self.w[path + ".weight"], self.adapters.get(path))

    def __call__(self, x, caches: List[KVCacheRef]):
        a, w = self.a, self.w
        h = x.astype(F32)
        for i in range(a.num_hidden_layers):
            p = f"{self.p}.layers.{i}"
            r = self.attention(i, rms_norm(h, w[f"{p}.input_layernorm.weight"], a.rms_norm_eps), caches[i])
            h = (h + r).astype(F32)
            n = rms_norm(h, w[f"{p}.post_attention_layernorm.weight"], a.rms_norm_eps)
            g = self.lin(n, f"{p}.mlp.gate_proj")
            u = self.lin(n, f"{p}.mlp.up_proj")
            h = (h + self.lin((silu(g) * u).astype(F32), f"{p}.mlp.down_proj")).astype(F32)
        return rms_norm(h, w[f"{self.p}.norm.weight"], a.rms_norm_eps)


# ----------------------------------------------------------------------------- sampler (build's own RNG)
MASK64 = (1 << 64) - 1


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & np.uint64(MASK64)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def gumbel_u(seed: int, step: int, n: int) -> np.ndarray:
    """Uniform (0,1) doubles for vocab indices 0..n-1 of one sampling event.

    key = splitmix64(splitmix64(seed) ^ step) ; u_v = ((splitmix64(key ^ v) >> 11) + 0.5) * 2^-53
    (csm-mlx_amd/csrc/csm_kernels.hip ``sample_gumbel`` implements the same).
    """
    with np.errstate(over="ignore"):
        k = splitmix64(np.array([seed & MASK64], dtype=np.uint64))
        k = splitmix64(k ^ np.uint64(step & MASK64))
        h = splitmix64(k ^ np.arange(n, dtype=np.uint64))
    return ((h >> np.uint64(11)).astype(np.float64) + 0.5) * (2.0 ** -53)


def topk_threshold(logits: np.ndarray, k: int) -> float:
    """k-th largest value; every logit >= it is kept (ties at the boundary all kept)."""
    if k <= 0 or k >= logits.shape[-1]:
        return -np.inf
    return float(np.sort(logits)[::-1][k - 1])


def filter_keep(logits: np.ndarray, top_k: int, top_p: float, min_p: float, min_keep: int) -> np.ndarray:
    """The kept set of mlx_lm ``make_sampler``'s filter chain (sample_utils: apply_top_k, then
    apply_top_p, then apply_min_p, then categorical_sampling), restated on the log-probabilities
    ``lp = logits - logsumexp(logits)`` that mlx_lm's generate hands its sampler:

      * top_k: keep lp >= the k-th largest (ties at the k-th value kept; mlx argpartition breaks them
        arbitrarily);
      * top_p: probs = exp(lp) (0 where masked, not renormalised), cumulative sum in ascending
        order; keep where it exceeds float32(1 - top_p);
      * min_p: keep lp >= max(kept lp) + float32(log(min_p)), and always the first min_keep entries
        of the descending order (if still kept).
    Order for the sorts: lp descending, equal values by index ascending (ascending = its reverse).
    Sums are float32 (np.cumsum order); the GPU sums the same values in a parallel order, so a
    top_p boundary within float32 rounding of 1 - top_p may fall differently (never seen in tests).
    The same holds for min_p: lse (np.sum order here, a DPP / wave-ordered sum on the GPU) enters every
    lp, so an entry within float32 rounding of the min_p threshold may be kept on one side only.
    If every entry is removed the arg-max is kept (mlx would sample from an all -inf row).
    Parity of this chain against mlx_lm itself is unpinned (mlx_lm is not importable here and the
    reference holds no sampler fixture; its generate() samples with plain categorical,
    generation.py:51-54)."""
    l = logits.astype(F32)
    n = l.shape[-1]
    keep = l >= topk_threshold(l, top_k)
    if (0.0 < top_p < 1.0) or min_p != 0.0:
        mx_ = l.max()
        lse = F32(mx_ + F32(np.log(np.sum(np.exp(l - mx_, dtype=F32), dtype=F32))))
        lp = (l - lse).astype(F32)
        order = np.lexsort((np.arange(n), -lp.astype(np.float64)))        # lp desc, index asc
        if 0.0 < top_p < 1.0:
            p_desc = np.where(keep[order], np.exp(lp[order]), F32(0)).astype(F32)
            cum_asc = np.cumsum(p_desc[::-1], dtype=F32)[::-1]           # ascending cumsum, back in desc order
            kp = np.zeros(n, bool)
            kp[order] = cum_asc > F32(1.0 - top_p)
            keep &= kp
        if min_p != 0.0 and keep.any():
            top = lp[keep].max()
            tmin = F32(top + F32(math.log(min_p)))
            rank = np.empty(n, np.int64)
            rank[order] = np.arange(n)
            keep &= ~(lp < tmin) | (rank < min_keep)
    if not keep.any():
        keep[int(np.argmax(l))] = True
    return keep


def sample_one(logits: np.ndarray, temperature: float, top_k: int, seed: int, step: int,
               top_p: float = 0.0, min_p: float = 0.0, min_keep: int = 1) -> int:
    """Greedy = first max (mx.argmax); else Gumbel-max of logits*(1/temp) over the kept set
    (top-k; with top_p / min_p the mlx_lm filter chain, ``filter_keep``)."""
    logits = logits.astype(F32)
    if temperature == 0:
        return int(np.argmax(logits))
    keep = filter_keep(logits, top_k, top_p, min_p, min_keep)
    scaled = (logits * (F32(1.0) / F32(temperature))).astype(F32).astype(np.float64)
    u = gumbel_u(seed, step, logits.shape[-1])
    g = -np.log(-np.log(u))
    val = np.where(keep, scaled + g, -np.inf)
    return int(np.argmax(val))


# ----------------------------------------------------------------------------- CSM
class OracleCSM:
    """Restatement of ``CSM`` (models.py:31-92) + ``generate_frame`` (generation.py:21-92)."""

    def __init__(self, args, weights: Dict[str, np.ndarray], bb_args, dec_args,
                 adapters: Optional[Dict[str, dict]] = None):
        """adapters: module path -> LoRA/DoRA tensors (see ``adapted_linear``), applied unfused."""
        self.args = args
        self.w = {k: np.asarray(v, dtype=F32) for k, v in weights.items()}
        self.ad = adapters or {}
        self.backbone = LlamaRef(self.w, "backbone", bb_args, self.ad)
        self.decoder = LlamaRef(self.w, "decoder", dec_args, self.ad)
        self.bb_args, self.dec_args = bb_args, dec_args
        self.V, self.K = args.n_audio_vocab, args.n_audio_codebooks
        self.debug = {}

    def new_backbone_cache(self):
        return [KVCacheRef() for _ in range(self.bb_args.num_hidden_layers)]

    def embed_audio(self, codebook: int, tokens: np.ndarray) -> np.ndarray:
        return adapted_embedding(tokens + codebook * self.V, self.w["audio_embeddings.weight"],
                                 self.ad.get("audio_embeddings"))                    # models.py:79-80

    def embed_tokens(self, tokens: np.ndarray) -> np.ndarray:                   # models.py:82-92
        text = adapted_embedding(tokens[:, :, -1], self.w["text_embeddings.weight"],
                                 self.ad.get("text_embeddings"))[:, :, None, :]
        audio_tokens = tokens[:, :, :-1] + self.V * np.arange(self.K)
        audio = adapted_embedding(audio_tokens.reshape(-1), self.w["audio_embeddings.weight"],
                                  self.ad.get("audio_embeddings")).reshape(*tokens.shape[:2], self.K, -1)
        return np.concatenate([audio, text], axis=-2)

    def frame(self, tokens, mask, cache, temperature=0.0, top_k=0, seeds=None, frame_idx=0,
              processors=None, c0_history=None, top_p=0.0, min_p=0.0, min_keep=1, sampler=None):
        """generation.py:21-92.  tokens/mask (B,T,33).  Returns codes (B,K) int32.
        processors: logits processors on c0 (:44-49), called with (stack(c0_history) or zeros((0,)),
        logits); c0 (B,1) is appended to c0_history when it is a list (:60-61).
        sampler: a callable logits (B, V) -> codes (B,) used for every codebook instead of the built-in
        greedy / Gumbel sampler (the sampler= keyword of the reference CLI, cli/generate.py:197-199)."""
        B = tokens.shape[0]
        emb = self.embed_tokens(tokens) * mask[..., None].astype(F32)              # :34-35
        x = np.zeros(emb.shape[:2] + emb.shape[3:], F32)
        for j in range(emb.shape[2]):                                              # :36 sum over 33, in order
            x = x + emb[:, :, j]
        h = self.backbone(x, cache)                                                # :39
        h_last = h[:, -1, :]                                                       # :40
        c0_logits = adapted_linear(h_last, self.w["codebook0_head.weight"], self.ad.get("codebook0_head"))  # :42
        for proc in processors or []:                                              # :44-49
            hist = np.stack(c0_history, 0) if c0_history else np.zeros((0,), np.int32)
            c0_logits = np.asarray(proc(hist, c0_logits), F32)
        self.debug["c0_logits"] = c0_logits
        self.debug["h_last"] = h_last
        seeds = seeds if seeds is not None else [0] * B
        flt = dict(top_p=top_p, min_p=min_p, min_keep=min_keep)
        if sampler is not None:
            c0 = np.asarray(sampler(c0_logits), np.int64).reshape(B)
        else:
            c0 = np.array([sample_one(c0_logits[b], temperature, top_k, seeds[b], frame_idx * self.K, **flt)
                           for b in range(B)], dtype=np.int64)                    # :51-54
        out = np.zeros((B, self.K), np.int32)
        out[:, 0] = c0
        if c0_history is not None:
            c0_history.append(c0[:, None].astype(np.int32))
        dec_in = np.stack([h_last, self.embed_audio(0, c0)], axis=1)               # :57-64
        dcache = [KVCacheRef() for _ in range(self.dec_args.num_hidden_layers)]   # :70 fresh per frame
        ci_logits_all = []
        for i in range(1, self.K):                                                 # :72
            z = self.decoder(adapted_linear(dec_in, self.w["projection.weight"], self.ad.get("projection")),
                             dcache)                                               # :74-77
            logits = np.matmul(z[:, -1, :], self.w["audio_head"][i - 1]).astype(F32)   # :79 (in,out) layout
            ci_logits_all.append(logits)
            if sampler is not None:
                ci = np.asarray(sampler(logits), np.int64).reshape(B)
            else:
                ci = np.array([sample_one(logits[b], temperature, top_k, seeds[b], frame_idx * self.K + i, **flt)
                               for b in range(B)], dtype=np.int64)
            out[:, i] = ci
            dec_in = self.embed_audio(i, ci)[:, None, :]                          # :87-89
        self.debug["ci_logits"] = np.stack(ci_logits_all, axis=1)
        return out

    def generate_codes(self, prompt_tokens: np.ndarray, prompt_mask: np.ndarray, max_frames: int,
                       temperature=0.0, top_k=0, seed=0, max_seq_len=2048, collect_logits=False,
                       processors=None, top_p=0.0, min_p=0.0, min_keep=1, sampler=None):
        """generation.py:95-178 up to (not including) decode_audio.  prompt (L,33).

        Returns (codes (F,K) int32 up to EOS, logits list if requested)."""
        L = prompt_tokens.shape[0]
        if L >= max_seq_len - max_frames:                                          # :132-137
            raise ValueError(f"Inputs too long ({L}), must be below max_seq_len - max_audio_frames: "
                             f"{max_seq_len - max_frames}")
        cache = self.new_backbone_cache()
        inp, msk = prompt_tokens[None].astype(np.int64), prompt_mask[None].astype(bool)
        samples, logs, c0_history = [], [], []                                     # :128
        for f in range(max_frames):                                                # :139
            s = self.frame(inp, msk, cache, temperature, top_k, [seed], f, processors, c0_history,
                           top_p=top_p, min_p=min_p, min_keep=min_keep, sampler=sampler)
            if collect_logits:
                logs.append((self.debug["c0_logits"][0].copy(), self.debug["ci_logits"][0].copy()))
            if not s.any():                                                        # :151 EOS
                break
            samples.append(s[0])
            inp = np.concatenate([s, np.zeros((1, 1), np.int32)], axis=1)[:, None, :].astype(np.int64)   # :156
            msk = np.concatenate([np.ones_like(s, bool), np.zeros((1, 1), bool)], axis=1)[:, None, :]   # :159
        codes = np.stack(samples) if samples else np.zeros((0, self.K), np.int32)
        return (codes, logs) if collect_logits else codes


def text_frame(ids, n_codebooks: int = 32) -> (np.ndarray, np.ndarray):
    """tokenizers.py:43-58 given already-tokenized ids: (n,K+1) tokens with ids in the last col."""
    ids = np.asarray(ids, dtype=np.int32)
    t = np.zeros((len(ids), n_codebooks + 1), np.int32)
    m = np.zeros((len(ids), n_codebooks + 1), bool)
    t[:, -1] = ids
    m[:, -1] = True
    return t, m


def audio_frame(codes_kt: np.ndarray) -> (np.ndarray, np.ndarray):
    """tokenizers.py:69-85: (K,T) codes -> append EOS zero frame -> (T+1, 33) rows, mask cols 0..K-1."""
    K, T = codes_kt.shape
    c = np.concatenate([codes_kt, np.zeros((K, 1), codes_kt.dtype)], axis=1)
    t = np.zeros((T + 1, K + 1), np.int32)
    m = np.zeros((T + 1, K + 1), bool)
    t[:, :-1] = c.T
    m[:, :-1] = True
    return t, m


# ----------------------------------------------------------------------------- compute_loss
def compute_loss_ref(o: "OracleCSM", batch, per_sample: bool = False, cause_mismatch: bool = False):
    """/root/reference/csm_mlx/finetune/trainer.py:203-318, whole-sequence form: one causal backbone
    call over rows [0, S-1), codebook0_head on every position, one causal decoder call over the
    (B*(S-1), K+1) rows [h_t, E_0(c_0), ..., E_{K-1}(c_{K-1})] of the next frame, masked means of
    the cross entropies."""
    tokens = np.asarray(batch["tokens"]).astype(np.int64)
    masks = np.asarray(batch["masks"]).astype(bool)
    loss_masks = np.asarray(batch["loss_masks"]).astype(bool)
    w0 = F32(batch["first_codebook_weight_multiplier"])
    B, S, n_cb = tokens.shape
    K = n_cb - 1
    tgt = tokens[:, 1:, :K]                                                        # :220-221
    lm = masks[:, 1:, :K] & loss_masks[:, 1:, :K]                                  # :263-265
    emb = o.embed_tokens(tokens) * masks[..., None].astype(F32)                    # :232-233
    x = np.zeros(emb.shape[:2] + emb.shape[3:], F32)
    for j in range(emb.shape[2]):
        x = x + emb[:, :, j]
    h = o.backbone(x[:, :-1], o.new_backbone_cache())                              # :234-239
    c0_logits = adapted_linear(h, o.w["codebook0_head.weight"], o.ad.get("codebook0_head"))
    ci = np.stack([o.embed_audio(i, tgt[:, :, i]) for i in range(K)], axis=-2)     # :243-249
    dec_in = np.concatenate([h[:, :, None, :], ci], axis=-2).reshape(-1, n_cb, h.shape[-1])
    dcache = [KVCacheRef() for _ in range(o.dec_args.num_hidden_layers)]
    proj = adapted_linear(dec_in, o.w["projection.weight"], o.ad.get("projection"))
    dh = o.decoder(proj, dcache).reshape(B, S - 1, n_cb, -1)[:, :, 1:-1, :]        # :257-262
    if cause_mismatch:                                                             # :266-269
        tgt = np.concatenate([tgt[:, 1:], tgt[:, :1]], axis=1)

    def ce(logits, t):
        lg = logits.astype(np.float64)
        m = lg.max(-1, keepdims=True)
        lse = np.log(np.exp(lg - m).sum(-1)) + m[..., 0]
        return lse - np.take_along_axis(lg, t[..., None], -1)[..., 0]

    def masked_mean(v, msk):
        return (v * msk).sum(-1) / msk.sum(-1) if per_sample else (v * msk).sum() / msk.sum()
    with np.errstate(invalid="ignore", divide="ignore"):
        total = masked_mean(ce(c0_logits, tgt[:, :, 0]), lm[:, :, 0]) * w0 / K         # :271-289
        for i in range(1, K):                                                          # :291-312
            logits = np.matmul(dh[:, :, i - 1, :], o.w["audio_head"][i - 1])
            total = total + masked_mean(ce(logits, tgt[:, :, i]), lm[:, :, i]) / K
    return total
