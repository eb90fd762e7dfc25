"""Parameter inventories and seeded synthetic weights (CSM + Mimi).

The real checkpoints (``senstella/csm-1b-mlx``, ``kyutai/moshiko-pytorch-bf16``)
are not available offline, so every run uses synthetic weights generated from
a seed.  Each tensor draws from its own NumPy PCG64
stream keyed by ``(seed, crc32(name))`` so any subset can be regenerated
independently and bit-identically on the GPU box and in the CPU oracle.

CSM key names follow the MLX module tree of the reference
(/root/reference/csm_mlx/models.py:31-77, mlx_lm ``LlamaModel`` children).
Mimi key names follow the Kyutai PyTorch checkpoint that the reference feeds
to ``Mimi.load_pytorch_weights`` (/root/reference/csm_mlx/tokenizers.py:16-19);
those names are recalled from moshi, not verifiable offline.
"""
from __future__ import annotations

import math
import zlib
from typing import Dict, Iterable, Optional, Tuple

import numpy as np

from .config import BACKBONE_CONFIGURATION, DECODER_CONFIGURATION, LlamaArgs, MimiArgs

# ----------------------------------------------------------------------------- bf16 helpers


def bf16_bits(a: np.ndarray) -> np.ndarray:
    """float32 -> bf16 bit pattern (uint16), round-to-nearest-even."""
    u = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)
    r = (u + np.uint32(0x7FFF) + ((u >> np.uint32(16)) & np.uint32(1))) >> np.uint32(16)
    return r.astype(np.uint16)


def bf16_to_f32(b: np.ndarray) -> np.ndarray:
    return (b.astype(np.uint32) << np.uint32(16)).view(np.float32)


def bf16_round(a: np.ndarray) -> np.ndarray:
    """Round a float32 array to the nearest bf16 value (returned as float32)."""
    return bf16_to_f32(bf16_bits(a))


# ----------------------------------------------------------------------------- CSM inventory

# kind: ("uniform", bound) | ("normal", std) | ("ones",) | ("zeros",) | ("const", v)
Spec = Tuple[Tuple[int, ...], tuple]


def _llama_specs(prefix: str, a: LlamaArgs) -> Dict[str, Spec]:
    d, hd = a.hidden_size, a.head_dim
    q, kv, f = a.num_attention_heads * hd, a.num_key_value_heads * hd, a.intermediate_size
    u = lambda fan_in: ("uniform", 1.0 / math.sqrt(fan_in))
    out: Dict[str, Spec] = {}
    for i in range(a.num_hidden_layers):
        p = f"{prefix}.layers.{i}"
        out[f"{p}.self_attn.q_proj.weight"] = ((q, d), u(d))
        out[f"{p}.self_attn.k_proj.weight"] = ((kv, d), u(d))
        out[f"{p}.self_attn.v_proj.weight"] = ((kv, d), u(d))
        out[f"{p}.self_attn.o_proj.weight"] = ((d, q), u(q))
        out[f"{p}.mlp.gate_proj.weight"] = ((f, d), u(d))
        out[f"{p}.mlp.up_proj.weight"] = ((f, d), u(d))
        out[f"{p}.mlp.down_proj.weight"] = ((d, f), u(f))
        out[f"{p}.input_layernorm.weight"] = ((d,), ("ones",))
        out[f"{p}.post_attention_layernorm.weight"] = ((d,), ("ones",))
    out[f"{prefix}.norm.weight"] = ((d,), ("ones",))
    return out


def csm_param_specs(args) -> Dict[str, Spec]:
    """Every parameter of ``CSM(args)`` with its shape and synthetic init.

    Shapes follow models.py:50-67: Linear weights are (out, in); ``audio_head`` is
    a raw (K-1, d_dec, V) array in (in, out) layout (used as ``h @ audio_head[i]``,
    generation.py:79).
    """
    bb = BACKBONE_CONFIGURATION[args.backbone_name]
    dec = DECODER_CONFIGURATION[args.decoder_name]
    D, Dd = bb.num_attention_heads * bb.head_dim, dec.num_attention_heads * dec.head_dim
    V, K = args.n_audio_vocab, args.n_audio_codebooks
    out: Dict[str, Spec] = {}
    out.update(_llama_specs("backbone", bb))
    out.update(_llama_specs("decoder", dec))
    out["text_embeddings.weight"] = ((args.n_text_vocab, D), ("normal", 1.0 / math.sqrt(D)))
    out["audio_embeddings.weight"] = ((V * K, D), ("normal", 1.0 / math.sqrt(D)))
    out["projection.weight"] = ((Dd, D), ("uniform", 1.0 / math.sqrt(D)))
    out["codebook0_head.weight"] = ((V, D), ("uniform", 1.0 / math.sqrt(D)))
    # reference inits zeros (models.py:65) which would make every ci == 0; use N(0, 1/sqrt(d_dec))
    out["audio_head"] = ((K - 1, Dd, V), ("normal", 1.0 / math.sqrt(Dd)))
    return out


def _rng(seed: int, name: str) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64([seed, zlib.crc32(name.encode())]))


def _draw(shape, kind, seed, name) -> np.ndarray:
    tag = kind[0]
    if tag == "ones":
        return np.ones(shape, np.float32)
    if tag == "zeros":
        return np.zeros(shape, np.float32)
    if tag == "const":
        return np.full(shape, kind[1], np.float32)
    g = _rng(seed, name)
    if tag == "uniform":
        b = np.float32(kind[1])
        x = g.random(shape, dtype=np.float32)
        x *= np.float32(2.0) * b
        x -= b
        return x
    if tag == "normal":
        x = g.standard_normal(shape, dtype=np.float32)
        x *= np.float32(kind[1])
        return x
    raise ValueError(kind)


def synthetic_csm_weights(args, seed: int = 0, names: Optional[Iterable[str]] = None,
                          mimi_bins: Optional[int] = None) -> Dict[str, np.ndarray]:
    """Seeded synthetic CSM weights (float32).

    Rows/columns of the c0/ci heads for ids >= ``mimi_bins`` (2048..2050 for csm_1b)
    are zeroed so greedy decoding never emits an id the Mimi codebook lacks
    (SURVEY.md section 8(d)).
    """
    specs = csm_param_specs(args)
    bins = mimi_bins if mimi_bins is not None else args.n_audio_vocab - 3
    out = {}
    for n in (names if names is not None else specs.keys()):
        shape, kind = specs[n]
        w = _draw(shape, kind, seed, n)
        if n == "codebook0_head.weight":
            w[bins:] = 0.0
        elif n == "audio_head":
            w[:, :, bins:] = 0.0
        out[n] = w
    return out


# ----------------------------------------------------------------------------- Mimi inventory


def mimi_layout(m: MimiArgs):
    """SEANet layer lists as (kind, key-prefix, meta) in execution order.

    Encoder indices follow moshi ``SEANetEncoder.model`` (ELU modules occupy
    indices too): 0 conv, then per ratio (4,5,6,8): resblock, ELU, strided conv;
    then ELU, final conv.  Decoder mirrors it with transposed convs.
    """
    enc, dec = [], []
    nf, rk = m.n_filters, m.residual_kernel_size
    idx = 0
    mult = 1
    enc.append(("conv", f"encoder.model.{idx}", dict(cin=m.channels, cout=mult * nf, k=m.kernel_size, stride=1, dil=1, elu=False)))
    idx += 1
    for ratio in reversed(m.ratios):
        ch = mult * nf
        enc.append(("res", f"encoder.model.{idx}", dict(ch=ch, hidden=ch // m.compress, k=rk, dil=1)))
        idx += 1
        idx += 1  # ELU
        enc.append(("conv", f"encoder.model.{idx}", dict(cin=ch, cout=ch * 2, k=ratio * 2, stride=ratio, dil=1, elu=True)))
        idx += 1
        mult *= 2
    idx += 1  # ELU
    enc.append(("conv", f"encoder.model.{idx}", dict(cin=mult * nf, cout=m.dimension, k=m.last_kernel_size, stride=1, dil=1, elu=True)))

    idx = 0
    mult = 2 ** len(m.ratios)
    dec.append(("conv", f"decoder.model.{idx}", dict(cin=m.dimension, cout=mult * nf, k=m.kernel_size, stride=1, dil=1, elu=False)))
    idx += 1
    for ratio in m.ratios:
        ch = mult * nf
        idx += 1  # ELU
        dec.append(("convtr", f"decoder.model.{idx}", dict(cin=ch, cout=ch // 2, k=ratio * 2, stride=ratio, elu=True)))
        idx += 1
        dec.append(("res", f"decoder.model.{idx}", dict(ch=ch // 2, hidden=ch // 2 // m.compress, k=rk, dil=1)))
        idx += 1
        mult //= 2
    idx += 1  # ELU
    dec.append(("conv", f"decoder.model.{idx}", dict(cin=nf, cout=m.channels, k=m.last_kernel_size, stride=1, dil=1, elu=True)))
    return enc, dec


def mimi_param_specs(m: MimiArgs) -> Dict[str, Spec]:
    out: Dict[str, Spec] = {}
    # variance-preserving conv init (uniform with var 1/fan_in) keeps the synthetic
    # signal O(1) through the ~15-conv SEANet stacks so RVQ codes stay diverse.
    cu = lambda fan_in: ("uniform", math.sqrt(3.0 / fan_in))
    enc, dec = mimi_layout(m)
    for kind, p, meta in enc + dec:
        if kind == "conv":
            fan = meta["cin"] * meta["k"]
            out[f"{p}.conv.conv.weight"] = ((meta["cout"], meta["cin"], meta["k"]), cu(fan))
            out[f"{p}.conv.conv.bias"] = ((meta["cout"],), ("uniform", 1.0 / math.sqrt(fan)))
        elif kind == "convtr":
            fan = meta["cin"] * meta["k"] // meta["stride"]
            out[f"{p}.convtr.convtr.weight"] = ((meta["cin"], meta["cout"], meta["k"]), cu(fan))
            out[f"{p}.convtr.convtr.bias"] = ((meta["cout"],), ("uniform", 1.0 / math.sqrt(fan)))
        else:  # resblock: block.1 = conv(k, ch->hidden), block.3 = conv(1, hidden->ch)
            ch, hid, k = meta["ch"], meta["hidden"], meta["k"]
            out[f"{p}.block.1.conv.conv.weight"] = ((hid, ch, k), cu(ch * k))
            out[f"{p}.block.1.conv.conv.bias"] = ((hid,), ("uniform", 1.0 / math.sqrt(ch * k)))
            out[f"{p}.block.3.conv.conv.weight"] = ((ch, hid, 1), cu(hid))
            out[f"{p}.block.3.conv.conv.bias"] = ((ch,), ("uniform", 1.0 / math.sqrt(hid)))
    d, f = m.dimension, m.dim_feedforward
    for tname in ("encoder_transformer", "decoder_transformer"):
        for l in range(m.num_layers):
            p = f"{tname}.transformer.layers.{l}"
            out[f"{p}.self_attn.in_proj_weight"] = ((3 * d, d), ("uniform", 1.0 / math.sqrt(d)))
            out[f"{p}.self_attn.out_proj.weight"] = ((d, d), ("uniform", 1.0 / math.sqrt(d)))
            out[f"{p}.norm1.weight"] = ((d,), ("ones",))
            out[f"{p}.norm1.bias"] = ((d,), ("zeros",))
            out[f"{p}.norm2.weight"] = ((d,), ("ones",))
            out[f"{p}.norm2.bias"] = ((d,), ("zeros",))
            out[f"{p}.linear1.weight"] = ((f, d), ("uniform", 1.0 / math.sqrt(d)))
            out[f"{p}.linear2.weight"] = ((d, f), ("uniform", 1.0 / math.sqrt(f)))
            out[f"{p}.layer_scale_1.scale"] = ((d,), ("const", m.layer_scale))
            out[f"{p}.layer_scale_2.scale"] = ((d,), ("const", m.layer_scale))
    s = m.downsample_stride
    out["downsample.conv.conv.conv.weight"] = ((d, d, 2 * s), cu(d * 2 * s))
    out["upsample.convtr.convtr.convtr.weight"] = ((d, 1, 2 * s), cu(2 * s // s))
    cd = m.codebook_dim
    for q, nq in (("rvq_first", 1), ("rvq_rest", m.n_q - 1)):
        out[f"quantizer.{q}.input_proj.weight"] = ((cd, d, 1), ("uniform", 1.0 / math.sqrt(d)))
        out[f"quantizer.{q}.output_proj.weight"] = ((d, cd, 1), ("uniform", 1.0 / math.sqrt(cd)))
        for k in range(nq):
            # codebook scale ~ the projected-embedding scale so nearest-neighbour picks vary
            out[f"quantizer.{q}.vq.layers.{k}._codebook.embedding_sum"] = ((m.bins, cd), ("normal", 0.1))
            out[f"quantizer.{q}.vq.layers.{k}._codebook.cluster_usage"] = ((m.bins,), ("ones",))
    return out


def synthetic_mimi_weights(m: MimiArgs, seed: int = 0) -> Dict[str, np.ndarray]:
    return {n: _draw(shape, kind, seed, n) for n, (shape, kind) in mimi_param_specs(m).items()}


def mimi_codebook(w: Dict[str, np.ndarray], q: str, k: int, eps: float = 1e-5) -> np.ndarray:
    """Effective codebook = embedding_sum / clamp(cluster_usage, eps) (moshi EuclideanCodebook)."""
    p = f"quantizer.{q}.vq.layers.{k}._codebook"
    usage = np.maximum(w[f"{p}.cluster_usage"], np.float32(eps))
    return (w[f"{p}.embedding_sum"] / usage[:, None]).astype(np.float32)
