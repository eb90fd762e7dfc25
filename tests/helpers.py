"""Shared builders for the parity tests (test infrastructure)."""
import dataclasses
import functools

import numpy as np

from csm_mlx.config import BACKBONE_CONFIGURATION as BB, DECODER_CONFIGURATION as DC
from csm_mlx.weights import bf16_round, synthetic_csm_weights


@functools.lru_cache(maxsize=4)
def csm_weights(args_key, seed=0):
    from csm_mlx.models import csm_1b, csm_tiny
    args = {"tiny": csm_tiny, "1b": csm_1b}[args_key]()
    return args, synthetic_csm_weights(args, seed)


_ORACLES = {}


def oracle_for(args, weights, bf16=False, q4=False):
    """bf16: every weight rounded to bf16 (CSM dtype "bf16").  q4: nn.quantize'd CSM (dtype "q4"):
    Linear / Embedding weights quantize->dequantize (oracle/quant_oracle.py), audio_head bf16.
    Memoised per weight dict (the csm_weights dicts are cached): the csm_1b bf16 / int4 conversions
    take 10-45 s each (6 GB of fp32 per variant)."""
    key = (id(weights), bool(bf16), bool(q4))
    if key not in _ORACLES:
        _ORACLES[key] = _oracle_for(args, weights, bf16, q4)
    return _ORACLES[key]


def _oracle_for(args, weights, bf16, q4):
    from oracle.csm_oracle import OracleCSM
    from oracle.quant_oracle import quantize_dequantize_weights
    w = {k: bf16_round(v) for k, v in weights.items()} if bf16 else weights
    if q4:
        w = quantize_dequantize_weights(weights)
        w["audio_head"] = bf16_round(weights["audio_head"])
    return OracleCSM(args, w, BB[args.backbone_name], DC[args.decoder_name])


def prompt_ids(seed: int, n_mid: int = 12, vocab: int = 128000, bos: int = 128000, eos: int = 128001):
    """SURVEY 8(d) prompt recipe: BOS + n ids ~ U[0, vocab) + EOS."""
    rng = np.random.default_rng(seed)
    return [bos] + [int(x) for x in rng.integers(0, vocab, n_mid)] + [eos]


def tiny_prompt_ids(seed: int, n_mid: int = 5):
    rng = np.random.default_rng(seed)
    return [998] + [int(x) for x in rng.integers(0, 990, n_mid)] + [999]


def first_divergence(a: np.ndarray, b: np.ndarray):
    n = min(len(a), len(b))
    for i in range(n):
        if not np.array_equal(a[i], b[i]):
            return i
    return None if len(a) == len(b) else n


def make_adapters(model_handle, weights, fine_tune_type="lora", keys=("attn",), rank=4, scale=2.0,
                  seed=7, b_std=0.05):
    """Synthetic trained adapters for ``keys`` (mlx_lm LoRALinear naming: <module>.lora_a (in, r),
    .lora_b (r, out); LoRAEmbedding: lora_a (n, r), lora_b (r, d); DoRA adds .m).  Returns
    (adapter_config dict, flat tensors for adapters.safetensors, oracle adapters {path: dict})."""
    from csm_mlx.adapters import converted_modules
    rng = np.random.default_rng(seed)
    tensors, oracle_ad = {}, {}
    for path, kind in converted_modules(model_handle, list(keys)).items():
        w = np.asarray(weights[path + ".weight"], np.float32)
        n_in = w.shape[1] if kind == "linear" else w.shape[0]
        n_out = w.shape[0] if kind == "linear" else w.shape[1]
        bound = 1.0 / np.sqrt(n_in) if kind == "linear" else 1.0 / np.sqrt(rank)
        a = rng.uniform(-bound, bound, (n_in, rank)).astype(np.float32)
        b = (rng.standard_normal((rank, n_out)) * b_std).astype(np.float32)
        tensors[path + ".lora_a"], tensors[path + ".lora_b"] = a, b
        ad = {"a": a, "b": b, "scale": scale, "m": None}
        if fine_tune_type == "dora":
            m = (np.linalg.norm(w, axis=1) * rng.uniform(0.8, 1.2, w.shape[0])).astype(np.float32)
            tensors[path + ".m"] = m
            ad["m"] = m
        oracle_ad[path] = ad
    config = {"fine_tune_type": fine_tune_type,
              "lora_parameters": {"rank": rank, "scale": scale, "dropout": 0.0, "keys": list(keys)}}
    return config, tensors, oracle_ad


def write_adapter_dir(path, config, tensors):
    import json
    from safetensors.numpy import save_file
    path.mkdir(parents=True, exist_ok=True)
    (path / "adapter_config.json").write_text(json.dumps(config))
    save_file({k: np.ascontiguousarray(v) for k, v in tensors.items()}, str(path / "adapters.safetensors"))
    return path


def oracle_batch(o, prompts, frames, collect_logits=False, temperature=0.0, top_k=0, seeds=None, **flt):
    """Greedy oracle frames for many utterances at once: prompts (tokens, mask) of equal length run as
    one (B, L, 33) batch through OracleCSM.frame (the reference's generate_frame is batch-agnostic,
    generation.py:21-92).  Returns per utterance (codes (F_b, K), [(c0, ci) per frame] or None);
    an utterance that reaches EOS is re-run alone so its frame count follows generation.py:151.
    Sampling (temperature > 0) uses the oracle's restatement of the engine's counter-based RNG with
    one seed per utterance."""
    seeds = [0] * len(prompts) if seeds is None else list(seeds)
    groups = {}
    for i, (t, _) in enumerate(prompts):
        groups.setdefault(t.shape[0], []).append(i)
    out = [None] * len(prompts)
    for L, idx in groups.items():
        toks = np.stack([prompts[i][0] for i in idx]).astype(np.int64)
        msk = np.stack([prompts[i][1] for i in idx]).astype(bool)
        cache = o.new_backbone_cache()
        codes, logs = [], []
        for f in range(frames):
            s = o.frame(toks, msk, cache, temperature, top_k, [seeds[i] for i in idx], f, **flt)
            codes.append(s)
            if collect_logits:
                logs.append((o.debug["c0_logits"].copy(), o.debug["ci_logits"].copy()))
            toks = np.concatenate([s, np.zeros((len(idx), 1), np.int32)], 1)[:, None, :].astype(np.int64)
            msk = np.concatenate([np.ones_like(s, bool), np.zeros((len(idx), 1), bool)], 1)[:, None, :]
        codes = np.stack(codes, 1)                                    # (b, F, K)
        for j, i in enumerate(idx):
            if not codes[j].any(-1).all():                            # EOS inside the window: run alone
                res = o.generate_codes(prompts[i][0], prompts[i][1], frames, temperature, top_k, seeds[i],
                                       collect_logits=collect_logits, **flt)
                out[i] = res if collect_logits else (res, None)
            else:
                out[i] = (codes[j], [(c0[j], ci[j]) for c0, ci in logs] if collect_logits else None)
    return out


# ----------------------------------------------------------------------------- EOS-capable weights
EOS_RIG = dict(alpha=2.5, emb_norm=20.0, head_gain=0.5, seed=77)


def eos_rig(args, w, alpha=EOS_RIG["alpha"], emb_norm=EOS_RIG["emb_norm"], head_gain=EOS_RIG["head_gain"],
            seed=EOS_RIG["seed"]):
    """Seeded synthetic weights in which an utterance CAN end (test infrastructure).

    The reference stops an utterance at the first all-zero frame (generation.py:151).  With plain random
    weights all 32 codes are never 0 together, so EOS is never exercised.  The rig (documented here and
    in DESIGN.md; nothing else changes):
      * audio_embeddings row ``0 + V*j`` (code 0 of codebook j, j < K-1) = ``emb_norm`` x a seeded unit
        vector u_j -- ~20x a normal row, so when c_j = 0 the decoder's residual stream at the next step
        is dominated by projection(u_j);
      * audio_head[j][:, 0] (code 0 of codebook j+1) = ``head_gain`` x the unit direction of
        projection(u_j) -- logit 0 then leads by ~10 whenever c_j = 0: a zero code chains to the end of
        the frame (greedy and sampled alike);
      * codebook0_head row 0 scaled by ``alpha`` -- c0 = 0 (and so the all-zero frame) becomes an
        occasional event whose timing depends on the utterance.
    Returns a new dict (the input is not modified)."""
    V, K = args.n_audio_vocab, args.n_audio_codebooks
    rng = np.random.default_rng(seed)
    out = dict(w)
    emb = np.array(w["audio_embeddings.weight"], np.float32)
    ah = np.array(w["audio_head"], np.float32)
    wp = np.asarray(w["projection.weight"], np.float32)
    for j in range(K - 1):
        u = rng.standard_normal(emb.shape[1]).astype(np.float32)
        u *= emb_norm / np.linalg.norm(u)
        emb[j * V] = u
        d = wp @ u
        ah[j][:, 0] = head_gain * d / np.linalg.norm(d)
    c0 = np.array(w["codebook0_head.weight"], np.float32)
    c0[0] *= alpha
    out["audio_embeddings.weight"], out["audio_head"], out["codebook0_head.weight"] = emb, ah, c0
    return out


@functools.lru_cache(maxsize=2)
def eos_weights(args_key="1b", seed=0):
    args, w = csm_weights(args_key, seed)
    return args, eos_rig(args, w)
