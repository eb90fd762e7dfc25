"""LoRA / DoRA / full fine-tune adapters at inference: ``load_adapters(model, adapter_path)``.

Reference: /root/reference/csm_mlx/finetune/utils.py:16-108 (``linear_to_lora_layers`` +
``load_adapters``, itself mlx_lm.tuner.utils), which wraps the selected Linear / Embedding modules
in mlx_lm ``LoRALinear`` / ``DoRALinear`` / ``LoRAEmbedding`` / ``DoRAEmbedding`` and loads
``adapters.safetensors`` into them with ``strict=False``.

The frame engine keeps its weights resident on the GPU in the layouts its kernels read (QKV rows
stacked, gate/up interleaved, folded tables), so an adapter is applied the way mlx_lm's
``fuse`` does it: the low-rank update is folded into the base weight once, on load, and the
frame graph runs unchanged (no extra launches per step).  Per adapted module, in the stored dtype:

  LoRA Linear      W' = W + dt(scale * lora_b.T @ lora_a.T)         lora_a (in, r), lora_b (r, out)
  LoRA Embedding   E' = E + dt(scale * lora_a @ lora_b)             lora_a (n, r),  lora_b (r, d)
  DoRA (either)    the LoRA W' above, then rows rescaled by m / ||W'_row||   m (out,) / (n,)

``dt`` rounds to the engine's weight dtype (bf16 engines: the delta is rounded to bf16 before the
add, as ``delta.astype(dtype)`` does).  The unfused forward of the reference,
``x W^T + scale (x A) B``, differs from this only by rounding (tests/test_adapters_*.py).

Which modules are adapted follows ``linear_to_lora_layers``: for each transformer layer of the
backbone and decoder, the layer-relative names in ``lora_parameters.keys`` ("attn" adds the four
attention and three MLP projections); names relative to a stack; and CSM-level names
("projection", "codebook0_head", "text_embeddings", "audio_embeddings").  Adapter tensors for
modules that were not converted are ignored, as ``load_weights(strict=False)`` ignores them.
"""
from __future__ import annotations

import json
from pathlib import Path
from typing import Callable, Dict, Iterable, Optional, Set, Tuple

import numpy as np

from .weights import bf16_round, bf16_to_f32

_LAYER_LINEARS = ("self_attn.q_proj", "self_attn.k_proj", "self_attn.v_proj", "self_attn.o_proj",
                  "mlp.gate_proj", "mlp.up_proj", "mlp.down_proj")
_LAYER_OTHER = ("self_attn", "mlp", "input_layernorm", "post_attention_layernorm", "self_attn.rope")
_TOP_LINEARS = ("projection", "codebook0_head")
_TOP_EMBEDDINGS = ("text_embeddings", "audio_embeddings")
_TOP_OTHER = ("backbone", "decoder", "backbone.norm", "decoder.norm")


def _expand_keys(keys: Optional[Iterable[str]]) -> Set[str]:
    """finetune/utils.py:55-71: "attn" adds the attention and MLP projections."""
    ks = set(keys) if keys is not None else set()
    if "attn" in ks:
        ks.update(_LAYER_LINEARS)
    return ks


def converted_modules(model, keys: Optional[Iterable[str]]) -> Dict[str, str]:
    """Full module path -> "linear" | "embedding" for every module ``linear_to_lora_layers`` would
    wrap (finetune/utils.py:73-84).  Naming a module that is neither raises the reference's
    ``ValueError("Can't convert layer of type ...")`` (finetune/utils.py:43-45)."""
    ks = _expand_keys(keys)
    out: Dict[str, str] = {}

    def take(path: str, kind: Optional[str]):
        if kind is None:
            raise ValueError(f"Can't convert layer of type {path} to LoRA")
        out[path] = kind

    for stack, st in (("backbone", model.backbone), ("decoder", model.decoder)):
        for i in range(len(st.layers)):
            for rel in _LAYER_LINEARS + _LAYER_OTHER:
                full_rel = f"layers.{i}.{rel}"
                if rel in ks or full_rel in ks or f"{stack}.{full_rel}" in ks:   # layer / stack / CSM pass
                    take(f"{stack}.{full_rel}", "linear" if rel in _LAYER_LINEARS else None)
        if "norm" in ks:
            take(f"{stack}.norm", None)
    for name in _TOP_LINEARS:
        if name in ks:
            take(name, "linear")
    for name in _TOP_EMBEDDINGS:
        if name in ks:
            take(name, "embedding")
    for name in _TOP_OTHER:
        if name in ks:
            take(name, None)
    return out


def read_adapter_dir(adapter_path) -> Tuple[dict, Dict[str, np.ndarray]]:
    """adapter_config.json + adapters.safetensors (finetune/utils.py:96-107), as fp32 numpy."""
    p = Path(adapter_path)
    if not p.exists():
        raise FileNotFoundError(f"The adapter path does not exist: {p}")
    with open(p / "adapter_config.json", "r") as fid:
        config = json.load(fid)
    from safetensors import safe_open
    tensors: Dict[str, np.ndarray] = {}
    with safe_open(str(p / "adapters.safetensors"), framework="pt") as f:
        for k in f.keys():
            tensors[k] = f.get_tensor(k).float().numpy()
    return config, tensors


def _as_f32(a: np.ndarray) -> np.ndarray:
    a = np.asarray(a)
    if a.dtype == np.uint16:          # bf16 bit patterns (how bf16 checkpoints are handed over)
        return bf16_to_f32(a)
    if a.dtype == np.uint32:
        raise NotImplementedError("adapters over MLX-packed int4 base weights: load the float "
                                  "checkpoint, load_adapters, then nn.quantize")
    return np.ascontiguousarray(a, dtype=np.float32)


def fuse_module(base: np.ndarray, kind: str, lora_a: Optional[np.ndarray], lora_b: Optional[np.ndarray],
                scale: float, m: Optional[np.ndarray], dtype: str) -> np.ndarray:
    """One adapted module's fused weight (mlx_lm LoRALinear/DoRALinear/LoRAEmbedding/DoRAEmbedding
    ``fuse``), fp32 holding values of ``dtype`` ("float32" | "bf16").  ``lora_a``/``lora_b`` None:
    the zero-initialised update (a DoRA module whose file holds only ``m``)."""
    rnd = bf16_round if dtype == "bf16" else (lambda z: np.asarray(z, dtype=np.float32))
    w = rnd(_as_f32(base))
    fused = w
    if lora_a is not None and lora_b is not None:
        a = lora_a.astype(np.float32)
        b = lora_b.astype(np.float32)
        if kind == "linear":
            if a.shape[0] != w.shape[1] or b.shape[1] != w.shape[0] or a.shape[1] != b.shape[0]:
                raise ValueError(f"LoRA shapes {a.shape} x {b.shape} do not fit weight {w.shape}")
            delta = (np.float32(scale) * b.T) @ a.T
        else:
            if a.shape[0] != w.shape[0] or b.shape[1] != w.shape[1] or a.shape[1] != b.shape[0]:
                raise ValueError(f"LoRA shapes {a.shape} x {b.shape} do not fit embedding {w.shape}")
            delta = a @ (np.float32(scale) * b)
        fused = rnd(w + rnd(delta.astype(np.float32)))
    if m is not None:                                    # DoRA: rows rescaled to magnitude m
        if m.shape != (w.shape[0],):
            raise ValueError(f"DoRA magnitude {m.shape} does not fit {w.shape}")
        norm = np.sqrt(np.sum(fused.astype(np.float64) ** 2, axis=1)).astype(np.float32)
        fused = rnd((m.astype(np.float32) / norm)[:, None] * fused)
    return fused


def fuse_adapters(model, config: dict, tensors: Dict[str, np.ndarray],
                  base_weight: Callable[[str], np.ndarray]):
    """Yield (weight name, fused fp32 array) for every converted module with adapter tensors."""
    fine_tune_type = config.get("fine_tune_type", "lora")
    if fine_tune_type == "full":                         # finetune/utils.py:100-107: weights as-is
        yield from tensors.items()
        return
    lp = config["lora_parameters"]
    scale = float(lp["scale"])
    dora = fine_tune_type == "dora"
    for path, kind in converted_modules(model, lp.get("keys")).items():
        a, b = tensors.get(path + ".lora_a"), tensors.get(path + ".lora_b")
        m = tensors.get(path + ".m") if dora else None
        if (a is None or b is None) and m is None:
            continue                     # never trained: LoRA's zero-init lora_b leaves W unchanged
        name = path + ".weight"
        base = base_weight(name)
        if dora and m is None:
            # DoRALinear / DoRAEmbedding.from_base set m = ||W_base|| per row and load_weights(strict=False)
            # keeps it when the file has no .m: the fused rows are rescaled back to the base norms
            w = bf16_round(_as_f32(base)) if model.dtype == "bf16" else _as_f32(base)
            m = np.sqrt(np.sum(w.astype(np.float64) ** 2, axis=1)).astype(np.float32)
        yield name, fuse_module(base, kind, a, b, scale, m, model.dtype)


def load_adapters(model, adapter_path, base_weights=None):
    """finetune/utils.py:87-108.  Returns ``model`` with the adapters folded into its weights.

    The base weights are re-read from what ``model.load_weights`` was given (a checkpoint path or a
    dict); pass ``base_weights`` (path or dict) when the model was loaded from a one-shot iterator."""
    config, tensors = read_adapter_dir(adapter_path)
    if model.dtype == "q4":
        raise NotImplementedError("load_adapters on an int4 engine: load_adapters first, then nn.quantize")
    lookup = model.base_weight_lookup(base_weights)
    model.load_weights(list(fuse_adapters(model, config, tensors, lookup)), strict=False)
    return model
